// SpiralConv forward / backward kernels for gfx950 (CDNA4), fp32.
//
// Reference: SpiralConv.forward (model.py:27-41) = index_select of the
// spiral neighbourhood + nn.Linear(S*Cin -> Cout), and its autograd
// (index_add_ / addmm backward).  Here the gather is fused with the
// contraction: every 32-row output tile is one v_mfma_f32_32x32x2_f32
// accumulator chain whose A operand is gathered straight from HBM/L2 into
// VGPRs (each lane pair reads one 128-B neighbour row with 16-B loads) and
// whose B operand (the weights) is staged once per persistent workgroup in LDS.
//
// K ordering inside one spiral slot is permuted (lane half h owns channels
// [h*C/2, h*C/2 + C/2)): MFMA step j sums A[i][h]*B[h][n] over h, so slot s's
// dot product is accumulated as pairs (j, j + C/2).  This is exact f32 (the
// f32 MFMA is a k-ordered fmaf chain), only the summation order differs from
// ATen's sgemm.
//
// Channel counts of 3 (xyz in/out: the first Enblock and the last decoder
// conv) would waste 29/32 of an MFMA tile, so those layers run on VALU
// kernels shaped for them (lane-per-output-channel or 8-lanes-per-row).
#include "cfsd_common.h"
#include "conv_bf16.h"
#include "conv_vm32.h"
#include "conv_coarse.h"
#include "conv_lat.h"

namespace cfsd {


// Occupancy target per channel shape (min waves per SIMD -> VGPR budget).
constexpr int mfma_occ(int cin, int cout) { return (cin == 32 && cout == 32) ? 4 : 2; }

// ==========================================================================
// Forward, MFMA path: CIN, COUT in {32, 64}.  A wave owns 32-row tiles
// (two 16-row groups) of the flattened (b, r) row space and all COUT
// columns, in a persistent XCD-aware sweep.  MFMA v_mfma_f32_16x16x4_f32:
// lane (i = l&15, kg = l>>4) holds row i's 16-B chunks kg, kg+4, ... of each
// gathered neighbour row, so ONE gather instruction covers 16 rows x 64
// contiguous bytes (16 cache sectors) -- the 32x32x2 lane map needed 64 and
// made the gathers address-(TA-)bound.  K order inside a slot is permuted
// consistently for A and B (chunk-major), exact f32 as before.
// Slot groups: blockIdx.y = g handles slots [g*SPG, g*SPG + SPG); with
// SPG < 9 (layers with few rows) the partials go to ws[g][m][COUT] and
// conv_combine adds the groups (fixed order), bias and activation.
// W slice staged in LDS as [COUT][SPG*CIN + 8] (pad 8: conflict-free
// ds_read_b128 for this lane map).
template <int CIN, int COUT, int ACT, int SPG>
__global__ __launch_bounds__(256, mfma_occ(CIN, COUT)) void conv_fwd_mfma(
    const float* __restrict__ x, const int* __restrict__ idx, const float* __restrict__ w,
    const float* __restrict__ bias, float* __restrict__ y, float* __restrict__ ws, int vsrc,
    int rows, long total_rows) {
  constexpr int CH = CIN / 16;    // 16-B chunks per lane per neighbour row
  constexpr int NCT = COUT / 16;  // 16-column output tiles
  constexpr int K = kSeq * CIN;
  constexpr int KG = SPG * CIN;
  constexpr int KP = KG + 8;
  extern __shared__ float lds_w[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = blockIdx.y, s0 = g * SPG;
  coop_copy<8, f32x4>(
      COUT * (KG / 4), [&](int e) { return ld4(&w[(long)(e / (KG / 4)) * K + s0 * CIN + 4 * (e % (KG / 4))]); },
      [&](int e, f32x4 v) { st4(&lds_w[(e / (KG / 4)) * KP + 4 * (e % (KG / 4))], v); });
  __syncthreads();
  const int r16 = lane & 15, kg = lane >> 4;
  float bn[NCT];
#pragma unroll
  for (int t = 0; t < NCT; ++t) bn[t] = (SPG == kSeq && bias) ? bias[t * 16 + r16] : 0.f;
  const long n_tiles = (total_rows + 31) / 32;
  const TileSweep sw = xcd_sweep(n_tiles, 4, wave, n_tiles < kContigTiles);
  for (long tile = sw.begin; tile < sw.end; tile += sw.step) {
    const long m0 = tile * 32;
    const float* xb[2];
    int src[2][SPG];
#pragma unroll
    for (int rg = 0; rg < 2; ++rg) {
      long m = m0 + rg * 16 + r16;
      if (m >= total_rows) m = total_rows - 1;  // clamp loads, stores are masked
      int b, r;
    divmod32(m, rows, b, r);
      xb[rg] = x + (long)b * vsrc * CIN + 4 * kg;
      const int* ir = idx + (long)r * kSeq + s0;
#pragma unroll
      for (int s = 0; s < SPG; ++s) src[rg][s] = ir[s];
    }
    // materialise all indices here: a compiler load sunk into the slot loop
    // would carry a waitcnt that also drains the asm prefetch
#pragma unroll
    for (int rg = 0; rg < 2; ++rg)
#pragma unroll
      for (int s = 0; s < SPG; ++s) asm volatile("" : "+v"(src[rg][s]));
    f32x4 acc[2][NCT];
#pragma unroll
    for (int rg = 0; rg < 2; ++rg)
#pragma unroll
      for (int t = 0; t < NCT; ++t) acc[rg][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // Software pipeline, fully unrolled over the slots with two static
    // register buffers: slot s+1's rows are in flight while slot s runs its
    // MFMAs.  Gathers are inline-asm loads retired by a counted vmcnt
    // (hipcc's own placement drained the prefetch; see gload4_async).
    f32x4 buf[2][2][CH];
#pragma unroll
    for (int rg = 0; rg < 2; ++rg)
#pragma unroll
      for (int c = 0; c < CH; ++c)
        gload4_async(buf[0][rg][c], xb[rg] + (long)src[rg][0] * CIN + 16 * c);
#pragma unroll
    for (int s = 0; s < SPG; ++s) {
      f32x4(&cur)[2][CH] = buf[s & 1];
      if (s + 1 < SPG) {
#pragma unroll
        for (int rg = 0; rg < 2; ++rg)
#pragma unroll
          for (int c = 0; c < CH; ++c)
            gload4_async(buf[(s + 1) & 1][rg][c], xb[rg] + (long)src[rg][s + 1] * CIN + 16 * c);
        if (CH == 2) vm_wait4<4>(cur[0][0], cur[0][1 % CH], cur[1][0], cur[1][1 % CH]);
        else vm_wait8<8>(cur[0][0], cur[0][1 % CH], cur[0][2 % CH], cur[0][3 % CH], cur[1][0],
                         cur[1][1 % CH], cur[1][2 % CH], cur[1][3 % CH]);
      } else {
        if (CH == 2) vm_wait4<0>(cur[0][0], cur[0][1 % CH], cur[1][0], cur[1][1 % CH]);
        else vm_wait8<0>(cur[0][0], cur[0][1 % CH], cur[0][2 % CH], cur[0][3 % CH], cur[1][0],
                         cur[1][1 % CH], cur[1][2 % CH], cur[1][3 % CH]);
      }
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const f32x4 bw = ld4(&lds_w[(t * 16 + r16) * KP + s * CIN + 4 * (kg + 4 * c)]);
#pragma unroll
          for (int rg = 0; rg < 2; ++rg) {
            const f32x4 av = cur[rg][c];
            acc[rg][t] = mfma16(av.x, bw.x, acc[rg][t]);
            acc[rg][t] = mfma16(av.y, bw.y, acc[rg][t]);
            acc[rg][t] = mfma16(av.z, bw.z, acc[rg][t]);
            acc[rg][t] = mfma16(av.w, bw.w, acc[rg][t]);
          }
        }
      }
    }
    float* dst = (SPG == kSeq) ? y : ws + (long)g * total_rows * COUT;
#pragma unroll
    for (int rg = 0; rg < 2; ++rg)
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const int n = t * 16 + r16;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const long mo = m0 + rg * 16 + 4 * kg + rr;
          if (mo < total_rows) {
            float v = acc[rg][t][rr];
            if (SPG == kSeq) {
              v += bn[t];
              if (ACT == CFSD_ACT_ELU) v = elu_f(v);
            }
            dst[mo * COUT + n] = v;
          }
        }
      }
  }
}

// Slot-group combine: out = act(sum_g ws[g] + bias) (fwd) or
// out = (sum_g ws[g]) * elu'(elu_y) (bwd data); one thread per float4.
template <int ACT>
__global__ __launch_bounds__(256) void conv_combine(const float* __restrict__ ws,
                                                    const float* __restrict__ bias,
                                                    const float* __restrict__ elu_y,
                                                    float* __restrict__ out, int groups,
                                                    int cols, long n4) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n4) return;
  f32x4 v = ld4(ws + 4 * t);
  for (int g = 1; g < groups; ++g) v += ld4(ws + (long)g * n4 * 4 + 4 * t);
  if (bias) {
    const int c = (int)(4 * t) % cols;
    v.x += bias[c]; v.y += bias[c + 1]; v.z += bias[c + 2]; v.w += bias[c + 3];
  }
  if (ACT == CFSD_ACT_ELU) {
    v.x = elu_f(v.x); v.y = elu_f(v.y); v.z = elu_f(v.z); v.w = elu_f(v.w);
  }
  if (elu_y) {
    const f32x4 e = ld4(elu_y + 4 * t);
    v.x *= elu_grad_from_out(e.x); v.y *= elu_grad_from_out(e.y);
    v.z *= elu_grad_from_out(e.z); v.w *= elu_grad_from_out(e.w);
  }
  st4(out + 4 * t, v);
}

// Forward, small input (CS <= 4 channels, e.g. the xyz input conv): one
// thread per output row computing all COUT channels.  The 9 neighbour rows
// are CS floats each (one dwordx3 per slot); W's addresses are wave-uniform
// compile-time offsets -> scalar loads feeding the FMAs as SGPR operands.
template <int CS, int COUT, int ACT>
__global__ __launch_bounds__(256) void conv_fwd_in_small(const float* __restrict__ x,
                                                         const int* __restrict__ idx,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ y, int vsrc,
                                                         int rows, long total_rows) {
  constexpr int K = kSeq * CS;
  const long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= total_rows) return;
  int b, r;
    divmod32(m, rows, b, r);
  const float* xb = x + (long)b * vsrc * CS;
  const int* ir = idx + (long)r * kSeq;
  float xv[K];
#pragma unroll
  for (int s = 0; s < kSeq; ++s) {
    const float* p = xb + (long)ir[s] * CS;
#pragma unroll
    for (int c = 0; c < CS; ++c) xv[s * CS + c] = p[c];
  }
  float* out = y + m * COUT;
#pragma unroll
  for (int o4 = 0; o4 < COUT / 4; ++o4) {
    float acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 4 * o4 + j;
      float a = bias ? bias[o] : 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) a = fmaf(xv[k], w[o * K + k], a);
      acc[j] = ACT == CFSD_ACT_ELU ? elu_f(a) : a;
    }
    st4(out + 4 * o4, (f32x4){acc[0], acc[1], acc[2], acc[3]});
  }
}

// Forward, small output (CO <= 4 channels, e.g. the xyz output conv),
// persistent over rows: L = CIN/4 lanes per row, each lane owns a float4 of
// input channels of every neighbour row (one coalesced 16*L-byte read per
// neighbour), the CO partial dots are reduced across the L lanes.
template <int CIN, int CO, int ACT, typename TX = float>
__global__ __launch_bounds__(256, CIN == 32 ? 8 : 4) void conv_fwd_out_small(const TX* __restrict__ x,
                                                          const int* __restrict__ idx,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ y, int vsrc,
                                                          int rows, long total_rows, int batch,
                                                          int xvm, int yvm) {
  constexpr int L = CIN / 4;
  constexpr int RPW = 64 / L;
  constexpr int K = kSeq * CIN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane % L, slot = lane / L;
  // Weights live in LDS (CO*K floats), not registers: 27 float4 of weights per
  // lane capped occupancy at 3 waves/SIMD and this kernel is gather-latency bound.
  __shared__ f32x4 lw[CO * K / 4];
  for (int i = threadIdx.x; i < CO * K / 4; i += blockDim.x) lw[i] = ld4(w + 4 * i);
  __syncthreads();
  float bo[CO];
#pragma unroll
  for (int o = 0; o < CO; ++o) bo[o] = bias ? bias[o] : 0.f;
  // XCD-aware sweep over RPW-row groups: each XCD walks a contiguous 1/8 of
  // the rows (two meshes at batch 16), so the neighbour rows a mesh gathers 9x
  // stay in that XCD's L2 instead of every L2 seeing every mesh
  const TileSweep sw = xcd_sweep((total_rows + RPW - 1) / RPW, 4, wave);
  for (long grp = sw.begin; grp < sw.end; grp += sw.step) {  // whole waves stay in the loop
    const long mm = grp * RPW + slot;
    const bool valid = mm < total_rows;
    const long m = valid ? mm : total_rows - 1;
    // rows visited in x's layout (vertex-major: RPW meshes of one vertex, so
    // the wave's neighbour loads are contiguous), y addressed in its own
    int b, r;
    split_row(m, xvm, batch, rows, b, r);
    const Lay lx = make_lay(xvm, batch, vsrc);
    const TX* xb = x + (long)b * lx.bs * CIN + 4 * q;
    const int* ir = idx + (long)r * kSeq;
    float acc[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) acc[o] = 0.f;
    int wq = q;
    asm volatile("" : "+v"(wq));  // opaque per iteration: keeps the weight reads from being hoisted into VGPRs
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      const f32x4 v = ld4f(xb + (long)ir[s] * lx.vs * CIN);
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        const f32x4 wv = lw[(o * K + s * CIN) / 4 + wq];
        acc[o] = fmaf(v.x, wv.x, acc[o]);
        acc[o] = fmaf(v.y, wv.y, acc[o]);
        acc[o] = fmaf(v.z, wv.z, acc[o]);
        acc[o] = fmaf(v.w, wv.w, acc[o]);
      }
    }
#pragma unroll
    for (int o = 0; o < CO; ++o)
#pragma unroll
      for (int d = L / 2; d >= 1; d >>= 1) acc[o] += __shfl_xor(acc[o], d);
    if (valid && q == 0) {
      const long yo = xvm == yvm ? m : (long)row_of(make_lay(yvm, batch, rows), b, r);
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        float v = acc[o] + bo[o];
        if (ACT == CFSD_ACT_ELU) v = elu_f(v);
        y[yo * CO + o] = v;
      }
    }
  }
}

// Forward, small input (CS <= 3; the xyz input conv) on MFMA: a 32-row tile
// is (32 x 27) gathered inputs times W^T (27 x COUT).  Every lane gathers its
// row's 27 values (9 idx + 9 x CS floats, L1-shared by the two lane halves)
// and keeps the half it feeds to v_mfma_f32_32x32x2_f32 (k-permuted: half h
// owns k in [h*KH, h*KH + KH)); W^T lives in registers.  Output rows are
// stored as 128-B coalesced segments.
// SWAP: the input is NOT read from x but gathered straight from the
// resident set through the feature swap (SwapSrc: each neighbour row's
// source mesh), so the swap and this conv need no order between them
// (conv_fwd_in_swap runs both as two roles of one launch).
template <int CS, int COUT, int ACT, typename TY, bool SWAP>
__device__ __forceinline__ void conv_fwd_in_body(int vb, int nvb, const float* __restrict__ x,
                                                 const SwapSrc& sw, const int* __restrict__ idx,
                                                 const float* __restrict__ w, const float* __restrict__ bias,
                                                 TY* __restrict__ y, int vsrc, int rows, long total_rows,
                                                 int batch, int xvm, int yvm) {
  constexpr int K = kSeq * CS, KH = (K + 1) / 2, NCT = COUT / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  float wb[NCT][KH];
  float bn[NCT];
#pragma unroll
  for (int t = 0; t < NCT; ++t) {
    bn[t] = bias ? bias[t * 32 + i] : 0.f;
#pragma unroll
    for (int kk = 0; kk < KH; ++kk) {
      const int k = h * KH + kk;
      wb[t][kk] = k < K ? w[(t * 32 + i) * K + k] : 0.f;
    }
  }
  const long n_tiles = (total_rows + 31) / 32;
  const int key = SWAP ? *sw.key : 0;
  for (long tile = (long)vb * 4 + wave; tile < n_tiles; tile += (long)nvb * 4) {
    long m = tile * 32 + i;
    if (m >= total_rows) m = total_rows - 1;
    int b, r;
    // rows visited in x's layout (the xyz input is batch-major: a tile's
    // neighbour rows are one mesh's), each 128-B output row stored in y's
    split_row(m, xvm, batch, rows, b, r);
    const Lay lx = make_lay(xvm, batch, vsrc);
    const float* xb = x + (long)b * lx.bs * CS;
    const int* ir = idx + (long)r * kSeq;
    float g[2 * KH];
    if constexpr (SWAP) {
      long src[kSeq];
#pragma unroll
      for (int s = 0; s < kSeq; ++s) src[s] = swap_src_mesh(sw, key, b, ir[s], vsrc);
#pragma unroll
      for (int s = 0; s < kSeq; ++s) ld_row<CS>(sw.data + (src[s] * vsrc + ir[s]) * CS, &g[s * CS]);
    } else {
#pragma unroll
      for (int s = 0; s < kSeq; ++s) {
        ld_row<CS>(xb + (long)ir[s] * lx.vs * CS, &g[s * CS]);
      }
    }
#pragma unroll
    for (int k = K; k < 2 * KH; ++k) g[k] = 0.f;
    f32x16 acc[NCT];
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[t] = (f32x16){0.f};
#pragma unroll
    for (int kk = 0; kk < KH; ++kk) {
      const float a = h ? g[KH + kk] : g[kk];
#pragma unroll
      for (int t = 0; t < NCT; ++t) acc[t] = mfma32(a, wb[t][kk], acc[t]);
    }
#pragma unroll
    for (int t = 0; t < NCT; ++t)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const long mo = tile * 32 + acc_row(rr, lane);
        if (mo < total_rows) {
          long yo = mo;
          if (xvm != yvm) {
            int bo, ro;
            split_row(mo, xvm, batch, rows, bo, ro);
            yo = row_of(make_lay(yvm, batch, rows), bo, ro);
          }
          const float v = acc[t][rr] + bn[t];
          stf(&y[yo * COUT + t * 32 + i], ACT == CFSD_ACT_ELU ? elu_f(v) : v);
        }
      }
  }
}
template <int CS, int COUT, int ACT, typename TY = float>
__global__ __launch_bounds__(256) void conv_fwd_in_mfma(const float* __restrict__ x,
                                                        const int* __restrict__ idx,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        TY* __restrict__ y, int vsrc, int rows,
                                                        long total_rows, int batch, int xvm,
                                                        int yvm) {
  conv_fwd_in_body<CS, COUT, ACT, TY, false>(blockIdx.x, gridDim.x, x, SwapSrc{}, idx, w, bias, y, vsrc, rows,
                                             total_rows, batch, xvm, yvm);
}

// The feature swap (swap_k: x = the swapped batch, every vertex) and the
// first Enblock's conv (gathering through the swap from the resident set)
// as two independent roles of ONE launch: workgroups [0, n_conv) the conv,
// the rest one swap row per thread.  Same values as swap_features + the
// conv launch (the conv's inputs are the same copies).
template <int CS, int COUT, int ACT, typename TY>
__global__ __launch_bounds__(256) void conv_fwd_in_swap(const SwapSrc sw, float* __restrict__ x, int n_conv,
                                                        long swap_total, const int* __restrict__ idx,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ bias, TY* __restrict__ y,
                                                        int vsrc, int rows, long total_rows, int batch,
                                                        int xvm, int yvm) {
  if ((int)blockIdx.x < n_conv) {
    conv_fwd_in_body<CS, COUT, ACT, TY, true>(blockIdx.x, n_conv, x, sw, idx, w, bias, y, vsrc, rows, total_rows,
                                              batch, xvm, yvm);
    return;
  }
  const long t = (long)((int)blockIdx.x - n_conv) * blockDim.x + threadIdx.x;
  if (t >= swap_total) return;
  int ob, v;  // row t of x's storage
  split_row(t, xvm, batch, vsrc, ob, v);
  const long src_mesh = swap_src_mesh(sw, *sw.key, ob, v, vsrc);
  float r3[CS];
  ld_row<CS>(sw.data + (src_mesh * vsrc + v) * CS, r3);
  st_row<CS>(x + t * CS, r3);
}

// ==========================================================================
// Backward data, MFMA path.  dx rows are source vertices u (flattened with
// b).  For slot s the A operand is T_s[u, :] = sum_{r in inv(u,s)} dpre[r, :]
// (gather-sum through the inverse spiral, fixed order -> deterministic); the
// B operand is W_s^T staged in LDS as [s][c][COUT + 4].
// inv_head[u*S + s] = the first four rows of inv(u,s) (-1 if absent), one
// int4 per key, prefetched two slots ahead.  Rows 0/1 are loaded
// unconditionally one slot ahead (clamped, weighted 0 when absent: 77 % of
// keys have <= 1 entry, 96 % <= 2); rows 2/3 (exec-masked loads) only for
// the lanes whose list has them; entries beyond the head (0.03 % of keys)
// walk inv_ptr/inv_row from offset 4.  Sum order = list order.
// Slot groups as in conv_fwd_mfma (partials -> ws, conv_combine).
constexpr int kInvHead = CFSD_INV_HEAD;
__device__ __forceinline__ float present(int r) { return r >= 0 ? 1.f : 0.f; }

// Small-channel (CO-wide dpre rows) list folding, entries 2.. of NS keys
// key0 + j (rows 0/1 already in t): the head's rows 2/3 as exec-masked loads,
// then the CSR tail from offset 4 (rare).  Adds in list order.
template <int NS, int CO>
__device__ __forceinline__ void fold_head_tail(const int4 (&hd)[NS], long key0,
                                               const float* __restrict__ db_,
                                               const int* __restrict__ inv_ptr,
                                               const int* __restrict__ inv_row,
                                               float (&t)[NS][CO]) {
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    if (hd[j].z >= 0) {
#pragma unroll
      for (int o = 0; o < CO; ++o) t[j][o] += db_[hd[j].z * CO + o];
      if (hd[j].w >= 0) {
#pragma unroll
        for (int o = 0; o < CO; ++o) t[j][o] += db_[hd[j].w * CO + o];
        const long key = key0 + j;
        for (int e = inv_ptr[key] + kInvHead; e < inv_ptr[key + 1]; ++e) {
#pragma unroll
          for (int o = 0; o < CO; ++o) t[j][o] += db_[inv_row[e] * CO + o];
        }
      }
    }
  }
}


// dpre through a buffer descriptor: 32-bit per-lane byte offsets, and an
// absent list row is an out-of-range offset that returns 0 with no memory
// access.  Every row load is then ONE unconditional instruction -- no exec
// branches, whose joins made hipcc drain the in-flight prefetch.
constexpr int kAbsentRow = 0x7ffff000;
__device__ __forceinline__ f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

constexpr int kDxOcc = 3;
constexpr int dx_occ(int cin, int cout) { return (cin == 32 && cout == 32) ? kDxOcc : 2; }

template <int CIN, int COUT, int SPG>
__global__ __launch_bounds__(256, dx_occ(CIN, COUT)) void conv_dx_mfma(
    const float* __restrict__ dpre, const int* __restrict__ inv_ptr,
    const int* __restrict__ inv_row, const int4* __restrict__ inv_head,
    const float* __restrict__ w, const float* __restrict__ elu_y, float* __restrict__ dx,
    float* __restrict__ ws, int vsrc, int rows, long total_rows) {
  constexpr int HALF = COUT / 2, Q = HALF / 4;
  // K map inside a slot: lane half h, load q covers dpre channels
  // 4*h + 8*q + [0, 4) (the two lane halves read the two 16-B halves of one
  // 32-B segment of the row)
  constexpr int NT = CIN / 32;
  constexpr int OP = COUT + 4;
  constexpr int K = kSeq * CIN;
  constexpr int RB = COUT * (int)sizeof(float);  // dpre row bytes
  extern __shared__ float lds_wt[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = blockIdx.y, s0 = g * SPG;
  // lds_wt[(sl*CIN + c) * OP + o] = w[o, (s0+sl)*CIN + c]
  coop_copy<12, float>(
      COUT * SPG * CIN, [&](int e) { return w[(long)(e / (SPG * CIN)) * K + s0 * CIN + e % (SPG * CIN)]; },
      [&](int e, float v) { lds_wt[(e % (SPG * CIN)) * OP + e / (SPG * CIN)] = v; });
  __syncthreads();
  const int nbytes = (int)(total_rows / vsrc * rows * RB);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dpre), 0, nbytes, 0x00020000);
  const int i = lane & 31, h = lane >> 5;
  const long n_tiles = (total_rows + 31) / 32;
  const TileSweep sw = xcd_sweep(n_tiles, 4, wave, n_tiles < kContigTiles);
  for (long tile = sw.begin; tile < sw.end; tile += sw.step) {
    const long m0 = tile * 32;
    long m = m0 + i;
    if (m >= total_rows) m = total_rows - 1;
    int b, u;
    divmod32(m, vsrc, b, u);
    const int base = b * rows * RB + 16 * h;
    const int4* pu = inv_head + (long)u * kSeq + s0;
    auto roff = [&](int r) { return r >= 0 ? base + r * RB : kAbsentRow; };
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x16){0.f};
    // slot pipeline: list rows 0..2 of slot s+1 and the head of slot s+2
    // are in flight while slot s computes (row 2: 3.6 % of keys but ~70 %
    // of 32-row wave-slots).  Every load is unconditional, so hipcc's
    // counters stay exact and the wait at the top of a slot only retires
    // the previous slot's prefetch.
    f32x4 c0[Q], c1[Q], c2[Q];
    const int4 none = make_int4(-1, -1, -1, -1);
    int4 pc = pu[0], pn = SPG > 1 ? pu[1] : none;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      c0[q] = buf_ld4(rsrc, roff(pc.x) + 32 * q);
      c1[q] = buf_ld4(rsrc, roff(pc.y) + 32 * q);
      c2[q] = buf_ld4(rsrc, roff(pc.z) + 32 * q);
    }
#pragma unroll 1
    for (int s = 0; s < SPG; ++s) {
      const int4 cur = pc;
      f32x4 a[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) a[q] = (c0[q] + c1[q]) + c2[q];  // absent rows read as 0
      // past the last slot the head is `none` (out-of-range loads, no
      // traffic) rather than a branch: a branch made hipcc merge the two
      // paths' counters into vmcnt(0), draining the prefetch every slot
      int4 pnn = pu[min(s + 2, SPG - 1)];
      if (s + 2 >= SPG) pnn = none;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        c0[q] = buf_ld4(rsrc, roff(pn.x) + 32 * q);
        c1[q] = buf_ld4(rsrc, roff(pn.y) + 32 * q);
        c2[q] = buf_ld4(rsrc, roff(pn.z) + 32 * q);
      }
      pc = pn;
      pn = pnn;
      if (cur.w >= 0) {  // 0.3 % of keys: rows 3.. of the list
        const long key = (long)u * kSeq + s0 + s;
        const float* db_ = dpre + base / (int)sizeof(float);
#pragma unroll
        for (int q = 0; q < Q; ++q) a[q] += ld4(db_ + (long)cur.w * COUT + 8 * q);
        for (int e = inv_ptr[key] + kInvHead; e < inv_ptr[key + 1]; ++e) {
          const float* p = db_ + (long)inv_row[e] * COUT;
#pragma unroll
          for (int q = 0; q < Q; ++q) a[q] += ld4(p + 8 * q);
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float* wr = &lds_wt[(s * CIN + t * 32 + i) * OP + 4 * h];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const f32x4 bw = ld4(wr + 8 * q);
          acc[t] = mfma32(a[q].x, bw.x, acc[t]);
          acc[t] = mfma32(a[q].y, bw.y, acc[t]);
          acc[t] = mfma32(a[q].z, bw.z, acc[t]);
          acc[t] = mfma32(a[q].w, bw.w, acc[t]);
        }
      }
    }
    float* dst = (SPG == kSeq) ? dx : ws + (long)g * total_rows * CIN;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = t * 32 + i;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const long mo = m0 + acc_row(rr, lane);
        if (mo < total_rows) {
          float v = acc[t][rr];
          if (SPG == kSeq && elu_y) v *= elu_grad_from_out(elu_y[mo * CIN + c]);
          dst[mo * CIN + c] = v;
        }
      }
    }
  }
}

// ==========================================================================
// Layers with few rows (the coarse levels: <= ~2k 32-row tiles, where the
// persistent kernels above cannot fill 256 CUs without splitting the slots
// over workgroups and combining partials in a second launch).  Here a wave
// owns one 16-row x 16-column output tile and ALL 9 slots, so there is no
// partial and no combine launch; the slots run in batches of 3 whose
// gathers and weight loads are all in flight together (3 memory-latency
// exposures per tile instead of 9).  v_mfma_f32_16x16x4_f32 lane map as in
// conv_fwd_mfma (lane (i, kg) holds row i's 16-B chunks kg, kg+4, ..);
// two accumulators (even / odd chunk) halve the dependent-MFMA chain.
// Tasks are numbered column-tile fastest, so the waves of a workgroup
// gather the same rows (L1 hits).
constexpr int kFwdLatSb = 3;
constexpr int kDxLatSb = 3;
template <int CIN, int COUT, int ACT, int CTW>
__global__ __launch_bounds__(256) void conv_fwd_lat(const float* __restrict__ x,
                                                    const int* __restrict__ idx,
                                                    const float* __restrict__ w,
                                                    const float* __restrict__ bias,
                                                    float* __restrict__ y, int vsrc, int rows,
                                                    long total_rows, int batch, int xvm, int yvm) {
  // CTW column tiles per wave share the wave's A gathers
  constexpr int CH = CIN / 16, NCT = COUT / 16, K = kSeq * CIN, NTW = NCT / CTW;
  constexpr int FSB = kFwdLatSb;
  static_assert(kSeq % FSB == 0, "slot batches");
  static_assert(NCT % CTW == 0, "column tiles per wave");
  const int lane = threadIdx.x & 63, r16 = lane & 15, kg = lane >> 4;
  const long task = (long)xcd_block() * 4 + (threadIdx.x >> 6);
  const long n_rt = (total_rows + 15) / 16;
  if (task >= n_rt * NTW) return;
  const int ct0 = (int)(task % NTW) * CTW;
  const long rt = task / NTW;
  long m = rt * 16 + r16;
  if (m >= total_rows) m = total_rows - 1;  // clamp loads, stores are masked
  int b, r;
  split_row(m, xvm, batch, rows, b, r);  // rows in x's layout (vertex-major: 16 meshes of a vertex)
  const Lay lx = make_lay(xvm, batch, vsrc);
  const float* xb = x + (long)b * lx.bs * CIN + 4 * kg;
  const int* ir = idx + (long)r * kSeq;
  const float* wb = w + (long)(ct0 * 16 + r16) * K + 4 * kg;  // + t*16*K
  int src[kSeq];
#pragma unroll
  for (int s = 0; s < kSeq; ++s) src[s] = ir[s] * lx.vs;
  f32x4 acc[CTW][2];
#pragma unroll
  for (int t = 0; t < CTW; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s0 = 0; s0 < kSeq; s0 += FSB) {
    f32x4 av[FSB][CH], bw[FSB][CH][CTW];
#pragma unroll
    for (int sl = 0; sl < FSB; ++sl)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        av[sl][c] = ld4(xb + (long)src[s0 + sl] * CIN + 16 * c);
#pragma unroll
        for (int t = 0; t < CTW; ++t)
          bw[sl][c][t] = ld4(wb + (long)t * 16 * K + (s0 + sl) * CIN + 16 * c);
      }
    // keep the batch's loads ahead of its MFMAs (hipcc otherwise interleaves
    // them with vmcnt waits to save registers, re-exposing the latency)
    __builtin_amdgcn_sched_group_barrier(0x020, (1 + CTW) * FSB * CH, 0);  // VMEM reads
    __builtin_amdgcn_sched_group_barrier(0x008, 4 * CTW * FSB * CH, 0);    // MFMA
#pragma unroll
    for (int sl = 0; sl < FSB; ++sl)
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int t = 0; t < CTW; ++t) {
          f32x4& a = acc[t][c & 1];
          a = mfma16(av[sl][c].x, bw[sl][c][t].x, a);
          a = mfma16(av[sl][c].y, bw[sl][c][t].y, a);
          a = mfma16(av[sl][c].z, bw[sl][c][t].z, a);
          a = mfma16(av[sl][c].w, bw[sl][c][t].w, a);
        }
  }
#pragma unroll
  for (int t = 0; t < CTW; ++t) {
    const int n = (ct0 + t) * 16 + r16;
    const float bn = bias ? bias[n] : 0.f;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const long mo = rt * 16 + 4 * kg + rr;
      if (mo < total_rows) {
        float v = acc[t][0][rr] + acc[t][1][rr] + bn;
        if (ACT == CFSD_ACT_ELU) v = elu_f(v);
        long yo = mo;
        if (xvm != yvm) {
          int bo, ro;
          split_row(mo, xvm, batch, rows, bo, ro);
          yo = row_of(make_lay(yvm, batch, rows), bo, ro);
        }
        y[yo * COUT + n] = v;
      }
    }
  }
}

// Backward data for layers with few source rows, same tiling as
// conv_fwd_lat: a wave owns 16 source rows u x CTW*16 input channels c and
// all 9 slots (CTW = 2 for 32 input channels: the list gathers of A are
// shared by both column tiles).  A = T_s[u][o] (gather-sum of dpre rows through the inverse
// spiral: the inv_head rows of a batch of 3 slots are loaded together,
// rare further entries added after), B = W_s^T read straight from W (4
// strided dwords per 4-chunk of o; W is L2-resident), in flight with A.
// (body shared by the conv_dx_lat kernel and the dx half of
// conv_bwd_lat_pair; vb / vnb = this workgroup's number / count in its grid)
template <int CIN, int COUT, int CTW, int DSB = kDxLatSb>
__device__ __forceinline__ void conv_dx_lat_body(int vb, int vnb, const float* __restrict__ dpre,
                                                 const int* __restrict__ inv_ptr,
                                                 const int* __restrict__ inv_row,
                                                 const int4* __restrict__ inv_head,
                                                 const float* __restrict__ w,
                                                 const float* __restrict__ elu_y,
                                                 float* __restrict__ dx, int vsrc, int rows,
                                                 long total_rows) {
  constexpr int CH = COUT / 16, NCT = CIN / 16, K = kSeq * CIN, NTW = NCT / CTW;
  static_assert(kSeq % DSB == 0, "slot batches");
  static_assert(NCT % CTW == 0, "column tiles per wave");
  const int lane = threadIdx.x & 63, r16 = lane & 15, kg = lane >> 4;
  const long task = (long)xcd_block_of(vb, vnb) * 4 + (threadIdx.x >> 6);
  const long n_rt = (total_rows + 15) / 16;
  if (task >= n_rt * NTW) return;
  const int ct0 = (int)(task % NTW) * CTW;
  const long rt = task / NTW;
  long m = rt * 16 + r16;
  if (m >= total_rows) m = total_rows - 1;
  int b, u;
    divmod32(m, vsrc, b, u);
  const float* db_ = dpre + (long)b * rows * COUT + 4 * kg;
  constexpr int RB = COUT * (int)sizeof(float);
  const int base = (b * rows * COUT + 4 * kg) * (int)sizeof(float);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dpre), 0,
                                                      (int)(total_rows / vsrc * rows * RB), 0x00020000);
  const int4* pu = inv_head + (long)u * kSeq;
  const float* wb = w + (long)(4 * kg) * K + ct0 * 16 + r16;  // + ct*16 + o_off*K + s*CIN
  f32x4 acc[CTW][2];
#pragma unroll
  for (int t = 0; t < CTW; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s0 = 0; s0 < kSeq; s0 += DSB) {
    int4 pr[DSB];
#pragma unroll
    for (int sl = 0; sl < DSB; ++sl) pr[sl] = pu[s0 + sl];
    f32x4 bw[DSB][CH][CTW];
#pragma unroll
    for (int sl = 0; sl < DSB; ++sl)
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int t = 0; t < CTW; ++t) {
          const float* q = wb + (long)(16 * c) * K + (s0 + sl) * CIN + 16 * t;
          bw[sl][c][t] = f32x4{q[0], q[K], q[2 * K], q[3 * K]};
        }
    // list rows 0..2 of the batch's keys: unconditional buffer loads, absent
    // rows out of range (read as 0, no traffic), all in flight together
    f32x4 a[DSB][CH];
#pragma unroll
    for (int sl = 0; sl < DSB; ++sl) {
      f32x4 r[3][CH];
      const int hr[3] = {pr[sl].x, pr[sl].y, pr[sl].z};
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int c = 0; c < CH; ++c)
          r[j][c] = buf_ld4(rsrc, hr[j] >= 0 ? base + hr[j] * RB + 64 * c : kAbsentRow);
#pragma unroll
      for (int c = 0; c < CH; ++c) a[sl][c] = (r[0][c] + r[1][c]) + r[2][c];
    }
    // rows 3.. (0.3 % of keys): exec branch
#pragma unroll
    for (int sl = 0; sl < DSB; ++sl) {
      {
        if (pr[sl].w >= 0) {
#pragma unroll
          for (int c = 0; c < CH; ++c) a[sl][c] += ld4(db_ + (long)pr[sl].w * COUT + 16 * c);
          const long key = (long)u * kSeq + s0 + sl;
          for (int e = inv_ptr[key] + kInvHead; e < inv_ptr[key + 1]; ++e) {
            const float* p = db_ + (long)inv_row[e] * COUT;
#pragma unroll
            for (int c = 0; c < CH; ++c) a[sl][c] += ld4(p + 16 * c);
          }
        }
      }
    }
#pragma unroll
    for (int sl = 0; sl < DSB; ++sl)
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int t = 0; t < CTW; ++t) {
          f32x4& ac = acc[t][c & 1];
          ac = mfma16(a[sl][c].x, bw[sl][c][t].x, ac);
          ac = mfma16(a[sl][c].y, bw[sl][c][t].y, ac);
          ac = mfma16(a[sl][c].z, bw[sl][c][t].z, ac);
          ac = mfma16(a[sl][c].w, bw[sl][c][t].w, ac);
        }
  }
#pragma unroll
  for (int t = 0; t < CTW; ++t) {
    const int c = (ct0 + t) * 16 + r16;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const long mo = rt * 16 + 4 * kg + rr;
      if (mo < total_rows) {
        float v = acc[t][0][rr] + acc[t][1][rr];
        if (elu_y) v *= elu_grad_from_out(elu_y[mo * CIN + c]);
        dx[mo * CIN + c] = v;
      }
    }
  }
}
template <int CIN, int COUT, int CTW>
__global__ __launch_bounds__(256) void conv_dx_lat(const float* __restrict__ dpre,
                                                   const int* __restrict__ inv_ptr,
                                                   const int* __restrict__ inv_row,
                                                   const int4* __restrict__ inv_head,
                                                   const float* __restrict__ w,
                                                   const float* __restrict__ elu_y,
                                                   float* __restrict__ dx, int vsrc, int rows,
                                                   long total_rows) {
  conv_dx_lat_body<CIN, COUT, CTW>(blockIdx.x, gridDim.x, dpre, inv_ptr, inv_row, inv_head, w,
                                   elu_y, dx, vsrc, rows, total_rows);
}
// Backward data, small dpre (CO <= 4 channels; the xyz output conv): one
// thread per source row (b, u) computing all CIN outputs.  The spiral
// transpose is first folded in the CO-wide dpre space,
//   t[s][o] = sum_{r : idx[r][s] = u} dpre[b][r][o]   (inv_head + rare overflow),
// then dx[c] = sum_{s,o} t[s][o] * W[o][s*CIN + c].  W's addresses are
// wave-uniform compile-time offsets, so they are scalar loads (SGPR operands
// of the FMAs, no LDS, no per-lane W registers).  All 9 inv_head loads and
// the 18 dpre row loads of a thread are independent and issued together.
template <int CIN, int CO>
__global__ __launch_bounds__(256) void conv_dx_out_small(const float* __restrict__ dpre,
                                                         const int* __restrict__ inv_ptr,
                                                         const int* __restrict__ inv_row,
                                                         const int4* __restrict__ inv_head,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ elu_y,
                                                         float* __restrict__ dx, int vsrc,
                                                         int rows, long total_rows) {
  constexpr int K = kSeq * CIN;
  const long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= total_rows) return;
  int b, u;
    divmod32(m, vsrc, b, u);
  const float* db_ = dpre + (long)b * rows * CO;
  const int4* pu = inv_head + (long)u * kSeq;
  int4 pr[kSeq];
#pragma unroll
  for (int s = 0; s < kSeq; ++s) pr[s] = pu[s];
  float tt[kSeq][CO];
#pragma unroll
  for (int s = 0; s < kSeq; ++s) {
    const float* p0 = db_ + (long)max(pr[s].x, 0) * CO;
    const float* p1 = db_ + (long)max(pr[s].y, 0) * CO;
    const float f0 = present(pr[s].x), f1 = present(pr[s].y);
#pragma unroll
    for (int o = 0; o < CO; ++o) tt[s][o] = p0[o] * f0 + p1[o] * f1;
  }
  fold_head_tail<kSeq, CO>(pr, (long)u * kSeq, db_, inv_ptr, inv_row, tt);
  float* out = dx + m * CIN;
  const float* ey = elu_y ? elu_y + m * CIN : nullptr;
#pragma unroll
  for (int c4 = 0; c4 < CIN / 4; ++c4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kSeq; ++s)
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        const float* wp = w + o * K + s * CIN + 4 * c4;
        acc.x = fmaf(tt[s][o], wp[0], acc.x);
        acc.y = fmaf(tt[s][o], wp[1], acc.y);
        acc.z = fmaf(tt[s][o], wp[2], acc.z);
        acc.w = fmaf(tt[s][o], wp[3], acc.w);
      }
    if (ey) {
      const f32x4 g = ld4(ey + 4 * c4);
      acc.x *= elu_grad_from_out(g.x);
      acc.y *= elu_grad_from_out(g.y);
      acc.z *= elu_grad_from_out(g.z);
      acc.w *= elu_grad_from_out(g.w);
    }
    st4(out + 4 * c4, acc);
  }
}

// ==========================================================================
// Backward weight, MFMA path, LDS-staged.  A block owns 32-row tiles in a
// persistent loop.  Per tile, all threads stage dpre[32][COUT] and the
// gathered x for every slot, x_lds[s][32][CIN], into LDS (coalesced 16-B
// loads, the NEXT tile's loads are in flight in registers during this tile's
// MFMAs).  The U = kSeq*(COUT/32)*(CIN/32) output tiles (s, ot, ct) of
// dW[32 o][32 c] are split evenly over the block's WAVES waves, each keeping
// its UPW accumulators across all tiles: A = dpre^T (o on lanes), B = x
// (c on lanes), MFMA step j reduces rows (j, j+16).  The block writes one
// slab [U][32][32] + db partial; cfsd_dw_reduce sums slabs in fixed order.
template <int CIN, int COUT>
struct DwCfg {
  static constexpr int U = kSeq * (COUT / 32) * (CIN / 32);
  static constexpr int WAVES = (U % 12 == 0) ? 12 : 9;  // 36 units -> 12 x 3, else 9 x U/9
  static constexpr int UPW = U / WAVES;
  static constexpr int THREADS = WAVES * 64;
  static constexpr int XF4 = kSeq * 32 * CIN / 4;  // float4s of gathered x per tile
  static constexpr int DF4 = 32 * COUT / 4;        // float4s of dpre per tile
  static constexpr int XPT = (XF4 + THREADS - 1) / THREADS;
  static constexpr int DPT = (DF4 + THREADS - 1) / THREADS;
  static constexpr int LDS_FLOATS = 32 * COUT + kSeq * 32 * CIN;
  static_assert(U % WAVES == 0, "unit split");
};

template <int CIN, int COUT>
__global__ __launch_bounds__(768) void conv_dw_mfma(
    const float* __restrict__ x, const int* __restrict__ idx, const float* __restrict__ dpre,
    float* __restrict__ ws, float* __restrict__ ws_db, int vsrc, int rows, long total_rows, int batch,
    int xvm, int dpvm) {
  using C = DwCfg<CIN, COUT>;
  constexpr int OT = COUT / 32, CT = CIN / 32;
  extern __shared__ float lds[];
  float* dp_lds = lds;               // [32][COUT]
  float* x_lds = lds + 32 * COUT;    // [kSeq][32][CIN]
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const long n_tiles = (total_rows + 31) / 32;

  f32x16 acc[C::UPW];
#pragma unroll
  for (int q = 0; q < C::UPW; ++q) acc[q] = (f32x16){0.f};
  float db_acc = 0.f;

  // K (rows) is visited in x's layout (vertex-major: a 32-row tile is 2
  // vertices x 16 meshes, so each slot's gathered rows are two contiguous
  // blocks); dpre rows are addressed in their own layout
  const Lay lx = make_lay(xvm, batch, vsrc), ldp = make_lay(dpvm, batch, rows);
  // (loading the spiral indices one tile ahead of the gathers measured
  // slower: D3 74 -> 91 us)
  f32x4 xs[C::XPT], ds[C::DPT];
  auto load_tile = [&](long tile) {
    const long m0 = tile * 32;
#pragma unroll
    for (int e = 0; e < C::XPT; ++e) {
      const int f = tid + e * C::THREADS;  // f in [0, XF4): (s, row, c4)
      if (f < C::XF4) {
        const int c4 = f % (CIN / 4);
        const int row = (f / (CIN / 4)) % 32;
        const int s = f / (32 * CIN / 4);
        long m = m0 + row;
        if (m >= total_rows) m = total_rows - 1;
        int b, r;  // < 2^31 rows: 32-bit division
        split_row(m, xvm, batch, rows, b, r);
        const int src = idx[r * kSeq + s];
        xs[e] = ld4(x + ((long)b * lx.bs + (long)src * lx.vs) * CIN + 4 * c4);
      }
    }
#pragma unroll
    for (int e = 0; e < C::DPT; ++e) {
      const int f = tid + e * C::THREADS;  // (row, o4)
      if (f < C::DF4) {
        const int row = f / (COUT / 4);
        const long m = m0 + row;
        long dr = m;
        if (xvm != dpvm && m < total_rows) {
          int b, r;
          split_row(m, xvm, batch, rows, b, r);
          dr = row_of(ldp, b, r);
        }
        ds[e] = m < total_rows ? ld4(dpre + dr * COUT + 4 * (f % (COUT / 4)))
                               : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  const TileSweep sw = xcd_sweep(n_tiles, 1, 0);
  long tile = sw.begin;
  if (tile < sw.end) load_tile(tile);
  for (; tile < sw.end; tile += sw.step) {
#pragma unroll
    for (int e = 0; e < C::XPT; ++e) {
      const int f = tid + e * C::THREADS;
      if (f < C::XF4) st4(&x_lds[4 * f], xs[e]);
    }
#pragma unroll
    for (int e = 0; e < C::DPT; ++e) {
      const int f = tid + e * C::THREADS;
      if (f < C::DF4) st4(&dp_lds[4 * f], ds[e]);
    }
    __syncthreads();
    const long next = tile + sw.step;
    if (next < sw.end) load_tile(next);
    if (tid < COUT) {
#pragma unroll 8
      for (int row = 0; row < 32; ++row) db_acc += dp_lds[row * COUT + tid];
    }
#pragma unroll
    for (int q = 0; q < C::UPW; ++q) {
      const int un = wave * C::UPW + q;
      const int s = un / (OT * CT), ot = (un / CT) % OT, ct = un % CT;
      const float* ap = dp_lds + (16 * h) * COUT + ot * 32 + i;
      const float* bp = x_lds + (s * 32 + 16 * h) * CIN + ct * 32 + i;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[q] = mfma32(ap[j * COUT], bp[j * CIN], acc[q]);
    }
    __syncthreads();
  }
  float* slab = ws + (long)blockIdx.x * (C::U * 1024);
#pragma unroll
  for (int q = 0; q < C::UPW; ++q) {
    const int un = wave * C::UPW + q;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) slab[un * 1024 + acc_row(rr, lane) * 32 + i] = acc[q][rr];
  }
  if (tid < COUT) ws_db[(long)blockIdx.x * COUT + tid] = db_acc;
}

// dW/db slab reduction, coalesced: a 1024-thread block owns 64 consecutive
// slab offsets f, its 16 waves sum the slabs w, w+16, ... and the 16 partials
// are added in fixed order (deterministic); f is then mapped to dW's layout.
template <int CIN, int COUT>
__global__ __launch_bounds__(1024) void conv_dw_reduce(const float* __restrict__ ws,
                                                       const float* __restrict__ ws_db,
                                                       float* __restrict__ dw,
                                                       float* __restrict__ db, int n_slabs) {
  constexpr int OT = COUT / 32, CT = CIN / 32;
  constexpr int U = DwCfg<CIN, COUT>::U;
  constexpr int NW = U * 1024;
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int f = blockIdx.x * 64 + lane;
  const bool valid = f < NW + COUT;
  if (!valid) f = NW + COUT - 1;
  const float* src = f < NW ? ws + f : ws_db + (f - NW);
  const long stride = f < NW ? NW : COUT;
  float sum = 0.f;
#pragma unroll 4
  for (int p = wv; p < n_slabs; p += 16) sum += src[(long)p * stride];
  part[wv][lane] = sum;
  __syncthreads();
  if (wv == 0 && valid) {
    float t = part[0][lane];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += part[q][lane];
    if (f < NW) {
      const int un = f >> 10, within = f & 1023;
      const int cc = (un % CT) * 32 + (within & 31);
      const int o = ((un / CT) % OT) * 32 + (within >> 5);
      const int s = un / (CT * OT);
      dw[(long)o * (kSeq * CIN) + s * CIN + cc] = t;
    } else {
      db[f - NW] = t;
    }
  }
}

template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv_dw_lat(const float* __restrict__ x,
                                                   const int* __restrict__ idx,
                                                   const float* __restrict__ dpre,
                                                   float* __restrict__ ws,
                                                   float* __restrict__ ws_db, int vsrc, int rows,
                                                   int total_rows, int rchunk, int n_chunks, int batch,
                                                   int xvm, int dpvm) {
  __shared__ float red[lat_red_floats(4)];
  conv_dw_lat_body<CIN, COUT>(blockIdx.x, gridDim.x, x, idx, dpre, ws, ws_db, vsrc, rows,
                              total_rows, rchunk, n_chunks, batch, xvm, dpvm, red);
}

// Both gradients of one coarse-level conv in ONE launch (horizontal fusion):
// the dx and dW workgroups are independent and each set alone fills only part
// of the chip with latency-bound waves, so interleaving them (alternate
// workgroups while both sets last) overlaps their memory latencies instead of
// running two half-empty launches back to back.  Each half computes exactly
// what conv_dx_lat / conv_dw_lat compute.
struct DxLatArgs {
  const float* dpre;
  const int* inv_ptr;
  const int* inv_row;
  const int4* inv_head;
  const float* w;
  const float* elu_y;
  float* dx;
  int vsrc, rows;
  long total_rows;
  int nb;
};
#ifdef CFSD_LAT_STAMPS
// diagnostic build only (tools/kbench.py KB_LATSTAMPS): per-workgroup role, start, end
__device__ unsigned long long g_lat_stamps[4096 * 3];
extern "C" int cfsd_debug_lat_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lat_stamps), sizeof(g_lat_stamps), 0, hipMemcpyDeviceToHost);
}
#endif
// The pair's data-gradient role gathers ONE slot per trip (the standalone
// conv_dx_lat three): 94 VGPRs + 32 AGPRs instead of 162 + 32, so four waves
// per SIMD fit and BOTH roles are resident from the start.  At 196 registers
// (two waves per SIMD) D1's 533 dx workgroups alone filled the chip and its
// 486 dW workgroups were dispatched only as dx ones retired (per-workgroup
// stamps: dW starts 9.0-15.8 us, span 24.4 us); now every workgroup starts
// by 0.6 us, span 22.6 us.  Same slot order: bit-identical.  D1 pair 25.9 ->
// 24.1 us, step fp32 -1..-7 us, bf16 -3 us (profiles/round8j_*).
constexpr int kPairDxSb = 1;
constexpr int kPairMinWaves = 4;
template <int CIN, int COUT, int CTW>
__global__ __launch_bounds__(256, kPairMinWaves) void conv_bwd_lat_pair(const DxLatArgs a, const DwLatArgs d) {
  // the data-gradient role first: it is the longer one, and the dW
  // workgroups fill the slots its retiring waves free (alternating the
  // roles: D1 27.4 vs 25.8 us, D0 24.2 vs 19.6 us, same box)
  const int bid = (int)blockIdx.x;
  const bool is_dx = bid < a.nb;
  const int vb = is_dx ? bid : bid - a.nb;
  __shared__ float red[lat_red_floats(4)];
#ifdef CFSD_LAT_STAMPS
  const unsigned long long t0 = wall_clock64();
#endif
  if (is_dx)
    conv_dx_lat_body<CIN, COUT, CTW, kPairDxSb>(vb, a.nb, a.dpre, a.inv_ptr, a.inv_row, a.inv_head, a.w,
                                                a.elu_y, a.dx, a.vsrc, a.rows, a.total_rows);
  else
    conv_dw_lat_body<CIN, COUT>(vb, d.nb, d.x, d.idx, d.dpre, d.ws, d.ws_db, d.vsrc, d.rows,
                                d.total_rows, d.rchunk, d.n_chunks, d.batch, d.xvm, d.dpvm, red);
#ifdef CFSD_LAT_STAMPS
  __syncthreads();
  if (threadIdx.x == 0 && bid < 4096) {
    g_lat_stamps[3 * bid] = is_dx ? 1 : 2;
    g_lat_stamps[3 * bid + 1] = t0;
    g_lat_stamps[3 * bid + 2] = wall_clock64();
  }
#endif
}

// ==========================================================================
// Backward data of a conv evaluated on a ROW SUBSET (the Enblocks: the conv
// runs only at the vertices the 0/1 down-sample keeps).  There a source row
// has ~2.25 non-empty (u, s) inverse lists of its 9, so the inverse-spiral
// formulation (A = per-slot gather-sum of dpre, MFMA over all 9 slots of
// every source row) spends ~3/4 of its MFMA work on zero rows.  Instead the
// reference's own two steps (autograd of model.py:40 then :34):
//  (1) AddmmBackward at the kept rows only: dG[b,r, s*CIN+c] =
//      sum_o dpre[b,r,o] w[o, s*CIN+c], a dense [rows, COUT] x [COUT, 9*CIN]
//      MFMA product (conv_dg_body; it shares a launch with the dW slabs);
//  (2) IndexSelectBackward (index_add_): dx[b,u,:] = g * sum_{p in flat(u)}
//      dG[b, p, :] where flat(u) lists the flattened spiral positions
//      p = r*9 + s with idx[r,s] == u in ASCENDING p -- the sequential
//      index_add_ order of the reference (conv_dx_rowsub_gather).
// dG row-major [batch*rows][9*CIN] fp32 in the workspace, behind the slabs.
struct DgArgs {
  const float* dpre;
  const float* w;
  float* dg;
  int total_rows;  // batch * rows
  int n_groups;    // column groups per 16-row tile (divides 9*CIN/16)
  int nb;          // workgroups of this half
};
// LDS of a dG workgroup: W^T of its column group, [ntg*16][COUT + 4]
template <int CIN, int COUT>
constexpr int dg_lds_floats(int n_groups) { return kSeq * CIN / n_groups * (COUT + 4); }

// v_mfma_f32_16x16x4_f32.  A workgroup owns one column group (ntg 16-wide
// n-tiles, the same for its 4 waves) and 4 consecutive 16-row tiles, a wave
// one tile.  Lane (i, kg) holds dpre row i's channels [kg*COUT/4, +COUT/4)
// (MFMA step t uses o = kg*COUT/4 + t, B permuted the same way: exact f32
// sums over o); B from the group's W^T staged in LDS as wl[n][o] (row pad 4:
// conflict-free ds_read_b128 for 16 consecutive n).  Every dG element is
// written exactly once.
template <int CIN, int COUT>
__device__ __forceinline__ void conv_dg_body(int vb, int vnb, const DgArgs& g, float* wl) {
  constexpr int K = kSeq * CIN, NT = K / 16, KP = COUT / 4, LDW = COUT + 4;
  const int lane = threadIdx.x & 63, j = lane & 15, kg = lane >> 4;
  const int wgi = xcd_block_of(vb, vnb);
  const int ntg = NT / g.n_groups, grp = wgi % g.n_groups;
  const int rt = (wgi / g.n_groups) * 4 + (threadIdx.x >> 6);
  const int row = min(rt * 16 + j, g.total_rows - 1);  // clamp loads, stores masked
  f32x4 a[KP / 4];
#pragma unroll
  for (int q = 0; q < KP / 4; ++q) a[q] = ld4(g.dpre + (long)row * COUT + kg * KP + 4 * q);
  // stage the group's W^T (A loads in flight); consecutive threads take
  // consecutive o (conflict-free LDS writes)
  const int n0 = grp * ntg * 16;
  // (4 loads per thread in flight per batch: a load -> store loop exposed one
  // memory latency per element)
  for (int e0 = threadIdx.x; e0 < COUT * ntg * 4; e0 += 4 * (int)blockDim.x) {
    f32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = min(e0 + q * (int)blockDim.x, COUT * ntg * 4 - 1);
      v[q] = ld4(g.w + (e % COUT) * K + n0 + (e / COUT) * 4);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = e0 + q * (int)blockDim.x;
      if (e < COUT * ntg * 4) {
        const int o = e % COUT, n4 = (e / COUT) * 4;
        wl[(n4 + 0) * LDW + o] = v[q].x;
        wl[(n4 + 1) * LDW + o] = v[q].y;
        wl[(n4 + 2) * LDW + o] = v[q].z;
        wl[(n4 + 3) * LDW + o] = v[q].w;
      }
    }
  }
  __syncthreads();
  if (rt * 16 >= g.total_rows) return;
  // transposed orientation: D[i = n][j = row] (A = W^T from LDS, B = dpre),
  // so a lane's 4 accumulator values are dG[row j][n 4kg .. 4kg+3], one 16-B
  // store (the [row][n] orientation needed 4 dword stores per lane)
  const int row_out = rt * 16 + j;
  float* out = g.dg + (long)row_out * K + n0 + 4 * kg;
  for (int nt = 0; nt < ntg; ++nt) {
    const float* bp = wl + (nt * 16 + j) * LDW + kg * KP;
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) {
      const f32x4 wv = *reinterpret_cast<const f32x4*>(bp + 4 * q);
      f32x4& ac = acc[q & 1];
      ac = mfma16(wv.x, a[q].x, ac);
      ac = mfma16(wv.y, a[q].y, ac);
      ac = mfma16(wv.z, a[q].z, ac);
      ac = mfma16(wv.w, a[q].w, ac);
    }
    if (row_out < g.total_rows) st4(out + nt * 16, acc[0] + acc[1]);
  }
}

// dG workgroups and dW-slab workgroups (conv_dw_lat_body) of one Enblock conv
// interleaved in one launch, as conv_bwd_lat_pair.
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv_bwd_rowsub_pair(const DgArgs a, const DwLatArgs d) {
  extern __shared__ float wl[];
  __shared__ float red[lat_red_floats(4)];
  // the data-gradient role first: it is the longer one, and the dW
  // workgroups fill the slots its retiring waves free (alternating the
  // roles: D1 27.4 vs 25.8 us, D0 24.2 vs 19.6 us, same box)
  const int bid = (int)blockIdx.x;
  const bool is_dg = bid < a.nb;
  const int vb = is_dg ? bid : bid - a.nb;
  if (is_dg)
    conv_dg_body<CIN, COUT>(vb, a.nb, a, wl);
  else
    conv_dw_lat_body<CIN, COUT>(vb, d.nb, d.x, d.idx, d.dpre, d.ws, d.ws_db, d.vsrc, d.rows,
                                d.total_rows, d.rchunk, d.n_chunks, d.batch, d.xvm, d.dpvm, red);
}

// (2): a thread per (source row, 16-B channel chunk); the row's flat list
// (4*G entries, -1 padded) is read as G int4 loads (one address per row ->
// broadcast), every dG load is an unconditional buffer load (an absent entry
// is an out-of-range offset: 0.0, no memory access), all in flight together;
// summed in list order; elu'(elu_y) epilogue.
template <int CIN, int G, typename TY = float>
__global__ __launch_bounds__(256) void conv_dx_rowsub_gather(const float* __restrict__ dg,
                                                             const int4* __restrict__ flat,
                                                             const TY* __restrict__ elu_y,
                                                             TY* __restrict__ dx, int vsrc,
                                                             int rows, int total_src,
                                                             int dg_bytes, int batch, int dxvm) {
  constexpr int Q = CIN / 4;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total_src * Q) return;
  const int m = t / Q, q = t - m * Q;
  int b, u;
  split_row(m, dxvm, batch, vsrc, b, u);  // dx / elu_y rows in dx's layout; dG batch-major
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dg), 0, dg_bytes, 0x00020000);
  const int base = (b * rows * kSeq * CIN + 4 * q) * (int)sizeof(float);
  int4 e[G];
#pragma unroll
  for (int k = 0; k < G; ++k) e[k] = flat[u * G + k];
  auto off = [&](int p) { return p >= 0 ? base + p * (CIN * (int)sizeof(float)) : kAbsentRow; };
  f32x4 v[4 * G];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    v[4 * k + 0] = buf_ld4(rsrc, off(e[k].x));
    v[4 * k + 1] = buf_ld4(rsrc, off(e[k].y));
    v[4 * k + 2] = buf_ld4(rsrc, off(e[k].z));
    v[4 * k + 3] = buf_ld4(rsrc, off(e[k].w));
  }
  f32x4 s = v[0];
#pragma unroll
  for (int k = 1; k < 4 * G; ++k) s += v[k];
  if (elu_y) {
    const f32x4 y = ld4f(elu_y + (long)m * CIN + 4 * q);
    s.x *= elu_grad_from_out(y.x);
    s.y *= elu_grad_from_out(y.y);
    s.z *= elu_grad_from_out(y.z);
    s.w *= elu_grad_from_out(y.w);
  }
  st4f(dx + (long)m * CIN + 4 * q, s);  // bf16 storage: one rounding of the fp32 sum
}

// Batched weight-gradient reduction: ONE launch reduces the deferred slab
// sets of several layers (each left in its own workspace by a deferred
// cfsd_spiral_conv_bwd_weight / cfsd_spiral_conv_bwd call), instead of one
// reduce launch per layer.  Item kinds: 0 = conv_dw_mfma slabs
// ([nslab][U*1024] + db [nslab][COUT], mapped like conv_dw_reduce), 1 =
// plain slabs [nslab][COUT*K + COUT] (small-channel kernels, fused xyz
// backward).  Same fixed summation order as the per-layer reduces.
struct DwRedItem {
  const float* ws;
  const float* ws_db;
  float* dw;
  float* db;
  int kind, cin, cout, n_slabs, n_el, blk0;
};
constexpr int kMaxDwRed = 16;
// Optional Adam step fused into the reduction (single-process training: no
// gradient exchange between the reduce and the update).  Every reduced
// element is updated by the thread that produced its gradient; the elements
// no item covers ([lo, hi) ranges of the flat buffers, e.g. the Linears)
// by the workgroups past the reduction's.
constexpr int kMaxAdamRest = 2 * kMaxDwRed + 2;
struct DwAdam {
  float* p;
  const float* g;  // flat gradient buffer the items' dw/db point into
  float* m;
  float* v;
  bf16_t* shadow;
  const int* step;
  float lr, b1, b2, eps, wd;
  int n_rest;
  long rest_lo[kMaxAdamRest], rest_hi[kMaxAdamRest], rest_blk0[kMaxAdamRest + 1];
};
struct DwRedBatch {
  DwRedItem it[kMaxDwRed];
  int n;
  int blk_end;  // first workgroup past the reductions
  DwAdam adam;  // adam.p == nullptr: no fused update
};

__device__ __forceinline__ void adam_consts(const DwAdam& a, float& step_size, float& sqrt_bc2) {
  const int t = *a.step;
  step_size = a.lr / (1.f - powf(a.b1, (float)t));
  sqrt_bc2 = sqrtf(1.f - powf(a.b2, (float)t));
}
// Adam on the element whose gradient (value g) was just written at gp.
__device__ __forceinline__ void adam_at(const DwAdam& a, const float* gp, float g, float step_size,
                                        float sqrt_bc2) {
  const long o = gp - a.g;
  float pv = a.p[o], mv = a.m[o], vv = a.v[o];
  adam_elem(pv, g, mv, vv, a.b1, a.b2, a.eps, a.wd, step_size, sqrt_bc2);
  a.p[o] = pv;
  a.m[o] = mv;
  a.v[o] = vv;
  if (a.shadow) stf(a.shadow + o, pv);
}

// Adam on 4 consecutive elements (gradients g) starting at gp: every load
// issued before the first update (the per-element helper's store-to-load
// order serialised four memory round trips); same arithmetic per element.
__device__ __forceinline__ void adam_at4(const DwAdam& a, const float* gp, const f32x4 g, float step_size,
                                         float sqrt_bc2) {
  const long o = gp - a.g;
  float pv[4], mv[4], vv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    pv[e] = a.p[o + e];
    mv[e] = a.m[o + e];
    vv[e] = a.v[o + e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    adam_elem(pv[e], g[e], mv[e], vv[e], a.b1, a.b2, a.eps, a.wd, step_size, sqrt_bc2);
    a.p[o + e] = pv[e];
    a.m[o + e] = mv[e];
    a.v[o + e] = vv[e];
    if (a.shadow) stf(a.shadow + o + e, pv[e]);
  }
}

// Items whose slab length is a multiple of 4 (every conv_dw_mfma / lat
// item: U*1024 + cout) are reduced four consecutive elements per lane with
// 16-B loads (256 elements per workgroup); the others (small-channel slabs)
// one element per lane.  Same per-element summation order either way.
#ifndef CFSD_RED_LOADS
#define CFSD_RED_LOADS 8
#endif
constexpr int kRedLoads = CFSD_RED_LOADS;
__device__ __forceinline__ void dw_reduce_batch_body(const DwRedBatch& B, const int vb) {
  const bool fuse = B.adam.p != nullptr;
  if (fuse && vb >= B.blk_end) {  // Adam on the elements no item covers
    const DwAdam& a = B.adam;
    float step_size, sqrt_bc2;
    adam_consts(a, step_size, sqrt_bc2);
    const int rb = vb - B.blk_end;
    int ri = 0;
    while (ri + 1 < a.n_rest && rb >= a.rest_blk0[ri + 1]) ++ri;
    const long base = a.rest_lo[ri] + (long)(rb - a.rest_blk0[ri]) * 4096;
    const long hi = a.rest_hi[ri];
    float gv[4], pv[4], mv[4], vv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // all loads first (clamped), then the updates
      const long o = min(base + k * 1024 + threadIdx.x, hi - 1);
      gv[k] = a.g[o];
      pv[k] = a.p[o];
      mv[k] = a.m[o];
      vv[k] = a.v[o];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long o = base + k * 1024 + threadIdx.x;
      if (o < hi) {
        adam_elem(pv[k], gv[k], mv[k], vv[k], a.b1, a.b2, a.eps, a.wd, step_size, sqrt_bc2);
        a.p[o] = pv[k];
        a.m[o] = mv[k];
        a.v[o] = vv[k];
        if (a.shadow) stf(a.shadow + o, pv[k]);
      }
    }
    return;
  }
  int li = 0;
  while (li + 1 < B.n && vb >= B.it[li + 1].blk0) ++li;
  const DwRedItem d = B.it[li];
  __shared__ f32x4 part[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int K = kSeq * d.cin;
  const int nw = d.n_el - d.cout;  // kind 0: dW part of a slab
  const bool vec = d.kind == 0;     // n_el, nw and cout are multiples of 4
  const int per_blk = vec ? 256 : 64;
  int f = (vb - d.blk0) * per_blk + (vec ? 4 * lane : lane);
  const bool valid = f < d.n_el;
  if (!valid) f = vec ? d.n_el - 4 : d.n_el - 1;
  const float* src;
  long stride;
  if (d.kind == 0) {
    src = f < nw ? d.ws + f : d.ws_db + (f - nw);
    stride = f < nw ? nw : d.cout;
  } else {
    src = d.ws + f;
    stride = d.n_el;
  }
  // slabs p = wv, wv + 16, ... summed in that order; every pass issues its
  // 16 loads together, the partial last pass too (clamped loads, masked adds:
  // a per-slab tail loop paid one memory round trip per slab -- up to 14 for
  // the ~200-slab lat items)
  // (kRedLoads slabs per batch: 8 keeps the kernel at <= 64 VGPRs, two
  // workgroups per CU, so one workgroup's combine / Adam tail overlaps the
  // other's loads; the per-element order is unchanged)
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  const int last = d.n_slabs - 1;
  if (vec) {
    for (int p = wv; p < d.n_slabs; p += 16 * kRedLoads) {
      f32x4 t[kRedLoads];
#pragma unroll
      for (int j = 0; j < kRedLoads; ++j) t[j] = ld4(src + (long)min(p + 16 * j, last) * stride);
#pragma unroll
      for (int j = 0; j < kRedLoads; ++j)
        if (p + 16 * j < d.n_slabs) sum += t[j];
    }
  } else {
    for (int p = wv; p < d.n_slabs; p += 16 * kRedLoads) {
      float t[kRedLoads];
#pragma unroll
      for (int j = 0; j < kRedLoads; ++j) t[j] = src[(long)min(p + 16 * j, last) * stride];
#pragma unroll
      for (int j = 0; j < kRedLoads; ++j)
        if (p + 16 * j < d.n_slabs) sum.x += t[j];
    }
  }
  part[wv][lane] = sum;
  __syncthreads();
  if (wv == 0 && valid) {
    f32x4 t = part[0][lane];
#pragma unroll 3
    for (int q = 1; q < 16; ++q) t += part[q][lane];
    float step_size = 0.f, sqrt_bc2 = 1.f;
    if (fuse) adam_consts(B.adam, step_size, sqrt_bc2);
    if (!vec) {
      float* dst = f >= nw ? d.db + (f - nw) : d.dw + f;
      *dst = t.x;
      if (fuse) adam_at(B.adam, dst, t.x, step_size, sqrt_bc2);
    } else if (f >= nw) {
#pragma unroll
      for (int e = 0; e < 4; ++e) d.db[f - nw + e] = t[e];
      if (fuse) adam_at4(B.adam, d.db + f - nw, t, step_size, sqrt_bc2);
    } else {
      // 4 consecutive elements of one 32-wide unit row: 4 consecutive c
      const int CT = d.cin / 32, OT = d.cout / 32;
      const int un = f >> 10, within = f & 1023;
      const int cc = (un % CT) * 32 + (within & 31);
      const int o = ((un / CT) % OT) * 32 + (within >> 5);
      const int sl = un / (CT * OT);
      float* dst = d.dw + (long)o * K + sl * d.cin + cc;  // 8-B aligned in the flat buffer
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = t[e];
      if (fuse) adam_at4(B.adam, dst, t, step_size, sqrt_bc2);
    }
  }
}
#ifdef CFSD_LAT_STAMPS
// diagnostic build only (tools/kbench.py KB_STAMPFN=cfsd_debug_red_stamps): role (1 reduce, 2 Adam rest), start, end
__device__ unsigned long long g_red_stamps[4096 * 3];
extern "C" int cfsd_debug_red_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_red_stamps), sizeof(g_red_stamps), 0, hipMemcpyDeviceToHost);
}
#endif
__global__ __launch_bounds__(1024, kRedLoads <= 8 ? 8 : 4) void dw_reduce_batch_k(const DwRedBatch B) {
#ifdef CFSD_LAT_STAMPS
  const unsigned long long t0 = wall_clock64();
#endif
  // the Adam-only workgroups (the elements no item covers: the Linears) are
  // dispatched FIRST: the launch is 704 workgroups at two per CU, and as the
  // last of the grid they waited ~7 us for slots the slab reductions held
  // (role stamps, profiles/round8o_*), then ran their own trips at the end
  const int nrest = (B.adam.p != nullptr) ? (int)gridDim.x - B.blk_end : 0;
  const int vb = (int)blockIdx.x < nrest ? B.blk_end + (int)blockIdx.x : (int)blockIdx.x - nrest;
  dw_reduce_batch_body(B, vb);
#ifdef CFSD_LAT_STAMPS
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x < 4096) {
    g_red_stamps[3 * blockIdx.x] = vb >= B.blk_end ? 2 : 1;
    g_red_stamps[3 * blockIdx.x + 1] = t0;
    g_red_stamps[3 * blockIdx.x + 2] = wall_clock64();
  }
#endif
}

// Backward weight, small input (CS <= 4; first Enblock): lane = output
// channel o, 64/COUT rows per wave in flight; each lane accumulates its
// kSeq*CS weight partials over a strided row range; waves are combined in
// LDS in fixed order; one slab [COUT*K + COUT] per block.
template <int CS, int COUT>
__global__ __launch_bounds__(256) void conv_dw_in_small(const float* __restrict__ x,
                                                        const int* __restrict__ idx,
                                                        const float* __restrict__ dpre,
                                                        float* __restrict__ ws, int vsrc,
                                                        int rows, long total_rows) {
  constexpr int K = kSeq * CS;
  constexpr int RPW = 64 / COUT;  // row slots per wave
  constexpr int NEL = COUT * K + COUT;
  __shared__ float red[NEL];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int o = lane % COUT, slot = lane / COUT;
  float acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = 0.f;
  const long stride = (long)gridDim.x * 4 * RPW;
  for (long m = ((long)blockIdx.x * 4 + wave) * RPW + slot; m < total_rows; m += stride) {
    int b, r;
    divmod32(m, rows, b, r);
    const float d = dpre[m * COUT + o];
    const float* xb = x + (long)b * vsrc * CS;
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      const float* p = xb + (long)idx[(long)r * kSeq + s] * CS;
#pragma unroll
      for (int c = 0; c < CS; ++c) acc[s * CS + c] = fmaf(d, p[c], acc[s * CS + c]);
    }
    acc[K] += d;
  }
  // combine row slots inside the wave (lanes with equal o)
#pragma unroll
  for (int k = 0; k <= K; ++k)
#pragma unroll
    for (int d = COUT; d < 64; d <<= 1) acc[k] += __shfl_xor(acc[k], d);
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv && slot == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int e = o * K + k;
        red[e] = wv == 0 ? acc[k] : red[e] + acc[k];
      }
      const int e = COUT * K + o;
      red[e] = wv == 0 ? acc[K] : red[e] + acc[K];
    }
    __syncthreads();
  }
  for (int e = tid; e < NEL; e += 256) ws[(long)blockIdx.x * NEL + e] = red[e];
}

// Backward weight, small output (CO <= 4; last decoder conv): L = CIN/4
// lanes per row; lane q accumulates dW[o][s*CIN + 4q .. +4] for all o, s.
template <int CIN, int CO>
__global__ __launch_bounds__(256) void conv_dw_out_small(const float* __restrict__ x,
                                                         const int* __restrict__ idx,
                                                         const float* __restrict__ dpre,
                                                         float* __restrict__ ws, int vsrc,
                                                         int rows, long total_rows) {
  constexpr int L = CIN / 4;
  constexpr int K = kSeq * CIN;
  constexpr int RPW = 64 / L;
  constexpr int NEL = CO * K + CO;
  __shared__ float red[NEL];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int q = lane % L, slot = lane / L;
  f32x4 acc[kSeq][CO];
  float dbs[CO];
#pragma unroll
  for (int s = 0; s < kSeq; ++s)
#pragma unroll
    for (int o = 0; o < CO; ++o) acc[s][o] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < CO; ++o) dbs[o] = 0.f;
  const long stride = (long)gridDim.x * 4 * RPW;
  for (long m = ((long)blockIdx.x * 4 + wave) * RPW + slot; m < total_rows; m += stride) {
    int b, r;
    divmod32(m, rows, b, r);
    float d[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) d[o] = dpre[m * CO + o];
    const float* xb = x + (long)b * vsrc * CIN + 4 * q;
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      const f32x4 v = ld4(xb + (long)idx[(long)r * kSeq + s] * CIN);
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        acc[s][o].x = fmaf(d[o], v.x, acc[s][o].x);
        acc[s][o].y = fmaf(d[o], v.y, acc[s][o].y);
        acc[s][o].z = fmaf(d[o], v.z, acc[s][o].z);
        acc[s][o].w = fmaf(d[o], v.w, acc[s][o].w);
      }
    }
#pragma unroll
    for (int o = 0; o < CO; ++o) dbs[o] += d[o];
  }
#pragma unroll
  for (int s = 0; s < kSeq; ++s)
#pragma unroll
    for (int o = 0; o < CO; ++o)
#pragma unroll
      for (int dd = L; dd < 64; dd <<= 1) {
        acc[s][o].x += __shfl_xor(acc[s][o].x, dd);
        acc[s][o].y += __shfl_xor(acc[s][o].y, dd);
        acc[s][o].z += __shfl_xor(acc[s][o].z, dd);
        acc[s][o].w += __shfl_xor(acc[s][o].w, dd);
      }
#pragma unroll
  for (int o = 0; o < CO; ++o)
#pragma unroll
    for (int dd = L; dd < 64; dd <<= 1) dbs[o] += __shfl_xor(dbs[o], dd);
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv && slot == 0) {
#pragma unroll
      for (int s = 0; s < kSeq; ++s)
#pragma unroll
        for (int o = 0; o < CO; ++o) {
          const int e = o * K + s * CIN + 4 * q;
          const f32x4 v = acc[s][o];
          if (wv == 0) {
            red[e] = v.x; red[e + 1] = v.y; red[e + 2] = v.z; red[e + 3] = v.w;
          } else {
            red[e] += v.x; red[e + 1] += v.y; red[e + 2] += v.z; red[e + 3] += v.w;
          }
        }
      if (q == 0)
#pragma unroll
        for (int o = 0; o < CO; ++o) red[CO * K + o] = wv == 0 ? dbs[o] : red[CO * K + o] + dbs[o];
    }
    __syncthreads();
  }
  for (int e = tid; e < NEL; e += 256) ws[(long)blockIdx.x * NEL + e] = red[e];
}

// ==========================================================================
// Rank-64 MFMA update used by the 3-channel weight gradients.  A wave holds
// a 64-row tile whose per-row 27/28-vector (gathered xyz, or the spiral-
// transposed dpre) was written transposed into wave-private LDS,
// At[i][k] (i < 32 padded with zero rows, k = tile row), and multiplies it by
// the tile's rows of a dense row-major matrix B (dpre, or the layer input):
//   acc[ct] (32 x 32) += At (32 x 64) . B[row0 .. row0+64)[ct*32 .. +32).
// v_mfma_f32_32x32x2_f32 with k-order (kk, kk+32) per step so each lane
// reads its A values as one ds_read_b128 per 4 steps.
constexpr int kAts = 68;  // At row stride (floats): 16-B aligned, bank-spread

template <int NCT, typename TB>
__device__ __forceinline__ void rank64_mfma(const float* At, const TB* __restrict__ B,
                                            long row0, long nrows, int ldb, f32x16 (&acc)[NCT],
                                            int lane) {
  const int i = lane & 31, h = lane >> 5;
#pragma unroll
  for (int kk = 0; kk < 32; kk += 4) {
    const f32x4 a = ld4(&At[i * kAts + 32 * h + kk]);
    float bv[4][NCT];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      long rr = row0 + kk + j + 32 * h;
      if (rr >= nrows) rr = nrows - 1;  // its A column is zero
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) bv[j][ct] = ldf(&B[rr * ldb + ct * 32 + i]);
    }
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      acc[ct] = mfma32(a.x, bv[0][ct], acc[ct]);
      acc[ct] = mfma32(a.y, bv[1][ct], acc[ct]);
      acc[ct] = mfma32(a.z, bv[2][ct], acc[ct]);
      acc[ct] = mfma32(a.w, bv[3][ct], acc[ct]);
    }
  }
}

// LDS writes by some lanes -> reads by other lanes of the same wave: LDS
// executes a wave's instructions in order, so a counter wait plus a compiler
// barrier is enough (no s_barrier; waves run independent tile counts).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Backward weight, small input (CS <= 3; first Enblock) on MFMA:
//   dW^T[(s,c)][o] = sum_m G[m][(s,c)] dpre[m][o],   db[o] = sum_m 1 * dpre[m][o]
// where G is the gathered input (27 values per row); row 27 of At is the
// all-ones row so db falls out of the same MFMAs.  Persistent waves over
// 64-row tiles, block partials combined in fixed order -> one slab
// [COUT*K + COUT] per block (reduced by slab_reduce).
template <int CS, int COUT, typename TD = float>
__global__ __launch_bounds__(256) void conv_dw_in_mfma(const float* __restrict__ x,
                                                       const int* __restrict__ idx,
                                                       const TD* __restrict__ dpre,
                                                       float* __restrict__ ws, int vsrc, int rows,
                                                       long total_rows, int batch, int xvm,
                                                       int dpvm) {
  constexpr int K = kSeq * CS, NI = K + 1, NCT = COUT / 32, NEL = COUT * K + COUT;
  static_assert(NI <= 32 && COUT % 32 == 0, "shape");
  __shared__ float at_all[4 * 32 * kAts];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* At = at_all + wave * 32 * kAts;
  for (int e = lane; e < (32 - NI) * kAts; e += 64) At[NI * kAts + e] = 0.f;
  f32x16 acc[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ct][r] = 0.f;
  const long n_tiles = (total_rows + 63) / 64;
  for (long tile = (long)blockIdx.x * 4 + wave; tile < n_tiles; tile += (long)gridDim.x * 4) {
    const long m = tile * 64 + lane;
    const bool valid = m < total_rows;
    const long mm = valid ? m : total_rows - 1;
    int b, r;
    split_row(mm, dpvm, batch, rows, b, r);  // K (rows) in dpre's layout
    const Lay lx = make_lay(xvm, batch, vsrc);
    const float* xb = x + (long)b * lx.bs * CS;
    const int* ir = idx + (long)r * kSeq;
    float xv[K];
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      ld_row<CS>(xb + (long)ir[s] * lx.vs * CS, &xv[s * CS]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) At[k * kAts + lane] = valid ? xv[k] : 0.f;
    At[K * kAts + lane] = valid ? 1.f : 0.f;
    wave_lds_sync();
    rank64_mfma<NCT>(At, dpre, tile * 64, total_rows, COUT, acc, lane);
    wave_lds_sync();
  }
  __syncthreads();
  float* red = at_all;  // reuse: NEL floats
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int i = acc_row(rr, lane), o = ct * 32 + (lane & 31);
          if (i < NI) {
            const int e = i < K ? o * K + i : COUT * K + o;
            red[e] = wv == 0 ? acc[ct][rr] : red[e] + acc[ct][rr];
          }
        }
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < NEL; e += 256) ws[(long)blockIdx.x * NEL + e] = red[e];
}

// Backward of a small-output conv (CO*kSeq <= 32; the xyz output conv),
// data + weight fused, in source-row space.  Per source row (b, u) a thread
// folds the spiral transpose in the CO-wide dpre space,
//   t[s][o] = sum_{r : idx[r][s] = u} dpre[b][r][o]       (inv_head + overflow)
// and then produces
//   dx[b][u][c]  = g * sum_{s,o} t[s][o] W[o][s*CIN + c]   (VALU, W as SGPRs)
//   dW[o][s*CIN + c] += t[s][o] x[b][u][c]                  (rank-64 MFMA per tile)
//   db[o] += t[0][o]        (every row r appears once in slot 0's lists)
// The dW identity is the same double sum as sum_r dpre[r] x[idx[r][s]],
// regrouped by source row, so x is read densely instead of gathered.
template <int CIN, int CO>
__global__ __launch_bounds__(256) void conv_bwd_out_small(
    const float* __restrict__ dpre, const int* __restrict__ inv_ptr,
    const int* __restrict__ inv_row, const int4* __restrict__ inv_head,
    const float* __restrict__ w, const float* __restrict__ elu_y, const float* __restrict__ x,
    float* __restrict__ dx, float* __restrict__ ws, int vsrc, int rows, long total_rows) {
  constexpr int K = kSeq * CIN, NI = kSeq * CO, NCT = CIN / 32, NEL = CO * K + CO;
  static_assert(NI <= 32 && CIN % 32 == 0, "shape");
  __shared__ float at_all[4 * 32 * kAts];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* At = at_all + wave * 32 * kAts;
  for (int e = lane; e < (32 - NI) * kAts; e += 64) At[NI * kAts + e] = 0.f;
  f32x16 acc[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ct][r] = 0.f;
  float dbs[CO];
#pragma unroll
  for (int o = 0; o < CO; ++o) dbs[o] = 0.f;
  const long n_tiles = (total_rows + 63) / 64;
  for (long tile = (long)blockIdx.x * 4 + wave; tile < n_tiles; tile += (long)gridDim.x * 4) {
    const long m = tile * 64 + lane;
    const bool valid = m < total_rows;
    const long mm = valid ? m : total_rows - 1;
    int b, u;
    divmod32(mm, vsrc, b, u);
    const float* db_ = dpre + (long)b * rows * CO;
    const int4* pu = inv_head + (long)u * kSeq;
    int4 pr[kSeq];
#pragma unroll
    for (int s = 0; s < kSeq; ++s) pr[s] = pu[s];
    float tt[kSeq][CO];
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      const float* p0 = db_ + (long)max(pr[s].x, 0) * CO;
      const float* p1 = db_ + (long)max(pr[s].y, 0) * CO;
      const float f0 = present(pr[s].x), f1 = present(pr[s].y);
#pragma unroll
      for (int o = 0; o < CO; ++o) tt[s][o] = p0[o] * f0 + p1[o] * f1;
    }
    fold_head_tail<kSeq, CO>(pr, (long)u * kSeq, db_, inv_ptr, inv_row, tt);
    if (!valid) {
#pragma unroll
      for (int s = 0; s < kSeq; ++s)
#pragma unroll
        for (int o = 0; o < CO; ++o) tt[s][o] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < kSeq; ++s)
#pragma unroll
      for (int o = 0; o < CO; ++o) At[(s * CO + o) * kAts + lane] = tt[s][o];
#pragma unroll
    for (int o = 0; o < CO; ++o) dbs[o] += tt[0][o];
    if (dx && valid) {
      float* out = dx + mm * CIN;
      const float* ey = elu_y ? elu_y + mm * CIN : nullptr;
#pragma unroll
      for (int c4 = 0; c4 < CIN / 4; ++c4) {
        f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kSeq; ++s)
#pragma unroll
          for (int o = 0; o < CO; ++o) {
            const float* wp = w + o * K + s * CIN + 4 * c4;
            a4.x = fmaf(tt[s][o], wp[0], a4.x);
            a4.y = fmaf(tt[s][o], wp[1], a4.y);
            a4.z = fmaf(tt[s][o], wp[2], a4.z);
            a4.w = fmaf(tt[s][o], wp[3], a4.w);
          }
        if (ey) {
          const f32x4 g = ld4(ey + 4 * c4);
          a4.x *= elu_grad_from_out(g.x);
          a4.y *= elu_grad_from_out(g.y);
          a4.z *= elu_grad_from_out(g.z);
          a4.w *= elu_grad_from_out(g.w);
        }
        st4(out + 4 * c4, a4);
      }
    }
    wave_lds_sync();
    rank64_mfma<NCT>(At, x, tile * 64, total_rows, CIN, acc, lane);
    wave_lds_sync();
  }
#pragma unroll
  for (int o = 0; o < CO; ++o)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) dbs[o] += __shfl_xor(dbs[o], d);
  __syncthreads();
  float* red = at_all;
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int i = acc_row(rr, lane), c = ct * 32 + (lane & 31);
          if (i < NI) {
            const int e = (i % CO) * K + (i / CO) * CIN + c;
            red[e] = wv == 0 ? acc[ct][rr] : red[e] + acc[ct][rr];
          }
        }
      if (lane == 0)
#pragma unroll
        for (int o = 0; o < CO; ++o) red[CO * K + o] = wv == 0 ? dbs[o] : red[CO * K + o] + dbs[o];
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < NEL; e += 256) ws[(long)blockIdx.x * NEL + e] = red[e];
}

// Same fused backward on MFMA (the kernel the step uses).  A wave owns
// 32-source-row tiles (XCD-aware persistent sweep).  Lane (i, h) = (row,
// half) folds only HALF of the row's spiral transpose: slots
// s = 5h .. 5h + 4 (s < 9), i.e. t values k = s*CO + o in [h*KH, h*KH + KH),
// KH = 5*CO, which is exactly the A operand it feeds to
//   dx (32 x CIN) = T (32 x 2KH) . Wt (2KH x CIN),  Wt[k][c] = W[o][s*CIN + c]
// (v_mfma_f32_32x32x2_f32, step j pairs k = j and k = KH + j; Wt in VGPRs).
// T is also written to wave-private LDS as At[k][row] and
//   dW^T (32 x CIN) += At (2KH x 32 rows) . x_tile (32 rows x CIN)
// runs as 16 more MFMA steps whose K order (rows) is the accumulator row
// order acc_row(j, lane): the x values that feed B are then the same
// registers the dx epilogue needs for elu'(y) when elu_y == x (the model's
// case: the output conv's input is the last Deblock's ELU output).
// CO (1..3) consecutive floats of one dpre row in ONE buffer load.
template <int CO>
__device__ __forceinline__ void load_row(__amdgpu_buffer_rsrc_t rsrc, int off, float (&v)[CO]) {
  // (bit-cast whole vectors: a bit_cast of a vector ELEMENT lvalue miscompiles
  // to element 0 on this clang)
  if constexpr (CO == 3) {
    typedef float f32x3 __attribute__((ext_vector_type(3)));
    const f32x3 t = __builtin_bit_cast(f32x3, __builtin_amdgcn_raw_buffer_load_b96(rsrc, off, 0, 0));
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
  } else if constexpr (CO == 2) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 t = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, 0, 0));
    v[0] = t.x;
    v[1] = t.y;
  } else {
    v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
  }
}
constexpr int kAtS = 36;  // At row stride: conflict-free ds_read_b128 of the dW A operand
constexpr int kBwdOutOcc = 1;
template <int CIN, int CO, typename TX = float>
__global__ __launch_bounds__(256, kBwdOutOcc) void conv_bwd_out_mfma(
    const float* __restrict__ dpre, const int* __restrict__ inv_ptr,
    const int* __restrict__ inv_row, const int4* __restrict__ inv_head,
    const float* __restrict__ w, const TX* __restrict__ elu_y, const TX* __restrict__ x,
    TX* __restrict__ dx, float* __restrict__ ws, int vsrc, int rows, long total_rows, int batch,
    int xvm, int dpvm) {
  constexpr int SPH = 5, KH = SPH * CO, K = kSeq * CIN, NCT = CIN / 32, NEL = CO * K + CO;
  static_assert(2 * KH <= 32 && CIN % 32 == 0, "shape");
  __shared__ float at_all[4 * 32 * kAtS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, h = lane >> 5;
  float* At = at_all + wave * 32 * kAtS;
  for (int e = lane; e < (32 - 2 * KH) * kAtS; e += 64) At[2 * KH * kAtS + e] = 0.f;
  // Wt (B operand of dx): lane (c, h) holds Wt[h*KH + j][ct*32 + c]
  float wt[NCT][KH];
#pragma unroll
  for (int j = 0; j < KH; ++j) {
    const int k = h * KH + j, sl = k / CO, o = k % CO;
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
      wt[ct][j] = sl < kSeq ? w[o * K + sl * CIN + ct * 32 + li] : 0.f;
  }
  f32x16 dwacc[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) dwacc[ct][r] = 0.f;
  float dbs[CO];
#pragma unroll
  for (int o = 0; o < CO; ++o) dbs[o] = 0.f;
  const int ey_mode = elu_y == nullptr ? 0 : (elu_y == x ? 1 : 2);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(dpre), 0, (int)(total_rows / vsrc * rows * CO * (long)sizeof(float)), 0x00020000);
  const Lay ldp = make_lay(dpvm, batch, rows);
  const long n_tiles = (total_rows + 31) / 32;
  const TileSweep sw = xcd_sweep(n_tiles, 4, wave);
  for (long tile = sw.begin; tile < sw.end; tile += sw.step) {
    const long row0 = tile * 32;
    // half-row spiral transpose in the CO-wide dpre space
    const long m = row0 + li;
    const bool valid = m < total_rows;
    const long mm = valid ? m : total_rows - 1;
    int b, u;
    split_row(mm, xvm, batch, vsrc, b, u);  // source rows (x, dx, elu_y) in x's layout
    // x tile in accumulator-row order (B operand of dW, elu' source); issued
    // first: independent of the inverse-spiral chain, so their latency hides
    // behind it
    float xv[NCT][16];
    const TX* xt = x + row0 * CIN + li;
    const int last = (int)(total_rows - 1 - row0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int rr = min(acc_row(j, lane), last);  // clamped rows have a zero At column
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) xv[ct][j] = ldf(&xt[rr * CIN + ct * 32]);
    }
    const float* db_ = dpre + (long)b * ldp.bs * CO;
    const int dstride = ldp.vs * CO;  // floats between consecutive rows of one mesh's dpre
    const int4 none = make_int4(-1, -1, -1, -1);
    int4 pr[SPH];
#pragma unroll
    for (int sl = 0; sl < SPH; ++sl) {
      const int sg = h * SPH + sl;
      pr[sl] = sg < kSeq ? inv_head[u * kSeq + sg] : none;
    }
    // list rows 0..2 of the 5 keys: 45 unconditional buffer dword loads in
    // flight together (absent rows out of range: 0, no traffic); rows 3..
    // (0.3 % of keys) through an exec branch
    float tt[SPH][CO];
    const int base = b * ldp.bs * CO * (int)sizeof(float);
#pragma unroll
    for (int sl = 0; sl < SPH; ++sl) {
      const int hr[3] = {pr[sl].x, pr[sl].y, pr[sl].z};
      float v[3][CO];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int off = hr[j] >= 0 ? base + hr[j] * dstride * (int)sizeof(float) : kAbsentRow;
        // one load per list row: the texture path costs a cycle per distinct
        // cache line per instruction, so per-channel dword loads tripled it
        load_row<CO>(rsrc, off, v[j]);
      }
#pragma unroll
      for (int o = 0; o < CO; ++o) tt[sl][o] = (v[0][o] + v[1][o]) + v[2][o];
    }
#pragma unroll
    for (int sl = 0; sl < SPH; ++sl) {
      if (pr[sl].w >= 0) {
#pragma unroll
        for (int o = 0; o < CO; ++o) tt[sl][o] += db_[pr[sl].w * dstride + o];
        const long key = (long)u * kSeq + h * SPH + sl;
        for (int e = inv_ptr[key] + kInvHead; e < inv_ptr[key + 1]; ++e) {
#pragma unroll
          for (int o = 0; o < CO; ++o) tt[sl][o] += db_[inv_row[e] * dstride + o];
        }
      }
    }
    if (!valid) {
#pragma unroll
      for (int q = 0; q < KH; ++q) tt[q / CO][q % CO] = 0.f;
    }
#pragma unroll
    for (int q = 0; q < KH; ++q) At[(h * KH + q) * kAtS + li] = tt[q / CO][q % CO];
    if (h == 0) {  // slot 0 lists hold every output row once: db = sum_u t[0][o]
#pragma unroll
      for (int o = 0; o < CO; ++o) dbs[o] += tt[0][o];
    }
    // dx = T . Wt
    f32x16 dxacc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
#pragma unroll
      for (int r = 0; r < 16; ++r) dxacc[ct][r] = 0.f;
#pragma unroll
      for (int j = 0; j < KH; ++j) dxacc[ct] = mfma32(tt[j / CO][j % CO], wt[ct][j], dxacc[ct]);
    }
    wave_lds_sync();
    // dW^T += At . x_tile, K (rows) in accumulator-row order
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      const f32x4 a = ld4(&At[li * kAtS + 8 * t4 + 4 * h]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        dwacc[ct] = mfma32(a.x, xv[ct][4 * t4 + 0], dwacc[ct]);
        dwacc[ct] = mfma32(a.y, xv[ct][4 * t4 + 1], dwacc[ct]);
        dwacc[ct] = mfma32(a.z, xv[ct][4 * t4 + 2], dwacc[ct]);
        dwacc[ct] = mfma32(a.w, xv[ct][4 * t4 + 3], dwacc[ct]);
      }
    }
    if (dx) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long rr = row0 + acc_row(r, lane);
        if (rr < total_rows) {
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) {
            float v = dxacc[ct][r];
            if (ey_mode == 1) v *= elu_grad_from_out(xv[ct][r]);
            else if (ey_mode == 2) v *= elu_grad_from_out(ldf(&elu_y[rr * CIN + ct * 32 + li]));
            stf(&dx[rr * CIN + ct * 32 + li], v);
          }
        }
      }
    }
    wave_lds_sync();
  }
  // block combine (fixed wave order) -> one slab [CO*K + CO]
#pragma unroll
  for (int o = 0; o < CO; ++o)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) dbs[o] += __shfl_xor(dbs[o], d);
  __syncthreads();
  float* red = at_all;
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int k = acc_row(rr, lane), c = ct * 32 + li;
          const int sl = k / CO;
          if (sl < kSeq && k < 2 * KH) {
            const int e = (k % CO) * K + sl * CIN + c;
            red[e] = wv == 0 ? dwacc[ct][rr] : red[e] + dwacc[ct][rr];
          }
        }
      if (lane == 0)
#pragma unroll
        for (int o = 0; o < CO; ++o) red[CO * K + o] = wv == 0 ? dbs[o] : red[CO * K + o] + dbs[o];
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < NEL; e += 256) ws[(long)blockIdx.x * NEL + e] = red[e];
}

__global__ __launch_bounds__(1024) void slab_reduce(const float* __restrict__ ws, int n_slabs,
                                                    int n_el, float* __restrict__ out_a, int n_a,
                                                    float* __restrict__ out_b) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int e = blockIdx.x * 64 + lane;
  const bool valid = e < n_el;
  if (!valid) e = n_el - 1;
  float sum = 0.f;
#pragma unroll 4
  for (int p = wv; p < n_slabs; p += 16) sum += ws[(long)p * n_el + e];
  part[wv][lane] = sum;
  __syncthreads();
  if (wv == 0 && valid) {
    float t = part[0][lane];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += part[q][lane];
    if (e < n_a) out_a[e] = t;
    else out_b[e - n_a] = t;
  }
}

// Materialising gather (HBM roofline probe): g[b, r, s*cin + c] = x[b, idx[r,s], c].
// blockIdx.y = mesh b; a block covers GU*256 consecutive 16-B output chunks
// of that mesh (thread i: chunks i, i+256, ...), so every store instruction
// is 4 KB contiguous per wave-pair and all GU loads are in flight before the
// first store.  Index math is 32-bit with compile-time divisors (C4 chunks
// per neighbour row, kSeq slots): the 64-bit divisions of a flat index cost
// more VALU time than the store stream itself.  Output stores are
// non-temporal (write-once stream, no L2 allocation).
constexpr int GU = 4;
template <int C4>
__global__ __launch_bounds__(256) void spiral_gather_k(const float* __restrict__ x,
                                                       const int* __restrict__ idx,
                                                       float* __restrict__ g, int vsrc,
                                                       int per_mesh) {
  const int b = blockIdx.y;
  const float* xb = x + (long)b * vsrc * (4 * C4);
  f32x4* gb = reinterpret_cast<f32x4*>(g) + (long)b * per_mesh;
  const int t0 = blockIdx.x * (256 * GU) + threadIdx.x;
  int src[GU];
#pragma unroll
  for (int u = 0; u < GU; ++u) {
    const int t = min(t0 + u * 256, per_mesh - 1);
    src[u] = idx[t / C4];  // (r*kSeq + s) = t / C4: idx is [rows, kSeq] row-major
  }
  f32x4 v[GU];
#pragma unroll
  for (int u = 0; u < GU; ++u) {
    const int t = t0 + u * 256;
    v[u] = ld4(xb + (long)src[u] * (4 * C4) + 4 * (t % C4));
  }
#pragma unroll
  for (int u = 0; u < GU; ++u) {
    const int t = t0 + u * 256;
    if (t < per_mesh) __builtin_nontemporal_store(v[u], gb + t);
  }
}

// Any other channel count: one thread per chunk, runtime divisors (32-bit).
__global__ __launch_bounds__(256) void spiral_gather_any_k(const float* __restrict__ x,
                                                           const int* __restrict__ idx,
                                                           float* __restrict__ g, int vsrc,
                                                           int c4, int per_mesh) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= per_mesh) return;
  const int src = idx[t / c4];
  st4(g + ((long)b * per_mesh + t) * 4, ld4(x + ((long)b * vsrc + src) * (4 * c4) + 4 * (t % c4)));
}

}  // namespace cfsd

using namespace cfsd;

// ============================================================== C ABI
static int check_conv_args(const void* a, const void* b, const void* c, int batch, int vsrc,
                           int rows, int seq, int cin, int cout) {
  if (!a || !b || !c) return set_error(CFSD_EINVAL, "null pointer");
  if (batch <= 0 || vsrc <= 0 || rows <= 0 || seq <= 0 || cin <= 0 || cout <= 0)
    return set_error(CFSD_EINVAL, "non-positive size (batch=%d vsrc=%d rows=%d seq=%d cin=%d cout=%d)",
                     batch, vsrc, rows, seq, cin, cout);
  if (seq != kSeq) return set_error(CFSD_EINVAL, "spiral length %d unsupported (built for %d)", seq, kSeq);
  if ((long)batch * (vsrc > rows ? vsrc : rows) >= (1L << 31))
    return set_error(CFSD_EINVAL, "batch x vertices >= 2^31 (32-bit row indices)");
  return CFSD_OK;
}

// Persistent VALU kernels: one resident round, never more blocks than rows/64.
template <typename K>
static unsigned small_grid(K kernel, long rows) {
  const long cap = resident_blocks_of(kernel, 256, 0);
  const long need = (rows + 63) / 64;
  return (unsigned)(need < cap ? (need > 0 ? need : 1) : cap);
}

// One thread per row, 256-thread blocks.
static unsigned row_grid(long rows) { return (unsigned)((rows + 255) / 256); }

// Slots per group for the MFMA fwd / bwd-data kernels: few rows -> split the
// 9 spiral slots over more waves (partials combined by conv_combine).
static int pick_spg(long m_rows, size_t ws_floats_avail, long out_cols) {
  const long tiles = (m_rows + 31) / 32;
  int spg = tiles >= 2048 ? 9 : (tiles >= 400 ? 3 : 1);
  while (spg < 9 && (size_t)(kSeq / spg) * m_rows * out_cols > ws_floats_avail) spg = spg == 1 ? 3 : 9;
  return spg;
}

static size_t slot_group_ws_floats(long m_rows, long out_cols) {
  return (size_t)kSeq * m_rows * out_cols;  // worst case: 9 groups of one slot
}

template <int CIN, int COUT, int ACT, int SPG>
static int launch_fwd_mfma(const float* x, const int* idx, const float* w, const float* bias,
                           float* y, float* ws, int vsrc, int rows, long M, hipStream_t st) {
  constexpr size_t lds = (size_t)COUT * (SPG * CIN + 8) * sizeof(float);
  static_assert(lds <= 80 * 1024, "W slice must fit LDS");
  const long n_tiles = (M + 31) / 32;
  auto kern = conv_fwd_mfma<CIN, COUT, ACT, SPG>;
  const long max_blocks = resident_blocks_of(kern, 256, lds) / (kSeq / SPG);
  dim3 grid(balanced_blocks(n_tiles, 4, max_blocks > 0 ? max_blocks : 1), kSeq / SPG);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, x, idx, w, bias, y, ws, vsrc, rows, M);
  int rc = launch_status("spiral_conv_fwd");
  if (rc || SPG == kSeq) return rc;
  const long n4 = M * COUT / 4;
  hipLaunchKernelGGL((conv_combine<ACT>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, ws,
                     bias, (const float*)nullptr, y, kSeq / SPG, COUT, n4);
  return launch_status("spiral_conv_fwd_combine");
}

// Rows below which the latency-shaped kernels (conv_fwd_lat / conv_dx_lat)
// beat the persistent ones (fewer 32-row tiles than ~8 per CU).
constexpr int kLatMaxRows = 65536;
constexpr int kLatFwdMax = kLatMaxRows;
constexpr int kLatDwMax = kLatMaxRows;


// coarse levels: slot groups in one workgroup, partials combined in LDS
// (spiral_conv_coarse.hip)
static int fwd_coarse(const float* x, int xvm, const int* idx, const float* w, const float* bias, float* y,
                      int yvm, int vsrc, int rows, int batch, int cin, int cout, int act, hipStream_t st) {
  coarse::FwdKsArgs a{};
  a.x = x;
  a.idx = idx;
  a.w = w;
  a.bias = bias;
  a.y = y;
  a.vsrc = vsrc;
  a.rows = rows;
  a.batch = batch;
  a.total_rows = (long)batch * rows;
  a.xvm = xvm;
  a.yvm = yvm;
  a.elu = act == CFSD_ACT_ELU;
  return coarse::launch_fwd_ks(a, cin, cout, st);
}

extern "C" int cfsd_spiral_conv_fwd_up_supported(int batch, int rows, int seq, int cin, int cout) {
  if (batch <= 0 || rows <= 0 || seq != kSeq) return 0;
  return coarse::fwd_up_supported((long)batch * rows, cin, cout) ? 1 : 0;
}

extern "C" int cfsd_spiral_conv_fwd_up(const float* xc, const int32_t* comp_col, const float* comp_val,
                                       const int32_t* idx, const float* w, const float* bias, float* y, float* y_up,
                                       int batch, int n_coarse, int rows, int seq, int cin, int cout, int act,
                                       void* stream) {
  int rc = check_conv_args(xc, idx, w, batch, n_coarse, rows, seq, cin, cout);
  if (rc) return rc;
  if (!comp_col || !comp_val || !y) return set_error(CFSD_EINVAL, "spiral_conv_fwd_up: null pointer");
  if (act != CFSD_ACT_NONE && act != CFSD_ACT_ELU) return set_error(CFSD_EINVAL, "bad act %d", act);
  if (!coarse::fwd_up_supported((long)batch * rows, cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_fwd_up: unsupported layer (%d x %d rows, %d -> %d)", batch, rows,
                     cin, cout);
  coarse::FwdKsArgs a{};
  a.x = xc;
  a.idx = idx;
  a.w = w;
  a.bias = bias;
  a.y = y;
  a.yup = y_up;
  a.up_col = comp_col;
  a.up_val = comp_val;
  a.vsrc = rows;
  a.rows = rows;
  a.batch = batch;
  a.n_coarse = n_coarse;
  a.total_rows = (long)batch * rows;
  a.elu = act == CFSD_ACT_ELU;
  return coarse::launch_fwd_ks(a, cin, cout, (hipStream_t)stream);
}

template <int CIN, int COUT, int ACT>
static int dispatch_fwd_mfma(const float* x, const int* idx, const float* w, const float* bias,
                             float* y, float* ws, size_t ws_floats, int vsrc, int rows, long M,
                             hipStream_t st) {
  if (coarse::fwd_ks_enabled(M, CIN, COUT))
    return fwd_coarse(x, 0, idx, w, bias, y, 0, vsrc, rows, (int)(M / rows), CIN, COUT, ACT, st);
  // (64 -> 32 excepted: measured slower there than slot groups + combine)
constexpr int kFwdLat6432 = 0;
  if (M < kLatFwdMax && (kFwdLat6432 || !(CIN == 64 && COUT == 32))) {
constexpr int kFwdLatCtw = 1;
    // one wave per column tile: sharing the A gathers across both 32 -> 32
    // column tiles (CTW 2) measured slower here (E1 16.8 vs 16.1 us, E2 11.0
    // vs 7.8 us, same-box A/B) -- unlike the dx, whose A is a list gather-sum
    // 64 -> 64 (the level-3 Deblock): two column tiles per wave, each A
    // gather feeding twice the MFMAs (D0 forward 19.1 -> 16.3 us)
    constexpr int ctw = (CIN == 32 && COUT == 32) ? kFwdLatCtw : (CIN == 64 ? 2 : 1);
    const long tasks = (M + 15) / 16 * (COUT / 16 / ctw);
    hipLaunchKernelGGL((conv_fwd_lat<CIN, COUT, ACT, ctw>), dim3((unsigned)((tasks + 3) / 4)),
                       dim3(256), 0, st, x, idx, w, bias, y, vsrc, rows, M, (int)(M / rows), 0, 0);
    return launch_status("spiral_conv_fwd_lat");
  }
  constexpr bool big = (size_t)COUT * (kSeq * CIN + 8) * sizeof(float) > 80 * 1024;
  int spg = ws ? pick_spg(M, ws_floats, COUT) : 9;
  if (big && spg == 9) spg = 3;  // whole W does not fit LDS
  if (spg != 9 && !ws) return set_error(CFSD_EWORKSPACE, "spiral_conv_fwd: workspace required");
  if (spg == 9)
    return launch_fwd_mfma<CIN, COUT, ACT, (big ? 3 : 9)>(x, idx, w, bias, y, ws, vsrc, rows, M, st);
  if (spg == 3) return launch_fwd_mfma<CIN, COUT, ACT, 3>(x, idx, w, bias, y, ws, vsrc, rows, M, st);
  return launch_fwd_mfma<CIN, COUT, ACT, 1>(x, idx, w, bias, y, ws, vsrc, rows, M, st);
}

extern "C" size_t cfsd_spiral_conv_workspace(int batch, int vsrc, int rows, int seq, int cin,
                                             int cout) {
  if (batch <= 0 || vsrc <= 0 || rows <= 0 || seq != kSeq || cin <= 0 || cout <= 0) return 0;
  const size_t a = slot_group_ws_floats((long)batch * rows, cout);
  const size_t b = slot_group_ws_floats((long)batch * vsrc, cin);
  return (a > b ? a : b) * sizeof(float);
}

extern "C" int cfsd_spiral_conv_fwd(const float* x, const int32_t* idx, const float* w,
                                    const float* bias, float* y, float* workspace,
                                    size_t workspace_bytes, int batch, int vsrc, int rows, int seq,
                                    int cin, int cout, int act, void* stream) {
  int rc = check_conv_args(x, idx, w, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if ((long)batch * rows >= (1L << 31) || (long)batch * vsrc >= (1L << 31))
    return set_error(CFSD_EINVAL, "spiral_conv_fwd: batch*rows must be < 2^31");
  if (!y) return set_error(CFSD_EINVAL, "null y");
  if (act != CFSD_ACT_NONE && act != CFSD_ACT_ELU) return set_error(CFSD_EINVAL, "bad act %d", act);
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * rows;
  const size_t wsf = workspace ? workspace_bytes / sizeof(float) : 0;
#define FWD(CIN_, COUT_)                                                                         \
  if (cin == CIN_ && cout == COUT_)                                                              \
    return act == CFSD_ACT_ELU                                                                   \
               ? dispatch_fwd_mfma<CIN_, COUT_, CFSD_ACT_ELU>(x, idx, w, bias, y, workspace, wsf, \
                                                              vsrc, rows, M, st)                 \
               : dispatch_fwd_mfma<CIN_, COUT_, CFSD_ACT_NONE>(x, idx, w, bias, y, workspace,    \
                                                               wsf, vsrc, rows, M, st);
  FWD(32, 32) FWD(32, 64) FWD(64, 32) FWD(64, 64)
#undef FWD
  if (cin <= 3 && (cout == 32 || cout == 64)) {
    const long tiles = (M + 31) / 32;
    const unsigned gp = (unsigned)((tiles + 3) / 4 < 2048 ? (tiles + 3) / 4 : 2048);
#define FIN(CS_, CO_)                                                                            \
  if (cin == CS_ && cout == CO_) {                                                               \
    if (act == CFSD_ACT_ELU)                                                                     \
      hipLaunchKernelGGL((conv_fwd_in_mfma<CS_, CO_, CFSD_ACT_ELU>), dim3(gp), dim3(256), 0, st,  \
                         x, idx, w, bias, y, vsrc, rows, M, batch, 0, 0);                        \
    else                                                                                         \
      hipLaunchKernelGGL((conv_fwd_in_mfma<CS_, CO_, CFSD_ACT_NONE>), dim3(gp), dim3(256), 0, st, \
                         x, idx, w, bias, y, vsrc, rows, M, batch, 0, 0);                        \
    return launch_status("spiral_conv_fwd_in");                                                  \
  }
    FIN(1, 32) FIN(2, 32) FIN(3, 32) FIN(1, 64) FIN(2, 64) FIN(3, 64)
#undef FIN
  }
#define FWD_SMALL(KERNEL, A_, B_, ...)                                                           \
  if (cin == A_ && cout == B_) {                                                                 \
    if (act == CFSD_ACT_ELU) {                                                                   \
      auto k = KERNEL<A_, B_, CFSD_ACT_ELU>;                                                     \
      hipLaunchKernelGGL(k, dim3(GRID(k)), dim3(256), 0, st, x, idx, w, bias, y, vsrc, rows, M __VA_ARGS__); \
    } else {                                                                                     \
      auto k = KERNEL<A_, B_, CFSD_ACT_NONE>;                                                    \
      hipLaunchKernelGGL(k, dim3(GRID(k)), dim3(256), 0, st, x, idx, w, bias, y, vsrc, rows, M __VA_ARGS__); \
    }                                                                                            \
    return launch_status("spiral_conv_fwd_small");                                               \
  }
#define GRID(k) row_grid(M)
  FWD_SMALL(conv_fwd_in_small, 3, 16)
#undef GRID
#define GRID(k) small_grid(k, M)
  FWD_SMALL(conv_fwd_out_small, 16, 3, , batch, 0, 0) FWD_SMALL(conv_fwd_out_small, 32, 3, , batch, 0, 0)
  FWD_SMALL(conv_fwd_out_small, 64, 3, , batch, 0, 0)
#undef GRID
#undef FWD_SMALL
  return set_error(CFSD_EINVAL, "spiral_conv_fwd: unsupported channels %d -> %d", cin, cout);
}

template <int CIN, int COUT, int SPG>
static int launch_dx_mfma(const float* dpre, const int* inv_ptr, const int* inv_row,
                          const int* inv_head, const float* w, const float* elu_y, float* dx,
                          float* ws, int vsrc, int rows, long M, hipStream_t st) {
  constexpr size_t lds = (size_t)SPG * CIN * (COUT + 4) * sizeof(float);
  static_assert(lds <= 80 * 1024, "W slice must fit LDS");
  auto kern = conv_dx_mfma<CIN, COUT, SPG>;
  const long max_blocks = resident_blocks_of(kern, 256, lds) / (kSeq / SPG);
  dim3 grid(balanced_blocks((M + 31) / 32, 4, max_blocks > 0 ? max_blocks : 1), kSeq / SPG);
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, dpre, inv_ptr,
                     inv_row, (const int4*)inv_head, w, elu_y, dx, ws, vsrc, rows, M);
  int rc = launch_status("spiral_conv_bwd_data");
  if (rc || SPG == kSeq) return rc;
  const long n4 = M * CIN / 4;
  hipLaunchKernelGGL((conv_combine<CFSD_ACT_NONE>), dim3((unsigned)((n4 + 255) / 256)), dim3(256),
                     0, st, ws, (const float*)nullptr, elu_y, dx, kSeq / SPG, CIN, n4);
  return launch_status("spiral_conv_bwd_data_combine");
}

// latency-shaped dx below ~64k dx rows (the persistent kernel cannot fill
// the chip there without slot groups), and up to 80k rows when the conv was
// evaluated on a row subset (Enblock: ~2.25 list entries per dx row instead
// of 9; each persistent block would stage W for ~2 tiles) -- measured on the
// 68k-row E1 dx: 33.8 us latency-shaped vs 38.8 us persistent
static bool dx_is_lat(long m_dx, long dpre_rows) {
  return m_dx < kLatMaxRows || (m_dx < 80000 && 2 * dpre_rows <= m_dx);
}
// 32 -> 32 with >= 32k rows: one wave covers both 16-column tiles (the list
// gathers are shared instead of repeated per column tile; measured E1 dx
// 33 -> 29 us; the fewer, fatter waves lose on the smaller levels)
constexpr int kDxLatCtw64 = 2;
constexpr int kDxLatCtw6432 = 2;
static int dx_lat_ctw(int cin, int cout, long m_dx) {
  // 64-wide inputs: two column tiles per wave share the list gather-sums
  // (D0 dx 18.6 -> 15.2 us; the D1 paired backward 40.7 -> 36.9 us)
  if (cin == 64 && cout == 64) return kDxLatCtw64;
  if (cin == 64 && cout == 32) return kDxLatCtw6432;
  return (cin == 32 && cout == 32 && m_dx >= 32768) ? 2 : 1;
}

template <int CIN, int COUT>
static int dispatch_dx_mfma(const float* dpre, const int* inv_ptr, const int* inv_row,
                            const int* inv_head, const float* w, const float* elu_y, float* dx,
                            float* ws, size_t ws_floats, int vsrc, int rows, long M,
                            hipStream_t st) {
  if (coarse::dx_ks_enabled(M, CIN, COUT)) {
    const coarse::DxKsArgs a{dpre, inv_ptr, inv_row, (const int4*)inv_head, w, elu_y, dx, vsrc, rows,
                             (int)(M / vsrc), M};
    return coarse::launch_dx_ks(a, CIN, COUT, st);
  }
  if (dx_is_lat(M, M / vsrc * rows)) {
    if (dx_lat_ctw(CIN, COUT, M) == 2) {
      constexpr int CTW2 = CIN / 16 >= 2 ? 2 : 1;
      const long tasks = (M + 15) / 16 * (CIN / 16 / CTW2);
      hipLaunchKernelGGL((conv_dx_lat<CIN, COUT, CTW2>), dim3((unsigned)((tasks + 3) / 4)), dim3(256),
                         0, st, dpre, inv_ptr, inv_row, (const int4*)inv_head, w, elu_y, dx, vsrc, rows, M);
      return launch_status("spiral_conv_bwd_data_lat");
    }
    const long tasks = (M + 15) / 16 * (CIN / 16);
    hipLaunchKernelGGL((conv_dx_lat<CIN, COUT, 1>), dim3((unsigned)((tasks + 3) / 4)), dim3(256), 0, st,
                       dpre, inv_ptr, inv_row, (const int4*)inv_head, w, elu_y, dx, vsrc, rows, M);
    return launch_status("spiral_conv_bwd_data_lat");
  }
  constexpr bool big = (size_t)kSeq * CIN * (COUT + 4) * sizeof(float) > 80 * 1024;
  int spg = ws ? pick_spg(M, ws_floats, CIN) : 9;
  if (big && spg == 9) spg = 3;
  if (spg != 9 && !ws) return set_error(CFSD_EWORKSPACE, "spiral_conv_bwd_data: workspace required");
  if (spg == 9)
    return launch_dx_mfma<CIN, COUT, (big ? 3 : 9)>(dpre, inv_ptr, inv_row, inv_head, w, elu_y, dx,
                                                    ws, vsrc, rows, M, st);
  if (spg == 3)
    return launch_dx_mfma<CIN, COUT, 3>(dpre, inv_ptr, inv_row, inv_head, w, elu_y, dx, ws, vsrc,
                                        rows, M, st);
  return launch_dx_mfma<CIN, COUT, 1>(dpre, inv_ptr, inv_row, inv_head, w, elu_y, dx, ws, vsrc,
                                      rows, M, st);
}

extern "C" int cfsd_spiral_conv_bwd_data(const float* dpre, const int32_t* inv_ptr,
                                         const int32_t* inv_row, const int32_t* inv_head,
                                         const float* w, const float* elu_y, float* dx,
                                         float* workspace, size_t workspace_bytes, int batch,
                                         int vsrc, int rows, int seq, int cin, int cout,
                                         void* stream) {
  int rc = check_conv_args(dpre, inv_ptr, inv_row, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!w || !dx || !inv_head) return set_error(CFSD_EINVAL, "null w/dx/inv_head");
  if ((uintptr_t)inv_head & 15) return set_error(CFSD_EINVAL, "inv_head must be 16-B aligned");
  if ((long)batch * rows * cout * (long)sizeof(float) >= (1L << 31))
    return set_error(CFSD_EINVAL, "dpre larger than 2 GiB (32-bit buffer offsets)");
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * vsrc;
  const size_t wsf = workspace ? workspace_bytes / sizeof(float) : 0;
#define DXM(CIN_, COUT_)                                                                       \
  if (cin == CIN_ && cout == COUT_)                                                            \
    return dispatch_dx_mfma<CIN_, COUT_>(dpre, inv_ptr, inv_row, inv_head, w, elu_y, dx,       \
                                         workspace, wsf, vsrc, rows, M, st);
  DXM(32, 32) DXM(32, 64) DXM(64, 32) DXM(64, 64)
#undef DXM
#define DXS(CIN_, CO_)                                                                          \
  if (cin == CIN_ && cout == CO_) {                                                             \
    auto k = conv_dx_out_small<CIN_, CO_>;                                                      \
    hipLaunchKernelGGL(k, dim3(row_grid(M)), dim3(256), 0, st,                                  \
                       dpre, inv_ptr, inv_row, (const int4*)inv_head, w, elu_y, dx, vsrc, rows, M); \
    return launch_status("spiral_conv_bwd_data_small");                                        \
  }
  DXS(16, 3) DXS(32, 3) DXS(64, 3)
#undef DXS
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data: unsupported channels %d -> %d", cin, cout);
}

// ---- bwd weight: launch geometry shared by the workspace query and the launch
namespace {
enum DwKind { kDwMfma, kDwLat, kDwInMfma, kDwInSmall, kDwOutSmall, kDwNone };
struct DwGeom {
  DwKind kind;
  int gx;  // workgroups (= slabs), or row chunks for kDwLat
  size_t ws_floats;
  int rchunk;
};

size_t dw_units(int cin, int cout) { return (size_t)kSeq * (cout / 32) * (cin / 32); }

// Workgroups (= slabs) of a conv_dw_mfma launch: the geometry's gx capped at
// one resident round.
int dw_mfma_slabs(int cin, int cout, int gx) {
  int cap = gx;
#define CAP(CIN_, COUT_)                                                                         \
  if (cin == CIN_ && cout == COUT_) {                                                            \
    using C = DwCfg<CIN_, COUT_>;                                                                \
    cap = resident_blocks_of(conv_dw_mfma<CIN_, COUT_>, C::THREADS, C::LDS_FLOATS * sizeof(float)); \
  }
  CAP(32, 32) CAP(32, 64) CAP(64, 32) CAP(64, 64)
#undef CAP
  return gx < cap ? gx : cap;
}

constexpr int kDwLatWaves = 2048;
// one wave per (dW unit, row chunk), ~2k waves (the few-row layers).
// The 64 -> 64 few-tile layer (D0) pairs its dW slabs with the slot-group
// dx (coarse::conv_bwd_ks_pair: 9-wave workgroups, ONE per CU at its 160
// VGPRs), so its dW waves are sized to the CUs the dx role leaves: with
// 2048 waves (252 workgroups + 134 dx) half the dW workgroups were
// dispatched only as dx ones retired (stamps: starts up to 11.4 us, span
// 17.9 us); sized to fit, every workgroup of the launch starts at once.
DwGeom lat_geom(int batch, int rows, int cin, int cout) {
  DwGeom g{kDwLat, 0, 0, 0};
  const long M = (long)batch * rows;
  const long U = (long)dw_units(cin, cout);
  long R = (M * U / kDwLatWaves + 15) / 16 * 16;
  R = R < 32 ? 32 : (R > 512 ? 512 : R);
  if (cin == 64 && cout == 64 && M < coarse::kMaxTilesFew * 16) {
    // longer row chunks until the pair's dW workgroups (8 waves each, whole
    // chunk groups) fit beside its dx workgroups (rows == dx rows there)
    const long nb_dx = ((M + 15) / 16 + 1) / 2, free_wg = device_cus() - nb_dx;
    while (R < 512 && (lat_tasks((int)((M + R - 1) / R), (int)U) + 7) / 8 > free_wg) R += 16;
  }
  g.rchunk = (int)R;
  g.gx = (int)((M + R - 1) / R);
  g.ws_floats = (size_t)g.gx * U * 1024 + (size_t)g.gx * cout;
  return g;
}
DwGeom dw_geom(int batch, int rows, int cin, int cout) {
  DwGeom g{kDwNone, 0, 0, 0};
  const long M = (long)batch * rows;
  if ((cin == 32 || cin == 64) && (cout == 32 || cout == 64) && M < kLatDwMax) {
    g = lat_geom(batch, rows, cin, cout);  // few rows
  } else if ((cin == 32 || cin == 64) && (cout == 32 || cout == 64)) {
    g.kind = kDwMfma;
    const long n_tiles = (M + 31) / 32;
constexpr int kDwTpb = 4;
    long gx = (n_tiles + kDwTpb - 1) / kDwTpb;  // >= 4 tiles per block keeps the slab traffic bounded
constexpr int kDwMaxWg = 512;  // (768: same time, 1.5x the slab traffic)
    if (gx > kDwMaxWg) gx = kDwMaxWg;  // 2 blocks of 9 waves per CU
    g.gx = (int)(gx > 0 ? gx : 1);
    g.ws_floats = (size_t)g.gx * dw_units(cin, cout) * 1024 + (size_t)g.gx * cout;
  } else if (cin <= 3 && (cout == 32 || cout == 64)) {
    g.kind = kDwInMfma;
    long gx = ((M + 63) / 64 + 3) / 4;  // one 64-row tile per wave per pass
    g.gx = (int)(gx > 512 ? 512 : (gx < 1 ? 1 : gx));
    g.ws_floats = (size_t)g.gx * ((size_t)cout * kSeq * cin + cout);
  } else if (cin <= 4 && (cout == 16 || cout == 32 || cout == 64)) {
    g.kind = kDwInSmall;
    const long per_blk = 4 * (64 / cout);
    long gx = (M + per_blk * 8 - 1) / (per_blk * 8);  // >= 8 rows per row slot
    g.gx = (int)(gx > 512 ? 512 : (gx < 1 ? 1 : gx));
    g.ws_floats = (size_t)g.gx * ((size_t)cout * kSeq * cin + cout);
  } else if (cout <= 4 && (cin == 16 || cin == 32 || cin == 64)) {
    g.kind = kDwOutSmall;
    const long per_blk = 4 * (64 / (cin / 4));
    long gx = (M + per_blk * 8 - 1) / (per_blk * 8);
    g.gx = (int)(gx > 512 ? 512 : (gx < 1 ? 1 : gx));
    g.ws_floats = (size_t)g.gx * ((size_t)cout * kSeq * cin + cout);
  }
  return g;
}
}  // namespace

extern "C" size_t cfsd_spiral_conv_bwd_weight_workspace(int batch, int rows, int seq, int cin,
                                                        int cout) {
  if (batch <= 0 || rows <= 0 || seq != kSeq || cin <= 0 || cout <= 0) return 0;
  return dw_geom(batch, rows, cin, cout).ws_floats * sizeof(float);
}

constexpr int kDwVm32 = 1;  // 32 -> 32 with vertex-major x and dpre: vm32::conv_dw_vm32
// The fp32 weight gradient takes vm32::conv_dw_vm32 (its slabs: cfsd_dw_slabs.fused == 3)
static bool dw_vm32_path(int xvm, int dpvm, int cin, int cout, int batch) {
  return kDwVm32 && xvm && dpvm && cin == 32 && cout == 32 && batch % 16 == 0;
}
// dW / db of an fp32 conv, x and dpre each batch-major or vertex-major
// (xvm / dpvm; the small-channel kernels are batch-major only).
static int dw_f32(const float* x, int xvm, const int32_t* idx, const float* dpre, int dpvm, float* dw,
                  float* db, float* workspace, size_t workspace_bytes, int batch, int vsrc, int rows,
                  int cin, int cout, hipStream_t st) {
  int rc = CFSD_OK;
  if (!workspace) return set_error(CFSD_EINVAL, "null workspace");
  if ((dw == nullptr) != (db == nullptr))
    return set_error(CFSD_EINVAL, "dw and db must both be set (or both NULL: deferred)");
  const bool deferred = dw == nullptr;
  DwGeom g = dw_geom(batch, rows, cin, cout);
  if (g.kind == kDwNone)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight: unsupported channels %d -> %d", cin, cout);
  if (workspace_bytes < g.ws_floats * sizeof(float))
    return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes,
                     g.ws_floats * sizeof(float));
  if ((xvm || dpvm) && g.kind != kDwLat && g.kind != kDwMfma)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight: vertex-major operands need 32/64 channels");
  if ((long)batch * vsrc * cin >= (1L << 31))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight: x has >= 2^31 elements (32-bit offsets)");
  const long M = (long)batch * rows;
  const int n_el = cout * kSeq * cin + cout;
  const dim3 rg((unsigned)((n_el + 63) / 64));
  if (g.kind == kDwLat) {
    float* ws_db = workspace + (size_t)g.gx * dw_units(cin, cout) * 1024;
    const long tasks = lat_tasks(g.gx, dw_units(cin, cout));
#define DWL(CIN_, COUT_)                                                                        \
  if (cin == CIN_ && cout == COUT_) {                                                           \
    hipLaunchKernelGGL((conv_dw_lat<CIN_, COUT_>), dim3((unsigned)((tasks + 3) / 4)), dim3(256), \
                       0, st, x, idx, dpre, workspace, ws_db, vsrc, rows, (int)M, g.rchunk,      \
                       g.gx, batch, xvm, dpvm);                                                 \
    rc = launch_status("spiral_conv_bwd_weight_lat");                                           \
    if (rc || deferred) return rc;                                                              \
    hipLaunchKernelGGL((conv_dw_reduce<CIN_, COUT_>), rg, dim3(1024), 0, st, workspace, ws_db,  \
                       dw, db, lat_slabs(g.gx));                                                \
    return launch_status("spiral_conv_bwd_weight_reduce");                                      \
  }
    DWL(32, 32) DWL(32, 64) DWL(64, 32) DWL(64, 64)
#undef DWL
  }
  if (g.kind == kDwMfma) {
    float* ws_db = workspace + (size_t)g.gx * dw_units(cin, cout) * 1024;
    int nslab = g.gx;
#define DWM(CIN_, COUT_)                                                                        \
  if (cin == CIN_ && cout == COUT_) {                                                           \
    using C = DwCfg<CIN_, COUT_>;                                                               \
    auto k = conv_dw_mfma<CIN_, COUT_>;                                                         \
    if (dw_vm32_path(xvm, dpvm, cin, cout, batch)) {                                            \
      nslab = vm32::dw_slabs(batch, rows, g.gx);                                                \
      rc = vm32::launch_dw(x, idx, dpre, workspace, ws_db, nslab, vsrc, rows, batch, st);        \
    } else {                                                                                    \
      nslab = dw_mfma_slabs(cin, cout, g.gx);                                                   \
      hipLaunchKernelGGL(k, dim3(nslab), dim3(C::THREADS), C::LDS_FLOATS * sizeof(float), st, x, \
                         idx, dpre, workspace, ws_db, vsrc, rows, M, batch, xvm, dpvm);         \
      rc = launch_status("spiral_conv_bwd_weight");                                             \
    }                                                                                           \
    if (rc || deferred) return rc;                                                              \
    hipLaunchKernelGGL((conv_dw_reduce<CIN_, COUT_>), rg, dim3(1024), 0, st, workspace, ws_db,  \
                       dw, db, nslab);                                                          \
    return launch_status("spiral_conv_bwd_weight_reduce");                                      \
  }
    DWM(32, 32) DWM(32, 64) DWM(64, 32) DWM(64, 64)
#undef DWM
  }
#define DWS(KERNEL, A_, B_, ...)                                                                  \
  if (cin == A_ && cout == B_) {                                                                  \
    hipLaunchKernelGGL((KERNEL<A_, B_>), dim3(g.gx), dim3(256), 0, st, x, idx, dpre, workspace,   \
                       vsrc, rows, M __VA_ARGS__);                                                \
    rc = launch_status("spiral_conv_bwd_weight_small");                                           \
    if (rc || deferred) return rc;                                                                \
    hipLaunchKernelGGL(slab_reduce, rg, dim3(1024), 0, st, workspace, g.gx, n_el, dw,             \
                       cout * kSeq * cin, db);                                                    \
    return launch_status("spiral_conv_bwd_weight_small_reduce");                                  \
  }
  if (g.kind == kDwInMfma) {
    DWS(conv_dw_in_mfma, 3, 32, , batch, 0, 0) DWS(conv_dw_in_mfma, 3, 64, , batch, 0, 0)
    DWS(conv_dw_in_mfma, 2, 32, , batch, 0, 0) DWS(conv_dw_in_mfma, 2, 64, , batch, 0, 0)
    DWS(conv_dw_in_mfma, 1, 32, , batch, 0, 0) DWS(conv_dw_in_mfma, 1, 64, , batch, 0, 0)
  } else if (g.kind == kDwInSmall) {
    DWS(conv_dw_in_small, 3, 16) DWS(conv_dw_in_small, 3, 32) DWS(conv_dw_in_small, 3, 64)
  } else {
    DWS(conv_dw_out_small, 16, 3) DWS(conv_dw_out_small, 32, 3) DWS(conv_dw_out_small, 64, 3)
  }
#undef DWS
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight: unsupported channels %d -> %d", cin, cout);
}

extern "C" int cfsd_spiral_conv_bwd_weight(const float* x, const int32_t* idx, const float* dpre,
                                           float* dw, float* db, float* workspace,
                                           size_t workspace_bytes, int batch, int vsrc, int rows,
                                           int seq, int cin, int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  return dw_f32(x, 0, idx, dpre, 0, dw, db, workspace, workspace_bytes, batch, vsrc, rows, cin, cout,
                (hipStream_t)stream);
}

// ---- fused backward (data + weight)
namespace {
bool fused_small(int cin, int cout) { return cout * kSeq <= 32 && (cin == 32 || cin == 64); }
int fused_small_gx(long m_src) {  // ~2 32-row tiles per wave
  long gx = ((m_src + 31) / 32 + 7) / 8;
  constexpr int bpc = 0;  // workgroups per CU (0: the occupancy bound)
  const long cap = bpc > 0 ? (long)bpc * device_cus() : 1024;
  return (int)(gx > cap ? cap : (gx < 1 ? 1 : gx));
}
}  // namespace

namespace {
// Paired only for 32-wide dpre rows: the 64-wide dx body needs ~256 VGPRs,
// which would cap the dW workgroups sharing the kernel at 1 wave per SIMD
// (measured: dec 64->64 and E3 32->64 got 1-3 us slower paired, 64->32 and
// E2 32->32 3-5 us faster).
// the coarse few-tile layers: slot-group dx + dW slabs (conv_bwd_ks_pair)
bool bwd_ks_paired(int batch, int vsrc, int rows, int cin, int cout) {
  return (cin == 32 || cin == 64) && (cout == 32 || cout == 64) && coarse::dx_ks_enabled((long)batch * vsrc, cin, cout) &&
         dw_geom(batch, rows, cin, cout).kind == kDwLat;
}
bool bwd_paired(int batch, int vsrc, int rows, int cin, int cout) {
  if (bwd_ks_paired(batch, vsrc, rows, cin, cout)) return true;
  if (!((cin == 32 || cin == 64) && cout == 32)) return false;
  if (coarse::dx_ks_enabled((long)batch * vsrc, cin, cout)) return false;
  return dx_is_lat((long)batch * vsrc, (long)batch * rows) &&
         dw_geom(batch, rows, cin, cout).kind == kDwLat;
}
}  // namespace

extern "C" int cfsd_spiral_conv_bwd_paired(int batch, int vsrc, int rows, int seq, int cin,
                                           int cout) {
  if (batch <= 0 || vsrc <= 0 || rows <= 0 || seq != kSeq) return 0;
  return bwd_paired(batch, vsrc, rows, cin, cout) ? 1 : 0;
}

extern "C" size_t cfsd_spiral_conv_bwd_workspace(int batch, int vsrc, int rows, int seq, int cin,
                                                 int cout) {
  if (batch <= 0 || vsrc <= 0 || rows <= 0 || seq != kSeq || cin <= 0 || cout <= 0) return 0;
  if (fused_small(cin, cout))
    return (size_t)fused_small_gx((long)batch * vsrc) * ((size_t)cout * kSeq * cin + cout) *
           sizeof(float);
  const size_t a = cfsd_spiral_conv_workspace(batch, vsrc, rows, seq, cin, cout);
  const size_t b = cfsd_spiral_conv_bwd_weight_workspace(batch, rows, seq, cin, cout);
  return a > b ? a : b;
}

extern "C" int cfsd_spiral_conv_bwd(const float* x, const int32_t* idx, const float* dpre,
                                    const int32_t* inv_ptr, const int32_t* inv_row,
                                    const int32_t* inv_head, const float* w, const float* elu_y,
                                    float* dx, float* dw, float* db, float* workspace,
                                    size_t workspace_bytes, int batch, int vsrc, int rows, int seq,
                                    int cin, int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!inv_ptr || !inv_row || !inv_head || !w || !workspace)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd: null inverse table / w / workspace");
  if ((uintptr_t)inv_head & 15) return set_error(CFSD_EINVAL, "inv_head must be 16-B aligned");
  if ((long)batch * rows * cout * (long)sizeof(float) >= (1L << 31))
    return set_error(CFSD_EINVAL, "dpre larger than 2 GiB (32-bit buffer offsets)");
  if ((dw == nullptr) != (db == nullptr))
    return set_error(CFSD_EINVAL, "dw and db must both be set (or both NULL: deferred)");
  const size_t need = cfsd_spiral_conv_bwd_workspace(batch, vsrc, rows, seq, cin, cout);
  if (workspace_bytes < need)
    return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  if (dx && bwd_ks_paired(batch, vsrc, rows, cin, cout)) {
    const DwGeom g = dw_geom(batch, rows, cin, cout);
    float* ws_db = workspace + (size_t)g.gx * dw_units(cin, cout) * 1024;
    const coarse::DxKsArgs a{dpre, inv_ptr, inv_row, (const int4*)inv_head, w, elu_y, dx, vsrc, rows, batch,
                             (long)batch * vsrc};
    const DwLatArgs d{x, idx, dpre, workspace, ws_db, vsrc, rows, batch * rows, g.rchunk, g.gx, 0, batch, 0, 0};
    rc = coarse::launch_bwd_ks_pair(a, d, lat_tasks(g.gx, dw_units(cin, cout)), cin, cout, st);
    if (rc || !dw) return rc;
    const int n_el = cout * kSeq * cin + cout;
#define KSR(CIN_, COUT_)                                                                             \
  if (cin == CIN_ && cout == COUT_) {                                                                \
    hipLaunchKernelGGL((conv_dw_reduce<CIN_, COUT_>), dim3((unsigned)((n_el + 63) / 64)), dim3(1024), 0, st, \
                       workspace, ws_db, dw, db, lat_slabs(g.gx));                                   \
    return launch_status("spiral_conv_bwd_weight_reduce");                                           \
  }
    KSR(32, 32) KSR(32, 64) KSR(64, 32) KSR(64, 64)
#undef KSR
  }
  if (dx && bwd_paired(batch, vsrc, rows, cin, cout)) {
    const DwGeom g = dw_geom(batch, rows, cin, cout);
    const long M = (long)batch * vsrc;
    const long dw_tasks = lat_tasks(g.gx, dw_units(cin, cout));
    float* ws_db = workspace + (size_t)g.gx * dw_units(cin, cout) * 1024;
    DxLatArgs a{dpre, inv_ptr, inv_row, (const int4*)inv_head, w, elu_y, dx, vsrc, rows, M, 0};
    DwLatArgs d{x, idx, dpre, workspace, ws_db, vsrc, rows, batch * rows, g.rchunk, g.gx,
                (int)((dw_tasks + 3) / 4), batch, 0, 0};
    const int ctw = dx_lat_ctw(cin, cout, M);
    a.nb = (int)(((M + 15) / 16 * (cin / 16 / ctw) + 3) / 4);
    const dim3 grid((unsigned)(a.nb + d.nb));
    const int n_el = cout * kSeq * cin + cout;
#define PAIR(CIN_, COUT_, CTW_)                                                                 \
  if (cin == CIN_ && cout == COUT_ && ctw == CTW_) {                                            \
    hipLaunchKernelGGL((conv_bwd_lat_pair<CIN_, COUT_, CTW_>), grid, dim3(256), 0, st, a, d);    \
    rc = launch_status("spiral_conv_bwd_lat_pair");                                             \
    if (rc || !dw) return rc;                                                                   \
    hipLaunchKernelGGL((conv_dw_reduce<CIN_, COUT_>), dim3((unsigned)((n_el + 63) / 64)),        \
                       dim3(1024), 0, st, workspace, ws_db, dw, db, lat_slabs(g.gx));           \
    return launch_status("spiral_conv_bwd_weight_reduce");                                      \
  }
    PAIR(32, 32, 1) PAIR(32, 32, 2) PAIR(64, 32, 1) PAIR(64, 32, 2)
#undef PAIR
    return set_error(CFSD_EINVAL, "spiral_conv_bwd: unsupported channels %d -> %d", cin, cout);
  }
  if (!fused_small(cin, cout)) {
    if (dx) {
      rc = cfsd_spiral_conv_bwd_data(dpre, inv_ptr, inv_row, inv_head, w, elu_y, dx, workspace,
                                     workspace_bytes, batch, vsrc, rows, seq, cin, cout, stream);
      if (rc) return rc;
    }
    return cfsd_spiral_conv_bwd_weight(x, idx, dpre, dw, db, workspace, workspace_bytes, batch,
                                       vsrc, rows, seq, cin, cout, stream);
  }
  const long Ms = (long)batch * vsrc;
  const int gx = fused_small_gx(Ms);
  const int n_el = cout * kSeq * cin + cout;
#define BOS(CIN_, CO_)                                                                           \
  if (cin == CIN_ && cout == CO_) {                                                              \
    hipLaunchKernelGGL((conv_bwd_out_mfma<CIN_, CO_>), dim3(gx), dim3(256), 0, st, dpre,         \
                       inv_ptr, inv_row, (const int4*)inv_head, w, elu_y, x, dx, workspace, vsrc, \
                       rows, Ms, batch, 0, 0);                                                   \
    rc = launch_status("spiral_conv_bwd_small");                                                 \
    if (rc || !dw) return rc;                                                                    \
    hipLaunchKernelGGL(slab_reduce, dim3((unsigned)((n_el + 63) / 64)), dim3(1024), 0, st,        \
                       workspace, gx, n_el, dw, cout * kSeq * cin, db);                          \
    return launch_status("spiral_conv_bwd_small_reduce");                                        \
  }
  BOS(32, 1) BOS(32, 2) BOS(32, 3) BOS(64, 1) BOS(64, 2) BOS(64, 3)
#undef BOS
  return set_error(CFSD_EINVAL, "spiral_conv_bwd: unsupported channels %d -> %d", cin, cout);
}

// ---- row-subset backward (dG + dW slabs, then the flat-list gather)
namespace {
size_t rowsub_dg_floats(int batch, int rows, int cin) {
  return ((size_t)batch * rows * kSeq * cin + 63) / 64 * 64;
}
size_t rowsub_slab_floats(int batch, int rows, int cin, int cout) {
  return (dw_geom(batch, rows, cin, cout).ws_floats + 63) / 64 * 64;
}
// 32 input channels (every Enblock after the first in the reference configs;
// W^T of a 64-channel input would not leave LDS for a second workgroup)
bool rowsub_shape(int cin, int cout) { return cin == 32 && (cout == 32 || cout == 64); }
// column groups per 16-row tile: enough waves to cover the chip (~2k)
int rowsub_groups(long row_tiles, int n_tiles) {
  static const int divs[] = {1, 2, 3, 4, 6, 9, 12, 18, 36};
  for (int d : divs)
    if (n_tiles % d == 0 && row_tiles * d >= 1536) return d;
  return n_tiles;
}
}  // namespace

extern "C" size_t cfsd_spiral_conv_bwd_rowsub_workspace(int batch, int vsrc, int rows, int seq,
                                                        int cin, int cout) {
  if (batch <= 0 || vsrc <= 0 || rows <= 0 || seq != kSeq || !rowsub_shape(cin, cout)) return 0;
  return (rowsub_slab_floats(batch, rows, cin, cout) + rowsub_dg_floats(batch, rows, cin)) *
         sizeof(float);
}

static int bwd_rowsub(const float* x, int xvm, const int32_t* idx, const float* dpre, const int32_t* inv_flat,
                      int flat_width, const float* w, const float* elu_y, float* dx, float* dw, float* db,
                      float* workspace, size_t workspace_bytes, int batch, int vsrc, int rows, int seq, int cin,
                      int cout, void* stream);

extern "C" int cfsd_spiral_conv_bwd_rowsub(const float* x, const int32_t* idx, const float* dpre,
                                           const int32_t* inv_flat, int flat_width,
                                           const float* w, const float* elu_y, float* dx,
                                           float* dw, float* db, float* workspace,
                                           size_t workspace_bytes, int batch, int vsrc, int rows,
                                           int seq, int cin, int cout, void* stream) {
  return bwd_rowsub(x, 0, idx, dpre, inv_flat, flat_width, w, elu_y, dx, dw, db, workspace, workspace_bytes, batch,
                    vsrc, rows, seq, cin, cout, stream);
}

extern "C" int cfsd_spiral_conv_bwd_rowsub_x(const float* x, int x_dt, const int32_t* idx, const float* dpre,
                                             const int32_t* inv_flat, int flat_width, const float* w,
                                             const float* elu_y, float* dx, float* dw, float* db, float* workspace,
                                             size_t workspace_bytes, int batch, int vsrc, int rows, int seq, int cin,
                                             int cout, void* stream) {
  if (CFSD_DT_TYPE(x_dt) != CFSD_DT_F32 || (x_dt & ~(CFSD_VM | 0xf)))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_x: x must be fp32 (either layout)");
  return bwd_rowsub(x, (x_dt & CFSD_VM) != 0, idx, dpre, inv_flat, flat_width, w, elu_y, dx, dw, db, workspace,
                    workspace_bytes, batch, vsrc, rows, seq, cin, cout, stream);
}

static int bwd_rowsub(const float* x, int xvm, const int32_t* idx, const float* dpre, const int32_t* inv_flat,
                      int flat_width, const float* w, const float* elu_y, float* dx, float* dw, float* db,
                      float* workspace, size_t workspace_bytes, int batch, int vsrc, int rows, int seq, int cin,
                      int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!inv_flat || !w || !dx || !workspace)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub: null inv_flat / w / dx / workspace");
  if (!rowsub_shape(cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub: unsupported channels %d -> %d", cin, cout);
  if (flat_width <= 0 || flat_width > 16 || flat_width % 4)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub: flat_width %d not in {4, 8, 12, 16}", flat_width);
  if ((uintptr_t)inv_flat & 15) return set_error(CFSD_EINVAL, "inv_flat must be 16-B aligned");
  if ((dw == nullptr) != (db == nullptr))
    return set_error(CFSD_EINVAL, "dw and db must both be set (or both NULL: deferred)");
  const size_t need = cfsd_spiral_conv_bwd_rowsub_workspace(batch, vsrc, rows, seq, cin, cout);
  if (workspace_bytes < need)
    return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  const size_t dg_el = (size_t)batch * rows * kSeq * cin;
  if (dg_el * sizeof(float) >= (size_t)kAbsentRow)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub: dG of %zu floats exceeds 32-bit buffer offsets", dg_el);
  hipStream_t st = (hipStream_t)stream;
  const DwGeom g = dw_geom(batch, rows, cin, cout);
  float* dg = workspace + rowsub_slab_floats(batch, rows, cin, cout);
  const int total = batch * rows;
  const int n_tiles = kSeq * cin / 16;
  DgArgs a{dpre, w, dg, total, 0, 0};
  a.n_groups = rowsub_groups((total + 15) / 16, n_tiles);
  a.nb = (int)(((total + 15) / 16 + 3) / 4) * a.n_groups;
  const bool lat = g.kind == kDwLat;
  float* ws_db = workspace + (size_t)g.gx * dw_units(cin, cout) * 1024;
  DwLatArgs d{x, idx, dpre, workspace, ws_db, vsrc, rows, total, g.rchunk, g.gx, 0, batch, xvm, 0};
  if (lat) d.nb = (int)((lat_tasks(g.gx, dw_units(cin, cout)) + 3) / 4);
  if (xvm && !lat) return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_x: vertex-major x needs a few-row layer");
  const int n_el = cout * kSeq * cin + cout;
  if (lat && batch % 16 == 0 && cin == 32 && cout == 32 && (flat_width == 8 || flat_width == 12 || flat_width == 16)) {
    // 16-mesh batches, 32 -> 32: dx straight from dpre by the flat-list MFMA
    // kernel (one 16-mesh MFMA tile per list entry; dx in x's layout) paired
    // with the dW slabs in one launch -- no dG round trip, no gather launch
    // (the fp32 step's E1: 22.1 + 8.2 -> 22.0 us, E2: 8.5 + 5.1 -> 11.9 us;
    // E3, 32 -> 64 on 267 vertices: 14.9 vs 7.0 + 4.8 us, keeps the dG path).
    // dx sums each entry's MFMA products into one accumulator (the dG path
    // rounds every dG element first): equal to fp32 rounding, not bit for bit.
    rc = vm32::launch_bwd_flat_pair(dpre, inv_flat, flat_width, w, elu_y, dx, xvm, vsrc, rows, batch, cin, cout,
                                    d, lat_tasks(g.gx, dw_units(cin, cout)), st);
    if (rc || !dw) return rc;
#define RSR(CIN_, COUT_)                                                                          \
    if (cin == CIN_ && cout == COUT_)                                                             \
      hipLaunchKernelGGL((conv_dw_reduce<CIN_, COUT_>), dim3((unsigned)((n_el + 63) / 64)),       \
                         dim3(1024), 0, st, workspace, ws_db, dw, db, lat_slabs(g.gx));
    RSR(32, 32) RSR(32, 64)
#undef RSR
    return launch_status("spiral_conv_bwd_rowsub_reduce");
  }
  const dim3 grid((unsigned)(a.nb + d.nb));
#define RSP(CIN_, COUT_)                                                                          \
  if (cin == CIN_ && cout == COUT_) {                                                             \
    hipLaunchKernelGGL((conv_bwd_rowsub_pair<CIN_, COUT_>), grid, dim3(256),                      \
                       (dg_lds_floats<CIN_, COUT_>(a.n_groups) * sizeof(float)), st, a, d);                  \
    rc = launch_status("spiral_conv_bwd_rowsub_pair");                                           \
    if (!rc && lat && dw)                                                                         \
      hipLaunchKernelGGL((conv_dw_reduce<CIN_, COUT_>), dim3((unsigned)((n_el + 63) / 64)),       \
                         dim3(1024), 0, st, workspace, ws_db, dw, db, lat_slabs(g.gx));           \
  }
  RSP(32, 32) RSP(32, 64)
#undef RSP
  if (rc || (rc = launch_status("spiral_conv_bwd_rowsub_reduce"))) return rc;
  if (!lat) {  // many rows: the persistent dW kernel, same slab layout
    rc = cfsd_spiral_conv_bwd_weight(x, idx, dpre, dw, db, workspace, workspace_bytes, batch, vsrc,
                                     rows, seq, cin, cout, stream);
    if (rc) return rc;
  }
  const long threads = (long)batch * vsrc * (cin / 4);
  const dim3 gg((unsigned)((threads + 255) / 256));
  const int G = flat_width / 4, M = batch * vsrc;
#define RSG(CIN_, G_)                                                                             \
  if (cin == CIN_ && G == G_) {                                                                   \
    hipLaunchKernelGGL((conv_dx_rowsub_gather<CIN_, G_>), gg, dim3(256), 0, st, dg,               \
                       (const int4*)inv_flat, elu_y, dx, vsrc, rows, M, (int)(dg_el * sizeof(float)), batch, xvm); \
    return launch_status("spiral_conv_bwd_rowsub_gather");                                       \
  }
  RSG(32, 1) RSG(32, 2) RSG(32, 3) RSG(32, 4)
#undef RSG
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub: unsupported channels %d -> %d", cin, cout);
}

extern "C" size_t cfsd_spiral_conv_bwd_data_rowsub_workspace(int batch, int rows, int seq, int cin) {
  if (batch <= 0 || rows <= 0 || seq != kSeq || cin != 32) return 0;
  return rowsub_dg_floats(batch, rows, cin) * sizeof(float);
}

extern "C" int cfsd_spiral_conv_bwd_data_rowsub(const float* dpre, const int32_t* inv_flat,
                                                int flat_width, const float* w, const void* elu_y,
                                                void* dx, int dx_dt, float* workspace,
                                                size_t workspace_bytes, int batch, int vsrc, int rows,
                                                int seq, int cin, int cout, void* stream) {
  int rc = check_conv_args(dpre, inv_flat, w, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!dx || !workspace) return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_rowsub: null dx / workspace");
  if (!rowsub_shape(cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_rowsub: unsupported channels %d -> %d", cin, cout);
  const int dxvm = (dx_dt & CFSD_VM) != 0;  // dx and elu_y vertex-major
  dx_dt = CFSD_DT_TYPE(dx_dt);
  if (dx_dt != CFSD_DT_F32 && dx_dt != CFSD_DT_BF16) return set_error(CFSD_EINVAL, "bad dx dtype %d", dx_dt);
  if (flat_width <= 0 || flat_width > 16 || flat_width % 4)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_rowsub: flat_width %d not in {4, 8, 12, 16}", flat_width);
  if ((uintptr_t)inv_flat & 15) return set_error(CFSD_EINVAL, "inv_flat must be 16-B aligned");
  const size_t dg_el = (size_t)batch * rows * kSeq * cin;
  if (workspace_bytes < rowsub_dg_floats(batch, rows, cin) * sizeof(float))
    return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes,
                     rowsub_dg_floats(batch, rows, cin) * sizeof(float));
  if (dg_el * sizeof(float) >= (size_t)kAbsentRow)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_rowsub: dG exceeds 32-bit buffer offsets");
  hipStream_t st = (hipStream_t)stream;
  if (batch % 16 == 0 && cout == 32 && (flat_width == 4 || flat_width == 8 || flat_width == 12 || flat_width == 16)) {
    // 16-mesh batches, 32 -> 32: dx straight from dpre by the flat-list MFMA
    // kernel (no dG round trip, no gather launch; the bf16 step's E1: dG 11.0
    // + gather 7.0 us), the fp32 sum rounded once for bf16 storage
    if (dx_dt == CFSD_DT_BF16)
      return vm32::launch_dx_flat_b16(dpre, inv_flat, flat_width, w, (const bf16_t*)elu_y, (bf16_t*)dx, dxvm, vsrc,
                                      rows, batch, cin, cout, st);
    return vm32::launch_dx_flat(dpre, 0, dxvm, inv_flat, flat_width, w, (const float*)elu_y, (float*)dx, vsrc, rows,
                                batch, cin, cout, st);
  }
  const int total = batch * rows;
  DgArgs a{dpre, w, workspace, total, rowsub_groups((total + 15) / 16, kSeq * cin / 16), 0};
  a.nb = (int)(((total + 15) / 16 + 3) / 4) * a.n_groups;
  DwLatArgs d{};  // no dW half
  if (cout == 32)
    hipLaunchKernelGGL((conv_bwd_rowsub_pair<32, 32>), dim3(a.nb), dim3(256),
                       (dg_lds_floats<32, 32>(a.n_groups) * sizeof(float)), st, a, d);
  else
    hipLaunchKernelGGL((conv_bwd_rowsub_pair<32, 64>), dim3(a.nb), dim3(256),
                       (dg_lds_floats<32, 64>(a.n_groups) * sizeof(float)), st, a, d);
  if ((rc = launch_status("spiral_conv_bwd_data_rowsub_dg"))) return rc;
  const long threads = (long)batch * vsrc * (cin / 4);
  const dim3 gg((unsigned)((threads + 255) / 256));
  const int G = flat_width / 4, M = batch * vsrc, dgb = (int)(dg_el * sizeof(float));
#define RSG2(G_)                                                                                   \
  if (G == G_) {                                                                                   \
    if (dx_dt == CFSD_DT_BF16)                                                                     \
      hipLaunchKernelGGL((conv_dx_rowsub_gather<32, G_, bf16_t>), gg, dim3(256), 0, st, workspace, \
                         (const int4*)inv_flat, (const bf16_t*)elu_y, (bf16_t*)dx, vsrc, rows, M, dgb, batch, dxvm); \
    else                                                                                           \
      hipLaunchKernelGGL((conv_dx_rowsub_gather<32, G_, float>), gg, dim3(256), 0, st, workspace,  \
                         (const int4*)inv_flat, (const float*)elu_y, (float*)dx, vsrc, rows, M, dgb, batch, dxvm); \
    return launch_status("spiral_conv_bwd_data_rowsub_gather");                                   \
  }
  RSG2(1) RSG2(2) RSG2(3) RSG2(4)
#undef RSG2
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_rowsub: bad flat_width");
}

extern "C" int cfsd_spiral_gather(const float* x, const int32_t* idx, float* g, int batch,
                                  int vsrc, int rows, int seq, int cin, void* stream) {
  if (!x || !idx || !g) return set_error(CFSD_EINVAL, "spiral_gather: null pointer");
  if (batch <= 0 || vsrc <= 0 || rows <= 0 || seq <= 0 || cin <= 0 || (cin % 4))
    return set_error(CFSD_EINVAL, "spiral_gather: bad sizes");
  const long per_mesh = (long)rows * seq * (cin / 4);
  if (per_mesh >= (1L << 31) || batch > 65535)
    return set_error(CFSD_EINVAL, "spiral_gather: %ld chunks per mesh / batch %d too large", per_mesh, batch);
  const hipStream_t st = (hipStream_t)stream;
  const int pm = (int)per_mesh;
  if (cin == 32 || cin == 64) {
    const dim3 grid((unsigned)((per_mesh + 256 * GU - 1) / (256 * GU)), (unsigned)batch);
    if (cin == 32) hipLaunchKernelGGL(spiral_gather_k<8>, grid, dim3(256), 0, st, x, idx, g, vsrc, pm);
    else hipLaunchKernelGGL(spiral_gather_k<16>, grid, dim3(256), 0, st, x, idx, g, vsrc, pm);
  } else {
    hipLaunchKernelGGL(spiral_gather_any_k, dim3((unsigned)((per_mesh + 255) / 256), (unsigned)batch),
                       dim3(256), 0, st, x, idx, g, vsrc, cin / 4, pm);
  }
  return launch_status("spiral_gather");
}

// ============================================================== mixed precision (bf16 path)
// The bf16 path of the step stores the level-0/1 activations and gradients
// in bf16 (engine precision "bf16"); these entry points take each operand's
// storage type and route the 32/64-channel layers to the bf16 MFMA kernels
// (spiral_conv_bf16.hip) and the xyz layers to the small-channel kernels
// above, instantiated for bf16 operands.  Weights: `w` fp32 master (small
// layers), `w_bf16` its bf16 shadow (MFMA layers).
static bool mfma_shape(int cin, int cout) {
  return (cin == 32 || cin == 64) && (cout == 32 || cout == 64);
}
static bool dt_ok(int dt) {
  return (dt & ~(CFSD_VM | 0xf)) == 0 && (CFSD_DT_TYPE(dt) == CFSD_DT_F32 || CFSD_DT_TYPE(dt) == CFSD_DT_BF16);
}
static int vm_of(int dt) { return (dt & CFSD_VM) != 0; }

extern "C" int cfsd_spiral_conv_fwd_in_swap(const float* data, const int32_t* batch_idx,
                                            const uint8_t* region_mask, const int32_t* key, int bs, int n_meshes,
                                            int n_regions, float* x, int x_dt, const int32_t* idx, const float* w,
                                            const float* bias, void* y, int y_dt, int vsrc, int rows, int cin,
                                            int cout, int act, void* stream) {
  if (!data || !batch_idx || !region_mask || !key || !x || !idx || !w || !y)
    return set_error(CFSD_EINVAL, "spiral_conv_fwd_in_swap: null pointer");
  if (bs <= 0 || n_meshes <= 0 || n_regions <= 0 || vsrc <= 0 || rows <= 0)
    return set_error(CFSD_EINVAL, "spiral_conv_fwd_in_swap: bad sizes");
  if (cin != 3 || (cout != 32 && cout != 64))
    return set_error(CFSD_EINVAL, "spiral_conv_fwd_in_swap: the xyz input conv (3 -> 32/64) only");
  if (act != CFSD_ACT_NONE && act != CFSD_ACT_ELU) return set_error(CFSD_EINVAL, "bad act %d", act);
  if (!dt_ok(x_dt) || !dt_ok(y_dt) || CFSD_DT_TYPE(x_dt) != CFSD_DT_F32)
    return set_error(CFSD_EINVAL, "spiral_conv_fwd_in_swap: fp32 x, fp32 or bf16 y");
  const int batch = bs * bs;
  const long M = (long)batch * rows, swap_total = (long)batch * vsrc;
  if (swap_total >= (1L << 31)) return set_error(CFSD_EINVAL, "spiral_conv_fwd_in_swap: bs^2 x nv >= 2^31");
  const int xvm = vm_of(x_dt), yvm = vm_of(y_dt);
  const SwapSrc sw{data, batch_idx, region_mask, key, bs, n_meshes, n_regions};
  const long tiles = (M + 31) / 32;
  const int n_conv = (int)((tiles + 3) / 4 < 2048 ? (tiles + 3) / 4 : 2048);
  const dim3 grid((unsigned)(n_conv + (swap_total + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
  const bool ybf = CFSD_DT_TYPE(y_dt) == CFSD_DT_BF16;
#define FSW(CO_, ACT_, TY_)                                                                                 \
  hipLaunchKernelGGL((conv_fwd_in_swap<3, CO_, ACT_, TY_>), grid, dim3(256), 0, st, sw, x, n_conv, swap_total, \
                     idx, w, bias, (TY_*)y, vsrc, rows, M, batch, xvm, yvm)
  if (cout == 32) {
    if (act == CFSD_ACT_ELU) {
      if (ybf) FSW(32, CFSD_ACT_ELU, bf16_t); else FSW(32, CFSD_ACT_ELU, float);
    } else {
      if (ybf) FSW(32, CFSD_ACT_NONE, bf16_t); else FSW(32, CFSD_ACT_NONE, float);
    }
  } else {
    if (act == CFSD_ACT_ELU) {
      if (ybf) FSW(64, CFSD_ACT_ELU, bf16_t); else FSW(64, CFSD_ACT_ELU, float);
    } else {
      if (ybf) FSW(64, CFSD_ACT_NONE, bf16_t); else FSW(64, CFSD_ACT_NONE, float);
    }
  }
#undef FSW
  return launch_status("spiral_conv_fwd_in_swap");
}

extern "C" int cfsd_spiral_conv_fwd_x(const void* x, int x_dt, const int32_t* idx, const float* w,
                                      const uint16_t* w_bf16, const float* bias, void* y, int y_dt,
                                      int batch, int vsrc, int rows, int seq, int cin, int cout,
                                      int act, void* stream) {
  int rc = check_conv_args(x, idx, y, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!dt_ok(x_dt) || !dt_ok(y_dt)) return set_error(CFSD_EINVAL, "spiral_conv_fwd_x: bad dtype");
  if (act != CFSD_ACT_NONE && act != CFSD_ACT_ELU) return set_error(CFSD_EINVAL, "bad act %d", act);
  const hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * rows;
  const int xvm = vm_of(x_dt), yvm = vm_of(y_dt);
  x_dt = CFSD_DT_TYPE(x_dt);
  if (mfma_shape(cin, cout) && x_dt == CFSD_DT_BF16) {
    if (!w_bf16) return set_error(CFSD_EINVAL, "spiral_conv_fwd_x: w_bf16 required");
    return bf::launch_fwd((const bf16_t*)x, xvm, idx, (const bf16_t*)w_bf16, bias, y, y_dt, vsrc, rows, M, cin,
                          cout, act, st);
  }
  y_dt = CFSD_DT_TYPE(y_dt);
  if (!w) return set_error(CFSD_EINVAL, "spiral_conv_fwd_x: w required");
  if (mfma_shape(cin, cout) && x_dt == CFSD_DT_F32 && xvm) {  // fp32 vertex-major
    if (y_dt != CFSD_DT_F32) return set_error(CFSD_EINVAL, "spiral_conv_fwd_x: fp32 x needs fp32 y");
    if (coarse::fwd_ks_enabled(M, cin, cout))
      return fwd_coarse((const float*)x, xvm, idx, w, bias, (float*)y, yvm, vsrc, rows, batch, cin, cout, act, st);
    if (M < kLatFwdMax && cin == 32 && cout == 32) {  // few rows (an Enblock's kept rows): 16x16 tasks
      const long tasks = (M + 15) / 16 * 2;
      if (act == CFSD_ACT_ELU)
        hipLaunchKernelGGL((conv_fwd_lat<32, 32, CFSD_ACT_ELU, 1>), dim3((unsigned)((tasks + 3) / 4)), dim3(256),
                           0, st, (const float*)x, idx, w, bias, (float*)y, vsrc, rows, M, batch, xvm, yvm);
      else
        hipLaunchKernelGGL((conv_fwd_lat<32, 32, CFSD_ACT_NONE, 1>), dim3((unsigned)((tasks + 3) / 4)), dim3(256),
                           0, st, (const float*)x, idx, w, bias, (float*)y, vsrc, rows, M, batch, xvm, yvm);
      return launch_status("spiral_conv_fwd_lat_x");
    }
    return vm32::launch_fwd((const float*)x, idx, w, bias, (float*)y, yvm, vsrc, rows, batch, cin, cout, act, st);
  }
  if (cin <= 3 && (cout == 32 || cout == 64) && x_dt == CFSD_DT_F32 && y_dt == CFSD_DT_F32) {
#define FINF(CS_, CO_)                                                                           \
  if (cin == CS_ && cout == CO_) {                                                               \
    if (act == CFSD_ACT_ELU)                                                                     \
      hipLaunchKernelGGL((conv_fwd_in_mfma<CS_, CO_, CFSD_ACT_ELU, float>), dim3(gp), dim3(256),  \
                         0, st, (const float*)x, idx, w, bias, (float*)y, vsrc, rows, M, batch,  \
                         xvm, yvm);                                                              \
    else                                                                                         \
      hipLaunchKernelGGL((conv_fwd_in_mfma<CS_, CO_, CFSD_ACT_NONE, float>), dim3(gp), dim3(256), \
                         0, st, (const float*)x, idx, w, bias, (float*)y, vsrc, rows, M, batch,  \
                         xvm, yvm);                                                              \
    return launch_status("spiral_conv_fwd_in_x");                                                \
  }
    const long tiles = (M + 31) / 32;
    const unsigned gp = (unsigned)((tiles + 3) / 4 < 2048 ? (tiles + 3) / 4 : 2048);
    FINF(1, 32) FINF(2, 32) FINF(3, 32) FINF(1, 64) FINF(2, 64) FINF(3, 64)
#undef FINF
  }
  if (cout <= 3 && cin == 32 && xvm && batch % 8 == 0 && y_dt == CFSD_DT_F32)  // xyz output conv, vertex-major x
    return vm32::launch_fwd_out(x, x_dt == CFSD_DT_BF16, idx, w, bias, (float*)y, yvm, vsrc, rows, batch, cout, act,
                                st);
  if (cout <= 3 && (cin == 16 || cin == 32 || cin == 64) && x_dt == CFSD_DT_F32 && y_dt == CFSD_DT_F32) {
#define FOUTF(CI_, CO_)                                                                           \
  if (cin == CI_ && cout == CO_) {                                                                \
    if (act == CFSD_ACT_ELU) {                                                                    \
      auto k = conv_fwd_out_small<CI_, CO_, CFSD_ACT_ELU, float>;                                 \
      hipLaunchKernelGGL(k, dim3(small_grid(k, M)), dim3(256), 0, st, (const float*)x, idx, w,    \
                         bias, (float*)y, vsrc, rows, M, batch, xvm, yvm);                        \
    } else {                                                                                      \
      auto k = conv_fwd_out_small<CI_, CO_, CFSD_ACT_NONE, float>;                                \
      hipLaunchKernelGGL(k, dim3(small_grid(k, M)), dim3(256), 0, st, (const float*)x, idx, w,    \
                         bias, (float*)y, vsrc, rows, M, batch, xvm, yvm);                        \
    }                                                                                             \
    return launch_status("spiral_conv_fwd_out_x");                                                \
  }
    FOUTF(16, 3) FOUTF(32, 3) FOUTF(64, 3) FOUTF(32, 1) FOUTF(32, 2)
#undef FOUTF
  }
  if (cin <= 3 && (cout == 32 || cout == 64) && x_dt == CFSD_DT_F32 && y_dt == CFSD_DT_BF16) {
    const long tiles = (M + 31) / 32;
    const unsigned gp = (unsigned)((tiles + 3) / 4 < 2048 ? (tiles + 3) / 4 : 2048);
#define FINB(CS_, CO_)                                                                           \
  if (cin == CS_ && cout == CO_) {                                                               \
    if (act == CFSD_ACT_ELU)                                                                     \
      hipLaunchKernelGGL((conv_fwd_in_mfma<CS_, CO_, CFSD_ACT_ELU, bf16_t>), dim3(gp), dim3(256), \
                         0, st, (const float*)x, idx, w, bias, (bf16_t*)y, vsrc, rows, M, batch, \
                         xvm, yvm);                                                              \
    else                                                                                         \
      hipLaunchKernelGGL((conv_fwd_in_mfma<CS_, CO_, CFSD_ACT_NONE, bf16_t>), dim3(gp), dim3(256), \
                         0, st, (const float*)x, idx, w, bias, (bf16_t*)y, vsrc, rows, M, batch, \
                         xvm, yvm);                                                              \
    return launch_status("spiral_conv_fwd_in_bf16");                                             \
  }
    FINB(1, 32) FINB(2, 32) FINB(3, 32) FINB(1, 64) FINB(2, 64) FINB(3, 64)
#undef FINB
  }
  if (cout <= 3 && (cin == 16 || cin == 32 || cin == 64) && x_dt == CFSD_DT_BF16 && y_dt == CFSD_DT_F32) {
#define FOUTB(CI_, CO_)                                                                           \
  if (cin == CI_ && cout == CO_) {                                                                \
    if (act == CFSD_ACT_ELU) {                                                                    \
      auto k = conv_fwd_out_small<CI_, CO_, CFSD_ACT_ELU, bf16_t>;                                \
      hipLaunchKernelGGL(k, dim3(small_grid(k, M)), dim3(256), 0, st, (const bf16_t*)x, idx, w,   \
                         bias, (float*)y, vsrc, rows, M, batch, xvm, yvm);                        \
    } else {                                                                                      \
      auto k = conv_fwd_out_small<CI_, CO_, CFSD_ACT_NONE, bf16_t>;                               \
      hipLaunchKernelGGL(k, dim3(small_grid(k, M)), dim3(256), 0, st, (const bf16_t*)x, idx, w,   \
                         bias, (float*)y, vsrc, rows, M, batch, xvm, yvm);                        \
    }                                                                                             \
    return launch_status("spiral_conv_fwd_out_bf16");                                             \
  }
    FOUTB(16, 3) FOUTB(32, 3) FOUTB(64, 3) FOUTB(32, 1) FOUTB(32, 2)
#undef FOUTB
  }
  return set_error(CFSD_EINVAL, "spiral_conv_fwd_x: unsupported %d -> %d with dtypes %d -> %d", cin, cout,
                   x_dt, y_dt);
}

extern "C" int cfsd_spiral_conv_bwd_data_x(const void* dpre, int dpre_dt, const int32_t* inv_ptr,
                                           const int32_t* inv_row, const int32_t* inv_head,
                                           const uint16_t* w_bf16, const uint16_t* elu_y,
                                           uint16_t* dx, int dx_dt, int batch, int vsrc, int rows,
                                           int seq, int cin, int cout, void* stream) {
  int rc = check_conv_args(dpre, inv_ptr, inv_row, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!w_bf16 || !dx || !inv_head) return set_error(CFSD_EINVAL, "null w_bf16/dx/inv_head");
  if (!dt_ok(dpre_dt) || !dt_ok(dx_dt) || CFSD_DT_TYPE(dx_dt) != CFSD_DT_BF16)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_x: bad dtype");
  if ((uintptr_t)inv_head & 15) return set_error(CFSD_EINVAL, "inv_head must be 16-B aligned");
  if ((long)batch * rows * cout * (CFSD_DT_TYPE(dpre_dt) == CFSD_DT_F32 ? 4L : 2L) >= (1L << 31))
    return set_error(CFSD_EINVAL, "dpre larger than 2 GiB (32-bit buffer offsets)");
  if (!mfma_shape(cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_x: unsupported channels %d -> %d", cin, cout);
  return bf::launch_dx(dpre, dpre_dt, inv_ptr, inv_row, inv_head, (const bf16_t*)w_bf16,
                       (const bf16_t*)elu_y, (bf16_t*)dx, vm_of(dx_dt), vsrc, rows, (long)batch * vsrc,
                       cin, cout, (hipStream_t)stream);
}

extern "C" int cfsd_spiral_conv_bwd_data_flat(const void* dpre, int dpre_dt, const int32_t* inv_flat,
                                              int flat_width, const void* w, const void* elu_y, void* dx,
                                              int dx_dt, int batch, int vsrc, int rows, int seq, int cin,
                                              int cout, void* stream) {
  int rc = check_conv_args(dpre, inv_flat, w, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!dx) return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat: null dx");
  if (!dt_ok(dpre_dt) || !dt_ok(dx_dt) || !vm_of(dpre_dt) || !vm_of(dx_dt))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat: dpre and dx must be vertex-major (CFSD_VM)");
  if (CFSD_DT_TYPE(dx_dt) == CFSD_DT_F32) {  // fp32 operands and weights (spiral_conv_vm32.hip)
    if (CFSD_DT_TYPE(dpre_dt) != CFSD_DT_F32)
      return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat: fp32 dx needs fp32 dpre");
    if ((uintptr_t)inv_flat & 15) return set_error(CFSD_EINVAL, "inv_flat must be 16-B aligned");
    return vm32::launch_dx_flat((const float*)dpre, 1, 1, inv_flat, flat_width, (const float*)w, (const float*)elu_y,
                                (float*)dx, vsrc, rows, batch, cin, cout, (hipStream_t)stream);
  }
  if (!bf::vm16_ok(batch, cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat: batch %% 16 == 0 and 32 -> 32/64 channels only");
  if ((uintptr_t)inv_flat & 15) return set_error(CFSD_EINVAL, "inv_flat must be 16-B aligned");
  if ((long)batch * rows * cout * (CFSD_DT_TYPE(dpre_dt) == CFSD_DT_F32 ? 4L : 2L) >= (long)kAbsentRow)
    return set_error(CFSD_EINVAL, "dpre exceeds 32-bit buffer offsets");
  return bf::launch_dx_flat_vm16(dpre, dpre_dt, inv_flat, flat_width, (const bf16_t*)w,
                                 (const bf16_t*)elu_y, (bf16_t*)dx, vsrc, rows, batch, cin, cout,
                                 (hipStream_t)stream);
}

// ---- vertex-major pair (ABI 4.10): flat-list dx + vm32 dW slabs in one launch
static bool vm_pair_shape(int batch, int rows, int cin, int cout) {
  return cin == 32 && cout == 32 && batch % 16 == 0 && dw_geom(batch, rows, cin, cout).kind == kDwMfma;
}
extern "C" size_t cfsd_spiral_conv_bwd_flat_pair_workspace(int batch, int rows, int seq, int cin, int cout) {
  if (batch <= 0 || rows <= 0 || seq != kSeq || !vm_pair_shape(batch, rows, cin, cout)) return 0;
  return dw_geom(batch, rows, cin, cout).ws_floats * sizeof(float);
}

extern "C" int cfsd_spiral_conv_bwd_flat_pair(const float* x, const int32_t* idx, const float* dpre,
                                              const int32_t* inv_flat, int flat_width, const float* w,
                                              const float* elu_y, float* dx, float* dw, float* db, float* workspace,
                                              size_t workspace_bytes, int batch, int vsrc, int rows, int seq, int cin,
                                              int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!inv_flat || !w || !dx || !workspace)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair: null inv_flat / w / dx / workspace");
  if (!vm_pair_shape(batch, rows, cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair: 32 -> 32, batch %% 16 == 0, batch x rows >= %d only",
                     kLatDwMax);
  if (flat_width <= 0 || flat_width > 20 || flat_width % 4)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair: flat_width %d not in {4, ..., 20}", flat_width);
  if ((uintptr_t)inv_flat & 15) return set_error(CFSD_EINVAL, "inv_flat must be 16-B aligned");
  if ((dw == nullptr) != (db == nullptr))
    return set_error(CFSD_EINVAL, "dw and db must both be set (or both NULL: deferred)");
  if ((long)batch * rows * cout * 4 >= (long)kAbsentRow || (long)batch * vsrc * cin * 4 >= (long)kAbsentRow)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair: operands exceed 32-bit buffer offsets");
  const size_t need = cfsd_spiral_conv_bwd_flat_pair_workspace(batch, rows, seq, cin, cout);
  if (workspace_bytes < need) return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const DwGeom g = dw_geom(batch, rows, cin, cout);
  float* ws_db = workspace + (size_t)g.gx * dw_units(cin, cout) * 1024;
  const int nslab = vm32::dw_slabs(batch, rows, g.gx);  // as cfsd_dw_reduce_batch's fused = 3 items
  rc = vm32::launch_bwd_vm_pair(dpre, inv_flat, flat_width, w, elu_y, dx, x, idx, workspace, ws_db, nslab, vsrc,
                                rows, batch, st);
  if (rc || !dw) return rc;
  const int n_el = cout * kSeq * cin + cout;
  hipLaunchKernelGGL((conv_dw_reduce<32, 32>), dim3((unsigned)((n_el + 63) / 64)), dim3(1024), 0, st, workspace,
                     ws_db, dw, db, nslab);
  return launch_status("spiral_conv_bwd_flat_pair_reduce");
}

// ---- the bf16 step's Enblock pair (ABI 4.11): row-subset flat dx + vm16 dW slabs
extern "C" int cfsd_spiral_conv_bwd_rowsub_pair_bf16(const void* x, const int32_t* idx, const float* dpre,
                                                     const int32_t* inv_flat, int flat_width, const float* w,
                                                     const void* elu_y, void* dx, float* workspace,
                                                     size_t workspace_bytes, int batch, int vsrc, int rows, int seq,
                                                     int cin, int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!inv_flat || !w || !dx || !workspace)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_pair_bf16: null inv_flat / w / dx / workspace");
  if (cin != 32 || cout != 32 || batch % 16)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_pair_bf16: 32 -> 32, batch %% 16 == 0 only");
  if (flat_width <= 0 || flat_width > 16 || flat_width % 4)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_pair_bf16: flat_width %d not in {4, 8, 12, 16}",
                     flat_width);
  if ((uintptr_t)inv_flat & 15) return set_error(CFSD_EINVAL, "inv_flat must be 16-B aligned");
  if ((long)batch * rows * cout * 4 >= (long)kAbsentRow)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_pair_bf16: dpre exceeds 32-bit buffer offsets");
  const int nslab = bf::dw_slabs(batch, rows, cin, cout);  // as cfsd_dw_reduce_batch's fused = 2 items
  const size_t need = (size_t)nslab * ((size_t)cout * kSeq * cin + cout) * sizeof(float);
  if (workspace_bytes < need) return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  return bf::launch_bwd_rowsub16_pair((const bf16_t*)x, idx, dpre, inv_flat, flat_width, w, (const bf16_t*)elu_y,
                                      (bf16_t*)dx, workspace, nslab, vsrc, rows, batch, (hipStream_t)stream);
}

// ---- the same pair on the bf16 step's tensors (ABI 4.11)
extern "C" int cfsd_spiral_conv_bwd_flat_pair_bf16(const void* x, const int32_t* idx, const void* dpre,
                                                   const int32_t* inv_flat, int flat_width, const void* w,
                                                   const void* elu_y, void* dx, float* workspace,
                                                   size_t workspace_bytes, int batch, int vsrc, int rows, int seq,
                                                   int cin, int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!inv_flat || !w || !dx || !workspace)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair_bf16: null inv_flat / w / dx / workspace");
  if (cin != 32 || cout != 32 || batch % 16)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair_bf16: 32 -> 32, batch %% 16 == 0 only");
  if (flat_width <= 0 || flat_width > 20 || flat_width % 4)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair_bf16: flat_width %d not in {4, ..., 20}", flat_width);
  if ((uintptr_t)inv_flat & 15) return set_error(CFSD_EINVAL, "inv_flat must be 16-B aligned");
  const int nslab = bf::dw_slabs(batch, rows, cin, cout);  // as cfsd_dw_reduce_batch's fused = 2 items
  const size_t need = (size_t)nslab * ((size_t)cout * kSeq * cin + cout) * sizeof(float);
  if (workspace_bytes < need) return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  return bf::launch_bwd_vm16_pair((const bf16_t*)x, idx, (const bf16_t*)dpre, inv_flat, flat_width, (const bf16_t*)w,
                                  (const bf16_t*)elu_y, (bf16_t*)dx, workspace, nslab, vsrc, rows, batch,
                                  (hipStream_t)stream);
}

extern "C" size_t cfsd_spiral_conv_bwd_weight_x_workspace(int batch, int rows, int seq, int cin,
                                                          int cout) {
  if (batch <= 0 || rows <= 0 || seq != kSeq || cin <= 0 || cout <= 0) return 0;
  if (mfma_shape(cin, cout))
    return (size_t)bf::dw_slabs(batch, rows, cin, cout) * ((size_t)cout * kSeq * cin + cout) * sizeof(float);
  return cfsd_spiral_conv_bwd_weight_workspace(batch, rows, seq, cin, cout);
}

extern "C" int cfsd_spiral_conv_bwd_weight_x(const void* x, int x_dt, const int32_t* idx,
                                             const void* dpre, int dpre_dt, float* dw, float* db,
                                             float* workspace, size_t workspace_bytes, int batch,
                                             int vsrc, int rows, int seq, int cin, int cout,
                                             void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!dt_ok(x_dt) || !dt_ok(dpre_dt)) return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight_x: bad dtype");
  if (!workspace) return set_error(CFSD_EINVAL, "null workspace");
  if ((dw == nullptr) != (db == nullptr))
    return set_error(CFSD_EINVAL, "dw and db must both be set (or both NULL: deferred)");
  const size_t need = cfsd_spiral_conv_bwd_weight_x_workspace(batch, rows, seq, cin, cout);
  if (workspace_bytes < need)
    return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  const hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * rows;
  const int n_el = cout * kSeq * cin + cout;
  const dim3 rg((unsigned)((n_el + 63) / 64));
  const int xvm = vm_of(x_dt), dpvm = vm_of(dpre_dt);
  x_dt = CFSD_DT_TYPE(x_dt);
  int n_slabs = 0;
  if (mfma_shape(cin, cout) && x_dt == CFSD_DT_F32) {  // fp32: the fp32 kernels, x / dpre in any layout
    if (CFSD_DT_TYPE(dpre_dt) != CFSD_DT_F32)
      return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight_x: fp32 x needs fp32 dpre");
    return dw_f32((const float*)x, xvm, idx, (const float*)dpre, dpvm, dw, db, workspace, workspace_bytes, batch,
                  vsrc, rows, cin, cout, st);
  }
  if (mfma_shape(cin, cout) && x_dt == CFSD_DT_BF16) {
    rc = bf::launch_dw((const bf16_t*)x, xvm, idx, dpre, dpre_dt, workspace, vsrc, rows, M, cin, cout, st);
    n_slabs = bf::dw_slabs(batch, rows, cin, cout);
  } else if (cin <= 3 && (cout == 32 || cout == 64) && x_dt == CFSD_DT_F32) {
    const DwGeom g = dw_geom(batch, rows, cin, cout);
    if (g.kind != kDwInMfma) return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight_x: geometry");
    const bool dbf = CFSD_DT_TYPE(dpre_dt) == CFSD_DT_BF16;
#define DWIB(CS_, CO_)                                                                             \
  if (cin == CS_ && cout == CO_) {                                                                 \
    if (dbf)                                                                                       \
      hipLaunchKernelGGL((conv_dw_in_mfma<CS_, CO_, bf16_t>), dim3(g.gx), dim3(256), 0, st,        \
                         (const float*)x, idx, (const bf16_t*)dpre, workspace, vsrc, rows, M, batch, \
                         xvm, dpvm);                                                               \
    else                                                                                           \
      hipLaunchKernelGGL((conv_dw_in_mfma<CS_, CO_, float>), dim3(g.gx), dim3(256), 0, st,         \
                         (const float*)x, idx, (const float*)dpre, workspace, vsrc, rows, M, batch,  \
                         xvm, dpvm);                                                               \
  }
    DWIB(1, 32) DWIB(2, 32) DWIB(3, 32) DWIB(1, 64) DWIB(2, 64) DWIB(3, 64)
#undef DWIB
    rc = launch_status("spiral_conv_bwd_weight_in_bf16");
    n_slabs = g.gx;
  } else {
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight_x: unsupported %d -> %d with dtypes %d/%d", cin,
                     cout, x_dt, dpre_dt);
  }
  if (rc || !dw) return rc;
  hipLaunchKernelGGL(slab_reduce, rg, dim3(1024), 0, st, workspace, n_slabs, n_el, dw, cout * kSeq * cin, db);
  return launch_status("spiral_conv_bwd_weight_x_reduce");
}

extern "C" int cfsd_spiral_conv_bwd_x(const void* x, int x_dt, const int32_t* idx, const float* dpre,
                                      int dpre_dt, const int32_t* inv_ptr, const int32_t* inv_row,
                                      const int32_t* inv_head, const float* w, const void* elu_y,
                                      void* dx, float* dw, float* db, float* workspace,
                                      size_t workspace_bytes, int batch, int vsrc, int rows, int seq,
                                      int cin, int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!dt_ok(x_dt)) return set_error(CFSD_EINVAL, "spiral_conv_bwd_x: bad x dtype");
  const bool xbf = CFSD_DT_TYPE(x_dt) == CFSD_DT_BF16;  // x, elu_y and dx share x's storage
  if (!dt_ok(dpre_dt) || CFSD_DT_TYPE(dpre_dt) != CFSD_DT_F32)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_x: dpre must be fp32");
  if (!fused_small(cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_x: small-output layers only (%d -> %d)", cin, cout);
  if (!inv_ptr || !inv_row || !inv_head || !w || !workspace)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_x: null inverse table / w / workspace");
  if ((uintptr_t)inv_head & 15) return set_error(CFSD_EINVAL, "inv_head must be 16-B aligned");
  if ((dw == nullptr) != (db == nullptr))
    return set_error(CFSD_EINVAL, "dw and db must both be set (or both NULL: deferred)");
  const size_t need = cfsd_spiral_conv_bwd_workspace(batch, vsrc, rows, seq, cin, cout);
  if (workspace_bytes < need) return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  const hipStream_t st = (hipStream_t)stream;
  const long Ms = (long)batch * vsrc;
  const int gx = fused_small_gx(Ms);
  const int n_el = cout * kSeq * cin + cout;
#define BOSB(CIN_, CO_)                                                                          \
  if (cin == CIN_ && cout == CO_) {                                                              \
    if (xbf)                                                                                     \
      hipLaunchKernelGGL((conv_bwd_out_mfma<CIN_, CO_, bf16_t>), dim3(gx), dim3(256), 0, st, dpre, \
                         inv_ptr, inv_row, (const int4*)inv_head, w, (const bf16_t*)elu_y,        \
                         (const bf16_t*)x, (bf16_t*)dx, workspace, vsrc, rows, Ms, batch,         \
                         vm_of(x_dt), vm_of(dpre_dt));                                            \
    else                                                                                         \
      hipLaunchKernelGGL((conv_bwd_out_mfma<CIN_, CO_, float>), dim3(gx), dim3(256), 0, st, dpre, \
                         inv_ptr, inv_row, (const int4*)inv_head, w, (const float*)elu_y,         \
                         (const float*)x, (float*)dx, workspace, vsrc, rows, Ms, batch,           \
                         vm_of(x_dt), vm_of(dpre_dt));                                            \
    rc = launch_status("spiral_conv_bwd_small_bf16");                                            \
    if (rc || !dw) return rc;                                                                    \
    hipLaunchKernelGGL(slab_reduce, dim3((unsigned)((n_el + 63) / 64)), dim3(1024), 0, st,        \
                       workspace, gx, n_el, dw, cout * kSeq * cin, db);                          \
    return launch_status("spiral_conv_bwd_small_reduce");                                        \
  }
  BOSB(32, 1) BOSB(32, 2) BOSB(32, 3) BOSB(64, 1) BOSB(64, 2) BOSB(64, 3)
#undef BOSB
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_x: unsupported channels %d -> %d", cin, cout);
}

// Fused dx + dW of the xyz output conv for vertex-major operands through the
// flat inverse list (spiral_conv_vm32.hip conv_bwd_out_vm): same workspace
// and slab layout as cfsd_spiral_conv_bwd_x (deferred items use fused = 1).
extern "C" int cfsd_spiral_conv_bwd_out_flat(const void* x, int x_dt, const int32_t* idx, const float* dpre,
                                             int dpre_dt, const int32_t* inv_flat, int flat_width, const float* w,
                                             const void* elu_y, void* dx, float* dw, float* db, float* workspace,
                                             size_t workspace_bytes, int batch, int vsrc, int rows, int seq, int cin,
                                             int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!dt_ok(x_dt) || !dt_ok(dpre_dt) || CFSD_DT_TYPE(dpre_dt) != CFSD_DT_F32 || !vm_of(x_dt) || !vm_of(dpre_dt))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_out_flat: x (and elu_y, dx) and fp32 dpre must be vertex-major");
  if (cin != 32 || cout != 3 || vsrc != rows)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_out_flat: the 32 -> 3 output conv only (%d -> %d)", cin, cout);
  if (!inv_flat || !w || !workspace) return set_error(CFSD_EINVAL, "spiral_conv_bwd_out_flat: null flat / w / workspace");
  if ((uintptr_t)inv_flat & 15) return set_error(CFSD_EINVAL, "inv_flat must be 16-B aligned");
  if ((dw == nullptr) != (db == nullptr))
    return set_error(CFSD_EINVAL, "dw and db must both be set (or both NULL: deferred)");
  const size_t need = cfsd_spiral_conv_bwd_workspace(batch, vsrc, rows, seq, cin, cout);
  if (workspace_bytes < need) return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes, need);
  const hipStream_t st = (hipStream_t)stream;
  const int gx = fused_small_gx((long)batch * vsrc);
  rc = vm32::launch_bwd_out(dpre, inv_flat, flat_width, w, elu_y, x, dx, CFSD_DT_TYPE(x_dt) == CFSD_DT_BF16,
                            workspace, gx, vsrc, rows, batch, st);
  if (rc || !dw) return rc;
  const int n_el = cout * kSeq * cin + cout;
  hipLaunchKernelGGL(slab_reduce, dim3((unsigned)((n_el + 63) / 64)), dim3(1024), 0, st, workspace, gx, n_el, dw,
                     cout * kSeq * cin, db);
  return launch_status("spiral_conv_bwd_out_flat_reduce");
}

// Slab geometry of one deferred weight-gradient item (kind, slab count,
// slab length, db partials): what the producing launch chose.
template <typename Item>
static int fill_red_item(const cfsd_dw_slabs& q, int i, Item& d) {
  if (!q.workspace || !q.dw || !q.db) return set_error(CFSD_EINVAL, "dw_reduce_batch: item %d null", i);
  if (q.batch <= 0 || q.rows <= 0 || q.vsrc <= 0 || q.cin <= 0 || q.cout <= 0)
    return set_error(CFSD_EINVAL, "dw_reduce_batch: item %d bad sizes", i);
  d.ws = q.workspace;
  d.ws_db = nullptr;
  d.dw = q.dw;
  d.db = q.db;
  d.cin = q.cin;
  d.cout = q.cout;
  const int K = kSeq * q.cin;
  if (q.fused == 2 && mfma_shape(q.cin, q.cout)) {  // bf16 MFMA dW: plain slabs
    d.kind = 1;
    d.n_slabs = bf::dw_slabs(q.batch, q.rows, q.cin, q.cout);
    d.n_el = q.cout * K + q.cout;
  } else if (q.fused && fused_small(q.cin, q.cout)) {
    d.kind = 1;
    d.n_slabs = fused_small_gx((long)q.batch * q.vsrc);
    d.n_el = q.cout * K + q.cout;
  } else {
    const DwGeom g = dw_geom(q.batch, q.rows, q.cin, q.cout);
    if (g.kind == kDwNone) return set_error(CFSD_EINVAL, "dw_reduce_batch: item %d unsupported channels", i);
    if (g.kind == kDwMfma || g.kind == kDwLat) {
      const int U = (int)dw_units(q.cin, q.cout);
      d.kind = 0;
      const bool vm = q.fused == 3 && dw_vm32_path(1, 1, q.cin, q.cout, q.batch);  // as dw_f32 chose
      d.n_slabs = g.kind == kDwLat ? lat_slabs(g.gx)
                  : vm             ? vm32::dw_slabs(q.batch, q.rows, g.gx)
                                   : dw_mfma_slabs(q.cin, q.cout, g.gx);
      d.n_el = U * 1024 + q.cout;
      d.ws_db = q.workspace + (size_t)g.gx * U * 1024;
    } else {
      d.kind = 1;
      d.n_slabs = g.gx;
      d.n_el = q.cout * K + q.cout;
    }
  }
  return CFSD_OK;
}

static int dw_reduce_batch_launch(const cfsd_dw_slabs* items, int n, const DwAdam* adam, long n_params,
                                  void* stream) {
  if (n <= 0 && !adam) return CFSD_OK;
  if (!items) return set_error(CFSD_EINVAL, "dw_reduce_batch: null items");
  if (n > kMaxDwRed) return set_error(CFSD_EINVAL, "dw_reduce_batch: %d items > %d", n, kMaxDwRed);
  DwRedBatch B{};
  B.n = n;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    DwRedItem& d = B.it[i];
    const int rc = fill_red_item(items[i], i, d);
    if (rc) return rc;
    d.blk0 = blk;
    blk += d.kind == 0 ? (d.n_el + 255) / 256 : (d.n_el + 63) / 64;
  }
  B.blk_end = blk;
  B.adam.p = nullptr;
  if (adam) {
    // the items' dw/db ranges inside [0, n_params) of the flat gradient, sorted;
    // everything else is updated by the rest workgroups
    B.adam = *adam;
    long lo[2 * kMaxDwRed], hi[2 * kMaxDwRed];
    int nr = 0;
    for (int i = 0; i < n; ++i) {
      const long K = (long)kSeq * items[i].cin;
      const long w0 = items[i].dw - adam->g, b0 = items[i].db - adam->g;
      const long wn = (long)items[i].cout * K, bn = items[i].cout;
      if (w0 < 0 || w0 + wn > n_params || b0 < 0 || b0 + bn > n_params)
        return set_error(CFSD_EINVAL, "dw_reduce_batch_adam: item %d outside the flat gradient", i);
      lo[nr] = w0; hi[nr++] = w0 + wn;
      lo[nr] = b0; hi[nr++] = b0 + bn;
    }
    for (int i = 1; i < nr; ++i)  // insertion sort by start
      for (int j = i; j > 0 && lo[j] < lo[j - 1]; --j) {
        long t = lo[j]; lo[j] = lo[j - 1]; lo[j - 1] = t;
        t = hi[j]; hi[j] = hi[j - 1]; hi[j - 1] = t;
      }
    long cur = 0;
    int nrest = 0, rblk = 0;
    auto add_rest = [&](long a0, long a1) {
      if (a1 <= a0) return true;
      if (nrest >= kMaxAdamRest) return false;
      B.adam.rest_lo[nrest] = a0;
      B.adam.rest_hi[nrest] = a1;
      B.adam.rest_blk0[nrest] = rblk;
      rblk += (int)((a1 - a0 + 4095) / 4096);
      ++nrest;
      return true;
    };
    for (int i = 0; i < nr; ++i) {
      if (lo[i] < cur) return set_error(CFSD_EINVAL, "dw_reduce_batch_adam: overlapping items");
      if (!add_rest(cur, lo[i])) return set_error(CFSD_EINVAL, "dw_reduce_batch_adam: too many gaps");
      cur = hi[i];
    }
    if (!add_rest(cur, n_params)) return set_error(CFSD_EINVAL, "dw_reduce_batch_adam: too many gaps");
    B.adam.n_rest = nrest;
    B.adam.rest_blk0[nrest] = rblk;
    blk += rblk;
  }
  if (blk == 0) return CFSD_OK;
  hipLaunchKernelGGL(dw_reduce_batch_k, dim3(blk), dim3(1024), 0, (hipStream_t)stream, B);
  return launch_status("dw_reduce_batch");
}

extern "C" int cfsd_dw_reduce_batch(const cfsd_dw_slabs* items, int n, void* stream) {
  return dw_reduce_batch_launch(items, n, nullptr, 0, stream);
}

extern "C" int cfsd_dw_reduce_batch_adam(const cfsd_dw_slabs* items, int n, float* param,
                                         const float* grad, float* exp_avg, float* exp_avg_sq,
                                         const int32_t* step, size_t n_params, float lr, float beta1,
                                         float beta2, float eps, float weight_decay,
                                         uint16_t* param_bf16, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !step || n_params <= 0)
    return set_error(CFSD_EINVAL, "dw_reduce_batch_adam: null buffer / bad size");
  DwAdam a{};
  a.p = param;
  a.g = grad;
  a.m = exp_avg;
  a.v = exp_avg_sq;
  a.shadow = reinterpret_cast<bf16_t*>(param_bf16);
  a.step = step;
  a.lr = lr;
  a.b1 = beta1;
  a.b2 = beta2;
  a.eps = eps;
  a.wd = weight_decay;
  return dw_reduce_batch_launch(items, n, &a, (long)n_params, stream);
}
