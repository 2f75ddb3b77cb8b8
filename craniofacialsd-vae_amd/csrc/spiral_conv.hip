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

namespace cfsd {

constexpr int kSeq = 9;  // spiral length of every configuration (craniofacial/body/default.yaml)

// Persistent-grid geometry: enough blocks for ~4 per CU, tiles spread evenly.
static inline unsigned persistent_blocks(long n_tiles, int tiles_per_block_unit, long max_blocks) {
  long units = (n_tiles + tiles_per_block_unit - 1) / tiles_per_block_unit;
  if (units <= max_blocks) return (unsigned)(units > 0 ? units : 1);
  long per = (units + max_blocks - 1) / max_blocks;
  return (unsigned)((units + per - 1) / per);
}

// Occupancy target per channel shape (min waves per SIMD -> VGPR budget).
constexpr int mfma_occ(int cin, int cout) { return (cin == 32 && cout == 32) ? 4 : 2; }

// ==========================================================================
// Forward, MFMA path: CIN, COUT in {32, 64}.  Each wave owns 32-row tiles of
// the flattened (b, r) row space (all COUT columns) and loops over them.
// Slot groups: blockIdx.y = g handles spiral slots [g*SPG, g*SPG + SPG); with
// SPG < 9 (layers with few rows) the partial sums go to ws[g][m][COUT] and
// conv_combine adds the groups (fixed order), bias and activation.
// W slice staged in LDS as [COUT][SPG*CIN + 4] (pad: 16-lane ds_read_b128
// groups hit distinct 16-B slots).
template <int CIN, int COUT, int ACT, int SPG>
__global__ __launch_bounds__(256, mfma_occ(CIN, COUT)) void conv_fwd_mfma(
    const float* __restrict__ x, const int* __restrict__ idx, const float* __restrict__ w,
    const float* __restrict__ bias, float* __restrict__ y, float* __restrict__ ws, int vsrc,
    int rows, long total_rows) {
  constexpr int HALF = CIN / 2;
  constexpr int NT = COUT / 32;
  constexpr int K = kSeq * CIN;
  constexpr int KG = SPG * CIN;
  constexpr int KP = KG + 4;
  extern __shared__ float lds_w[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = blockIdx.y, s0 = g * SPG;
  for (int e = threadIdx.x; e < COUT * (KG / 4); e += 256) {
    const int n = e / (KG / 4), k4 = e % (KG / 4);
    st4(&lds_w[n * KP + 4 * k4], ld4(&w[(long)n * K + s0 * CIN + 4 * k4]));
  }
  __syncthreads();
  const int i = lane & 31, h = lane >> 5;
  float bn[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bn[t] = (SPG == kSeq && bias) ? bias[t * 32 + i] : 0.f;
  const long n_tiles = (total_rows + 31) / 32;
  for (long tile = (long)blockIdx.x * 4 + wave; tile < n_tiles; tile += (long)gridDim.x * 4) {
    const long m0 = tile * 32;
    long m = m0 + i;
    if (m >= total_rows) m = total_rows - 1;  // clamp loads, stores are masked
    const int b = (int)(m / rows), r = (int)(m % rows);
    const float* xb = x + (long)b * vsrc * CIN + h * HALF;
    const int* ir = idx + (long)r * kSeq + s0;
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x16){0.f};
    // software pipeline: neighbour row of slot s+1 and index of slot s+2 are
    // in flight while slot s runs its MFMAs (loop kept rolled: a full unroll
    // makes hipcc hoist all nine gathers and spill).
    f32x4 a[HALF / 4], an[HALF / 4];
    int src_n = SPG > 1 ? ir[1] : 0;
#pragma unroll
    for (int q = 0; q < HALF / 4; ++q) a[q] = ld4(xb + (long)ir[0] * CIN + 4 * q);
#pragma unroll 1
    for (int s = 0; s < SPG; ++s) {
      if (s + 1 < SPG) {
        const int src_nn = (s + 2 < SPG) ? ir[s + 2] : 0;
#pragma unroll
        for (int q = 0; q < HALF / 4; ++q) an[q] = ld4(xb + (long)src_n * CIN + 4 * q);
        src_n = src_nn;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float* wr = &lds_w[(t * 32 + i) * KP + s * CIN + h * HALF];
#pragma unroll
        for (int q = 0; q < HALF / 4; ++q) {
          const f32x4 bw = ld4(wr + 4 * q);
          acc[t] = mfma32(a[q].x, bw.x, acc[t]);
          acc[t] = mfma32(a[q].y, bw.y, acc[t]);
          acc[t] = mfma32(a[q].z, bw.z, acc[t]);
          acc[t] = mfma32(a[q].w, bw.w, acc[t]);
        }
      }
      if (s + 1 < SPG) {
#pragma unroll
        for (int q = 0; q < HALF / 4; ++q) a[q] = an[q];
      }
    }
    float* dst = (SPG == kSeq) ? y : ws + (long)g * total_rows * COUT;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = t * 32 + i;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const long mo = m0 + acc_row(rr, lane);
        if (mo < total_rows) {
          float v = acc[t][rr];
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
    const int c = (int)((4 * t) % cols);
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

// Forward, small input (CS <= 4 channels, e.g. the xyz input of the first
// Enblock): one lane per (row, output channel), persistent over rows.  The
// CS*kSeq gathered inputs of a row are the same for its COUT lanes
// (broadcast loads); each lane keeps its weight row in registers.
template <int CS, int COUT, int ACT>
__global__ __launch_bounds__(256) void conv_fwd_in_small(const float* __restrict__ x,
                                                         const int* __restrict__ idx,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ y, int vsrc,
                                                         int rows, long total_rows) {
  constexpr int K = kSeq * CS;
  constexpr int RPW = 64 / COUT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int o = lane % COUT, slot = lane / COUT;
  float wr[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wr[k] = w[o * K + k];
  const float bo = bias ? bias[o] : 0.f;
  const long stride = (long)gridDim.x * 4 * RPW;
  for (long m = ((long)blockIdx.x * 4 + wave) * RPW + slot; m < total_rows; m += stride) {
    const int b = (int)(m / rows), r = (int)(m % rows);
    const float* xb = x + (long)b * vsrc * CS;
    const int* ir = idx + (long)r * kSeq;
    float acc = bo;
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      const float* p = xb + (long)ir[s] * CS;
#pragma unroll
      for (int c = 0; c < CS; ++c) acc = fmaf(p[c], wr[s * CS + c], acc);
    }
    if (ACT == CFSD_ACT_ELU) acc = elu_f(acc);
    y[m * COUT + o] = acc;
  }
}

// Forward, small output (CO <= 4 channels, e.g. the xyz output conv),
// persistent over rows: L = CIN/4 lanes per row, each lane owns a float4 of
// input channels of every neighbour row (one coalesced 16*L-byte read per
// neighbour), the CO partial dots are reduced across the L lanes.
template <int CIN, int CO, int ACT>
__global__ __launch_bounds__(256) void conv_fwd_out_small(const float* __restrict__ x,
                                                          const int* __restrict__ idx,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ y, int vsrc,
                                                          int rows, long total_rows) {
  constexpr int L = CIN / 4;
  constexpr int RPW = 64 / L;
  constexpr int K = kSeq * CIN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane % L, slot = lane / L;
  f32x4 wr[kSeq][CO];
#pragma unroll
  for (int s = 0; s < kSeq; ++s)
#pragma unroll
    for (int o = 0; o < CO; ++o) wr[s][o] = ld4(w + (long)o * K + s * CIN + 4 * q);
  float bo[CO];
#pragma unroll
  for (int o = 0; o < CO; ++o) bo[o] = bias ? bias[o] : 0.f;
  const long n_rows_pad = (total_rows + RPW - 1) / RPW * RPW;  // whole waves stay in the loop
  const long stride = (long)gridDim.x * 4 * RPW;
  for (long mm = ((long)blockIdx.x * 4 + wave) * RPW + slot; mm < n_rows_pad; mm += stride) {
    const bool valid = mm < total_rows;
    const long m = valid ? mm : total_rows - 1;
    const int b = (int)(m / rows), r = (int)(m % rows);
    const float* xb = x + (long)b * vsrc * CIN + 4 * q;
    const int* ir = idx + (long)r * kSeq;
    float acc[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) acc[o] = 0.f;
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      const f32x4 v = ld4(xb + (long)ir[s] * CIN);
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        acc[o] = fmaf(v.x, wr[s][o].x, acc[o]);
        acc[o] = fmaf(v.y, wr[s][o].y, acc[o]);
        acc[o] = fmaf(v.z, wr[s][o].z, acc[o]);
        acc[o] = fmaf(v.w, wr[s][o].w, acc[o]);
      }
    }
#pragma unroll
    for (int o = 0; o < CO; ++o)
#pragma unroll
      for (int d = L / 2; d >= 1; d >>= 1) acc[o] += __shfl_xor(acc[o], d);
    if (valid && q == 0) {
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        float v = acc[o] + bo[o];
        if (ACT == CFSD_ACT_ELU) v = elu_f(v);
        y[m * CO + o] = v;
      }
    }
  }
}

// ==========================================================================
// Backward data, MFMA path.  dx rows are source vertices u (flattened with
// b).  For slot s the A operand is T_s[u, :] = sum_{r in inv(u,s)} dpre[r, :]
// (gather-sum through the inverse spiral, fixed order -> deterministic); the
// B operand is W_s^T staged in LDS as [s][c][COUT + 4].
// inv_pair[u*S + s] = the first two rows of inv(u,s) (-1 if absent): those
// loads are issued unconditionally one slot ahead; the rare further entries
// (inv_ptr/inv_row from offset 2) are summed in a short loop.
// Slot groups as in conv_fwd_mfma (partials -> ws, conv_combine).
template <int CIN, int COUT, int SPG>
__global__ __launch_bounds__(256, mfma_occ(CIN, COUT)) void conv_dx_mfma(
    const float* __restrict__ dpre, const int* __restrict__ inv_ptr,
    const int* __restrict__ inv_row, const int2* __restrict__ inv_pair,
    const float* __restrict__ w, const float* __restrict__ elu_y, float* __restrict__ dx,
    float* __restrict__ ws, int vsrc, int rows, long total_rows) {
  constexpr int HALF = COUT / 2;
  constexpr int NT = CIN / 32;
  constexpr int OP = COUT + 4;
  constexpr int K = kSeq * CIN;
  extern __shared__ float lds_wt[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = blockIdx.y, s0 = g * SPG;
  // lds_wt[(sl*CIN + c) * OP + o] = w[o, (s0+sl)*CIN + c]
  for (int e = threadIdx.x; e < COUT * SPG * CIN; e += 256) {
    const int o = e / (SPG * CIN), k = e % (SPG * CIN);
    lds_wt[k * OP + o] = w[(long)o * K + s0 * CIN + k];
  }
  __syncthreads();
  const int i = lane & 31, h = lane >> 5;
  const long n_tiles = (total_rows + 31) / 32;
  for (long tile = (long)blockIdx.x * 4 + wave; tile < n_tiles; tile += (long)gridDim.x * 4) {
    const long m0 = tile * 32;
    long m = m0 + i;
    if (m >= total_rows) m = total_rows - 1;
    const int b = (int)(m / vsrc), u = (int)(m % vsrc);
    const float* db_ = dpre + (long)b * rows * COUT + h * HALF;
    const int2* pu = inv_pair + (long)u * kSeq + s0;
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x16){0.f};
    // slot pipeline: rows r0/r1 of slot s+1 and the pair of slot s+2 are in
    // flight while slot s computes (rolled loop, see conv_fwd_mfma).
    f32x4 c0[HALF / 4], c1[HALF / 4];
    int2 pc = pu[0], pn = SPG > 1 ? pu[1] : make_int2(-1, -1);
#pragma unroll
    for (int q = 0; q < HALF / 4; ++q) {
      c0[q] = ld4(db_ + (long)max(pc.x, 0) * COUT + 4 * q);
      c1[q] = ld4(db_ + (long)max(pc.y, 0) * COUT + 4 * q);
    }
#pragma unroll 1
    for (int s = 0; s < SPG; ++s) {
      f32x4 a[HALF / 4];
      const float f0 = pc.x >= 0 ? 1.f : 0.f, f1 = pc.y >= 0 ? 1.f : 0.f;
#pragma unroll
      for (int q = 0; q < HALF / 4; ++q) a[q] = c0[q] * f0 + c1[q] * f1;
      const bool more = pc.y >= 0;
      if (s + 1 < SPG) {
        const int2 pnn = (s + 2 < SPG) ? pu[s + 2] : make_int2(-1, -1);
#pragma unroll
        for (int q = 0; q < HALF / 4; ++q) {
          c0[q] = ld4(db_ + (long)max(pn.x, 0) * COUT + 4 * q);
          c1[q] = ld4(db_ + (long)max(pn.y, 0) * COUT + 4 * q);
        }
        pc = pn;
        pn = pnn;
      }
      if (more) {  // rare: entries beyond the first two
        const long key = (long)u * kSeq + s0 + s;
        const int beg = inv_ptr[key] + 2, end = inv_ptr[key + 1];
        for (int e = beg; e < end; ++e) {
          const float* p = db_ + (long)inv_row[e] * COUT;
#pragma unroll
          for (int q = 0; q < HALF / 4; ++q) a[q] += ld4(p + 4 * q);
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float* wr = &lds_wt[(s * CIN + t * 32 + i) * OP + h * HALF];
#pragma unroll
        for (int q = 0; q < HALF / 4; ++q) {
          const f32x4 bw = ld4(wr + 4 * q);
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

// Backward data, small dpre (CO <= 4 channels; the xyz output conv),
// persistent over source rows: L = CIN/4 lanes per row u, lane q owns dx
// channels [4q, 4q+4).  W (CO x kSeq*CIN) is staged once in LDS; the first
// two inverse entries of every slot come from inv_pair so all their dpre
// loads are issued together; further entries (rare) are looped.
template <int CIN, int CO>
__global__ __launch_bounds__(256) void conv_dx_out_small(const float* __restrict__ dpre,
                                                         const int* __restrict__ inv_ptr,
                                                         const int* __restrict__ inv_row,
                                                         const int2* __restrict__ inv_pair,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ elu_y,
                                                         float* __restrict__ dx, int vsrc,
                                                         int rows, long total_rows) {
  constexpr int L = CIN / 4;
  constexpr int RPW = 64 / L;
  constexpr int K = kSeq * CIN;
  __shared__ float wl[CO * K];
  for (int e = threadIdx.x; e < CO * K; e += blockDim.x) wl[e] = w[e];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane % L, slot = lane / L;
  const long stride = (long)gridDim.x * 4 * RPW;
  for (long m = ((long)blockIdx.x * 4 + wave) * RPW + slot; m < total_rows; m += stride) {
    const int b = (int)(m / vsrc), u = (int)(m % vsrc);
    const float* db_ = dpre + (long)b * rows * CO;
    const int2* pu = inv_pair + (long)u * kSeq;
    float tt[kSeq][CO];
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      const int2 pr = pu[s];
      const float* p0 = db_ + (long)max(pr.x, 0) * CO;
      const float* p1 = db_ + (long)max(pr.y, 0) * CO;
      const float f0 = pr.x >= 0 ? 1.f : 0.f, f1 = pr.y >= 0 ? 1.f : 0.f;
#pragma unroll
      for (int o = 0; o < CO; ++o) tt[s][o] = p0[o] * f0 + p1[o] * f1;
    }
#pragma unroll
    for (int s = 0; s < kSeq; ++s) {
      if (pu[s].y >= 0) {
        const long key = (long)u * kSeq + s;
        for (int e = inv_ptr[key] + 2; e < inv_ptr[key + 1]; ++e) {
          const float* p = db_ + (long)inv_row[e] * CO;
#pragma unroll
          for (int o = 0; o < CO; ++o) tt[s][o] += p[o];
        }
      }
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kSeq; ++s)
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        const f32x4 wv = ld4(&wl[o * K + s * CIN + 4 * q]);
        acc.x = fmaf(tt[s][o], wv.x, acc.x);
        acc.y = fmaf(tt[s][o], wv.y, acc.y);
        acc.z = fmaf(tt[s][o], wv.z, acc.z);
        acc.w = fmaf(tt[s][o], wv.w, acc.w);
      }
    if (elu_y) {
      const f32x4 g = ld4(elu_y + m * CIN + 4 * q);
      acc.x *= elu_grad_from_out(g.x);
      acc.y *= elu_grad_from_out(g.y);
      acc.z *= elu_grad_from_out(g.z);
      acc.w *= elu_grad_from_out(g.w);
    }
    st4(dx + m * CIN + 4 * q, acc);
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
    float* __restrict__ ws, float* __restrict__ ws_db, int vsrc, int rows, long total_rows) {
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
        const int b = (int)(m / rows), r = (int)(m % rows);
        const int src = idx[(long)r * kSeq + s];
        xs[e] = ld4(x + ((long)b * vsrc + src) * CIN + 4 * c4);
      }
    }
#pragma unroll
    for (int e = 0; e < C::DPT; ++e) {
      const int f = tid + e * C::THREADS;  // (row, o4)
      if (f < C::DF4) {
        const int row = f / (COUT / 4);
        const long m = m0 + row;
        ds[e] = m < total_rows ? ld4(dpre + m * COUT + 4 * (f % (COUT / 4)))
                               : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  long tile = blockIdx.x;
  if (tile < n_tiles) load_tile(tile);
  for (; tile < n_tiles; tile += gridDim.x) {
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
    const long next = tile + gridDim.x;
    if (next < n_tiles) load_tile(next);
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

// dw[o, s*CIN + c] = sum_p slab_p[unit(s, o/32, c/32)][o%32][c%32]; 16
// threads per output element, fixed-order xor tree (deterministic).
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv_dw_reduce(const float* __restrict__ ws,
                                                      const float* __restrict__ ws_db,
                                                      float* __restrict__ dw,
                                                      float* __restrict__ db, int n_slabs) {
  constexpr int OT = COUT / 32, CT = CIN / 32;
  constexpr int U = DwCfg<CIN, COUT>::U;
  constexpr long n_out = (long)COUT * kSeq * CIN;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long e = tid >> 4;
  const int sub = threadIdx.x & 15;
  const bool valid = e < n_out + COUT;
  if (!valid) e = n_out + COUT - 1;
  float sum = 0.f;
  if (e < n_out) {
    const int o = (int)(e / (kSeq * CIN));
    const int k = (int)(e % (kSeq * CIN));
    const int s = k / CIN, cc = k % CIN;
    const int un = (s * OT + o / 32) * CT + cc / 32;
    const long off = (long)un * 1024 + (o % 32) * 32 + (cc % 32);
    for (int p = sub; p < n_slabs; p += 16) sum += ws[(long)p * (U * 1024) + off];
  } else {
    const int o = (int)(e - n_out);
    for (int p = sub; p < n_slabs; p += 16) sum += ws_db[(long)p * COUT + o];
  }
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1) sum += __shfl_xor(sum, d);
  if (sub == 0 && valid) {
    if (e < n_out) dw[e] = sum;
    else db[e - n_out] = sum;
  }
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
    const int b = (int)(m / rows), r = (int)(m % rows);
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
    const int b = (int)(m / rows), r = (int)(m % rows);
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

__global__ __launch_bounds__(256) void slab_reduce(const float* __restrict__ ws, int n_slabs,
                                                   int n_el, float* __restrict__ out_a, int n_a,
                                                   float* __restrict__ out_b) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long e = tid >> 4;
  const int sub = threadIdx.x & 15;
  const bool valid = e < n_el;
  if (!valid) e = n_el - 1;
  float sum = 0.f;
  for (int p = sub; p < n_slabs; p += 16) sum += ws[(long)p * n_el + e];
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1) sum += __shfl_xor(sum, d);
  if (sub == 0 && valid) {
    if (e < n_a) out_a[e] = sum;
    else out_b[e - n_a] = sum;
  }
}

// Materialising gather (HBM roofline probe): g[m, s*cin + c] = x[b, idx[r,s], c].
// One thread per 16-B chunk of the output.
__global__ __launch_bounds__(256) void spiral_gather_k(const float* __restrict__ x,
                                                       const int* __restrict__ idx,
                                                       float* __restrict__ g, int vsrc, int rows,
                                                       int seq, int cin, long total_chunks) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total_chunks) return;
  const int c4 = cin / 4;
  const int q = (int)(t % c4);
  const long rs = t / c4;
  const int s = (int)(rs % seq);
  const long m = rs / seq;
  const int b = (int)(m / rows), r = (int)(m % rows);
  const float* src = x + ((long)b * vsrc + idx[(long)r * seq + s]) * cin + 4 * q;
  st4(g + t * 4, ld4(src));
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
  return CFSD_OK;
}

static const long kMaxPersistentBlocks = 1024;  // 4 per CU on 256 CUs
static const unsigned kSmallBlocks = 1024;       // persistent VALU kernels

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
  constexpr size_t lds = (size_t)COUT * (SPG * CIN + 4) * sizeof(float);
  static_assert(lds <= 80 * 1024, "W slice must fit LDS");
  const long n_tiles = (M + 31) / 32;
  dim3 grid(persistent_blocks(n_tiles, 4, kMaxPersistentBlocks / (kSeq / SPG) + 1), kSeq / SPG);
  hipLaunchKernelGGL((conv_fwd_mfma<CIN, COUT, ACT, SPG>), grid, dim3(256), lds, st, x, idx, w,
                     bias, y, ws, vsrc, rows, M);
  int rc = launch_status("spiral_conv_fwd");
  if (rc || SPG == kSeq) return rc;
  const long n4 = M * COUT / 4;
  hipLaunchKernelGGL((conv_combine<ACT>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, ws,
                     bias, (const float*)nullptr, y, kSeq / SPG, COUT, n4);
  return launch_status("spiral_conv_fwd_combine");
}

template <int CIN, int COUT, int ACT>
static int dispatch_fwd_mfma(const float* x, const int* idx, const float* w, const float* bias,
                             float* y, float* ws, size_t ws_floats, int vsrc, int rows, long M,
                             hipStream_t st) {
  constexpr bool big = (size_t)COUT * (kSeq * CIN + 4) * sizeof(float) > 80 * 1024;
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
#define FWD_SMALL(KERNEL, A_, B_)                                                                \
  if (cin == A_ && cout == B_) {                                                                 \
    if (act == CFSD_ACT_ELU)                                                                     \
      hipLaunchKernelGGL((KERNEL<A_, B_, CFSD_ACT_ELU>), dim3(kSmallBlocks), dim3(256), 0, st, x, \
                         idx, w, bias, y, vsrc, rows, M);                                        \
    else                                                                                         \
      hipLaunchKernelGGL((KERNEL<A_, B_, CFSD_ACT_NONE>), dim3(kSmallBlocks), dim3(256), 0, st,  \
                         x, idx, w, bias, y, vsrc, rows, M);                                     \
    return launch_status("spiral_conv_fwd_small");                                               \
  }
  FWD_SMALL(conv_fwd_in_small, 3, 16) FWD_SMALL(conv_fwd_in_small, 3, 32)
  FWD_SMALL(conv_fwd_in_small, 3, 64) FWD_SMALL(conv_fwd_out_small, 16, 3)
  FWD_SMALL(conv_fwd_out_small, 32, 3) FWD_SMALL(conv_fwd_out_small, 64, 3)
#undef FWD_SMALL
  return set_error(CFSD_EINVAL, "spiral_conv_fwd: unsupported channels %d -> %d", cin, cout);
}

template <int CIN, int COUT, int SPG>
static int launch_dx_mfma(const float* dpre, const int* inv_ptr, const int* inv_row,
                          const int* inv_pair, const float* w, const float* elu_y, float* dx,
                          float* ws, int vsrc, int rows, long M, hipStream_t st) {
  constexpr size_t lds = (size_t)SPG * CIN * (COUT + 4) * sizeof(float);
  static_assert(lds <= 80 * 1024, "W slice must fit LDS");
  dim3 grid(persistent_blocks((M + 31) / 32, 4, kMaxPersistentBlocks / (kSeq / SPG) + 1),
            kSeq / SPG);
  hipLaunchKernelGGL((conv_dx_mfma<CIN, COUT, SPG>), grid, dim3(256), lds, st, dpre, inv_ptr,
                     inv_row, (const int2*)inv_pair, w, elu_y, dx, ws, vsrc, rows, M);
  int rc = launch_status("spiral_conv_bwd_data");
  if (rc || SPG == kSeq) return rc;
  const long n4 = M * CIN / 4;
  hipLaunchKernelGGL((conv_combine<CFSD_ACT_NONE>), dim3((unsigned)((n4 + 255) / 256)), dim3(256),
                     0, st, ws, (const float*)nullptr, elu_y, dx, kSeq / SPG, CIN, n4);
  return launch_status("spiral_conv_bwd_data_combine");
}

template <int CIN, int COUT>
static int dispatch_dx_mfma(const float* dpre, const int* inv_ptr, const int* inv_row,
                            const int* inv_pair, const float* w, const float* elu_y, float* dx,
                            float* ws, size_t ws_floats, int vsrc, int rows, long M,
                            hipStream_t st) {
  constexpr bool big = (size_t)kSeq * CIN * (COUT + 4) * sizeof(float) > 80 * 1024;
  int spg = ws ? pick_spg(M, ws_floats, CIN) : 9;
  if (big && spg == 9) spg = 3;
  if (spg != 9 && !ws) return set_error(CFSD_EWORKSPACE, "spiral_conv_bwd_data: workspace required");
  if (spg == 9)
    return launch_dx_mfma<CIN, COUT, (big ? 3 : 9)>(dpre, inv_ptr, inv_row, inv_pair, w, elu_y, dx,
                                                    ws, vsrc, rows, M, st);
  if (spg == 3)
    return launch_dx_mfma<CIN, COUT, 3>(dpre, inv_ptr, inv_row, inv_pair, w, elu_y, dx, ws, vsrc,
                                        rows, M, st);
  return launch_dx_mfma<CIN, COUT, 1>(dpre, inv_ptr, inv_row, inv_pair, w, elu_y, dx, ws, vsrc,
                                      rows, M, st);
}

extern "C" int cfsd_spiral_conv_bwd_data(const float* dpre, const int32_t* inv_ptr,
                                         const int32_t* inv_row, const int32_t* inv_pair,
                                         const float* w, const float* elu_y, float* dx,
                                         float* workspace, size_t workspace_bytes, int batch,
                                         int vsrc, int rows, int seq, int cin, int cout,
                                         void* stream) {
  int rc = check_conv_args(dpre, inv_ptr, inv_row, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!w || !dx || !inv_pair) return set_error(CFSD_EINVAL, "null w/dx/inv_pair");
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * vsrc;
  const size_t wsf = workspace ? workspace_bytes / sizeof(float) : 0;
#define DXM(CIN_, COUT_)                                                                       \
  if (cin == CIN_ && cout == COUT_)                                                            \
    return dispatch_dx_mfma<CIN_, COUT_>(dpre, inv_ptr, inv_row, inv_pair, w, elu_y, dx,       \
                                         workspace, wsf, vsrc, rows, M, st);
  DXM(32, 32) DXM(32, 64) DXM(64, 32) DXM(64, 64)
#undef DXM
#define DXS(CIN_, CO_)                                                                          \
  if (cin == CIN_ && cout == CO_) {                                                             \
    hipLaunchKernelGGL((conv_dx_out_small<CIN_, CO_>), dim3(kSmallBlocks), dim3(256), 0, st,    \
                       dpre, inv_ptr, inv_row, (const int2*)inv_pair, w, elu_y, dx, vsrc, rows, M); \
    return launch_status("spiral_conv_bwd_data_small");                                        \
  }
  DXS(16, 3) DXS(32, 3) DXS(64, 3)
#undef DXS
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data: unsupported channels %d -> %d", cin, cout);
}

// ---- bwd weight: launch geometry shared by the workspace query and the launch
namespace {
enum DwKind { kDwMfma, kDwInSmall, kDwOutSmall, kDwNone };
struct DwGeom {
  DwKind kind;
  int gx;
  size_t ws_floats;
};

size_t dw_units(int cin, int cout) { return (size_t)kSeq * (cout / 32) * (cin / 32); }

DwGeom dw_geom(int batch, int rows, int cin, int cout) {
  DwGeom g{kDwNone, 0, 0};
  const long M = (long)batch * rows;
  if ((cin == 32 || cin == 64) && (cout == 32 || cout == 64)) {
    g.kind = kDwMfma;
    const long n_tiles = (M + 31) / 32;
    long gx = (n_tiles + 3) / 4;  // >= 4 tiles per block keeps the slab traffic bounded
    if (gx > 768) gx = 768;       // 3 blocks of 9 waves per CU
    g.gx = (int)(gx > 0 ? gx : 1);
    g.ws_floats = (size_t)g.gx * dw_units(cin, cout) * 1024 + (size_t)g.gx * cout;
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

extern "C" int cfsd_spiral_conv_bwd_weight(const float* x, const int32_t* idx, const float* dpre,
                                           float* dw, float* db, float* workspace,
                                           size_t workspace_bytes, int batch, int vsrc, int rows,
                                           int seq, int cin, int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!dw || !db || !workspace) return set_error(CFSD_EINVAL, "null dw/db/workspace");
  DwGeom g = dw_geom(batch, rows, cin, cout);
  if (g.kind == kDwNone)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight: unsupported channels %d -> %d", cin, cout);
  if (workspace_bytes < g.ws_floats * sizeof(float))
    return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes,
                     g.ws_floats * sizeof(float));
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * rows;
  const int n_el = cout * kSeq * cin + cout;
  const dim3 rg((unsigned)(((long)n_el * 16 + 255) / 256));
  if (g.kind == kDwMfma) {
    float* ws_db = workspace + (size_t)g.gx * dw_units(cin, cout) * 1024;
#define DWM(CIN_, COUT_)                                                                        \
  if (cin == CIN_ && cout == COUT_) {                                                           \
    using C = DwCfg<CIN_, COUT_>;                                                               \
    hipLaunchKernelGGL((conv_dw_mfma<CIN_, COUT_>), dim3(g.gx), dim3(C::THREADS),               \
                       C::LDS_FLOATS * sizeof(float), st, x, idx, dpre, workspace, ws_db, vsrc, \
                       rows, M);                                                                \
    rc = launch_status("spiral_conv_bwd_weight");                                               \
    if (rc) return rc;                                                                          \
    hipLaunchKernelGGL((conv_dw_reduce<CIN_, COUT_>), rg, dim3(256), 0, st, workspace, ws_db,   \
                       dw, db, g.gx);                                                           \
    return launch_status("spiral_conv_bwd_weight_reduce");                                      \
  }
    DWM(32, 32) DWM(32, 64) DWM(64, 32) DWM(64, 64)
#undef DWM
  }
#define DWS(KERNEL, A_, B_)                                                                       \
  if (cin == A_ && cout == B_) {                                                                  \
    hipLaunchKernelGGL((KERNEL<A_, B_>), dim3(g.gx), dim3(256), 0, st, x, idx, dpre, workspace,   \
                       vsrc, rows, M);                                                            \
    rc = launch_status("spiral_conv_bwd_weight_small");                                           \
    if (rc) return rc;                                                                            \
    hipLaunchKernelGGL(slab_reduce, rg, dim3(256), 0, st, workspace, g.gx, n_el, dw,              \
                       cout * kSeq * cin, db);                                                    \
    return launch_status("spiral_conv_bwd_weight_small_reduce");                                  \
  }
  if (g.kind == kDwInSmall) {
    DWS(conv_dw_in_small, 3, 16) DWS(conv_dw_in_small, 3, 32) DWS(conv_dw_in_small, 3, 64)
  } else {
    DWS(conv_dw_out_small, 16, 3) DWS(conv_dw_out_small, 32, 3) DWS(conv_dw_out_small, 64, 3)
  }
#undef DWS
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight: unsupported channels %d -> %d", cin, cout);
}

extern "C" int cfsd_spiral_gather(const float* x, const int32_t* idx, float* g, int batch,
                                  int vsrc, int rows, int seq, int cin, void* stream) {
  if (!x || !idx || !g) return set_error(CFSD_EINVAL, "spiral_gather: null pointer");
  if (batch <= 0 || vsrc <= 0 || rows <= 0 || seq <= 0 || cin <= 0 || (cin % 4))
    return set_error(CFSD_EINVAL, "spiral_gather: bad sizes");
  const long chunks = (long)batch * rows * seq * (cin / 4);
  hipLaunchKernelGGL(spiral_gather_k, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, idx, g, vsrc, rows, seq, cin, chunks);
  return launch_status("spiral_gather");
}
