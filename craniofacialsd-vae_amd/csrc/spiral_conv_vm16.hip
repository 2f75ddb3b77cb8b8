// SpiralConv forward / data gradient on bf16 MFMA for VERTEX-MAJOR operands
// (CFSD_VM) with a batch that is a multiple of 16 -- the bf16 step's level-0/1
// layers (configs C3/C5: 16 meshes per GPU).
//
// Reference: SpiralConv.forward (model.py:27-41) and the autograd of its
// index_select / Linear (model.py:34, 40).
//
// Vertex-major storage puts the 16 mesh rows of one vertex side by side, so a
// 16-row MFMA tile is ONE vertex x 16 meshes: every spiral index is the same
// for the whole wave (scalar loads, scalar buffer offsets: no per-lane index
// or address arithmetic), and every neighbour gather is one contiguous 1-KiB
// wave load (16 meshes x 32 bf16 channels).  The MFMA runs transposed,
// D^T[channel][mesh] = W . X^T, with the weight rows permuted in LDS so that a
// lane's accumulators are 4*NT CONSECUTIVE output channels of one mesh: the
// epilogue stores 16-B (bf16) / 32-B (fp32) vectors, a whole output block per
// wave instruction group, instead of 2-byte scalars.  Persistent waves walk an
// XCD-contiguous vertex range, the 4 waves of a block on neighbouring tiles.
// Measured at D3 (rocprofv3 device time, batch 16): 16 us against 22.7 us for
// the batch-major conv_fwd_b16; variants measured slower and not kept: W
// fragments in registers (20.8 us: occupancy), one contiguous run per wave
// with the run's indices in one vector load (20.8), the same with waves
// interleaved and an unconditional next-tile prefetch (18.5).
//
// Same products in the same K order per output as conv_fwd_b16 / conv_dx_b16
// (spiral_conv_bf16.hip); the MFMA runs in the transposed orientation and the
// ELU uses the hardware exp (elu_fast), so results agree with those kernels to
// fp32 rounding, not bit for bit.
#include "conv_bf16.h"
#include "dx_flat_vm32.h"
#include "spmm_sched.h"

namespace cfsd {
namespace bf {

namespace {
constexpr int kS = 9;
constexpr int kAbsent = 0x7ffff000;  // out-of-range buffer offset: reads 0, no traffic

__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// output channel of row i (0..15) of MFMA tile t: lane group g's four rows of
// every tile are channels CPL*g + 4t .. +3, so a lane owns CPL consecutive ones
template <int NT>
__device__ __forceinline__ int perm_ch(int t, int i) {
  return 4 * NT * (i >> 2) + 4 * t + (i & 3);
}

// store CPL = 4*NT consecutive channels (fp32 values v[t][rr], channel 4t+rr)
template <int NT>
__device__ __forceinline__ void store_row(bf16_t* p, const float (&v)[NT][4]) {
#pragma unroll
  for (int h = 0; h < NT / 2; ++h)
    *reinterpret_cast<u32x4*>(p + 8 * h) =
        (u32x4){pack_bf2(v[2 * h][0], v[2 * h][1]), pack_bf2(v[2 * h][2], v[2 * h][3]),
                pack_bf2(v[2 * h + 1][0], v[2 * h + 1][1]), pack_bf2(v[2 * h + 1][2], v[2 * h + 1][3])};
}
template <int NT>
__device__ __forceinline__ void store_row(float* p, const float (&v)[NT][4]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) *reinterpret_cast<f32x4*>(p + 4 * t) = (f32x4){v[t][0], v[t][1], v[t][2], v[t][3]};
}
}  // namespace

// ------------------------------------------------------------------ forward
// Wave = tile (output row r, mesh group mg of 16).  Lane (j, g): mesh j,
// input channels [32kc + 8g, +8) of every neighbour (B operand, one 16-B
// buffer load per slot, the spiral offset in an SGPR); A = permuted W rows
// from LDS.  y in either layout (E1 writes its batch-major level-2 output).
template <int CIN, int COUT, int ACT, typename TY>
__global__ __launch_bounds__(256) void conv_fwd_vm16(const bf16_t* __restrict__ x,
                                                     const int* __restrict__ idx,
                                                     const bf16_t* __restrict__ w,
                                                     const float* __restrict__ bias,
                                                     TY* __restrict__ y, int vsrc, int rows,
                                                     int batch, int yvm) {
  constexpr int K = kS * CIN, KP = K + 8, KC = CIN / 32, NT = COUT / 16, CPL = 4 * NT;
  extern __shared__ bf16_t lw[];  // [NT*16][KP], row t*16 + i = W row perm_ch<NT>(t, i)
  coop_copy<8, u32x4>(
      COUT * K / 8,
      [&](int e) { return *reinterpret_cast<const u32x4*>(&w[(e / (K / 8)) * K + 8 * (e % (K / 8))]); },
      [&](int e, u32x4 v) {
        const int o = e / (K / 8), rem = o % CPL;
        const int row = (rem >> 2) * 16 + 4 * (o / CPL) + (rem & 3);
        *reinterpret_cast<u32x4*>(&lw[row * KP + 8 * (e % (K / 8))]) = v;
      });
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  float bn[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) bn[t][rr] = bias ? bias[CPL * g + 4 * t + rr] : 0.f;
  const int G16 = batch >> 4;
  const long n_tiles = (long)rows * G16;
  const int xbytes = (int)((long)vsrc * batch * CIN * 2);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(x), 0, xbytes, 0x00020000);
  const int vstride = batch * CIN * 2;  // bytes between two vertices' blocks
  const TileSweep sw = xcd_sweep(n_tiles, 4, wave, true);

  auto gather = [&](long tile, u32x4 (&a)[kS][KC]) {
    const int tl = uni((int)tile);
    const int r = tl / G16, mg = tl - r * G16;
    const int voff = ((mg * 16 + j) * CIN + 8 * g) * 2;
#pragma unroll
    for (int s = 0; s < kS; ++s) {
      const int src = uni(idx[r * kS + s]);
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) a[s][kc] = bload16(rs, voff + 64 * kc, src * vstride);
    }
  };
  auto compute_store = [&](long tile, const u32x4 (&a)[kS][KC]) {
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kS; ++s)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const u32x4 wa = *reinterpret_cast<const u32x4*>(&lw[(t * 16 + j) * KP + s * CIN + 32 * kc + 8 * g]);
          acc[t] = mfma_bf16(wa, a[s][kc], acc[t]);
        }
    float v[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float z = acc[t][rr] + bn[t][rr];
        if (ACT == CFSD_ACT_ELU) z = elu_fast(z);
        v[t][rr] = z;
      }
    const int tl = (int)tile;
    const int r = tl / G16, mesh = (tl - r * G16) * 16 + j;
    const long row = yvm ? (long)r * batch + mesh : (long)mesh * rows + r;
    store_row<NT>(y + row * COUT + CPL * g, v);
  };

  // two tiles per iteration, the next one's gathers always in flight
  u32x4 a0[kS][KC], a1[kS][KC];
  long t0 = sw.begin;
  if (t0 < sw.end) gather(t0, a0);
  while (t0 < sw.end) {
    const long t1 = t0 + sw.step;
    if (t1 < sw.end) gather(t1, a1);
    compute_store(t0, a0);
    if (t1 >= sw.end) break;
    t0 = t1 + sw.step;
    if (t0 < sw.end) gather(t0, a0);
    compute_store(t1, a1);
  }
}

// ------------------------------------------------------------------ data gradient
// Wave = tile (source vertex u, mesh group).  Per slot s the B operand is
// T_s[mesh][o] = sum of the dpre rows of the inverse-spiral list (u, s): the
// list head (int4, scalar) gives rows 0-2 as unconditional buffer loads with
// scalar offsets (absent rows out of range: 0, no traffic), rows 3.. (0.3 %
// of keys) through a uniform branch; summed in fp32 in list order, rounded
// once to bf16.  A = W_s^T with permuted channel rows (LDS).  dx and elu_y
// vertex-major; dpre vertex-major (bf16 or fp32).
template <int CIN, int COUT, typename TD>
__global__ __launch_bounds__(256) void conv_dx_vm16(const TD* __restrict__ dpre,
                                                    const int* __restrict__ inv_ptr,
                                                    const int* __restrict__ inv_row,
                                                    const int4* __restrict__ inv_head,
                                                    const bf16_t* __restrict__ w,
                                                    const bf16_t* __restrict__ elu_y,
                                                    bf16_t* __restrict__ dx, int vsrc, int rows,
                                                    int batch) {
  constexpr int K = kS * CIN, OP = COUT + 8, OC = COUT / 32, NT = CIN / 16, CPL = 4 * NT;
  constexpr int RB = COUT * (int)sizeof(TD);  // dpre row bytes
  static_assert(OC >= 1, "shape");
  // lwt[(s*NT + t)*16 + i][o] = W[o][s*CIN + perm_ch(t, i)]
  extern __shared__ bf16_t lwt[];
  coop_copy<12, bf16_t>(
      COUT * K, [&](int e) { return w[e]; },
      [&](int e, bf16_t v) {
        const int o = e / K, k = e % K, s = k / CIN, c = k % CIN, rem = c % CPL;
        const int row = (s * NT + (rem >> 2)) * 16 + 4 * (c / CPL) + (rem & 3);
        lwt[row * OP + o] = v;
      });
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int G16 = batch >> 4;
  const long n_tiles = (long)vsrc * G16;
  const int nbytes = (int)((long)batch * rows * RB);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<TD*>(dpre), 0, nbytes, 0x00020000);
  const int rstride = batch * RB;  // bytes between two rows' blocks
  const TileSweep sw = xcd_sweep(n_tiles, 4, wave, true);
  constexpr int NL = sizeof(TD) == 2 ? 1 : 2;  // 16-B loads per 8 channels of a row

  for (long tile = sw.begin; tile < sw.end; tile += sw.step) {
    const int tl = uni((int)tile);
    const int u = tl / G16, mg = tl - u * G16;
    const int voff = (mg * 16 + j) * RB + 8 * g * (int)sizeof(TD);
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s0 = 0; s0 < kS; s0 += 3) {
      int4 hd[3];
      u32x4 v[3][OC][3][NL];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int4 h = inv_head[u * kS + s0 + q];
        hd[q] = make_int4(uni(h.x), uni(h.y), uni(h.z), uni(h.w));
      }
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int hr[3] = {hd[q].x, hd[q].y, hd[q].z};
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
          const int so = hr[jj] >= 0 ? hr[jj] * rstride : kAbsent;
#pragma unroll
          for (int oc = 0; oc < OC; ++oc)
#pragma unroll
            for (int l = 0; l < NL; ++l) v[q][oc][jj][l] = bload16(rs, voff + 32 * oc * (int)sizeof(TD) + 16 * l, so);
        }
      }
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int s = s0 + q;
#pragma unroll
        for (int oc = 0; oc < OC; ++oc) {
          float a8[8];
#pragma unroll
          for (int jj = 0; jj < 3; ++jj) {
            float r8[8];
            if constexpr (sizeof(TD) == 2) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                r8[2 * e] = __uint_as_float(v[q][oc][jj][0][e] << 16);
                r8[2 * e + 1] = __uint_as_float(v[q][oc][jj][0][e] & 0xffff0000u);
              }
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                r8[e] = __uint_as_float(v[q][oc][jj][0][e]);
                r8[4 + e] = __uint_as_float(v[q][oc][jj][NL - 1][e]);
              }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) a8[e] = jj == 0 ? r8[e] : a8[e] + r8[e];
          }
          if (hd[q].w >= 0) {  // 0.3 % of keys: list rows 3.. (uniform branch)
            const long key = (long)u * kS + s;
            const TD* db_ = dpre + (long)(mg * 16 + j) * COUT + 32 * oc + 8 * g;
#pragma unroll
            for (int e = 0; e < 8; ++e) a8[e] += ldf(&db_[(long)hd[q].w * batch * COUT + e]);
            for (int p = inv_ptr[key] + CFSD_INV_HEAD; p < inv_ptr[key + 1]; ++p) {
              const TD* rp = db_ + (long)inv_row[p] * batch * COUT;
#pragma unroll
              for (int e = 0; e < 8; ++e) a8[e] += ldf(&rp[e]);
            }
          }
          const u32x4 bt = {pack_bf2(a8[0], a8[1]), pack_bf2(a8[2], a8[3]), pack_bf2(a8[4], a8[5]),
                            pack_bf2(a8[6], a8[7])};
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const u32x4 wa = *reinterpret_cast<const u32x4*>(&lwt[((s * NT + t) * 16 + j) * OP + 32 * oc + 8 * g]);
            acc[t] = mfma_bf16(wa, bt, acc[t]);
          }
        }
      }
    }
    const long row = (long)u * batch + mg * 16 + j;
    float vv[NT][4];
    float ey[CPL];
    if (elu_y) {
      const bf16_t* ep = elu_y + row * CIN + CPL * g;
#pragma unroll
      for (int h = 0; h < CPL / 8; ++h) {
        const u32x4 q = *reinterpret_cast<const u32x4*>(ep + 8 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ey[8 * h + 2 * e] = __uint_as_float(q[e] << 16);
          ey[8 * h + 2 * e + 1] = __uint_as_float(q[e] & 0xffff0000u);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float z = acc[t][rr];
        if (elu_y) z *= elu_grad_from_out(ey[4 * t + rr]);
        vv[t][rr] = z;
      }
    store_row<NT>(dx + row * CIN + CPL * g, vv);
  }
}

// ------------------------------------------------------------------ data gradient, flat lists
// dx[u] = elu'(y[u]) * sum_e W_{s_e}^T dpre[r_e] over the FLAT inverse list of
// u: the spiral positions p_e = 9 r_e + s_e with idx[r_e][s_e] == u, in
// ascending p (topology.inverse_flat, the order IndexSelectBackward's
// index_add_ visits them, model.py:34).  By linearity this equals the
// per-slot form (sum the slot's rows, then W_s^T), but needs ONE load per
// entry (9 per vertex on average, FW padded with out-of-range loads) instead
// of 3 head rows per slot, and the products are exact bf16 x bf16 in fp32
// (no bf16 rounding of row sums).  One MFMA per entry and 16-column tile.
// (vb, nvb: the workgroup's index and count among the WPB-wave workgroups
// running this body; lwt: the W^T image, as conv_dx_vm16)
template <int CIN, int COUT, typename TD, int FW, int WPB = 8>
__device__ __forceinline__ void dx_flat_vm16_body(const TD* __restrict__ dpre, const int4* __restrict__ flat,
                                                  const bf16_t* __restrict__ w, const bf16_t* __restrict__ elu_y,
                                                  bf16_t* __restrict__ dx, int vsrc, int rows, int batch, int vb,
                                                  int nvb, bf16_t* lwt) {
  constexpr int K = kS * CIN, OP = COUT + 8, OC = COUT / 32, NT = CIN / 16, CPL = 4 * NT;
  constexpr int RB = COUT * (int)sizeof(TD);
  constexpr int NL = sizeof(TD) == 2 ? 1 : 2;
  constexpr int FQ = FW / 4, PD = 2, NB = PD + 1;
  coop_copy<12, bf16_t>(
      COUT * K, [&](int e) { return w[e]; },
      [&](int e, bf16_t v) {
        const int o = e / K, k = e % K, s = k / CIN, c = k % CIN, rem = c % CPL;
        const int row = (s * NT + (rem >> 2)) * 16 + 4 * (c / CPL) + (rem & 3);
        lwt[row * OP + o] = v;
      });
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int G16 = batch >> 4;
  const long n_tiles = (long)vsrc * G16;
  const int nbytes = (int)((long)batch * rows * RB);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<TD*>(dpre), 0, nbytes, 0x00020000);
  const int rstride = batch * RB;
  const TileSweep sw = xcd_sweep_v(n_tiles, WPB, wave, true, vb, nvb);
  // the walk stops at the list's first -1 (uniform branch), entries e + 1,
  // e + 2 in flight while e runs its MFMAs, the next tile's list loaded at
  // the start of this one (as the fp32 conv_dx_flat_vm32)
  auto load_list = [&](long tile, int (&pe)[FW]) {
    const int u = uni((int)tile) / G16;
#pragma unroll
    for (int q = 0; q < FQ; ++q) {
      const int4 f = flat[(long)u * FQ + q];
      pe[4 * q] = uni(f.x);
      pe[4 * q + 1] = uni(f.y);
      pe[4 * q + 2] = uni(f.z);
      pe[4 * q + 3] = uni(f.w);
    }
  };
  int pe[FW], pn[FW];
  if (sw.begin < sw.end) load_list(sw.begin, pe);
  for (long tile = sw.begin; tile < sw.end; tile += sw.step) {
    if (tile + sw.step < sw.end) load_list(tile + sw.step, pn);
    const int tl = uni((int)tile);
    const int u = tl / G16, mg = tl - u * G16;
    const int voff = (mg * 16 + j) * RB + 8 * g * (int)sizeof(TD);
    auto issue = [&](int e, u32x4(&d)[OC][NL]) {
      const int so = pe[e] >= 0 ? (pe[e] / kS) * rstride : kAbsent;
#pragma unroll
      for (int oc = 0; oc < OC; ++oc)
#pragma unroll
        for (int l = 0; l < NL; ++l) d[oc][l] = bload16(rs, voff + 32 * oc * (int)sizeof(TD) + 16 * l, so);
    };
    u32x4 v[NB][OC][NL];
#pragma unroll
    for (int e = 0; e < PD; ++e) issue(e, v[e]);
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < FW; ++e) {
      if (e + PD < FW) issue(e + PD, v[(e + PD) % NB]);
      if (pe[e] < 0) break;  // uniform: the rest of the list is padding
      const int s = pe[e] % kS;
      const u32x4(&cur)[OC][NL] = v[e % NB];
#pragma unroll
      for (int oc = 0; oc < OC; ++oc) {
        u32x4 bt;
        if constexpr (sizeof(TD) == 2) {
          bt = cur[oc][0];
        } else {
          const f32x4 a = __builtin_bit_cast(f32x4, cur[oc][0]), b = __builtin_bit_cast(f32x4, cur[oc][1]);
          bt = (u32x4){pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y), pack_bf2(b.z, b.w)};
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const u32x4 wa = *reinterpret_cast<const u32x4*>(&lwt[((s * NT + t) * 16 + j) * OP + 32 * oc + 8 * g]);
          acc[t] = mfma_bf16(wa, bt, acc[t]);
        }
      }
    }
    const long row = (long)u * batch + mg * 16 + j;
    float vv[NT][4];
    float ey[CPL];
    if (elu_y) {
      const bf16_t* ep = elu_y + row * CIN + CPL * g;
#pragma unroll
      for (int h = 0; h < CPL / 8; ++h) {
        const u32x4 q = *reinterpret_cast<const u32x4*>(ep + 8 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ey[8 * h + 2 * e] = __uint_as_float(q[e] << 16);
          ey[8 * h + 2 * e + 1] = __uint_as_float(q[e] & 0xffff0000u);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        float z = acc[t][rr];
        if (elu_y) z *= elu_grad_from_out(ey[4 * t + rr]);
        vv[t][rr] = z;
      }
    store_row<NT>(dx + row * CIN + CPL * g, vv);
#pragma unroll
    for (int e = 0; e < FW; ++e) pe[e] = pn[e];
  }
}

template <int CIN, int COUT, typename TD, int FW>
__global__ __launch_bounds__(512) void conv_dx_flat_vm16(const TD* __restrict__ dpre,
                                                         const int4* __restrict__ flat,
                                                         const bf16_t* __restrict__ w,
                                                         const bf16_t* __restrict__ elu_y,
                                                         bf16_t* __restrict__ dx, int vsrc, int rows,
                                                         int batch) {
  extern __shared__ bf16_t lwt[];
  dx_flat_vm16_body<CIN, COUT, TD, FW>(dpre, flat, w, elu_y, dx, vsrc, rows, batch, blockIdx.x, gridDim.x, lwt);
}

// ------------------------------------------------------------------ weight gradient (32 -> 32)
// dW_s[o][c] = sum over (vertex v, mesh m) of dpre[v][m][o] x[idx[v][s]][m][c]
// (model.py:34, 40) for vertex-major bf16 x and dpre, batch % 16 == 0.  A unit
// (vertex v, 16-mesh group) is exactly the K = 16 of ONE
// v_mfma_f32_32x32x16_bf16 per slot: A[o][k] = dpre[v][k][o], B[k][c] =
// x_s[k][c].  Both operands are columns of the unit's contiguous 1-KiB
// row-major blocks, so a wave writes its blocks to its OWN 1-KiB LDS slots
// (one 16-B ds_write per lane each) and reads the fragments back with
// ds_read_b64_tr_b16 (the hardware transpose): no workgroup barrier in the
// sweep (the batch-major conv_dw_b16 stages 32-row tiles behind two barriers
// per tile and runs 9 small MFMAs between them).  A wave owns 3 slots (slot
// group) over an XCD-interleaved unit range; the next unit's blocks are in
// flight in registers during this unit's MFMAs.  Workgroup = 4 ranges x 3
// slot groups (12 waves, one per CU), summed in LDS in fixed order into one
// plain slab [32 * 288 + 32] (the conv_dw_b16 layout, dw_reduce_batch kind 1).
constexpr int kDw16Pd = 2;
constexpr int DW16_NR = 4, DW16_WAVES = DW16_NR * 3, DW16_THREADS = DW16_WAVES * 64;
typedef short s16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4v;

// 32x32x16 fragment of a [16 rows][32 cols] bf16 block in LDS (64-B rows):
// lane l gets column 16(g & 1) + (l & 15) of rows 8(g >> 1) .. + 7, g = l >> 4
__device__ __forceinline__ bf16x8 tr_frag32(const bf16_t* blk, int lane) {
  const int li = lane & 15, g = lane >> 4, q = li >> 2, p = li & 3;
  const bf16_t* a = blk + (8 * (g >> 1) + q) * 32 + 16 * (g & 1) + 4 * p;
  const s16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4v*)a);
  const s16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4v*)(a + 4 * 32));
  const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
  return __builtin_bit_cast(bf16x8, (u32x4){l2.x, l2.y, h2.x, h2.y});
}

// TD = float: an Enblock's dpre, fp32 batch-major at the kept rows (rounded to
// bf16 when staged, as conv_dw_b16 rounds it).
constexpr int DW16_LDS_BYTES = DW16_WAVES * 4 * 16 * 32 * 2 + DW16_NR * 64 * 4;  // block slots (red) + db partials
// PD: units in flight (2: the dW-only kernel; 1: the pair, under 80 VGPRs);
// bid / nb: this workgroup's slab and the slab count; lds: DW16_LDS_BYTES.
template <typename TD, int PD>
__device__ __forceinline__ void dw_vm16_body(const bf16_t* __restrict__ x, const int* __restrict__ idx,
                                             const TD* __restrict__ dpre, float* __restrict__ ws, int vsrc, int rows,
                                             int batch, int bid, int nb, char* lds_raw) {
  constexpr int C = 32, K = kS * C, NEL = C * K + C, NS = 3;
  constexpr int SLOT = 16 * C;  // bf16 elements of one 1-KiB block
  bf16_t* lds = reinterpret_cast<bf16_t*>(lds_raw);  // 48 KiB, reused by red
  float* dbl = reinterpret_cast<float*>(lds_raw + DW16_WAVES * (1 + NS) * SLOT * 2);
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int sg = wave % 3, vg = wave / 3;
  bf16_t* my = lds + wave * (1 + NS) * SLOT;  // [dpre][x_0][x_1][x_2]
  const int G16 = batch >> 4;
  const long n_units = (long)rows * G16;
  const int G = nb < 8 ? nb : 8;
  const int grp = bid % G, lb = bid / G, nb_g = (nb - grp + G - 1) / G;
  const long per = (n_units + G - 1) / G;
  const long g0 = grp * per, g1 = min(n_units, g0 + per);
  const int nr = nb_g * DW16_NR;
  const long u0 = g0 + lb * DW16_NR + vg, u1 = g1, ustep = nr;  // XCD-interleaved unit range
  const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(x), 0, (int)((long)vsrc * batch * C * 2),
                                                    0x00020000);
  const auto rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<TD*>(dpre), 0,
                                                    (int)((long)rows * batch * C * sizeof(TD)), 0x00020000);
  const int voff = lane * 16;
  f32x16 acc[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) acc[k] = (f32x16){0.f};
  float dbs = 0.f;
  // PD units' blocks in flight (a unit is only 3 MFMAs: one unit ahead
  // left every unit waiting out a memory latency)
  u32x4 ring[PD][1 + NS];
  auto load_unit = [&](long un, u32x4 (&b)[1 + NS]) {
    const int uu = uni((int)un);
    const int v = uu / G16, mg = uu - v * G16;
    if constexpr (sizeof(TD) == 2) {
      b[0] = bload16(rd, voff, (v * batch + mg * 16) * C * 2);
    } else {  // fp32 batch-major: lane (mesh l / 4, channels 8 (l % 4) .. + 7) of row v
      const int vo = ((mg * 16 + (lane >> 2)) * rows) * C * 4 + 32 * (lane & 3);
      const f32x4 lo = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, vo, v * C * 4, 0));
      const f32x4 hi = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, vo + 16, v * C * 4, 0));
      b[0] = (u32x4){pack_bf2(lo.x, lo.y), pack_bf2(lo.z, lo.w), pack_bf2(hi.x, hi.y), pack_bf2(hi.z, hi.w)};
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) b[1 + k] = bload16(rx, voff, (uni(idx[v * kS + NS * sg + k]) * batch + mg * 16) * C * 2);
  };
#pragma unroll
  for (int d = 0; d < PD - 1; ++d)
    if (u0 + d * ustep < u1) load_unit(u0 + d * ustep, ring[d]);
  for (long base = u0; base < u1; base += PD * ustep) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const long un = base + d * ustep;
      if (un >= u1) break;  // uniform
      const long ahead = un + (PD - 1) * ustep;
      if (ahead < u1) load_unit(ahead, ring[(d + PD - 1) % PD]);
#pragma unroll
      for (int k = 0; k < 1 + NS; ++k) *reinterpret_cast<u32x4*>(my + k * SLOT + 8 * lane) = ring[d][k];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const bf16x8 af = tr_frag32(my, lane);
#pragma unroll
      for (int k = 0; k < NS; ++k)
        acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, tr_frag32(my + (1 + k) * SLOT, lane), acc[k], 0, 0, 0);
      if (sg == 0) {
        const u32x4 av = __builtin_bit_cast(u32x4, af);
#pragma unroll
        for (int e = 0; e < 4; ++e) dbs += bf2f(av[e] & 0xffffu) + bf2f(av[e] >> 16);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // fragments read before the slots are rewritten
      __builtin_amdgcn_wave_barrier();
    }
  }
  // ranges summed in fixed order in LDS (reused) -> one plain slab per workgroup
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);
  for (int g = 0; g < DW16_NR; ++g) {
    if (vg == g) {
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int e = acc_row(rr, lane) * K + (NS * sg + k) * C + (lane & 31);
          red[e] = g == 0 ? acc[k][rr] : red[e] + acc[k][rr];
        }
      if (sg == 0) dbl[g * 64 + lane] = dbs;
    }
    __syncthreads();
  }
  if (threadIdx.x < C) {  // lane o + 32 h of a range summed meshes 8h .. 8h + 7 of column o
    float t = 0.f;
    for (int g = 0; g < DW16_NR; ++g) t += dbl[g * 64 + threadIdx.x] + dbl[g * 64 + 32 + threadIdx.x];
    red[C * K + threadIdx.x] = t;
  }
  __syncthreads();
  float* slab = ws + (long)bid * NEL;
  for (int e = threadIdx.x; e < NEL; e += DW16_THREADS) slab[e] = red[e];
}
template <typename TD>
__global__ __launch_bounds__(DW16_THREADS) void conv_dw_vm16(const bf16_t* __restrict__ x,
                                                             const int* __restrict__ idx,
                                                             const TD* __restrict__ dpre,
                                                             float* __restrict__ ws, int vsrc, int rows, int batch) {
  __shared__ __attribute__((aligned(16))) char lds[DW16_LDS_BYTES];
  dw_vm16_body<TD, kDw16Pd>(x, idx, dpre, ws, vsrc, rows, batch, blockIdx.x, gridDim.x, lds);
}

// The bf16 step's vertex-major Deblock backward in ONE launch: flat-list dx
// workgroups (12 waves) and weight-gradient workgroups (one unit in flight,
// one slab each) interleaved; both fit 80 VGPRs, so a CU holds one of each
// (as vm32::conv_bwd_vm_pair for fp32).  Same values as the two kernels.
#ifdef CFSD_LAT_STAMPS
// diagnostic build only (tools/kbench.py KB_STAMPFN=cfsd_debug_vm16_stamps): role, start, end
__device__ unsigned long long g_vm16_stamps[4096 * 3];
extern "C" int cfsd_debug_vm16_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vm16_stamps), sizeof(g_vm16_stamps), 0, hipMemcpyDeviceToHost);
}
#endif
template <int FW>
__global__ __launch_bounds__(DW16_THREADS, 2 * DW16_WAVES / 4) void conv_bwd_vm16_pair(
    const bf16_t* __restrict__ x, const int* __restrict__ idx, const bf16_t* __restrict__ dpre,
    const int4* __restrict__ flat, const bf16_t* __restrict__ w, const bf16_t* __restrict__ elu_y,
    bf16_t* __restrict__ dx, float* __restrict__ ws, int vsrc, int rows, int batch, int nb_dx, int nb_dw) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  // the data-gradient role first (see conv_bwd_lat_pair)
  const int bid = (int)blockIdx.x;
  const bool is_dx = bid < nb_dx;
  const int vb = is_dx ? bid : bid - nb_dx;
#ifdef CFSD_LAT_STAMPS
  const unsigned long long t0 = wall_clock64();
#endif
  if (is_dx)
    dx_flat_vm16_body<32, 32, bf16_t, FW, DW16_WAVES>(dpre, flat, w, elu_y, dx, vsrc, rows, batch, vb, nb_dx,
                                                      reinterpret_cast<bf16_t*>(lds_raw));
  else
    dw_vm16_body<bf16_t, 1>(x, idx, dpre, ws, vsrc, rows, batch, vb, nb_dw, lds_raw);
#ifdef CFSD_LAT_STAMPS
  __syncthreads();
  if (threadIdx.x == 0 && bid < 4096) {
    g_vm16_stamps[3 * bid] = is_dx ? 1 : 2;
    g_vm16_stamps[3 * bid + 1] = t0;
    g_vm16_stamps[3 * bid + 2] = wall_clock64();
  }
#endif
}

// ------------------------------------------------------------------ launchers
template <typename Kern>
static int resident(Kern k, size_t lds) {
  const int r = resident_blocks_of(k, 256, lds);
  return r > 0 ? r : 1;
}

template <int CIN, int COUT, int ACT, typename TY>
static int fwd16_t(const bf16_t* x, const int* idx, const bf16_t* w, const float* bias, TY* y, int vsrc,
                   int rows, int batch, int yvm, hipStream_t st) {
  constexpr size_t lds = (size_t)COUT * (kS * CIN + 8) * sizeof(bf16_t);
  auto kern = conv_fwd_vm16<CIN, COUT, ACT, TY>;
  const long tiles = (long)rows * (batch / 16);
  constexpr int bpc = 0;
  const unsigned grid = bpc > 0 ? cu_blocks(tiles, 4, bpc)
                                : balanced_blocks(tiles, 8, resident(kern, lds));  // >= 2 tiles per wave
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, x, idx, w, bias, y, vsrc, rows, batch, yvm);
  return launch_status("spiral_conv_fwd_vm16");
}

bool dw_vm16_ok(int batch, int cin, int cout, int xvm, int dpvm, int dpre_bf16) {
  return kDwVm16 && batch % 16 == 0 && cin == 32 && cout == 32 && xvm &&
         ((dpre_bf16 && dpvm) || (kDwVm16F32dp && !dpre_bf16 && !dpvm));
}

int launch_dw_vm16(const bf16_t* x, const int* idx, const void* dpre, int dpre_bf16, float* ws, int n_slabs, int vsrc,
                   int rows, int batch, hipStream_t st) {
  if ((long)vsrc * batch * 64 >= (long)kAbsent || (long)rows * batch * 128 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight_vm16: operands exceed 32-bit offsets");
  if (dpre_bf16)
    hipLaunchKernelGGL(conv_dw_vm16<bf16_t>, dim3(n_slabs), dim3(DW16_THREADS), 0, st, x, idx, (const bf16_t*)dpre, ws,
                       vsrc, rows, batch);
  else
    hipLaunchKernelGGL(conv_dw_vm16<float>, dim3(n_slabs), dim3(DW16_THREADS), 0, st, x, idx, (const float*)dpre, ws,
                       vsrc, rows, batch);
  return launch_status("spiral_conv_bwd_weight_vm16");
}

// The bf16 step's Enblock E1 backward in ONE launch: the fp32-product flat
// dx of vm32::launch_dx_flat_b16 (fp32 batch-major dpre at the kept rows, bf16
// vertex-major dx / elu_y) and the conv_dw_vm16<float> slabs, interleaved
// workgroup roles, two per CU.  Same values as the two launches.
template <int FW>
__global__ __launch_bounds__(DW16_THREADS, 2 * DW16_WAVES / 4) void conv_bwd_rowsub16_pair(
    const bf16_t* __restrict__ x, const int* __restrict__ idx, const float* __restrict__ dpre,
    const int4* __restrict__ flat, const float* __restrict__ w, const bf16_t* __restrict__ elu_y,
    bf16_t* __restrict__ dx, float* __restrict__ ws, int vsrc, int rows, int batch, int nb_dx, int nb_dw) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  // the data-gradient role first (see conv_bwd_lat_pair)
  const int bid = (int)blockIdx.x;
  const bool is_dx = bid < nb_dx;
  const int vb = is_dx ? bid : bid - nb_dx;
  if (is_dx)
    vm32::dx_flat_body<32, 32, FW, bf16_t, DW16_WAVES>(dpre, flat, w, elu_y, dx, vsrc, rows, batch, 0, 1, vb, nb_dx,
                                                       reinterpret_cast<float*>(lds_raw));
  else
    dw_vm16_body<float, 1>(x, idx, dpre, ws, vsrc, rows, batch, vb, nb_dw, lds_raw);
}

int launch_bwd_rowsub16_pair(const bf16_t* x, const int* idx, const float* dpre, const int* flat, int width,
                             const float* w, const bf16_t* elu_y, bf16_t* dx, float* ws, int n_slabs, int vsrc,
                             int rows, int batch, hipStream_t st) {
  if (batch % 16) return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_pair_bf16: batch %% 16 != 0");
  if ((long)vsrc * batch * 64 >= (long)kAbsent || (long)rows * batch * 128 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_pair_bf16: operands exceed 32-bit offsets");
  constexpr size_t lds_dx = (size_t)kS * 32 * (32 + 8) * sizeof(float);
  constexpr size_t lds = lds_dx > (size_t)DW16_LDS_BYTES ? lds_dx : (size_t)DW16_LDS_BYTES;
  constexpr int dxb = 0;  // dx workgroups (0: one per CU)
  const int nb_dx = dxb > 0 ? dxb : device_cus();
#define BV(FW_)                                                                                               \
  if (width == FW_) {                                                                                         \
    hipLaunchKernelGGL((conv_bwd_rowsub16_pair<FW_>), dim3((unsigned)(nb_dx + n_slabs)), dim3(DW16_THREADS), lds, \
                       st, x, idx, dpre, (const int4*)flat, w, elu_y, dx, ws, vsrc, rows, batch, nb_dx, n_slabs);  \
    return launch_status("spiral_conv_bwd_rowsub16_pair");                                                    \
  }
  BV(4) BV(8) BV(12) BV(16)
#undef BV
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub_pair_bf16: flat width %d", width);
}

int launch_bwd_vm16_pair(const bf16_t* x, const int* idx, const bf16_t* dpre, const int* flat, int width,
                         const bf16_t* w, const bf16_t* elu_y, bf16_t* dx, float* ws, int n_slabs, int vsrc, int rows,
                         int batch, hipStream_t st) {
  if (batch % 16) return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair (bf16): batch %% 16 != 0");
  if ((long)vsrc * batch * 64 >= (long)kAbsent || (long)rows * batch * 64 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair (bf16): operands exceed 32-bit offsets");
  constexpr size_t lds_dx = (size_t)kS * 32 * (32 + 8) * sizeof(bf16_t);
  constexpr size_t lds = lds_dx > (size_t)DW16_LDS_BYTES ? lds_dx : (size_t)DW16_LDS_BYTES;
  constexpr int dxb = 0;  // dx workgroups (0: one per CU)
  const int nb_dx = dxb > 0 ? dxb : device_cus();
#define BV(FW_)                                                                                             \
  if (width == FW_) {                                                                                       \
    hipLaunchKernelGGL((conv_bwd_vm16_pair<FW_>), dim3((unsigned)(nb_dx + n_slabs)), dim3(DW16_THREADS), lds, st, \
                       x, idx, dpre, (const int4*)flat, w, elu_y, dx, ws, vsrc, rows, batch, nb_dx, n_slabs);   \
    return launch_status("spiral_conv_bwd_vm16_pair");                                                      \
  }
  BV(8) BV(12) BV(16) BV(20)
#undef BV
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair (bf16): flat width %d", width);
}

bool vm16_ok(int batch, int cin, int cout) {
  return batch % 16 == 0 && cin == 32 && (cout == 32 || cout == 64);
}

int launch_fwd_vm16(const bf16_t* x, const int* idx, const bf16_t* w, const float* bias, void* y, int y_dt,
                    int vsrc, int rows, int batch, int cin, int cout, int act, hipStream_t st) {
  const int yvm = (y_dt & CFSD_VM) != 0;
  const bool ybf = CFSD_DT_TYPE(y_dt) == DT_BF16;
#define F16(CO)                                                                                          \
  if (cout == CO) {                                                                                      \
    if (ybf)                                                                                             \
      return act == CFSD_ACT_ELU                                                                         \
                 ? fwd16_t<32, CO, CFSD_ACT_ELU, bf16_t>(x, idx, w, bias, (bf16_t*)y, vsrc, rows, batch, yvm, st) \
                 : fwd16_t<32, CO, CFSD_ACT_NONE, bf16_t>(x, idx, w, bias, (bf16_t*)y, vsrc, rows, batch, yvm, st); \
    return act == CFSD_ACT_ELU                                                                           \
               ? fwd16_t<32, CO, CFSD_ACT_ELU, float>(x, idx, w, bias, (float*)y, vsrc, rows, batch, yvm, st) \
               : fwd16_t<32, CO, CFSD_ACT_NONE, float>(x, idx, w, bias, (float*)y, vsrc, rows, batch, yvm, st); \
  }
  F16(32) F16(64)
#undef F16
  return set_error(CFSD_EINVAL, "spiral_conv_fwd_vm16: unsupported channels %d -> %d", cin, cout);
}

template <int CIN, int COUT, typename TD>
static int dx16_t(const TD* dpre, const int* inv_ptr, const int* inv_row, const int* inv_head, const bf16_t* w,
                  const bf16_t* elu_y, bf16_t* dx, int vsrc, int rows, int batch, hipStream_t st) {
  constexpr size_t lds = (size_t)kS * CIN * (COUT + 8) * sizeof(bf16_t);
  auto kern = conv_dx_vm16<CIN, COUT, TD>;
  const long tiles = (long)vsrc * (batch / 16);
  const unsigned grid = balanced_blocks(tiles, 4, resident(kern, lds));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, dpre, inv_ptr, inv_row, (const int4*)inv_head, w,
                     elu_y, dx, vsrc, rows, batch);
  return launch_status("spiral_conv_bwd_data_vm16");
}

int launch_dx_vm16(const void* dpre, int dpre_dt, const int* inv_ptr, const int* inv_row, const int* inv_head,
                   const bf16_t* w, const bf16_t* elu_y, bf16_t* dx, int vsrc, int rows, int batch, int cin,
                   int cout, hipStream_t st) {
  const bool dbf = CFSD_DT_TYPE(dpre_dt) == DT_BF16;
#define D16(CO)                                                                                          \
  if (cout == CO)                                                                                        \
    return dbf ? dx16_t<32, CO, bf16_t>((const bf16_t*)dpre, inv_ptr, inv_row, inv_head, w, elu_y, dx, vsrc, \
                                        rows, batch, st)                                                 \
               : dx16_t<32, CO, float>((const float*)dpre, inv_ptr, inv_row, inv_head, w, elu_y, dx, vsrc, \
                                       rows, batch, st);
  D16(32) D16(64)
#undef D16
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_vm16: unsupported channels %d -> %d", cin, cout);
}

// bf16 flat-list data gradient: 3 workgroups on every CU (19.6 vs 21.1 us
// with the balanced-iteration grid, profiles/round5r_kprof_grid_bf16_out.txt)
constexpr int kVm16DxBpc = 3;
template <int CIN, int COUT, typename TD, int FW>
static int dxf16_t(const TD* dpre, const int* flat, const bf16_t* w, const bf16_t* elu_y, bf16_t* dx, int vsrc,
                   int rows, int batch, hipStream_t st) {
  constexpr size_t lds = (size_t)kS * CIN * (COUT + 8) * sizeof(bf16_t);
  auto kern = conv_dx_flat_vm16<CIN, COUT, TD, FW>;
  const long tiles = (long)vsrc * (batch / 16);
  const int r = resident_blocks_of(kern, 512, lds);
  constexpr int bpc = kVm16DxBpc;
  const unsigned grid = bpc > 0 ? cu_blocks(tiles, 8, bpc) : balanced_blocks(tiles, 8, r > 0 ? r : 1);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, dpre, (const int4*)flat, w, elu_y, dx, vsrc, rows,
                     batch);
  return launch_status("spiral_conv_bwd_data_flat");
}

int launch_dx_flat_vm16(const void* dpre, int dpre_dt, const int* flat, int width, const bf16_t* w,
                        const bf16_t* elu_y, bf16_t* dx, int vsrc, int rows, int batch, int cin, int cout,
                        hipStream_t st) {
  const bool dbf = CFSD_DT_TYPE(dpre_dt) == DT_BF16;
#define DF(CO, FW_)                                                                                       \
  if (cout == CO && width == FW_)                                                                         \
    return dbf ? dxf16_t<32, CO, bf16_t, FW_>((const bf16_t*)dpre, flat, w, elu_y, dx, vsrc, rows, batch, st) \
               : dxf16_t<32, CO, float, FW_>((const float*)dpre, flat, w, elu_y, dx, vsrc, rows, batch, st);
  DF(32, 8) DF(32, 12) DF(32, 16) DF(32, 20) DF(64, 8) DF(64, 12) DF(64, 16) DF(64, 20)
#undef DF
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat: unsupported channels %d -> %d / width %d", cin,
                   cout, width);
}

}  // namespace bf
}  // namespace cfsd
