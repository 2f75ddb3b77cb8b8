// Coarse-level SpiralConv kernels (levels 2-4 of the craniofacial hierarchy:
// 1065 / 267 / 67 vertices, i.e. 17k / 4.3k / 1.1k rows at batch 16).
//
// Why a separate family: at these sizes the whole layer is a few hundred
// 16-row tiles, so a kernel that gives each wave a tile and ALL nine slots
// (conv_fwd_lat) occupies ~500-2k waves on a 1024-SIMD chip and every wave
// runs a 144-288 deep v_mfma_f32_16x16x4_f32 chain (32-cycle issue each):
// the counters of round 3 (profiles/r04a_pmc_coarse_sq_summary.txt) show
// those waves issue-stalled 65 % of their life with half the SIMDs idle.
// Here the nine slots are split over the waves of a workgroup (slot groups),
// each wave keeps ITS slots' weights in VGPRs and reuses them over RT row
// tiles, and the slot-group partials are combined in LDS in a fixed order
// (g = 0, 1, ..) by the same workgroup -- no workspace and no combine launch.
//
// The Deblock form (UP) also evaluates the Pool(up) of the input inside the
// gather (model.py:80-82: Pool(x, up) then SpiralConv): the up-sampled row of
// vertex v is sum_k val[3v+k] * xc[col[3v+k]] over its 3 barycentric taps,
// computed with the SpMM's exact arithmetic ((0 + x0 v0) + x1 v1) + x2 v2
// un-fused (bit-identical to spmm_uniform_k), so the separate up-sampling
// launch disappears; the slot-0 wave (spiral slot 0 is the vertex itself,
// checked on the host) stores the up-sampled rows of its tile, which the
// weight gradient of the backward reads.
#include "cfsd_common.h"
#include "conv_coarse.h"
#include "conv_lat.h"

namespace cfsd {
namespace coarse {

// x_up chunk of fine vertex v for mesh b: the three taps of up row v
// (spmm_uniform_k's order and rounding)
__device__ __forceinline__ f32x4 up_row4(const f32x4 x0, const f32x4 x1, const f32x4 x2, float v0, float v1,
                                         float v2) {
#pragma clang fp contract(off)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc.x = acc.x + x0.x * v0;
  acc.y = acc.y + x0.y * v0;
  acc.z = acc.z + x0.z * v0;
  acc.w = acc.w + x0.w * v0;
  acc.x = acc.x + x1.x * v1;
  acc.y = acc.y + x1.y * v1;
  acc.z = acc.z + x1.z * v1;
  acc.w = acc.w + x1.w * v1;
  acc.x = acc.x + x2.x * v2;
  acc.y = acc.y + x2.y * v2;
  acc.z = acc.z + x2.z * v2;
  acc.w = acc.w + x2.w * v2;
  return acc;
}

// One workgroup = NSG waves (slot groups of kSeq / NSG slots) x RT 16-row
// tiles x all COUT columns.  v_mfma_f32_16x16x4_f32 lane map as conv_fwd_lat:
// lane (i = l & 15, kg = l >> 4) holds row i's 16-B chunks of channels
// 16c + 4kg .. +3; B = W[o][s*CIN + 16c + 4kg + j] for the 4 MFMAs j of a chunk.
// 9-wave workgroups place 3 waves on one SIMD: two co-resident workgroups
// need <= 85 VGPRs (6 waves x 85 <= 512), else every second workgroup of a
// CU waits for the first to exit (measured: D0 forward 267 workgroups, 11 of
// them a whole wave-life late)
// (two-tile workgroups: 78 KB of partials in LDS, one workgroup per CU)
constexpr int ks_min_waves(int nsg, int rt) { return nsg == 9 ? (rt == 1 ? 6 : 3) : 2; }
template <int CIN, int COUT, int NSG, int RT, int UP>
__global__ __launch_bounds__(64 * NSG, ks_min_waves(NSG, RT)) void conv_fwd_ks(const FwdKsArgs a) {
  constexpr int CH = CIN / 16, NCT = COUT / 16, K = kSeq * CIN, SPW = kSeq / NSG;
  constexpr int LDC = COUT + 4;  // partial row stride (kg rows land on distinct banks)
  static_assert(kSeq % NSG == 0, "slot groups");
  // fused Pool(up) lives in conv_fwd_pt only (its composite [rows][9][3] table)
  static_assert(!UP, "conv_fwd_ks has no fused up-sampling: use conv_fwd_pt<.., 1>");
  __shared__ f32x4 part4[NSG * RT * 16 * LDC / 4];
  float* part = reinterpret_cast<float*>(part4);
  const int lane = threadIdx.x & 63, r16 = lane & 15, kg = lane >> 4;
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long rt0 = (long)xcd_block() * RT;
  const long M = a.total_rows;
  const Lay lx = make_lay(a.xvm, a.batch, a.vsrc);
  // this lane's row in each tile (x's layout), its mesh / vertex and spiral
  int bq[RT], src[RT][SPW];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    long m = (rt0 + rt) * 16 + r16;
    if (m >= M) m = M - 1;  // clamped rows: loads only, stores are masked
    int r;
    split_row(m, a.xvm, a.batch, a.rows, bq[rt], r);
#pragma unroll
    for (int j = 0; j < SPW; ++j) src[rt][j] = a.idx[r * kSeq + g * SPW + j];
  }
  // this wave's weight slices (reused by all RT tiles)
  f32x4 bw[SPW][CH][NCT];
  const float* wb = a.w + (long)r16 * K + 4 * kg;
#pragma unroll
  for (int j = 0; j < SPW; ++j)
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int t = 0; t < NCT; ++t) bw[j][c][t] = ld4(wb + (long)t * 16 * K + (g * SPW + j) * CIN + 16 * c);
  f32x4 av[RT][SPW][CH];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const float* xb = a.x + (long)bq[rt] * lx.bs * CIN + 4 * kg;
#pragma unroll
    for (int j = 0; j < SPW; ++j)
#pragma unroll
      for (int c = 0; c < CH; ++c) av[rt][j][c] = ld4(xb + (long)src[rt][j] * lx.vs * CIN + 16 * c);
  }
  f32x4 acc[RT][NCT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // consecutive MFMAs go to different (tile, column tile) accumulators
#define KS_MF(Q)                        \
  _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) \
  _Pragma("unroll") for (int t = 0; t < NCT; ++t) acc[rt][t] = mfma16(av[rt][j][c].Q, bw[j][c][t].Q, acc[rt][t]);
#pragma unroll
  for (int j = 0; j < SPW; ++j)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      KS_MF(x) KS_MF(y) KS_MF(z) KS_MF(w)
    }
#undef KS_MF
  // slot-group partials -> LDS, combined in fixed group order
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NCT; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        part[((g * RT + rt) * 16 + 4 * kg + rr) * LDC + t * 16 + r16] = acc[rt][t][rr];
  __syncthreads();
  constexpr int N4 = RT * 16 * COUT / 4;
  for (int q = threadIdx.x; q < N4; q += 64 * NSG) {
    const int rt = q / (16 * COUT / 4), rem = q % (16 * COUT / 4);
    const int row = rem / (COUT / 4), c4 = rem % (COUT / 4);
    const long m = (rt0 + rt) * 16 + row;
    if (m >= M) continue;
    f32x4 v = part4[((0 * RT + rt) * 16 + row) * (LDC / 4) + c4];
#pragma unroll
    for (int gg = 1; gg < NSG; ++gg) v += part4[((gg * RT + rt) * 16 + row) * (LDC / 4) + c4];
    if (a.bias) v += ld4(a.bias + 4 * c4);
    if (a.elu) {
      v.x = elu_f(v.x);
      v.y = elu_f(v.y);
      v.z = elu_f(v.z);
      v.w = elu_f(v.w);
    }
    long yo = m;
    if (a.xvm != a.yvm) {
      int bo, ro;
      split_row(m, a.xvm, a.batch, a.rows, bo, ro);
      yo = row_of(make_lay(a.yvm, a.batch, a.rows), bo, ro);
    }
    st4(a.y + yo * COUT + 4 * c4, v);
  }
}

// Persistent form for the layers with several tiles per CU (the 17k-row
// layers: E1, D1): one 9-wave workgroup per CU, wave g = slot g, its weight
// slice loaded ONCE into VGPRs, then the workgroup walks a contiguous range
// of 16-row tiles: the next tile's spiral row (UP: its composite up-sampling
// row -- the 3 coarse columns / values of every spiral neighbour, a static
// table) is in flight during this tile's MFMAs and its gathers during this
// tile's combine; partials double-buffered in LDS (one barrier per tile).
#ifdef CFSD_LAT_STAMPS
// diagnostic build only (tools/kbench.py KB_PTSTAMPS): per-workgroup phases of conv_fwd_pt's first tile
__device__ unsigned long long g_pt_stamps[2048 * 6];
extern "C" int cfsd_debug_pt_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pt_stamps), sizeof(g_pt_stamps), 0, hipMemcpyDeviceToHost);
}
#define PT_T(v) v = wall_clock64();
#else
#define PT_T(v)
#endif
template <int CIN, int COUT, int UP>
__global__ __launch_bounds__(576, 3) void conv_fwd_pt(const FwdKsArgs a) {
#ifdef CFSD_LAT_STAMPS
  unsigned long long pt0 = wall_clock64(), pt1 = 0, pt2 = 0, pt3 = 0, pt4 = 0;
#endif
  constexpr int CH = CIN / 16, NCT = COUT / 16, K = kSeq * CIN, LDC = COUT + 4;
  constexpr int PB = 9 * 16 * LDC;  // floats per partial buffer
  __shared__ f32x4 part4[2 * PB / 4];
  float* part = reinterpret_cast<float*>(part4);
  const int lane = threadIdx.x & 63, r16 = lane & 15, kg = lane >> 4;
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long M = a.total_rows, n_rt = (M + 15) / 16;
  const int nb = gridDim.x, blk = xcd_block();
  // every workgroup walks `full` whole tiles; the rem leftover tiles are cut
  // into S column groups of NCT / S column tiles each (S the largest split
  // with rem * S <= nb), at most one such unit per workgroup: the launch's
  // tail is a fraction of a tile's MFMAs instead of a whole extra tile
  const long full = n_rt / nb, rem = n_rt - full * nb;
  int S = NCT;
  while (S > 1 && rem * S > nb) S >>= 1;
  const long t0 = full * blk;
  const long nitems = full + (blk < rem * S ? 1 : 0);
  const int cw = NCT / S, clo_last = (blk % S) * cw;  // the unit's column tiles
  auto item_tile = [&](long i) { return i < full ? t0 + i : full * nb + blk / S; };
  const int nv_x = UP ? a.n_coarse : a.vsrc;
  const Lay lx = make_lay(a.xvm, a.batch, nv_x);
  f32x4 bw[CH][NCT];
  const float* wb = a.w + (long)r16 * K + g * CIN + 4 * kg;
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int t = 0; t < NCT; ++t) bw[c][t] = ld4(wb + (long)t * 16 * K + 16 * c);
#ifdef CFSD_LAT_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PT_T(pt1)
#endif
  // per tile: this lane's mesh b and spiral neighbour (UP: its 3 taps)
  struct Src {
    int b, v;
    int cc[UP ? 3 : 1];
    float vv[UP ? 3 : 1];
  };
  auto load_src = [&](long tile, Src& sr) {
    long m = tile * 16 + r16;
    if (m >= M) m = M - 1;
    int r;
    split_row(m, a.xvm, a.batch, a.rows, sr.b, r);
    if constexpr (UP) {
      const long e = ((long)r * kSeq + g) * 3;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        sr.cc[k] = a.up_col[e + k];
        sr.vv[k] = a.up_val[e + k];
      }
    } else {
      sr.v = a.idx[r * kSeq + g];
    }
  };
  auto load_x = [&](const Src& sr, f32x4 (&av)[CH]) {
    const float* xb = a.x + (long)sr.b * lx.bs * CIN + 4 * kg;
    if constexpr (UP) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const f32x4 x0 = ld4(xb + (long)sr.cc[0] * lx.vs * CIN + 16 * c);
        const f32x4 x1 = ld4(xb + (long)sr.cc[1] * lx.vs * CIN + 16 * c);
        const f32x4 x2 = ld4(xb + (long)sr.cc[2] * lx.vs * CIN + 16 * c);
        av[c] = up_row4(x0, x1, x2, sr.vv[0], sr.vv[1], sr.vv[2]);
      }
    } else {
#pragma unroll
      for (int c = 0; c < CH; ++c) av[c] = ld4(xb + (long)sr.v * lx.vs * CIN + 16 * c);
    }
  };
  if (nitems == 0) return;  // (grid <= tiles: never taken)
  Src cur;
  load_src(item_tile(0), cur);
#ifdef CFSD_LAT_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PT_T(pt2)
#endif
  f32x4 av[CH];
  load_x(cur, av);
#ifdef CFSD_LAT_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PT_T(pt3)
#endif
  for (long it = 0; it < nitems; ++it) {
    const long tile = item_tile(it);
    const bool whole = it < full;  // uniform
    const int clo = whole ? 0 : clo_last, chi = whole ? NCT : clo_last + cw;
    const bool more = it + 1 < nitems;  // uniform
    Src nxt;
    if (more) load_src(item_tile(it + 1), nxt);
    f32x4 acc[NCT];
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (whole) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
#pragma unroll
        for (int t = 0; t < NCT; ++t) acc[t] = mfma16(av[c].x, bw[c][t].x, acc[t]);
#pragma unroll
        for (int t = 0; t < NCT; ++t) acc[t] = mfma16(av[c].y, bw[c][t].y, acc[t]);
#pragma unroll
        for (int t = 0; t < NCT; ++t) acc[t] = mfma16(av[c].z, bw[c][t].z, acc[t]);
#pragma unroll
        for (int t = 0; t < NCT; ++t) acc[t] = mfma16(av[c].w, bw[c][t].w, acc[t]);
      }
    } else {  // a leftover unit: the same per-column chains, its columns only
#pragma unroll
      for (int t = 0; t < NCT; ++t)
        if (t >= clo && t < chi) {
#pragma unroll
          for (int c = 0; c < CH; ++c) {
            acc[t] = mfma16(av[c].x, bw[c][t].x, acc[t]);
            acc[t] = mfma16(av[c].y, bw[c][t].y, acc[t]);
            acc[t] = mfma16(av[c].z, bw[c][t].z, acc[t]);
            acc[t] = mfma16(av[c].w, bw[c][t].w, acc[t]);
          }
        }
    }
    if constexpr (UP) {  // slot 0 = the vertex itself: the tile's up-sampled rows
      if (g == 0 && a.yup && clo == 0) {
        const long m = tile * 16 + r16;
        if (m < M) {
#pragma unroll
          for (int c = 0; c < CH; ++c) st4(a.yup + m * CIN + 16 * c + 4 * kg, av[c]);
        }
      }
    }
    float* pb = part + (it & 1) * PB;
#pragma unroll
    for (int t = 0; t < NCT; ++t)
      if (t >= clo && t < chi)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) pb[(g * 16 + 4 * kg + rr) * LDC + t * 16 + r16] = acc[t][rr];
    if (more) load_x(nxt, av);  // next tile's gathers in flight during the combine
    __syncthreads();
    const f32x4* pb4 = reinterpret_cast<const f32x4*>(pb);
    const int lg = __builtin_ctz((chi - clo) * 4), N4 = 16 << lg;  // (column tiles: a power of two)
    for (int q = threadIdx.x; q < N4; q += 576) {
      const int row = q >> lg, c4 = clo * 4 + (q & ((1 << lg) - 1));
      const long m = tile * 16 + row;
      if (m >= M) continue;
      f32x4 v = pb4[row * (LDC / 4) + c4];
#pragma unroll
      for (int gg = 1; gg < 9; ++gg) v += pb4[(gg * 16 + row) * (LDC / 4) + c4];
      if (a.bias) v += ld4(a.bias + 4 * c4);
      if (a.elu) {
        v.x = elu_f(v.x);
        v.y = elu_f(v.y);
        v.z = elu_f(v.z);
        v.w = elu_f(v.w);
      }
      long yo = m;
      if (a.xvm != a.yvm) {
        int bo, ro;
        split_row(m, a.xvm, a.batch, a.rows, bo, ro);
        yo = row_of(make_lay(a.yvm, a.batch, a.rows), bo, ro);
      }
      st4(a.y + yo * COUT + 4 * c4, v);
    }
    cur = nxt;
#ifdef CFSD_LAT_STAMPS
    if (it == 0) PT_T(pt4)
#endif
  }
#ifdef CFSD_LAT_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 2048) {
    unsigned long long* o = g_pt_stamps + 6 * blockIdx.x;
    o[0] = pt0; o[1] = pt1; o[2] = pt2; o[3] = pt3; o[4] = pt4; o[5] = wall_clock64();
  }
#endif
}

// Backward data, same geometry: a workgroup owns RT 16-row tiles of SOURCE
// rows u (dx rows) x all CIN columns, wave g the slots of its group.  For slot
// s the A operand is T_s[u, :] = sum_{r in inv(u,s)} dpre[r, :] (the inverse
// spiral's head rows -- absent rows are out-of-range buffer loads that read 0
// -- summed (r0 + r1) + r2, then r3 and the rare CSR tail: conv_dx_lat's
// order), B = W_s^T (4 strided dwords per 4-chunk of o, kept in VGPRs over the
// tiles); partials combined in LDS in group order, then ELU' and the store.
constexpr int kInvHead = CFSD_INV_HEAD;
constexpr int kAbsentRow = 0x7ffff000;
__device__ __forceinline__ f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <int CIN, int NSG, int RT>
__host__ __device__ constexpr int dx_ks_lds_f4() { return NSG * RT * 16 * (CIN + 4) / 4; }
template <int CIN, int COUT, int NSG, int RT>
__device__ __forceinline__ void conv_dx_ks_body(int vb, int vnb, const DxKsArgs& a, f32x4* part4) {
  constexpr int CHO = COUT / 16, NCT = CIN / 16, K = kSeq * CIN, SPW = kSeq / NSG;
  constexpr int LDC = CIN + 4, RB = COUT * (int)sizeof(float);
  static_assert(kSeq % NSG == 0, "slot groups");
  float* part = reinterpret_cast<float*>(part4);
  const int lane = threadIdx.x & 63, r16 = lane & 15, kg = lane >> 4;
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long rt0 = (long)xcd_block_of(vb, vnb) * RT;
  const long M = a.total_rows;  // batch * vsrc
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dpre), 0,
                                                      (int)((long)a.batch * a.rows * RB), 0x00020000);
  int base[RT];
  int4 hd[RT][SPW];
  int uq[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    long m = (rt0 + rt) * 16 + r16;
    if (m >= M) m = M - 1;
    int b, u;
    divmod32(m, a.vsrc, b, u);
    uq[rt] = u;
    base[rt] = (b * a.rows * COUT + 4 * kg) * (int)sizeof(float);
#pragma unroll
    for (int j = 0; j < SPW; ++j) hd[rt][j] = a.inv_head[(long)u * kSeq + g * SPW + j];
  }
  f32x4 bw[SPW][CHO][NCT];
#pragma unroll
  for (int j = 0; j < SPW; ++j)
#pragma unroll
    for (int ch = 0; ch < CHO; ++ch)
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const float* q = a.w + (long)(16 * ch + 4 * kg) * K + (g * SPW + j) * CIN + 16 * t + r16;
        bw[j][ch][t] = f32x4{q[0], q[K], q[2 * K], q[3 * K]};
      }
  f32x4 av[RT][SPW][CHO];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
      const int hr[4] = {hd[rt][j].x, hd[rt][j].y, hd[rt][j].z, hd[rt][j].w};
      f32x4 r[4][CHO];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int ch = 0; ch < CHO; ++ch)
          r[e][ch] = buf_ld4(rsrc, hr[e] >= 0 ? base[rt] + hr[e] * RB + 64 * ch : kAbsentRow);
#pragma unroll
      for (int ch = 0; ch < CHO; ++ch) av[rt][j][ch] = ((r[0][ch] + r[1][ch]) + r[2][ch]) + r[3][ch];
    }
  // list rows past the head (0.03 % of keys at level 0): exec branch, list order
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < SPW; ++j) {
      if (hd[rt][j].w >= 0) {
        const long key = (long)uq[rt] * kSeq + g * SPW + j;
        for (int e = a.inv_ptr[key] + kInvHead; e < a.inv_ptr[key + 1]; ++e) {
#pragma unroll
          for (int ch = 0; ch < CHO; ++ch) av[rt][j][ch] += buf_ld4(rsrc, base[rt] + a.inv_row[e] * RB + 64 * ch);
        }
      }
    }
  f32x4 acc[RT][NCT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NCT; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#define KS_MF(Q)                                        \
  _Pragma("unroll") for (int rt = 0; rt < RT; ++rt)     \
  _Pragma("unroll") for (int t = 0; t < NCT; ++t) acc[rt][t] = mfma16(av[rt][j][ch].Q, bw[j][ch][t].Q, acc[rt][t]);
#pragma unroll
  for (int j = 0; j < SPW; ++j)
#pragma unroll
    for (int ch = 0; ch < CHO; ++ch) {
      KS_MF(x) KS_MF(y) KS_MF(z) KS_MF(w)
    }
#undef KS_MF
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int t = 0; t < NCT; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        part[((g * RT + rt) * 16 + 4 * kg + rr) * LDC + t * 16 + r16] = acc[rt][t][rr];
  __syncthreads();
  constexpr int N4 = RT * 16 * CIN / 4;
  for (int q = threadIdx.x; q < N4; q += 64 * NSG) {
    const int rt = q / (16 * CIN / 4), rem = q % (16 * CIN / 4);
    const int row = rem / (CIN / 4), c4 = rem % (CIN / 4);
    const long m = (rt0 + rt) * 16 + row;
    if (m >= M) continue;
    f32x4 v = part4[((0 * RT + rt) * 16 + row) * (LDC / 4) + c4];
#pragma unroll
    for (int gg = 1; gg < NSG; ++gg) v += part4[((gg * RT + rt) * 16 + row) * (LDC / 4) + c4];
    if (a.elu_y) {
      const f32x4 y = ld4(a.elu_y + m * CIN + 4 * c4);
      v.x *= elu_grad_from_out(y.x);
      v.y *= elu_grad_from_out(y.y);
      v.z *= elu_grad_from_out(y.z);
      v.w *= elu_grad_from_out(y.w);
    }
    st4(a.dx + m * CIN + 4 * c4, v);
  }
}
template <int CIN, int COUT, int NSG, int RT>
__global__ __launch_bounds__(64 * NSG, ks_min_waves(NSG, RT)) void conv_dx_ks(const DxKsArgs a) {
  __shared__ f32x4 part4[dx_ks_lds_f4<CIN, NSG, RT>()];
  conv_dx_ks_body<CIN, COUT, NSG, RT>(blockIdx.x, gridDim.x, a, part4);
}

// The data gradient and the weight-gradient slabs of one coarse conv in ONE
// launch (they are independent and each alone leaves most of the chip idle):
// workgroups alternate between the two halves while both last; the dW half
// is conv_dw_lat_body with NSG waves per workgroup (same slabs, same values).
#ifdef CFSD_LAT_STAMPS
// diagnostic build only (tools/kbench.py KB_KSSTAMPS): per-workgroup role, start, end
__device__ unsigned long long g_ks_stamps[4096 * 3];
extern "C" int cfsd_debug_ks_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ks_stamps), sizeof(g_ks_stamps), 0, hipMemcpyDeviceToHost);
}
#endif
template <int CIN, int COUT, int NSG, int RT>
__global__ __launch_bounds__(64 * NSG, ks_min_waves(NSG, RT)) void conv_bwd_ks_pair(const DxKsArgs a, const DwLatArgs d,
                                                                              int nb_dx) {
#ifdef CFSD_LAT_STAMPS
  const unsigned long long t0 = wall_clock64();
#endif
  // the data-gradient role first: it is the longer one, and the dW
  // workgroups fill the slots its retiring waves free (alternating the
  // roles: D1 27.4 vs 25.8 us, D0 24.2 vs 19.6 us, same box)
  const int bid = (int)blockIdx.x;
  const bool is_dx = bid < nb_dx;
  const int vb = is_dx ? bid : bid - nb_dx;
  // one LDS array for both roles (the dW role's chunk-group sums alias the dx partials)
  __shared__ f32x4 part4[dx_ks_lds_f4<CIN, NSG, RT>()];
  static_assert(dx_ks_lds_f4<CIN, NSG, RT>() * 4 >= lat_red_floats(NSG), "dW chunk-group LDS");
  if (is_dx)
    conv_dx_ks_body<CIN, COUT, NSG, RT>(vb, nb_dx, a, part4);
  else
    conv_dw_lat_body<CIN, COUT, NSG>(vb, d.nb, d.x, d.idx, d.dpre, d.ws, d.ws_db, d.vsrc, d.rows, d.total_rows,
                                     d.rchunk, d.n_chunks, d.batch, d.xvm, d.dpvm, reinterpret_cast<float*>(part4));
#ifdef CFSD_LAT_STAMPS
  __syncthreads();
  if (threadIdx.x == 0 && bid < 4096) {
    g_ks_stamps[3 * bid] = is_dx ? 1 : 2;
    g_ks_stamps[3 * bid + 1] = t0;
    g_ks_stamps[3 * bid + 2] = wall_clock64();
  }
#endif
}

// ------------------------------------------------------------------ host side
// Geometry, measured (kbench under rocprofv3 kernel trace, batch 16; same-box
// A/B of the slot-group / row-tile grids, profiles/r04*):
//  * the ~1k-tile layers (E1, D1: 17k rows) take the persistent form -- E1
//    32 -> 32 at 2 workgroups per CU 11.4 us (slot-group grids 11.3-13.8 us,
//    conv_fwd_lat 16.6 us), D1 64 -> 32 at 1 per CU 15.5 us (slot-group grids
//    18.5-22 us, conv_fwd_mfma + combine 22.2 us);
//  * the <= 267-tile layers (E2, E3, D0) one 9-wave workgroup per tile (E2
//    6.8, E3 6.6 us vs 7.7, 7.4 us); the fused up-sampling Deblock (D0) the
//    persistent form;
//  * the data gradient of the few-tile layers (D0) 9 slot groups x 2 tiles
//    per workgroup, paired with the dW slabs (26 us vs 14.7 + 14.6 us).
bool fwd_ks_enabled(long total_rows, int cin, int cout) {
  return total_rows < kMaxRows && (cin == 32 || cin == 64) && (cout == 32 || cout == 64);
}

// (fused only on the few-tile layers: D0 17.5 us fused vs 4.9 + 13.9 us; on D1
// the three-tap gathers cost more than the launch they save, 24.6 vs 6.4 + 15.5 us)
bool fwd_up_supported(long total_rows, int cin, int cout) {
  return total_rows < kMaxTilesFew * 16 && (cin == 32 || cin == 64) && (cout == 32 || cout == 64);
}

// (the ~1k-tile layers keep conv_bwd_lat_pair: D1 dx + dW 34.9 us paired vs
// 17.2 + 19.6 us on the slot-group dx and a separate dW)
bool dx_ks_enabled(long total_src_rows, int cin, int cout) {
  return total_src_rows < kMaxTilesFew * 16 && (cin == 32 || cin == 64) && (cout == 32 || cout == 64);
}

template <int CIN, int COUT, int UP>
static int launch_shape(const FwdKsArgs& a, hipStream_t st) {
  const long n_rt = (a.total_rows + 15) / 16;
  if (UP || n_rt >= kMaxTilesFew) {  // persistent: 1 (64-channel layers) or 2 workgroups per CU
    const long per_cu = (UP || CIN * COUT >= 64 * 32) ? 1 : 2;
    // (one workgroup per tile / balanced grids at 2-3 per CU measured slower:
    // D0 21.5 vs 18.3, D1 20.2 vs 15.9, E1 11.9 vs 11.0 us -- every workgroup
    // pays the weight-slice prologue, profiles/round5d_kprof_pt_grid.txt)
    const long grid = n_rt < 256 * per_cu ? n_rt : 256 * per_cu;
    hipLaunchKernelGGL((conv_fwd_pt<CIN, COUT, UP>), dim3((unsigned)grid), dim3(576), 0, st, a);
    return launch_status("spiral_conv_fwd_pt");
  }
  if constexpr (!UP) {
    hipLaunchKernelGGL((conv_fwd_ks<CIN, COUT, 9, 1, 0>), dim3((unsigned)n_rt), dim3(576), 0, st, a);
    return launch_status("spiral_conv_fwd_ks");
  }
  return CFSD_OK;
}

int launch_fwd_ks(const FwdKsArgs& a, int cin, int cout, hipStream_t st) {
  if (a.total_rows <= 0 || a.total_rows >= kMaxRows) return set_error(CFSD_EINVAL, "spiral_conv_fwd_ks: rows");
  const bool up = a.up_col != nullptr;
  if (up && a.xvm) return set_error(CFSD_EINVAL, "spiral_conv_fwd_ks: fused up-sampling needs batch-major input");
#define SHAPE(CI_, CO_)                                                         \
  if (cin == CI_ && cout == CO_) return up ? launch_shape<CI_, CO_, 1>(a, st) : launch_shape<CI_, CO_, 0>(a, st);
  SHAPE(32, 32) SHAPE(32, 64) SHAPE(64, 32) SHAPE(64, 64)
#undef SHAPE
  return set_error(CFSD_EINVAL, "spiral_conv_fwd_ks: unsupported channels %d -> %d", cin, cout);
}

int launch_bwd_ks_pair(const DxKsArgs& a, const DwLatArgs& d0, long dw_tasks, int cin, int cout, hipStream_t st) {
  if (a.total_rows <= 0 || a.total_rows >= kMaxTilesFew * 16)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_ks_pair: rows");
  const long n_rt = (a.total_rows + 15) / 16;
  const int nb_dx = (int)((n_rt + 1) / 2);
  DwLatArgs d = d0;
  d.nb = (int)((dw_tasks + 7) / 8);  // waves 0-7 of each 9-wave workgroup (whole chunk groups)
#define SHAPE(CI_, CO_)                                                                                   \
  if (cin == CI_ && cout == CO_) {                                                                        \
    hipLaunchKernelGGL((conv_bwd_ks_pair<CI_, CO_, 9, 2>), dim3((unsigned)(nb_dx + d.nb)), dim3(576), 0, st, a, \
                       d, nb_dx);                                                                         \
    return launch_status("spiral_conv_bwd_ks_pair");                                                      \
  }
  SHAPE(32, 32) SHAPE(32, 64) SHAPE(64, 32) SHAPE(64, 64)
#undef SHAPE
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_ks_pair: unsupported channels %d -> %d", cin, cout);
}

int launch_dx_ks(const DxKsArgs& a, int cin, int cout, hipStream_t st) {
  if (a.total_rows <= 0 || a.total_rows >= kMaxTilesFew * 16)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_ks: rows");
  const long n_rt = (a.total_rows + 15) / 16;
#define SHAPE(CI_, CO_)                                                                                          \
  if (cin == CI_ && cout == CO_) {                                                                               \
    hipLaunchKernelGGL((conv_dx_ks<CI_, CO_, 9, 2>), dim3((unsigned)((n_rt + 1) / 2)), dim3(576), 0, st, a);    \
    return launch_status("spiral_conv_bwd_data_ks");                                                             \
  }
  SHAPE(32, 32) SHAPE(32, 64) SHAPE(64, 32) SHAPE(64, 64)
#undef SHAPE
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_ks: unsupported channels %d -> %d", cin, cout);
}

}  // namespace coarse
}  // namespace cfsd
