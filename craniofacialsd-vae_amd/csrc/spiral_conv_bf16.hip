// SpiralConv forward / backward on bf16 MFMA (v_mfma_f32_16x16x32_bf16),
// gfx950.  The bf16 path of configs C3/C5 (BASELINE.json): bf16 activations
// and weights (the fp32 master parameters' shadow), fp32 accumulation.
//
// Reference: SpiralConv.forward (model.py:27-41) and its autograd
// (index_select backward = index_add_, addmm backward).  Same algorithm as the
// fp32 kernels of spiral_conv.hip (fused gather + contraction, deterministic
// inverse-spiral transpose, slab-reduced weight gradient), re-tiled for the
// bf16 MFMA: a 16-row tile x 32 input channels is ONE A fragment, and one
// 16-B load per lane gathers 16 neighbour rows x 64 contiguous bytes (a whole
// bf16 32-channel row) per spiral slot.
#include "conv_bf16.h"

namespace cfsd {
namespace bf {

constexpr int kS = 9;
constexpr int kAbsent = 0x7ffff000;  // out-of-range buffer offset: reads 0, no traffic

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ------------------------------------------------------------------ forward
// Wave = 16-row tile (rows of the flattened (b, r) space), all COUT columns,
// all 9 slots: lane (i = l&15, g = l>>4) gathers row i's channels
// [kc*32 + 8g, +8) of every neighbour (9 x CIN/32 16-B loads, all issued
// before the first MFMA), B = W[n][s*CIN + kc*32 + 8g ..] straight from the
// LDS copy of W (row-major, padded 16 B per row).  Persistent XCD-aware sweep.
template <int CIN, int COUT, int ACT, typename TY>
__global__ __launch_bounds__(256) void conv_fwd_b16(const bf16_t* __restrict__ x,
                                                    const int* __restrict__ idx,
                                                    const bf16_t* __restrict__ w,
                                                    const float* __restrict__ bias,
                                                    TY* __restrict__ y, int vsrc, int rows,
                                                    long total_rows, int batch, int xvm, int yvm) {
  constexpr int K = kS * CIN, KP = K + 8, KC = CIN / 32, NT = COUT / 16;
  extern __shared__ bf16_t lw[];  // [COUT][KP]
  coop_copy<8, u32x4>(
      COUT * K / 8,
      [&](int e) { return *reinterpret_cast<const u32x4*>(&w[(e / (K / 8)) * K + 8 * (e % (K / 8))]); },
      [&](int e, u32x4 v) { *reinterpret_cast<u32x4*>(&lw[(e / (K / 8)) * KP + 8 * (e % (K / 8))]) = v; });
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  float bn[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bn[t] = bias ? bias[t * 16 + i] : 0.f;
  // rows are visited in x's layout (vertex-major: a 16-row tile is one
  // vertex of 16 meshes, each neighbour gather one contiguous 1-KiB wave load)
  const Lay lx = make_lay(xvm, batch, vsrc), ly = make_lay(yvm, batch, rows);
  const long n_tiles = (total_rows + 15) / 16;
  const TileSweep sw = xcd_sweep(n_tiles, 4, wave, n_tiles < 2 * kContigTiles);
  for (long tile = sw.begin; tile < sw.end; tile += sw.step) {
    long m = tile * 16 + i;
    if (m >= total_rows) m = total_rows - 1;  // clamped loads, masked stores
    int b, r;
    split_row(m, xvm, batch, rows, b, r);
    const bf16_t* xb = x + (long)b * lx.bs * CIN + 8 * g;
    const int* ir = idx + r * kS;
    int src[kS];
#pragma unroll
    for (int s = 0; s < kS; ++s) src[s] = ir[s];
    u32x4 a[kS][KC];
#pragma unroll
    for (int s = 0; s < kS; ++s)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) a[s][kc] = ld8bf(xb + (long)src[s] * lx.vs * CIN + 32 * kc);
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kS; ++s)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const u32x4 bw = *reinterpret_cast<const u32x4*>(&lw[(t * 16 + i) * KP + s * CIN + 32 * kc + 8 * g]);
          acc[t] = mfma_bf16(a[s][kc], bw, acc[t]);
        }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const long mo = tile * 16 + 4 * g + rr;
      if (mo < total_rows) {
        long yo = mo;
        if (xvm != yvm) {
          int bo, ro;
          split_row(mo, xvm, batch, rows, bo, ro);
          yo = row_of(ly, bo, ro);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          float v = acc[t][rr] + bn[t];
          if (ACT == CFSD_ACT_ELU) v = elu_f(v);
          stf(&y[yo * COUT + t * 16 + i], v);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ backward data
// dx rows are source vertices u.  For slot s, A[u][o] = sum of dpre[r][o]
// over the inverse-spiral list (u, s) (head rows 0-2 as unconditional buffer
// loads -- absent rows read 0 with no memory access --, row 3 and the rare
// CSR tail through a branch), summed in fp32 in list order and rounded to
// bf16 once; B = W_s^T from an LDS image [s][c][o] (padded 16 B per row).
template <typename TD>
__device__ __forceinline__ void load_row8(__amdgpu_buffer_rsrc_t rs, int off, float (&v)[8]) {
  if constexpr (sizeof(TD) == 2) {
    const u32x4 q = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(q[j] << 16);
      v[2 * j + 1] = __uint_as_float(q[j] & 0xffff0000u);
    }
  } else {
    const f32x4 p = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    const f32x4 q = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
    v[0] = p.x; v[1] = p.y; v[2] = p.z; v[3] = p.w;
    v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
  }
}

template <int CIN, int COUT, typename TD>
__global__ __launch_bounds__(256) void conv_dx_b16(const TD* __restrict__ dpre,
                                                   const int* __restrict__ inv_ptr,
                                                   const int* __restrict__ inv_row,
                                                   const int4* __restrict__ inv_head,
                                                   const bf16_t* __restrict__ w,
                                                   const bf16_t* __restrict__ elu_y,
                                                   bf16_t* __restrict__ dx, int vsrc, int rows,
                                                   long total_rows, int batch, int dpvm, int dxvm) {
  constexpr int K = kS * CIN, OP = COUT + 8, OC = COUT / 32, NT = CIN / 16;
  constexpr int RB = COUT * (int)sizeof(TD);  // dpre row bytes
  extern __shared__ bf16_t lwt[];             // [kS*CIN][OP]: lwt[k*OP + o] = w[o*K + k]
  coop_copy<12, bf16_t>(
      COUT * K, [&](int e) { return w[e]; }, [&](int e, bf16_t v) { lwt[(e % K) * OP + e / K] = v; });
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, g = lane >> 4;
  const int nbytes = (int)(total_rows / vsrc * rows * RB);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<TD*>(dpre), 0, nbytes, 0x00020000);
  const Lay ld = make_lay(dpvm, batch, rows);
  const int rstride = ld.vs * RB;  // bytes between consecutive vertices of one mesh's dpre
  const long n_tiles = (total_rows + 15) / 16;
  const TileSweep sw = xcd_sweep(n_tiles, 4, wave, n_tiles < 2 * kContigTiles);
  for (long tile = sw.begin; tile < sw.end; tile += sw.step) {
    long m = tile * 16 + i;
    if (m >= total_rows) m = total_rows - 1;
    int b, u;
    split_row(m, dxvm, batch, vsrc, b, u);  // dx (and elu_y) rows in dx's layout
    const int base = b * ld.bs * RB + 8 * g * (int)sizeof(TD);
    const int4* pu = inv_head + u * kS;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s0 = 0; s0 < kS; s0 += 3) {
      int4 hd[3];
      float v[3][OC][3][8];
#pragma unroll
      for (int q = 0; q < 3; ++q) hd[q] = pu[s0 + q];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int hr[3] = {hd[q].x, hd[q].y, hd[q].z};
#pragma unroll
        for (int kc = 0; kc < OC; ++kc)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            load_row8<TD>(rs, hr[j] >= 0 ? base + hr[j] * rstride + 32 * kc * (int)sizeof(TD) : kAbsent,
                          v[q][kc][j]);
      }
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int s = s0 + q;
#pragma unroll
        for (int kc = 0; kc < OC; ++kc) {
          float a8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) a8[e] = (v[q][kc][0][e] + v[q][kc][1][e]) + v[q][kc][2][e];
          if (hd[q].w >= 0) {  // 0.3 % of keys: list rows 3..
            const TD* db_ = dpre + (long)b * ld.bs * COUT + 32 * kc + 8 * g;
            for (int e = 0; e < 8; ++e) a8[e] += ldf(&db_[(long)hd[q].w * ld.vs * COUT + e]);
            const long key = (long)u * kS + s;
            for (int p = inv_ptr[key] + CFSD_INV_HEAD; p < inv_ptr[key + 1]; ++p) {
              const TD* rp = db_ + (long)inv_row[p] * ld.vs * COUT;
              for (int e = 0; e < 8; ++e) a8[e] += ldf(&rp[e]);
            }
          }
          const u32x4 af = {pack_bf2(a8[0], a8[1]), pack_bf2(a8[2], a8[3]), pack_bf2(a8[4], a8[5]),
                            pack_bf2(a8[6], a8[7])};
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const u32x4 bw = *reinterpret_cast<const u32x4*>(&lwt[(s * CIN + t * 16 + i) * OP + 32 * kc + 8 * g]);
            acc[t] = mfma_bf16(af, bw, acc[t]);
          }
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const long mo = tile * 16 + 4 * g + rr;
      if (mo < total_rows) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int c = t * 16 + i;
          float val = acc[t][rr];
          if (elu_y) val *= elu_grad_from_out(bf2f(elu_y[mo * CIN + c]));
          dx[mo * CIN + c] = (bf16_t)f2bf(val);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ backward weight
// dW_s[o][c] = sum_rows dpre[row][o] * x[gather(row, s)][c]: K = rows, so both
// operands are columns of row-major tiles -> staged in LDS ([32 rows][COUT]
// dpre, [9][32 rows][CIN] gathered x, bf16) and read as MFMA fragments with
// ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group, delivered
// column-major: two reads = the 8 k-values of a lane).  A workgroup is G
// groups of WG = (COUT/16)(CIN/16) waves; a group sweeps its own 32-row tiles
// (next tile's loads in registers while the current tile's MFMAs run), a wave
// owns one (o-tile, c-tile) for all 9 slots (its A fragment is loaded once
// per tile).  The groups are summed in fixed order in LDS and the workgroup
// writes ONE plain slab [COUT*9*CIN + COUT] (dw_reduce_batch kind 1).
template <int CIN, int COUT>
struct DwB16Cfg {
  static constexpr int OT = COUT / 16, CT = CIN / 16;
  static constexpr int WG = OT * CT;                 // waves per group
  static constexpr int G = 16 / WG > 0 ? 16 / WG : 1;
  static constexpr int TG = WG * 64;                 // threads per group
  static constexpr int THREADS = G * TG;
  static constexpr int XCH = kS * 32 * CIN / 8;      // 16-B chunks of gathered x per tile
  static constexpr int DCH = 32 * COUT / 8;          // 16-B chunks of dpre per tile
  static constexpr int XPT = (XCH + TG - 1) / TG;
  static constexpr int DPT = (DCH + TG - 1) / TG;
  static constexpr int TILE_EL = 32 * COUT + kS * 32 * CIN;  // bf16 elements per group tile
  static constexpr int NEL = COUT * kS * CIN + COUT;
  static constexpr size_t LDS = (size_t)G * TILE_EL * 2 > (size_t)NEL * 4 ? (size_t)G * TILE_EL * 2
                                                                          : (size_t)NEL * 4;
};

__device__ __forceinline__ u32x4 tr_frag(const bf16_t* tile, int ld, int row0, int col0, int lane) {
  const int li = lane & 15, g = lane >> 4, q = li >> 2, p = li & 3;
  const bf16_t* a = tile + (row0 + 8 * g + q) * ld + col0 + 4 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * ld));
  const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
  return (u32x4){l2.x, l2.y, h2.x, h2.y};
}

template <int CIN, int COUT, typename TD>
__global__ __launch_bounds__(1024) void conv_dw_b16(const bf16_t* __restrict__ x,
                                                    const int* __restrict__ idx,
                                                    const TD* __restrict__ dpre,
                                                    float* __restrict__ ws, int vsrc, int rows,
                                                    long total_rows, int batch, int xvm, int dpvm) {
  using C = DwB16Cfg<CIN, COUT>;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(lds_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = wave / C::WG, wg = wave - grp * C::WG, gt = tid - grp * C::TG;
  bf16_t* dp_l = lds + grp * C::TILE_EL;  // [32][COUT]
  bf16_t* xg_l = dp_l + 32 * COUT;        // [kS][32][CIN]
  const int ot = wg / C::CT, ct = wg - ot * C::CT;
  const long n_tiles = (total_rows + 31) / 32;

  f32x4 acc[kS];
#pragma unroll
  for (int s = 0; s < kS; ++s) acc[s] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float db_acc = 0.f;

  // K (rows) is visited in x's layout: a vertex-major x tile is 2 vertices x
  // 16 meshes, its gathered rows two contiguous 1-KiB blocks per slot
  const Lay lx = make_lay(xvm, batch, vsrc), ldp = make_lay(dpvm, batch, rows);
  u32x4 xs[C::XPT], ds[C::DPT];
  auto load_tile = [&](long tile) {
    const long m0 = tile * 32;
#pragma unroll
    for (int e = 0; e < C::XPT; ++e) {
      const int f = gt + e * C::TG;
      if (f < C::XCH) {
        const int c8 = f % (CIN / 8), row = (f / (CIN / 8)) % 32, s = f / (32 * CIN / 8);
        long m = m0 + row;
        if (m >= total_rows) m = total_rows - 1;  // its dpre row is zero
        int b, r;
        split_row(m, xvm, batch, rows, b, r);
        xs[e] = ld8bf(x + ((long)b * lx.bs + (long)idx[r * kS + s] * lx.vs) * CIN + 8 * c8);
      }
    }
#pragma unroll
    for (int e = 0; e < C::DPT; ++e) {
      const int f = gt + e * C::TG;
      if (f < C::DCH) {
        const int row = f / (COUT / 8), c8 = f - row * (COUT / 8);
        const long m = m0 + row;
        long dr = m;
        if (xvm != dpvm && m < total_rows) {
          int b, r;
          split_row(m, xvm, batch, rows, b, r);
          dr = row_of(ldp, b, r);
        }
        ds[e] = m < total_rows ? ld8bf(dpre + dr * COUT + 8 * c8) : (u32x4){0u, 0u, 0u, 0u};
      }
    }
  };

  const TileSweep sw0 = xcd_sweep(n_tiles, C::G, 0), swg = xcd_sweep(n_tiles, C::G, grp);
  long tg = swg.begin;
  if (tg < swg.end) load_tile(tg);
  for (long t0 = sw0.begin; t0 < sw0.end; t0 += sw0.step, tg += swg.step) {
    const bool have = tg < swg.end;  // group-uniform
    if (have) {
#pragma unroll
      for (int e = 0; e < C::XPT; ++e) {
        const int f = gt + e * C::TG;
        if (f < C::XCH) *reinterpret_cast<u32x4*>(&xg_l[8 * f]) = xs[e];
      }
#pragma unroll
      for (int e = 0; e < C::DPT; ++e) {
        const int f = gt + e * C::TG;
        if (f < C::DCH) *reinterpret_cast<u32x4*>(&dp_l[8 * f]) = ds[e];
      }
    }
    __syncthreads();
    if (tg + swg.step < swg.end) load_tile(tg + swg.step);
    if (have) {
      if (gt < COUT) {
#pragma unroll 8
        for (int row = 0; row < 32; ++row) db_acc += bf2f(dp_l[row * COUT + gt]);
      }
      const u32x4 af = tr_frag(dp_l, COUT, 0, ot * 16, lane);
#pragma unroll
      for (int s = 0; s < kS; ++s) {
        const u32x4 bfr = tr_frag(xg_l + s * 32 * CIN, CIN, 0, ct * 16, lane);
        acc[s] = mfma_bf16(af, bfr, acc[s]);
      }
    }
    __syncthreads();
  }
  // groups summed in fixed order in LDS (reused), then one slab per workgroup
  float* red = reinterpret_cast<float*>(lds_raw);
  constexpr int K = kS * CIN;
  const int i = lane & 15, g = lane >> 4;
  for (int q = 0; q < C::G; ++q) {
    if (grp == q) {
#pragma unroll
      for (int s = 0; s < kS; ++s)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int e = (ot * 16 + 4 * g + rr) * K + s * CIN + ct * 16 + i;
          red[e] = (q == 0 ? 0.f : red[e]) + acc[s][rr];
        }
      if (gt < COUT) red[COUT * K + gt] = (q == 0 ? 0.f : red[COUT * K + gt]) + db_acc;
    }
    __syncthreads();
  }
  float* slab = ws + (long)blockIdx.x * C::NEL;
  for (int e = tid; e < C::NEL; e += C::THREADS) slab[e] = red[e];
}

// ------------------------------------------------------------------ launchers
template <typename K>
static int blocks_resident(K kern, int threads, size_t lds) {
  const int r = resident_blocks_of(kern, threads, lds);
  return r > 0 ? r : 1;
}

template <int CIN, int COUT, int ACT, typename TY>
static int fwd_t(const bf16_t* x, const int* idx, const bf16_t* w, const float* bias, TY* y,
                 int vsrc, int rows, long M, int xvm, int yvm, hipStream_t st) {
  constexpr size_t lds = (size_t)COUT * (kS * CIN + 8) * sizeof(bf16_t);
  auto kern = conv_fwd_b16<CIN, COUT, ACT, TY>;
  const long tiles = (M + 15) / 16;
  const unsigned grid = balanced_blocks(tiles, 4, blocks_resident(kern, 256, lds));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, x, idx, w, bias, y, vsrc, rows, M,
                     (int)(M / rows), xvm, yvm);
  return launch_status("spiral_conv_fwd_bf16");
}

int launch_fwd(const bf16_t* x, int xvm, const int* idx, const bf16_t* w, const float* bias, void* y,
               int y_dt, int vsrc, int rows, long M, int cin, int cout, int act, hipStream_t st) {
  const int yvm = (y_dt & CFSD_VM) != 0;
  if (xvm && vm16_ok((int)(M / rows), cin, cout))
    return launch_fwd_vm16(x, idx, w, bias, y, y_dt, vsrc, rows, (int)(M / rows), cin, cout, act, st);
#define F(CI, CO)                                                                                   \
  if (cin == CI && cout == CO) {                                                                    \
    if (CFSD_DT_TYPE(y_dt) == DT_BF16)                                                              \
      return act == CFSD_ACT_ELU                                                                    \
                 ? fwd_t<CI, CO, CFSD_ACT_ELU, bf16_t>(x, idx, w, bias, (bf16_t*)y, vsrc, rows, M, xvm, yvm, st) \
                 : fwd_t<CI, CO, CFSD_ACT_NONE, bf16_t>(x, idx, w, bias, (bf16_t*)y, vsrc, rows, M, xvm, yvm, st); \
    return act == CFSD_ACT_ELU                                                                      \
               ? fwd_t<CI, CO, CFSD_ACT_ELU, float>(x, idx, w, bias, (float*)y, vsrc, rows, M, xvm, yvm, st)  \
               : fwd_t<CI, CO, CFSD_ACT_NONE, float>(x, idx, w, bias, (float*)y, vsrc, rows, M, xvm, yvm, st); \
  }
  F(32, 32) F(32, 64) F(64, 32) F(64, 64)
#undef F
  return set_error(CFSD_EINVAL, "spiral_conv_fwd (bf16): unsupported channels %d -> %d", cin, cout);
}

template <int CIN, int COUT, typename TD>
static int dx_t(const TD* dpre, const int* inv_ptr, const int* inv_row, const int* inv_head,
                const bf16_t* w, const bf16_t* elu_y, bf16_t* dx, int vsrc, int rows, long M,
                int dpvm, int dxvm, hipStream_t st) {
  constexpr size_t lds = (size_t)kS * CIN * (COUT + 8) * sizeof(bf16_t);
  auto kern = conv_dx_b16<CIN, COUT, TD>;
  const long tiles = (M + 15) / 16;
  const unsigned grid = balanced_blocks(tiles, 4, blocks_resident(kern, 256, lds));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, dpre, inv_ptr, inv_row,
                     (const int4*)inv_head, w, elu_y, dx, vsrc, rows, M, (int)(M / vsrc), dpvm, dxvm);
  return launch_status("spiral_conv_bwd_data_bf16");
}

int launch_dx(const void* dpre, int dpre_dt, const int* inv_ptr, const int* inv_row,
              const int* inv_head, const bf16_t* w, const bf16_t* elu_y, bf16_t* dx, int dxvm, int vsrc,
              int rows, long M, int cin, int cout, hipStream_t st) {
  const int dpvm = (dpre_dt & CFSD_VM) != 0;
  if (dxvm && dpvm && vm16_ok((int)(M / vsrc), cin, cout))
    return launch_dx_vm16(dpre, dpre_dt, inv_ptr, inv_row, inv_head, w, elu_y, dx, vsrc, rows, (int)(M / vsrc),
                          cin, cout, st);
#define D(CI, CO)                                                                                 \
  if (cin == CI && cout == CO)                                                                    \
    return CFSD_DT_TYPE(dpre_dt) == DT_BF16                                                       \
               ? dx_t<CI, CO, bf16_t>((const bf16_t*)dpre, inv_ptr, inv_row, inv_head, w, elu_y,  \
                                      dx, vsrc, rows, M, dpvm, dxvm, st)                          \
               : dx_t<CI, CO, float>((const float*)dpre, inv_ptr, inv_row, inv_head, w, elu_y, dx, \
                                     vsrc, rows, M, dpvm, dxvm, st);
  D(32, 32) D(32, 64) D(64, 32) D(64, 64)
#undef D
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data (bf16): unsupported channels %d -> %d", cin, cout);
}

constexpr int kDw16Upb = 8;
int dw_slabs(int batch, int rows, int cin, int cout) {
  const long tiles = ((long)batch * rows + 31) / 32;
  const int G = 16 / ((cout / 16) * (cin / 16)) > 0 ? 16 / ((cout / 16) * (cin / 16)) : 1;
  // >= ~4 tiles per group (conv_dw_b16); conv_dw_vm16 (cin = cout = 32):
  // >= kDw16Upb 16-row units per workgroup
  long gx = (kDw16Upb > 0 && cin == 32 && cout == 32) ? (2 * tiles + kDw16Upb - 1) / kDw16Upb
                                                           : (tiles + 4 * G - 1) / (4 * G);
  if (gx > 256) gx = 256;                   // one workgroup per CU: bounded slab traffic
  return (int)(gx < 1 ? 1 : gx);
}

template <int CIN, int COUT, typename TD>
static int dw_t(const bf16_t* x, const int* idx, const TD* dpre, float* ws, int vsrc, int rows,
                long M, int xvm, int dpvm, hipStream_t st) {
  using C = DwB16Cfg<CIN, COUT>;
  const int gx = dw_slabs((int)(M / rows), rows, CIN, COUT);
  hipLaunchKernelGGL((conv_dw_b16<CIN, COUT, TD>), dim3(gx), dim3(C::THREADS), C::LDS, st, x, idx,
                     dpre, ws, vsrc, rows, M, (int)(M / rows), xvm, dpvm);
  return launch_status("spiral_conv_bwd_weight_bf16");
}

int launch_dw(const bf16_t* x, int xvm, const int* idx, const void* dpre, int dpre_dt, float* ws, int vsrc,
              int rows, long M, int cin, int cout, hipStream_t st) {
  const int dpvm = (dpre_dt & CFSD_VM) != 0;
  const int batch = (int)(M / rows);
  if (dw_vm16_ok(batch, cin, cout, xvm, dpvm, CFSD_DT_TYPE(dpre_dt) == DT_BF16))
    return launch_dw_vm16(x, idx, dpre, CFSD_DT_TYPE(dpre_dt) == DT_BF16, ws, dw_slabs(batch, rows, cin, cout), vsrc,
                          rows, batch, st);
#define W(CI, CO)                                                                                 \
  if (cin == CI && cout == CO)                                                                    \
    return CFSD_DT_TYPE(dpre_dt) == DT_BF16                                                       \
               ? dw_t<CI, CO, bf16_t>(x, idx, (const bf16_t*)dpre, ws, vsrc, rows, M, xvm, dpvm, st) \
               : dw_t<CI, CO, float>(x, idx, (const float*)dpre, ws, vsrc, rows, M, xvm, dpvm, st);
  W(32, 32) W(32, 64) W(64, 32) W(64, 64)
#undef W
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight (bf16): unsupported channels %d -> %d", cin, cout);
}

}  // namespace bf
}  // namespace cfsd
