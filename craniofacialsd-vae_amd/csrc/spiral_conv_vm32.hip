// SpiralConv forward and data gradient on fp32 MFMA for VERTEX-MAJOR operands
// (CFSD_VM) with a batch that is a multiple of 16: the fp32 step's level-0/1
// layers (the reference's arithmetic, config C2: 16 meshes per GPU).
//
// Reference: SpiralConv.forward (model.py:27-41) and the autograd of its
// index_select / Linear (model.py:34, 40).
//
// Vertex-major storage puts the 16 mesh rows of one vertex side by side, so a
// 16-row MFMA tile is ONE vertex x 16 meshes: the spiral indices are
// wave-uniform (scalar loads, scalar buffer offsets) and every neighbour
// gather reads one contiguous 2-KiB block (16 meshes x 32 fp32 channels).
// The MFMA runs transposed, D^T[channel][mesh] = W . X^T, so a lane's four
// accumulators are four CONSECUTIVE output channels of one mesh: the
// epilogue stores 16-B vectors instead of scalars.
//
// Forward: the same products in the same K order per output as the
// batch-major conv_fwd_mfma (spiral_conv.hip) -- x*w == w*x and the 16x16x4
// MFMA chain runs over k in the same order in either orientation -- so the
// two layouts give bit-identical outputs (GPU-tested).
//
// Data gradient: per source vertex u the FLAT inverse list (the spiral
// positions p = 9r + s with idx[r][s] == u, ascending p: the order in which
// IndexSelectBackward's index_add_ visits them, model.py:34) is walked once,
// one 2-KiB dpre block and 16 MFMAs per entry (9 entries per vertex on
// average).  The batch-major kernel instead sums each slot's list rows
// (three unconditional head loads per slot, 27 per vertex) before its MFMAs.
#include "conv_vm32.h"

namespace cfsd {
namespace vm32 {

namespace {
constexpr int kS = 9;
constexpr int kAbsent = 0x7ffff000;  // out-of-range buffer offset: reads 0, no memory access

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}
}  // namespace

// ------------------------------------------------------------------ forward
// Wave = tile of UPT units (vertex r, mesh group mg of 16) x all COUT
// columns.  Lane (j, g): mesh j, channel chunks g, g + 4 (16 B each) of every
// neighbour = the B operand X^T[k][mesh]; A = W rows from LDS (the batch-major
// kernel's B fragment, unchanged).  Slot s + PD's gathers are in flight while
// slot s runs its MFMAs.  y vertex-major (yvm) or batch-major (the Enblock
// evaluated at the kept rows writes the coarser, batch-major level).
#ifndef CFSD_VM32_FWD_OCC
#define CFSD_VM32_FWD_OCC 4  // waves per SIMD (VGPR budget 128)
#endif
template <int CIN, int COUT, int ACT, int UPT, int PD>
__global__ __launch_bounds__(256, CFSD_VM32_FWD_OCC) void conv_fwd_vm32(const float* __restrict__ x,
                                                     const int* __restrict__ idx,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ bias,
                                                     float* __restrict__ y, int vsrc, int rows,
                                                     int batch, int yvm) {
  constexpr int CH = CIN / 16, NCT = COUT / 16, K = kS * CIN, KP = K + 8, NB = PD + 1;
  extern __shared__ float lds_w[];  // [COUT][KP]
  coop_copy<8, f32x4>(
      COUT * (K / 4), [&](int e) { return ld4(&w[(long)(e / (K / 4)) * K + 4 * (e % (K / 4))]); },
      [&](int e, f32x4 v) { st4(&lds_w[(e / (K / 4)) * KP + 4 * (e % (K / 4))], v); });
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  float bn[NCT][4];
#pragma unroll
  for (int t = 0; t < NCT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) bn[t][rr] = bias ? bias[16 * t + 4 * g + rr] : 0.f;
  const int G16 = batch >> 4;
  const long n_units = (long)rows * G16;
  const long n_tiles = (n_units + UPT - 1) / UPT;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0,
                                                    (int)((long)vsrc * batch * CIN * 4), 0x00020000);
  const int vstride = batch * CIN * 4;  // bytes between two vertices' blocks
  const TileSweep sw = xcd_sweep(n_tiles, 4, wave, n_tiles < kContigTiles);
  for (long tile = sw.begin; tile < sw.end; tile += sw.step) {
    // compiler barrier: keeps the W fragments as per-MFMA-group LDS reads
    // (hipcc otherwise hoists the whole W slice out of the tile loop and spills)
    asm volatile("" ::: "memory");
    int vr[UPT], mgr[UPT], voff[UPT], soff[UPT][kS];
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      long un = tile * UPT + u;
      if (un >= n_units) un = n_units - 1;  // clamp loads, stores are skipped
      const int unit = uni((int)un);
      vr[u] = unit / G16;
      mgr[u] = unit - vr[u] * G16;
      voff[u] = ((mgr[u] * 16 + j) * CIN + 4 * g) * 4;
#pragma unroll
      for (int s = 0; s < kS; ++s) soff[u][s] = uni(idx[vr[u] * kS + s]) * vstride;
    }
    f32x4 acc[UPT][NCT];
#pragma unroll
    for (int u = 0; u < UPT; ++u)
#pragma unroll
      for (int t = 0; t < NCT; ++t) acc[u][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 buf[NB][UPT][CH];
    auto issue = [&](int s, f32x4(&d)[UPT][CH]) {
#pragma unroll
      for (int u = 0; u < UPT; ++u)
#pragma unroll
        for (int c = 0; c < CH; ++c) d[u][c] = bload4(rs, voff[u] + 64 * c, soff[u][s]);
    };
#pragma unroll
    for (int s = 0; s < PD; ++s) issue(s, buf[s]);
#pragma unroll
    for (int s = 0; s < kS; ++s) {
      if (s + PD < kS) issue(s + PD, buf[(s + PD) % NB]);
      f32x4(&cur)[UPT][CH] = buf[s % NB];
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const f32x4 bw = ld4(&lds_w[(t * 16 + j) * KP + s * CIN + 4 * (g + 4 * c)]);
#pragma unroll
          for (int u = 0; u < UPT; ++u) {
            const f32x4 av = cur[u][c];
            acc[u][t] = mfma16(bw.x, av.x, acc[u][t]);
            acc[u][t] = mfma16(bw.y, av.y, acc[u][t]);
            acc[u][t] = mfma16(bw.z, av.z, acc[u][t]);
            acc[u][t] = mfma16(bw.w, av.w, acc[u][t]);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      if (tile * UPT + u >= n_units) break;  // uniform
      const int mesh = mgr[u] * 16 + j;
      const long row = yvm ? (long)vr[u] * batch + mesh : (long)mesh * rows + vr[u];
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        f32x4 v;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          float z = acc[u][t][rr] + bn[t][rr];
          if (ACT == CFSD_ACT_ELU) z = elu_f(z);
          v[rr] = z;
        }
        st4(y + row * COUT + 16 * t + 4 * g, v);
      }
    }
  }
}

// ------------------------------------------------------------------ data gradient
// Wave = tile (source vertex u, mesh group mg).  Entry e of u's flat list is
// p_e = 9 r_e + s_e: B = dpre[r_e]^T (lane (j, g): mesh j, channels
// 16c + 4g .. +3, one 16-B buffer load per c with the row offset in an
// SGPR), A = W_{s_e}^T from LDS; entries e + 1, e + 2 are in flight while e
// runs its 16 MFMAs.  The list is padded to FW with -1 (ascending entries
// first), so the walk stops at the first -1 (uniform branch) and the
// prefetches past the end are out-of-range loads (no memory access).  The
// next tile's list is loaded at the start of this one.
template <int CIN, int COUT, int FW>
__global__ __launch_bounds__(512) void conv_dx_flat_vm32(const float* __restrict__ dpre,
                                                         const int4* __restrict__ flat,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ elu_y,
                                                         float* __restrict__ dx, int vsrc, int rows,
                                                         int batch) {
  constexpr int K = kS * CIN, OP = COUT + 8, NT = CIN / 16, OC = COUT / 16, FQ = FW / 4;
  constexpr int RB = COUT * 4;  // dpre row bytes
  // lwt[(s*CIN + ci)*OP + o] = W[o][s*CIN + ci]  (16-B reads conflict-free: OP = 40 / 72)
  extern __shared__ float lwt[];
  coop_copy<12, float>(
      COUT * K, [&](int e) { return w[e]; }, [&](int e, float v) { lwt[(e % K) * OP + e / K] = v; });
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int G16 = batch >> 4;
  const long n_tiles = (long)vsrc * G16;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dpre), 0,
                                                    (int)((long)batch * rows * RB), 0x00020000);
  const int rstride = batch * RB;  // bytes between two rows' blocks
  const TileSweep sw = xcd_sweep(n_tiles, 8, wave, true);

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
    const int voff = (mg * 16 + j) * RB + 16 * g;
    auto issue = [&](int e, f32x4(&d)[OC]) {
      const int so = pe[e] >= 0 ? (pe[e] / kS) * rstride : kAbsent;
#pragma unroll
      for (int c = 0; c < OC; ++c) d[c] = bload4(rs, voff + 64 * c, so);
    };
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 buf[3][OC];
    issue(0, buf[0]);
    issue(1, buf[1]);
#pragma unroll
    for (int e = 0; e < FW; ++e) {
      if (e + 2 < FW) issue(e + 2, buf[(e + 2) % 3]);
      if (pe[e] < 0) break;  // uniform: the rest of the list is padding
      const int s = pe[e] % kS;
      const float* wr = lwt + (s * CIN + j) * OP + 4 * g;
      const f32x4(&cur)[OC] = buf[e % 3];
#pragma unroll
      for (int c = 0; c < OC; ++c) {
        f32x4 a[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) a[t] = ld4(wr + t * 16 * OP + 16 * c);
        const f32x4 bv = cur[c];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16(a[t].x, bv.x, acc[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16(a[t].y, bv.y, acc[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16(a[t].z, bv.z, acc[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma16(a[t].w, bv.w, acc[t]);
      }
    }
    const long row = (long)u * batch + mg * 16 + j;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 v = acc[t];
      if (elu_y) {
        const f32x4 ey = ld4(elu_y + row * CIN + 16 * t + 4 * g);
        v.x *= elu_grad_from_out(ey.x);
        v.y *= elu_grad_from_out(ey.y);
        v.z *= elu_grad_from_out(ey.z);
        v.w *= elu_grad_from_out(ey.w);
      }
      st4(dx + row * CIN + 16 * t + 4 * g, v);
    }
#pragma unroll
    for (int e = 0; e < FW; ++e) pe[e] = pn[e];
  }
}

// ------------------------------------------------------------------ launchers
bool ok(int batch, int cin, int cout) { return batch % 16 == 0 && cin == 32 && (cout == 32 || cout == 64); }

template <typename Kern>
static int resident(Kern k, int threads, size_t lds) {
  const int r = resident_blocks_of(k, threads, lds);
  return r > 0 ? r : 1;
}

template <int CIN, int COUT, int ACT, int UPT, int PD>
static int fwd_t(const float* x, const int* idx, const float* w, const float* bias, float* y, int yvm,
                 int vsrc, int rows, int batch, hipStream_t st) {
  constexpr size_t lds = (size_t)COUT * (kS * CIN + 8) * sizeof(float);
  auto kern = conv_fwd_vm32<CIN, COUT, ACT, UPT, PD>;
  const long tiles = ((long)rows * (batch / 16) + UPT - 1) / UPT;
  const unsigned grid = balanced_blocks(tiles, 4, resident(kern, 256, lds));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, x, idx, w, bias, y, vsrc, rows, batch, yvm);
  return launch_status("spiral_conv_fwd_vm32");
}

// Units (vertex x 16 meshes) below which a wave takes ONE unit with two slots
// in flight (the level-1 row subset of an Enblock: ~1k units), else two units
// (more MFMA work per gathered slot) with one slot in flight.
#ifndef CFSD_VM32_UPT1_UNITS
#define CFSD_VM32_UPT1_UNITS 8192
#endif

template <int COUT, int ACT>
static int fwd_pick(const float* x, const int* idx, const float* w, const float* bias, float* y, int yvm,
                    int vsrc, int rows, int batch, hipStream_t st) {
  if ((long)rows * (batch / 16) < CFSD_VM32_UPT1_UNITS)
    return fwd_t<32, COUT, ACT, 1, 2>(x, idx, w, bias, y, yvm, vsrc, rows, batch, st);
  return fwd_t<32, COUT, ACT, 2, 1>(x, idx, w, bias, y, yvm, vsrc, rows, batch, st);
}

int launch_fwd(const float* x, const int* idx, const float* w, const float* bias, float* y, int yvm, int vsrc,
               int rows, int batch, int cin, int cout, int act, hipStream_t st) {
  if (!ok(batch, cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_fwd (fp32 vertex-major): batch %% 16 == 0 and 32 -> 32/64 only");
  if ((long)vsrc * batch * cin * 4 >= (long)kAbsent || (long)rows * batch >= (1L << 31))
    return set_error(CFSD_EINVAL, "spiral_conv_fwd (fp32 vertex-major): x exceeds 32-bit buffer offsets");
  if (cout == 32)
    return act == CFSD_ACT_ELU ? fwd_pick<32, CFSD_ACT_ELU>(x, idx, w, bias, y, yvm, vsrc, rows, batch, st)
                               : fwd_pick<32, CFSD_ACT_NONE>(x, idx, w, bias, y, yvm, vsrc, rows, batch, st);
  return act == CFSD_ACT_ELU ? fwd_pick<64, CFSD_ACT_ELU>(x, idx, w, bias, y, yvm, vsrc, rows, batch, st)
                             : fwd_pick<64, CFSD_ACT_NONE>(x, idx, w, bias, y, yvm, vsrc, rows, batch, st);
}

template <int CIN, int COUT, int FW>
static int dxf_t(const float* dpre, const int* flat, const float* w, const float* elu_y, float* dx, int vsrc,
                 int rows, int batch, hipStream_t st) {
  constexpr size_t lds = (size_t)kS * CIN * (COUT + 8) * sizeof(float);
  auto kern = conv_dx_flat_vm32<CIN, COUT, FW>;
  const long tiles = (long)vsrc * (batch / 16);
  const unsigned grid = balanced_blocks(tiles, 8, resident(kern, 512, lds));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, dpre, (const int4*)flat, w, elu_y, dx, vsrc, rows,
                     batch);
  return launch_status("spiral_conv_bwd_data_flat_vm32");
}

int launch_dx_flat(const float* dpre, const int* flat, int width, const float* w, const float* elu_y, float* dx,
                   int vsrc, int rows, int batch, int cin, int cout, hipStream_t st) {
  if (!ok(batch, cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (fp32): batch %% 16 == 0 and 32 -> 32/64 only");
  if ((long)batch * rows * cout * 4 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (fp32): dpre exceeds 32-bit buffer offsets");
#define DF(CO, FW_)                                                                                     \
  if (cout == CO && width == FW_) return dxf_t<32, CO, FW_>(dpre, flat, w, elu_y, dx, vsrc, rows, batch, st);
  DF(32, 8) DF(32, 12) DF(32, 16) DF(32, 20) DF(64, 8) DF(64, 12) DF(64, 16) DF(64, 20)
#undef DF
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (fp32): unsupported channels %d -> %d / width %d",
                   cin, cout, width);
}

}  // namespace vm32
}  // namespace cfsd
