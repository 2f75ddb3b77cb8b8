// The fp32 vertex-major flat-list data gradient as a device body (shared by
// the launches of spiral_conv_vm32.hip and the bf16 step's Enblock pair in
// spiral_conv_vm16.hip).  See spiral_conv_vm32.hip for the layout notes.
#pragma once
#include "cfsd_common.h"

namespace cfsd {
namespace vm32 {

namespace {
constexpr int kS = 9;
constexpr int kAbsent = 0x7ffff000;  // out-of-range buffer offset: reads 0, no memory access

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// LDS written by a wave and read back by other lanes of the same wave
__device__ __forceinline__ void wave_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}
}  // namespace

// ------------------------------------------------------------------ data gradient
// Wave = tile (source vertex u, mesh group mg).  Entry e of u's flat list is
// p_e = 9 r_e + s_e: B = dpre[r_e]^T (lane (j, g): mesh j, channels
// 16c + 4g .. +3, one 16-B buffer load per c with the row offset in an
// SGPR), A = W_{s_e}^T from LDS; entries e + 1, e + 2 are in flight while e
// runs its 16 MFMAs.  The list is padded to FW with -1 (ascending entries
// first), so the walk stops at the first -1 (uniform branch) and the
// prefetches past the end are out-of-range loads (no memory access).  The
// next tile's list is loaded at the start of this one.
constexpr int kVm32DxPd = 2;  // list entries in flight ahead of the one being multiplied
constexpr int kVm32DxOcc = 1;
// TY: storage of dx and elu_y (fp32, or bf16 for the bf16 step's E1: the
// fp32 sum rounded once)
template <int CIN, int COUT, int FW, typename TY = float, int WPB = 8>
__device__ __forceinline__ void dx_flat_body(const float* __restrict__ dpre, const int4* __restrict__ flat,
                                             const float* __restrict__ w, const TY* __restrict__ elu_y,
                                             TY* __restrict__ dx, int vsrc, int rows, int batch, int dpvm,
                                             int dxvm, int vb, int nvb, float* lwt) {
  constexpr int K = kS * CIN, OP = COUT + 8, NT = CIN / 16, OC = COUT / 16, FQ = FW / 4;
  constexpr int RB = COUT * 4;  // dpre row bytes
  // lwt[(s*CIN + ci)*OP + o] = W[o][s*CIN + ci]  (16-B reads conflict-free: OP = 40 / 72)
  coop_copy<12, float>(
      COUT * K, [&](int e) { return w[e]; }, [&](int e, float v) { lwt[(e % K) * OP + e / K] = v; });
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int G16 = batch >> 4;
  const long n_tiles = (long)vsrc * G16;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dpre), 0,
                                                    (int)((long)batch * rows * RB), 0x00020000);
  // dpre vertex-major (dpvm: a row's 16-mesh block contiguous) or batch-major
  // (the Enblock E1: dpre at the kept rows of the coarser, batch-major level):
  // mesh part per lane, row part as the entry's SGPR offset either way
  const int rstride = dpvm ? batch * RB : RB;  // bytes between two rows of one mesh
  const int mstride = dpvm ? RB : rows * RB;   // bytes between two meshes of one row
  const TileSweep sw = xcd_sweep_v(n_tiles, WPB, wave, true, vb, nvb);

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
    const int voff = (mg * 16 + j) * mstride + 16 * g;
    auto issue = [&](int e, f32x4(&d)[OC]) {
      const int so = pe[e] >= 0 ? (pe[e] / kS) * rstride : kAbsent;
#pragma unroll
      for (int c = 0; c < OC; ++c) d[c] = bload4(rs, voff + 64 * c, so);
    };
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    constexpr int PD = kVm32DxPd, NB = PD + 1;
    f32x4 buf[NB][OC];
#pragma unroll
    for (int e = 0; e < PD; ++e) issue(e, buf[e]);
#pragma unroll
    for (int e = 0; e < FW; ++e) {
      if (e + PD < FW) issue(e + PD, buf[(e + PD) % NB]);
      if (pe[e] < 0) break;  // uniform: the rest of the list is padding
      const int s = pe[e] % kS;
      const float* wr = lwt + (s * CIN + j) * OP + 4 * g;
      const f32x4(&cur)[OC] = buf[e % NB];
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
    // dx / elu_y row of (mesh, u): vertex-major, or batch-major (E2, E3)
    const long row = dxvm ? (long)u * batch + mg * 16 + j : (long)(mg * 16 + j) * vsrc + u;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 v = acc[t];
      if (elu_y) {
        const f32x4 ey = ld4f(elu_y + row * CIN + 16 * t + 4 * g);
        v.x *= elu_grad_from_out(ey.x);
        v.y *= elu_grad_from_out(ey.y);
        v.z *= elu_grad_from_out(ey.z);
        v.w *= elu_grad_from_out(ey.w);
      }
      st4f(dx + row * CIN + 16 * t + 4 * g, v);
    }
#pragma unroll
    for (int e = 0; e < FW; ++e) pe[e] = pn[e];
  }
}
}  // namespace vm32
}  // namespace cfsd
