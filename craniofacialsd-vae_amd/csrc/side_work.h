// Side work: independent, HBM-light tail work of the backward that rides in
// another launch as extra workgroups (horizontal fusion) instead of running
// in a launch of its own at the end of the step.
//
// What rides: (1) the reduction of a conv's deferred weight-gradient slabs
// into its dw / db (the reference's AddmmBackward dW = G^T.dY, model.py:40,
// summed over the per-workgroup partials), and (2) the Adam step
// (model_manager.py:316, torch.optim.Adam) of parameters whose gradient is
// final and that nothing later in the step reads -- on a single GPU the
// update of a layer can start as soon as its own backward is done.  The host
// launches chosen by the engine are latency-bound (the up-sampling transposes,
// the latent head backward), so most of their CUs idle; the side blocks fill
// them.  The final batched reduce then only sees what no host could take.
//
// Bit-identity with cfsd_dw_reduce_batch(_adam): every element is summed in
// the same order -- 16 partials, partial q over slabs q, q + 16, q + 32, ...
// ascending from 0, then ((p0 + p1) + p2) + ... + p15 -- and updated by the
// same adam_elem with the same step constants.  Here a side block of W waves
// owns 64 consecutive elements; wave w accumulates partials q = w, w + W, ..
// (one element per lane, 16 dword loads in flight), the partials meet in LDS
// and wave 0 adds them in q order, then applies Adam.
#pragma once
#include "cfsd_common.h"

namespace cfsd {

constexpr int kSideItems = 12;
constexpr int kSideRanges = 8;
constexpr int kSideRangeBlock = 1024;  // Adam elements per side block of a range

struct SideItem {
  const float* ws;     // slabs [n_slabs][stride]
  const float* ws_db;  // kind 0: db partials [n_slabs][cout] (else null)
  float* dw;
  float* db;
  int kind;  // 0: conv_dw_mfma / lat / vm32 unit-tiled slabs ([U][32 o][32 c] + db); 1: plain [cout*K + cout]
  int cin, cout, n_slabs, n_el, blk0;
};
struct SideJob {
  SideItem it[kSideItems];
  int n_items;
  long lo[kSideRanges], hi[kSideRanges];  // Adam-only flat ranges [lo, hi)
  int rblk0[kSideRanges + 1];             // first side block of each range (relative to the ranges' start)
  int n_ranges;
  int blk_items;  // side blocks of the reductions (ranges follow)
  int n_blocks;   // all side blocks
  // Adam (adam != 0): applied to every reduced element and every range element
  float* p;
  const float* g;  // flat gradient (items' dw / db point into it)
  float* m;
  float* v;
  bf16_t* shadow;
  const int* step;
  float lr, b1, b2, eps, wd;
  int adam;
};

__device__ __forceinline__ void side_adam_consts(const SideJob& J, float& step_size, float& sqrt_bc2) {
  const int t = *J.step;
  step_size = J.lr / (1.f - powf(J.b1, (float)t));
  sqrt_bc2 = sqrtf(1.f - powf(J.b2, (float)t));
}
__device__ __forceinline__ void side_adam_at(const SideJob& J, long o, float g, float step_size, float sqrt_bc2) {
  float pv = J.p[o], mv = J.m[o], vv = J.v[o];
  adam_elem(pv, g, mv, vv, J.b1, J.b2, J.eps, J.wd, step_size, sqrt_bc2);
  J.p[o] = pv;
  J.m[o] = mv;
  J.v[o] = vv;
  if (J.shadow) stf(J.shadow + o, pv);
}

// Side block `sb` (0 <= sb < J.n_blocks) of a launch whose workgroups have
// NW waves (NW = blockDim.x / 64 in {1, 2, 4, 8, 16}: it divides the 16
// partials).  Every thread of the block must call it (one barrier inside).
// Latency: every load a lane needs for one 256-slab pass is issued before the
// first add (a side block's life is ~one memory round trip per 256 slabs, not
// one per slab), and a range lane's 4 elements load together.
template <int NW>
__device__ __forceinline__ void side_block(const SideJob& J, int sb) {
  static_assert(16 % NW == 0, "waves per side block divide the 16 partials");
  constexpr int nw = NW, rpw = 16 / NW;
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (sb >= J.blk_items) {  // Adam over a final-gradient range
    const int rb = sb - J.blk_items;
    int ri = 0;
    while (ri + 1 < J.n_ranges && rb >= J.rblk0[ri + 1]) ++ri;
    float step_size, sqrt_bc2;
    side_adam_consts(J, step_size, sqrt_bc2);
    const long base = J.lo[ri] + (long)(rb - J.rblk0[ri]) * kSideRangeBlock, hi = J.hi[ri];
    for (int k0 = threadIdx.x; k0 < kSideRangeBlock; k0 += 4 * blockDim.x) {
      float pv[4], g[4], mv[4], vv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        long o = base + k0 + j * blockDim.x;
        if (o >= hi) o = hi - 1;
        pv[j] = J.p[o];
        g[j] = J.g[o];
        mv[j] = J.m[o];
        vv[j] = J.v[o];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long o = base + k0 + j * blockDim.x;
        if (o >= hi) continue;
        adam_elem(pv[j], g[j], mv[j], vv[j], J.b1, J.b2, J.eps, J.wd, step_size, sqrt_bc2);
        J.p[o] = pv[j];
        J.m[o] = mv[j];
        J.v[o] = vv[j];
        if (J.shadow) stf(J.shadow + o, pv[j]);
      }
    }
    return;
  }
  int li = 0;
  while (li + 1 < J.n_items && sb >= J.it[li + 1].blk0) ++li;
  const SideItem& d = J.it[li];
  const int nwd = d.n_el - d.cout;  // kind 0: the dW part of a slab (a multiple of 64: blocks never straddle)
  const int f0 = (sb - d.blk0) * 64;
  const int f = f0 + lane;
  const bool valid = f < d.n_el;
  // the block's 64 elements of slab p are at bp + p * stride + lane (wave-uniform
  // base and stride: buffer loads with the slab offset in an SGPR, so a load
  // costs no address VGPRs; lanes past the item read harmless or 0 words)
  const float* bp;
  int stride, off0;
  if (d.kind == 0 && f0 >= nwd) {
    bp = d.ws_db + (f0 - nwd);
    stride = d.cout;
    off0 = f0 - nwd;
  } else {
    bp = d.ws + f0;
    stride = d.kind == 0 ? nwd : d.n_el;
    off0 = f0;
  }
  const int ns = d.n_slabs;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bp), 0,
                                                    (int)(((long)ns * stride - off0) * 4), 0x00020000);
  const int vo = lane * 4;
  // partials q = wave + nw k (k < 16 / nw): slabs q, q + 16, ... ascending from 0;
  // per 256-slab pass all of this lane's loads are in flight together
  float s[rpw];
#pragma unroll
  for (int k = 0; k < rpw; ++k) s[k] = 0.f;
  for (int p0 = 0; p0 < ns; p0 += 256) {
    float t[rpw][16];
#pragma unroll
    for (int k = 0; k < rpw; ++k) {
      const int q = wave + nw * k;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int p = p0 + q + 16 * j;
        t[k][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                rs, vo, (p < ns ? p : ns - 1) * stride * 4, 0));
      }
    }
#pragma unroll
    for (int k = 0; k < rpw; ++k) {
      const int q = wave + nw * k;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (p0 + q + 16 * j < ns) s[k] += t[k][j];
    }
  }
#pragma unroll
  for (int k = 0; k < rpw; ++k) part[wave + nw * k][lane] = s[k];
  __syncthreads();
  if (wave != 0 || !valid) return;
  float t = part[0][lane];
#pragma unroll
  for (int q = 1; q < 16; ++q) t += part[q][lane];
  float* dst;
  if (f >= nwd) {
    dst = d.db + (f - nwd);
  } else if (d.kind == 1) {
    dst = d.dw + f;
  } else {  // unit-tiled: f = un * 1024 + o32 * 32 + c32
    const int CT = d.cin / 32, OT = d.cout / 32;
    const int un = f >> 10, within = f & 1023;
    const int cc = (un % CT) * 32 + (within & 31);
    const int o = ((un / CT) % OT) * 32 + (within >> 5);
    const int sl = un / (CT * OT);
    dst = d.dw + (long)o * (kSeq * d.cin) + sl * d.cin + cc;
  }
  *dst = t;
  if (J.adam) {
    float step_size, sqrt_bc2;
    side_adam_consts(J, step_size, sqrt_bc2);
    side_adam_at(J, dst - J.g, t, step_size, sqrt_bc2);
  }
}

// Side blocks go FIRST in a host grid (they start with the host's first
// blocks instead of queueing behind all of them), padded to a multiple of 8
// so block b of the host still lands on XCD b % 8: side_grid() blocks, of
// which the first n_blocks work.
__host__ __device__ inline int side_grid(const SideJob& J) { return (J.n_blocks + 7) / 8 * 8; }

// Host side (spiral_conv.hip): the device descriptor of a cfsd_side_work
// (item kinds and slab counts of each deferred slab set, as
// cfsd_dw_reduce_batch derives them).  n == 0 side blocks for w == NULL.
int make_side_job(const cfsd_side_work* w, SideJob& J);

}  // namespace cfsd
