// The visiting-order CSR SpMM (Pool(up)^T, long skewed rows) as a device body:
// its own launch (pool_swap.hip) and a workgroup role of a paired launch
// (spiral_conv_vm16.hip).
#pragma once
#include "cfsd_common.h"

namespace cfsd {

// The same SpMM for matrices with long, skewed rows (the transposes of the
// up-sampling matrices: level 0 has 12 entries per row on average but up to
// 96).  A row is a sequential fp32 fold in entry order (kept for
// bit-exactness), so the kernel cannot end before its longest row's chain of
// dependent chunks; spmm_csr_k's plain chunk loop paid two memory latencies
// (column list, then x rows) per 8 entries.  Here:
//  * rows are visited in `order` (rows by decreasing length, a host-built
//    schedule), slot-major inside each XCD's contiguous mesh group, so the
//    longest rows of every mesh start first and a wave's 8 rows have similar
//    lengths;
//  * the next chunk's columns / values are loaded while the current chunk's
//    x rows are in flight: one latency per chunk.
// one row's sequential fold, the next chunk's list prefetched
template <int CK, typename TX>
__device__ __forceinline__ void spmm_fold_prefetch(int beg, int end, const int* __restrict__ col,
                                                   const float* __restrict__ val,
                                                   const TX* __restrict__ xb, long rs, f32x4& acc) {
#pragma clang fp contract(off)
  int cc[CK];
  float vv[CK];
#pragma unroll
  for (int j = 0; j < CK; ++j) {
    const int e = min(beg + j, end - 1);
    cc[j] = col[e];
    vv[j] = val[e];
  }
  for (int e0 = beg; e0 < end; e0 += CK) {
    f32x4 xv[CK];
#pragma unroll
    for (int j = 0; j < CK; ++j) xv[j] = ld4f(xb + (long)cc[j] * rs);
    float vc[CK];
#pragma unroll
    for (int j = 0; j < CK; ++j) vc[j] = vv[j];
    if (e0 + CK < end) {  // next chunk's list while the x rows are in flight
#pragma unroll
      for (int j = 0; j < CK; ++j) {
        const int e = min(e0 + CK + j, end - 1);
        cc[j] = col[e];
        vv[j] = val[e];
      }
    }
#pragma unroll
    for (int j = 0; j < CK; ++j) {
      if (e0 + j < end) {
        acc.x = acc.x + xv[j].x * vc[j];
        acc.y = acc.y + xv[j].y * vc[j];
        acc.z = acc.z + xv[j].z * vc[j];
        acc.w = acc.w + xv[j].w * vc[j];
      }
    }
  }
}

// The same fold over 8 consecutive bf16 channels per thread (one 16-B load
// per entry instead of two 8-B ones; per element the same operations in the
// same order as two 4-wide threads: bit-identical)
template <int CK>
__device__ __forceinline__ void spmm_fold_prefetch8(int beg, int end, const int* __restrict__ col,
                                                    const float* __restrict__ val,
                                                    const bf16_t* __restrict__ xb, long rs, f32x4& acc0,
                                                    f32x4& acc1) {
#pragma clang fp contract(off)
  int cc[CK];
  float vv[CK];
#pragma unroll
  for (int j = 0; j < CK; ++j) {
    const int e = min(beg + j, end - 1);
    cc[j] = col[e];
    vv[j] = val[e];
  }
  for (int e0 = beg; e0 < end; e0 += CK) {
    u32x4 xv[CK];
#pragma unroll
    for (int j = 0; j < CK; ++j) xv[j] = *reinterpret_cast<const u32x4*>(xb + (long)cc[j] * rs);
    float vc[CK];
#pragma unroll
    for (int j = 0; j < CK; ++j) vc[j] = vv[j];
    if (e0 + CK < end) {  // next chunk's list while the x rows are in flight
#pragma unroll
      for (int j = 0; j < CK; ++j) {
        const int e = min(e0 + CK + j, end - 1);
        cc[j] = col[e];
        vv[j] = val[e];
      }
    }
#pragma unroll
    for (int j = 0; j < CK; ++j) {
      if (e0 + j < end) {
        const u32x4 q = xv[j];
        acc0.x = acc0.x + __uint_as_float(q.x << 16) * vc[j];
        acc0.y = acc0.y + __uint_as_float(q.x & 0xffff0000u) * vc[j];
        acc0.z = acc0.z + __uint_as_float(q.y << 16) * vc[j];
        acc0.w = acc0.w + __uint_as_float(q.y & 0xffff0000u) * vc[j];
        acc1.x = acc1.x + __uint_as_float(q.z << 16) * vc[j];
        acc1.y = acc1.y + __uint_as_float(q.z & 0xffff0000u) * vc[j];
        acc1.z = acc1.z + __uint_as_float(q.w << 16) * vc[j];
        acc1.w = acc1.w + __uint_as_float(q.w & 0xffff0000u) * vc[j];
      }
    }
  }
}

// spmm_sched_k over a CSR stored in visiting order: slot i is output row
// rows_s[i] with entries [ptr_s[i], ptr_s[i+1]) (the rows' entries in the
// original per-row order, so the same sums bit for bit).  The slot's row id
// and extent are independent loads, so the chain is extent -> list -> x rows,
// and a wave's entry lists are contiguous.
// One output element group (V channels of one row of one mesh) per thread of
// workgroup `bid` among the body's n_main workgroups (blockDim.x threads each).
template <typename TX, typename TY, int V, bool UNI>
__device__ __forceinline__ void spmm_sched_csr_body(const int* __restrict__ ptr_s, const int* __restrict__ col_s,
                                                    const float* __restrict__ val_s, const int* __restrict__ rows_s,
                                                    const TX* __restrict__ x, const TY* __restrict__ elu_y,
                                                    TY* __restrict__ y, int m, int n, int c4, int groups, int bpg,
                                                    int per, int xvm, int yvm, int n_main, int bid) {
  // vertex-major x (groups == 1): XCD k runs the k-th eighth of the schedule,
  // so the rows sharing a source block meet in one L2 (natural row order:
  // up0T 112.9 -> 64.1 MB of HBM traffic, 21.8 -> 20.0 us)
  const int blk = xvm ? xcd_block_of(bid, n_main) : bid;
  const int g = blk % groups;
  const int t = (blk / groups) * (int)blockDim.x + (int)threadIdx.x;
  if (t >= per) return;
  const int rowq = bpg * c4;  // threads per schedule slot
  // UNI (rowq % 64 == 0: a wave lies inside one slot): the slot, its extent
  // and entry list are wave-uniform -> scalar loads
  const int slot = UNI ? __builtin_amdgcn_readfirstlane(t / rowq) : t / rowq, rem = t - slot * rowq;
  const int bl = rem / c4, q = rem - bl * c4;
  const int b = g * bpg + bl, batch = groups * bpg;
  const Lay lx = make_lay(xvm, batch, n), ly = make_lay(yvm, batch, m);
  const int r = rows_s[slot], beg = ptr_s[slot], end = ptr_s[slot + 1];
  // (c4: V-channel groups per row; V = 8 for bf16 x, 4 otherwise)
  const TX* xb = x + (long)b * lx.bs * c4 * V + V * q;
  if constexpr (V == 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    spmm_fold_prefetch<8>(beg, end, col_s, val_s, xb, (long)lx.vs * c4 * 4, acc);
    const long o = (long)row_of(ly, b, r) * c4 + q;
    if (elu_y) {
      f32x4 gy = ld4f(elu_y + o * 4);
      acc.x *= elu_grad_from_out(gy.x);
      acc.y *= elu_grad_from_out(gy.y);
      acc.z *= elu_grad_from_out(gy.z);
      acc.w *= elu_grad_from_out(gy.w);
    }
    st4f(y + o * 4, acc);
  } else {
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    spmm_fold_prefetch8<8>(beg, end, col_s, val_s, xb, (long)lx.vs * c4 * 8, acc[0], acc[1]);
    const long o = ((long)row_of(ly, b, r) * c4 + q) * 8;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4 v = acc[h];
      if (elu_y) {
        const f32x4 gy = ld4f(elu_y + o + 4 * h);
        v.x *= elu_grad_from_out(gy.x);
        v.y *= elu_grad_from_out(gy.y);
        v.z *= elu_grad_from_out(gy.z);
        v.w *= elu_grad_from_out(gy.w);
      }
      st4f(y + o + 4 * h, v);
    }
  }
}


}  // namespace cfsd
