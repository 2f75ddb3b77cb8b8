// Pool (sparse down/up-sample) SpMM and the mini-batch feature swap, gfx950.
//
// Reference: Pool (model.py:50-55) = index_select(x, 1, col) * value, then
// torch_scatter.scatter_add(.., row, dim_size=M).  Here: row-sorted CSR whose
// per-row entry order is the COO file order, so each output is the same
// sequence of fp32 mul/add roundings as the reference's sequential
// scatter_add (multiply and add are issued un-fused on purpose).
//
// SwapFeatures (swap_batch_transform.py:13-52): bs base meshes -> bs^2 meshes,
// out[i*bs + j] = mesh i with the swapped region's feature vertices from j.
#include "cfsd_common.h"
#include "spmm_sched.h"

namespace cfsd {


// xb: the mesh's x base; rs: elements between consecutive vertices of one
// mesh (c for batch-major x, batch * c for vertex-major x).
template <int CK, typename TX>
__device__ __forceinline__ void spmm_row_chunks(int beg, int end, const int* __restrict__ col,
                                                const float* __restrict__ val,
                                                const TX* __restrict__ xb, long rs, f32x4& acc) {
#pragma clang fp contract(off)
  for (int e0 = beg; e0 < end; e0 += CK) {
    float v[CK];
    f32x4 xv[CK];
#pragma unroll
    for (int j = 0; j < CK; ++j) {
      const int e = e0 + j < end ? e0 + j : end - 1;
      v[j] = val[e];
      xv[j] = ld4f(xb + (long)col[e] * rs);
    }
#pragma unroll
    for (int j = 0; j < CK; ++j) {
      if (e0 + j < end) {
        acc.x = acc.x + xv[j].x * v[j];
        acc.y = acc.y + xv[j].y * v[j];
        acc.z = acc.z + xv[j].z * v[j];
        acc.w = acc.w + xv[j].w * v[j];
      }
    }
  }
}

// One thread per (b, r, 4-channel chunk).  Consecutive threads walk the
// channel chunks of one row, so a row of C fp32 is read/written as C/4
// 16-B accesses by C/4 adjacent lanes.
// XCD-aware: the dispatcher places block i on XCD i % 8, so block group
// g = blockIdx % 8 takes the g-th contiguous eighth of the (b, r, q) space
// (two meshes of a 16-mesh batch): the rows one XCD gathers then come from
// a ~2 x V x C x 4-byte slice that fits its 4 MB L2 instead of the whole
// batch.  Placement changes speed only, never results.
// Storage types: x TX, y / elu_y TY (fp32 or bf16; fp32 arithmetic).
template <typename TX, typename TY>
__global__ __launch_bounds__(256) void spmm_csr_k(const int* __restrict__ row_ptr,
                                                  const int* __restrict__ col,
                                                  const float* __restrict__ val,
                                                  const TX* __restrict__ x,
                                                  const TY* __restrict__ elu_y,
                                                  TY* __restrict__ y, int m, int n, int c4,
                                                  long total, int batch, int xvm, int yvm) {
  // hipcc contracts a*b+c into fma by default; the reference rounds the
  // product and the sum separately (index_select*value, then scatter_add).
#pragma clang fp contract(off)
  const long per = (total + 7) / 8;
  const long t = (long)(blockIdx.x & 7) * per + (long)(blockIdx.x >> 3) * blockDim.x + threadIdx.x;
  if (t >= total || t >= (long)((blockIdx.x & 7) + 1) * per) return;
  int br, q, b, r;
  divmod32(t, c4, br, q);
  split_row(br, yvm, batch, m, b, r);  // output rows in y's layout
  const Lay lx = make_lay(xvm, batch, n);
  const long rs = (long)lx.vs * c4 * 4;
  const TX* xb = x + (long)b * lx.bs * c4 * 4 + 4 * q;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int beg = row_ptr[r], end = row_ptr[r + 1];
  // Entries in chunks: the chunk's column/value and x loads are all issued
  // before the first add (independent), the adds stay in entry order.
  // Short rows (up-sampling: 3 barycentric taps) use 4-entry chunks, long
  // rows (its transpose: ~12) 8-entry chunks; past-the-end entries are
  // clamped to the row's last one (an L1 hit, not added) -- measured faster
  // than exec-masked loads.  The 3-tap rows get an exact 3-entry chunk
  // (no clamped 4th load: up0 16.4 -> 15.2 us, same add order).
  if (end - beg == 3) spmm_row_chunks<3>(beg, end, col, val, xb, rs, acc);
  else if (end - beg <= 4) spmm_row_chunks<4>(beg, end, col, val, xb, rs, acc);
  else spmm_row_chunks<8>(beg, end, col, val, xb, rs, acc);
  if (elu_y) {
    f32x4 g = ld4f(elu_y + t * 4);
    acc.x *= elu_grad_from_out(g.x);
    acc.y *= elu_grad_from_out(g.y);
    acc.z *= elu_grad_from_out(g.z);
    acc.w *= elu_grad_from_out(g.w);
  }
  // (non-temporal stores measured: this kernel ~0.8 us faster, the conv
  // reading y 0.5-1 us slower -> plain stores)
  st4f(y + t * 4, acc);
}

// SpMM for a matrix whose rows all hold exactly K entries (the barycentric
// up-sampling matrices: 3 per row), stored row-major in the CSR arrays:
// row r's entries are [r*K, r*K + K), so there is no row_ptr load and the
// dependent chain is column/value -> x rows (two memory latencies instead of
// three).  A thread owns RPT chunks 256 apart (each load instruction still
// covers 256 consecutive chunks), all their loads issued before the first
// add; the adds are the CSR kernel's: 0 + x0*v0, then + x1*v1, ... un-fused
// (bit-identical).  Same XCD grouping as spmm_csr_k.
template <int K, int RPT, typename TX, typename TY>
__global__ __launch_bounds__(256) void spmm_uniform_k(const int* __restrict__ col,
                                                      const float* __restrict__ val,
                                                      const TX* __restrict__ x,
                                                      const TY* __restrict__ elu_y,
                                                      TY* __restrict__ y, int m, int n, int c4,
                                                      long total, int batch, int xvm, int yvm) {
#pragma clang fp contract(off)
  const Lay lx = make_lay(xvm, batch, n);
  const long per = (total + 7) / 8;
  const int grp = blockIdx.x & 7;
  const long lim = min(total, (long)(grp + 1) * per);
  const long t0 = (long)grp * per + (long)(blockIdx.x >> 3) * (256 * RPT) + threadIdx.x;
  if (t0 >= lim) return;
  int cc[RPT][K], bq[RPT], qq[RPT];
  float vv[RPT][K];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const long t = min(t0 + 256 * j, lim - 1);  // clamped chunks: loads only
    int br, r;
    divmod32(t, c4, br, qq[j]);
    split_row(br, yvm, batch, m, bq[j], r);  // output rows in y's layout
#pragma unroll
    for (int k = 0; k < K; ++k) {
      cc[j][k] = col[r * K + k];
      vv[j][k] = val[r * K + k];
    }
  }
  f32x4 xv[RPT][K];
#pragma unroll
  for (int j = 0; j < RPT; ++j)
#pragma unroll
    for (int k = 0; k < K; ++k)
      xv[j][k] = ld4f(x + ((long)bq[j] * lx.bs + (long)cc[j][k] * lx.vs) * c4 * 4 + 4 * qq[j]);
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const long t = t0 + 256 * j;
    if (t >= lim) break;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      acc.x = acc.x + xv[j][k].x * vv[j][k];
      acc.y = acc.y + xv[j][k].y * vv[j][k];
      acc.z = acc.z + xv[j][k].z * vv[j][k];
      acc.w = acc.w + xv[j][k].w * vv[j][k];
    }
    if (elu_y) {
      const f32x4 g = ld4f(elu_y + t * 4);
      acc.x *= elu_grad_from_out(g.x);
      acc.y *= elu_grad_from_out(g.y);
      acc.z *= elu_grad_from_out(g.z);
      acc.w *= elu_grad_from_out(g.w);
    }
    st4f(y + t * 4, acc);
  }
}

// spmm_uniform_k for VERTEX-MAJOR x and y (the up-samplings of the
// vertex-major levels): output row r is one contiguous block of batch x c
// elements and a wave lies inside one row (batch * c / 4 % 64 == 0), so the
// row's K columns / values are wave-uniform scalar loads and each tap is one
// buffer load per lane with the source block's offset in an SGPR (the
// batch-major kernel loads every column / value per lane).  A wave runs RW
// rows (XCD-contiguous), all their tap loads issued before the first add;
// the adds are spmm_uniform_k's (bit-identical).
template <int K, int RW, typename TX, typename TY>
__global__ __launch_bounds__(256) void spmm_uniform_vm_k(const int* __restrict__ col, const float* __restrict__ val,
                                                         const TX* __restrict__ x, TY* __restrict__ y, int m, int n,
                                                         int rowq) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int wpr = rowq / 64;  // waves per row
  const long wg = (long)xcd_block() * 4 + (threadIdx.x >> 6);
  const long row0 = (wg / wpr) * RW;
  const int part = (int)(wg % wpr);
  if (row0 >= m) return;
  const int q = part * 64 + lane;  // 4-element chunk of the row block
  const int eb = (int)sizeof(TX);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<TX*>(x), 0, (int)((long)n * rowq * 4 * eb), 0x00020000);
  f32x4 xv[RW][K];
  float vv[RW][K];
#pragma unroll
  for (int w = 0; w < RW; ++w) {
    const int r = __builtin_amdgcn_readfirstlane((int)min(row0 + w, (long)m - 1));
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int c = col[r * K + k];
      vv[w][k] = val[r * K + k];
      if constexpr (sizeof(TX) == 4) {
        xv[w][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, q * 16, c * rowq * 16, 0));
      } else {
        const u32x2 h = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, q * 8, c * rowq * 8, 0));
        xv[w][k] = (f32x4){__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xffff0000u),
                           __uint_as_float(h.y << 16), __uint_as_float(h.y & 0xffff0000u)};
      }
    }
  }
#pragma unroll
  for (int w = 0; w < RW; ++w) {
    if (row0 + w >= m) break;  // uniform
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      acc.x = acc.x + xv[w][k].x * vv[w][k];
      acc.y = acc.y + xv[w][k].y * vv[w][k];
      acc.z = acc.z + xv[w][k].z * vv[w][k];
      acc.w = acc.w + xv[w][k].w * vv[w][k];
    }
    st4f(y + ((row0 + w) * rowq + q) * 4, acc);
  }
}

template <typename TX, typename TY>
__global__ __launch_bounds__(256) void spmm_sched_k(const int* __restrict__ row_ptr,
                                                    const int* __restrict__ col,
                                                    const float* __restrict__ val,
                                                    const int* __restrict__ order,
                                                    const TX* __restrict__ x,
                                                    const TY* __restrict__ elu_y,
                                                    TY* __restrict__ y, int m, int n, int c4,
                                                    int groups, int bpg, int per) {
  const int g = (int)blockIdx.x % groups;
  const int t = (int)(blockIdx.x / groups) * (int)blockDim.x + (int)threadIdx.x;
  if (t >= per) return;
  const int rowq = bpg * c4;  // threads per schedule slot
  const int slot = t / rowq, rem = t - slot * rowq;
  const int bl = rem / c4, q = rem - bl * c4;
  const int b = g * bpg + bl, r = order[slot];
  const TX* xb = x + (long)b * n * c4 * 4 + 4 * q;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int beg = row_ptr[r], end = row_ptr[r + 1];
  // (16-entry chunks for the > 32-entry rows measured no faster at level 0
  // and slower elsewhere: the wider branch's registers cost occupancy)
  spmm_fold_prefetch<8>(beg, end, col, val, xb, (long)c4 * 4, acc);
  const long o = ((long)b * m + r) * c4 + q;
  if (elu_y) {
    f32x4 gy = ld4f(elu_y + o * 4);
    acc.x *= elu_grad_from_out(gy.x);
    acc.y *= elu_grad_from_out(gy.y);
    acc.z *= elu_grad_from_out(gy.z);
    acc.w *= elu_grad_from_out(gy.w);
  }
  st4f(y + o * 4, acc);
}

// spmm_sched_k over a CSR stored in visiting order: slot i is output row
// rows_s[i] with entries [ptr_s[i], ptr_s[i+1]) (the rows' entries in the
// original per-row order, so the same sums bit for bit).  The slot's row id
// and extent are independent loads, so the chain is extent -> list -> x rows
// (spmm_sched_k: order -> row_ptr -> list -> x rows), and a wave's entry
// lists are contiguous.
template <typename TX, typename TY, int V = 4, bool UNI = false>
__global__ __launch_bounds__(256) void spmm_sched_csr_k(const int* __restrict__ ptr_s,
                                                        const int* __restrict__ col_s,
                                                        const float* __restrict__ val_s,
                                                        const int* __restrict__ rows_s,
                                                        const TX* __restrict__ x,
                                                        const TY* __restrict__ elu_y,
                                                        TY* __restrict__ y, int m, int n, int c4,
                                                        int groups, int bpg, int per, int xvm,
                                                        int yvm, int n_main) {
  spmm_sched_csr_body<TX, TY, V, UNI>(ptr_s, col_s, val_s, rows_s, x, elu_y, y, m, n, c4, groups, bpg, per, xvm, yvm,
                                      n_main, (int)blockIdx.x);
}

// out[(i*bs + j), v, :] = x[mesh(i or j), v, :]; one thread per (out mesh,
// vertex); c <= 4 channels per vertex (xyz) are copied as scalars, larger c
// in 16-B chunks.  Device-side indices are range-guarded so a bad value can
// never fault the GPU: a key outside [0, n_regions) swaps nothing (every
// output mesh is its base mesh) and a mesh index outside [0, n_meshes) is
// clamped into it (the host validates both before they reach the device).
__global__ __launch_bounds__(256) void swap_k(const float* __restrict__ x,
                                              const int* __restrict__ batch_idx,
                                              const unsigned char* __restrict__ mask,
                                              const int* __restrict__ key, float* __restrict__ out,
                                              int bs, int nv, int c, int n_meshes, int n_regions,
                                              long total, int yvm) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  int ob, v;  // thread t = row t of the output storage (vertex-major: the bs^2 meshes of a vertex adjacent)
  split_row(t, yvm, bs * bs, nv, ob, v);
  const SwapSrc sw{x, batch_idx, mask, key, bs, n_meshes, n_regions};
  const long src_mesh = swap_src_mesh(sw, *key, ob, v, nv);
  const float* src = x + (src_mesh * nv + v) * c;
  float* dst = out + t * c;
  if (c == 3) {  // xyz: one dwordx3 load and store
    float v3[3];
    ld_row<3>(src, v3);
    st_row<3>(dst, v3);
  } else {
    for (int q = 0; q < c; ++q) dst[q] = src[q];
  }
}

// The un-swapped batch (data config swap_features: False, data_loading.py:38
// with no feature_swapper): out mesh b = x[batch_idx[b]], one thread per
// (out mesh, vertex) row of out's storage; mesh indices clamped like swap_k.
__global__ __launch_bounds__(256) void gather_meshes_k(const float* __restrict__ x,
                                                       const int* __restrict__ batch_idx,
                                                       float* __restrict__ out, int bs, int nv, int c,
                                                       int n_meshes, long total, int yvm) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  int ob, v;
  split_row(t, yvm, bs, nv, ob, v);
  const long src_mesh = min(max(batch_idx[ob], 0), n_meshes - 1);
  const float* src = x + (src_mesh * nv + v) * c;
  float* dst = out + t * c;
  if (c == 3) {
    float v3[3];
    ld_row<3>(src, v3);
    st_row<3>(dst, v3);
  } else {
    for (int q = 0; q < c; ++q) dst[q] = src[q];
  }
}

// Storage conversion fp32 <-> bf16 (round to nearest even), 4 elements per
// thread (n % 4 tail by the last thread).
template <typename TS, typename TD>
__global__ __launch_bounds__(256) void cast_k(const TS* __restrict__ src, TD* __restrict__ dst, long n) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x, n4 = n / 4;
  if (q < n4) {
    st4f(dst + 4 * q, ld4f(src + 4 * q));
  } else if (q == n4) {
    for (long i = 4 * n4; i < n; ++i) stf(dst + i, ldf(src + i));
  }
}

// Spectral blend of the augmentation (utils.py:244-267): coefficients
// s4[p, j, :] = s1 + v[p, j] * (s2 - s1) for j < n_blend, else s1 (the
// reference's s3/s4 assembly; spectral_combination is the 0/1 special case of
// v).  s1, s2, s4 [pairs, k, c]; v [pairs, k].  Same operation order as numpy.
__global__ __launch_bounds__(256) void spectral_blend_k(const float* __restrict__ s1,
                                                        const float* __restrict__ s2,
                                                        const float* __restrict__ v,
                                                        float* __restrict__ s4, int k, int c,
                                                        int n_blend, long total) {
#pragma clang fp contract(off)
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const long pj = t / c;
  const int j = (int)(pj % k);
  const float a = s1[t];
  s4[t] = j < n_blend ? a + v[pj] * (s2[t] - a) : a;
}

// Dataset normalisation (data_loading.py:259-260, (verts - mean) / std with
// per-vertex [nv, c] statistics): subtraction then IEEE division, the two
// roundings of the reference's torch ops, so the result is bit-exact.
__global__ __launch_bounds__(256) void normalize_k(const float* x,  // may alias out (in-place normalisation)
                                                   const float* __restrict__ mean,
                                                   const float* __restrict__ std,
                                                   float* out, int per_mesh, long total) {
#pragma clang fp contract(off)
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int e = (int)(t % per_mesh);
  out[t] = (x[t] - mean[e]) / std[e];
}

__global__ void scale_k(float* __restrict__ y, long n, float alpha) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) y[t] *= alpha;
}

__global__ void elu_bwd_k(const float* __restrict__ dy, const float* __restrict__ y,
                          float* dx, long n) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) dx[t] = dy[t] * elu_grad_from_out(y[t]);
}

// Per-vertex reconstruction errors (model_manager.py:395-400, test.py:81-84,
// 280-301).  One thread per vertex row of 3 channels: optional
// un-normalisation (x*std + mean, rounded separately as torch does), then
// err = sqrt(((d0^2 + d1^2) + d2^2)) * to_mm and l1 = |d0| + |d1| + |d2|.
__global__ void vertex_errors_k(const float* __restrict__ out, const float* __restrict__ gt,
                                const float* __restrict__ mean, const float* __restrict__ std,
                                float* __restrict__ err, float* __restrict__ l1, int nv,
                                long total, float to_mm) {
#pragma clang fp contract(off)
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int v = (int)t % nv;  // total * 3 < 2^31 (checked at the ABI)
  float a[3], g[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    a[q] = out[t * 3 + q];
    g[q] = gt[t * 3 + q];
  }
  if (mean) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float s = std[v * 3 + q], m = mean[v * 3 + q];
      a[q] = a[q] * s + m;
      g[q] = g[q] * s + m;
    }
  }
  const float d0 = a[0] - g[0], d1 = a[1] - g[1], d2 = a[2] - g[2];
  if (err) err[t] = sqrtf(d0 * d0 + d1 * d1 + d2 * d2) * to_mm;
  if (l1) l1[t] = fabsf(d0) + fabsf(d1) + fabsf(d2);
}

// Per-mesh mean of the vertex errors (test.py:297 torch.mean(errors, dim=1)):
// one 256-thread workgroup per mesh, strided partial sums reduced in a fixed
// tree (deterministic; summation order differs from torch's CPU reduction).
__global__ void __launch_bounds__(256) row_mean_k(const float* __restrict__ err,
                                                  float* __restrict__ mesh_mean, int nv) {
  __shared__ float part[256];
  const float* row = err + (long)blockIdx.x * nv;
  float acc = 0.f;
  for (int v = threadIdx.x; v < nv; v += 256) acc += row[v];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) mesh_mean[blockIdx.x] = part[0] / (float)nv;
}

}  // namespace cfsd

using namespace cfsd;

extern "C" int cfsd_vertex_errors(const float* out, const float* gt, const float* mean,
                                  const float* std, float* err, float* l1, float* mesh_mean,
                                  int batch, int nv, float to_mm, void* stream) {
  if (!out || !gt) return set_error(CFSD_EINVAL, "vertex_errors: null pointer");
  if (!mean != !std) return set_error(CFSD_EINVAL, "vertex_errors: mean and std go together");
  if (mesh_mean && !err) return set_error(CFSD_EINVAL, "vertex_errors: mesh_mean needs err");
  if (batch <= 0 || nv <= 0) return set_error(CFSD_EINVAL, "vertex_errors: bad sizes");
  const long total = (long)batch * nv;
  if (total * 3 >= (1L << 31)) return set_error(CFSD_EINVAL, "vertex_errors: batch x nv too large");
  if (!err && !l1) return CFSD_OK;
  hipLaunchKernelGGL(vertex_errors_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, out, gt, mean, std, err, l1, nv, total, to_mm);
  if (mesh_mean)
    hipLaunchKernelGGL(row_mean_k, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream, err,
                       mesh_mean, nv);
  return launch_status("vertex_errors");
}

// storage descriptor (type | CFSD_VM) -> (type, vertex-major); false if invalid
static bool split_dt(int dt, int& type, int& vm) {
  type = CFSD_DT_TYPE(dt);
  vm = (dt & CFSD_VM) != 0;
  return (dt & ~(CFSD_VM | 0xf)) == 0 && (type == CFSD_DT_F32 || type == CFSD_DT_BF16);
}

static int spmm_launch(const int32_t* row_ptr, const int32_t* col, const float* val,
                       const int32_t* order, const void* x, int x_dt, const void* elu_y, void* y,
                       int y_dt, int batch, int m, int n, int c, void* stream) {
  if (!row_ptr || !col || !val || !x || !y) return set_error(CFSD_EINVAL, "spmm_csr: null pointer");
  int xvm, yvm;
  if (!split_dt(x_dt, x_dt, xvm) || !split_dt(y_dt, y_dt, yvm)) return set_error(CFSD_EINVAL, "spmm_csr: bad dtype");
  if (order && (xvm || yvm)) return set_error(CFSD_EINVAL, "spmm_csr_sched: batch-major operands only");
  if (batch <= 0 || m <= 0 || n <= 0 || c <= 0 || (c % 4))
    return set_error(CFSD_EINVAL, "spmm_csr: bad sizes batch=%d m=%d n=%d c=%d", batch, m, n, c);
  if ((x_dt != CFSD_DT_F32 && x_dt != CFSD_DT_BF16) || (y_dt != CFSD_DT_F32 && y_dt != CFSD_DT_BF16))
    return set_error(CFSD_EINVAL, "spmm_csr: bad dtype");
  const long total = (long)batch * m * (c / 4);
  if (total >= (1L << 31) || (long)batch * n >= (1L << 31))
    return set_error(CFSD_EINVAL, "spmm_csr: batch x rows >= 2^31 (32-bit indices)");
  const hipStream_t st0 = (hipStream_t)stream;
  if (order) {  // scheduled rows: XCD groups of whole meshes
    const int groups = batch % 8 == 0 ? 8 : 1, bpg = batch / groups;
    const int per = bpg * m * (c / 4);
    const unsigned nb = (unsigned)(groups * ((per + 255) / 256));
#define SPMS(TX, TY)                                                                             \
  hipLaunchKernelGGL((spmm_sched_k<TX, TY>), dim3(nb), dim3(256), 0, st0, row_ptr, col, val,     \
                     order, (const TX*)x, (const TY*)elu_y, (TY*)y, m, n, c / 4, groups, bpg, per)
    if (x_dt == CFSD_DT_F32 && y_dt == CFSD_DT_F32) SPMS(float, float);
    else if (x_dt == CFSD_DT_F32) SPMS(float, bf16_t);
    else if (y_dt == CFSD_DT_F32) SPMS(bf16_t, float);
    else SPMS(bf16_t, bf16_t);
#undef SPMS
    return launch_status("spmm_csr_sched");
  }
  const long per_grp = (total + 7) / 8;  // 8 XCD groups of equal block count
  const unsigned nblk = (unsigned)(8 * ((per_grp + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
#define SPMM(TX, TY)                                                                             \
  hipLaunchKernelGGL((spmm_csr_k<TX, TY>), dim3(nblk), dim3(256), 0, st, row_ptr, col, val,      \
                     (const TX*)x, (const TY*)elu_y, (TY*)y, m, n, c / 4, total, batch, xvm, yvm)
  if (x_dt == CFSD_DT_F32 && y_dt == CFSD_DT_F32) SPMM(float, float);
  else if (x_dt == CFSD_DT_F32) SPMM(float, bf16_t);
  else if (y_dt == CFSD_DT_F32) SPMM(bf16_t, float);
  else SPMM(bf16_t, bf16_t);
#undef SPMM
  return launch_status("spmm_csr");
}

extern "C" int cfsd_spmm_csr(const int32_t* row_ptr, const int32_t* col, const float* val,
                             const float* x, const float* elu_y, float* y, int batch, int m,
                             int n, int c, void* stream) {
  return spmm_launch(row_ptr, col, val, nullptr, x, CFSD_DT_F32, elu_y, y, CFSD_DT_F32, batch, m, n, c,
                     stream);
}

extern "C" int cfsd_spmm_csr_sched(const int32_t* row_ptr, const int32_t* col, const float* val,
                                   const int32_t* order, const void* x, int x_dt, const void* elu_y,
                                   void* y, int y_dt, int batch, int m, int n, int c, void* stream) {
  if (!order) return set_error(CFSD_EINVAL, "spmm_csr_sched: null order");
  return spmm_launch(row_ptr, col, val, order, x, x_dt, elu_y, y, y_dt, batch, m, n, c, stream);
}

extern "C" int cfsd_spmm_csr_x(const int32_t* row_ptr, const int32_t* col, const float* val,
                               const void* x, int x_dt, const void* elu_y, void* y, int y_dt,
                               int batch, int m, int n, int c, void* stream) {
  return spmm_launch(row_ptr, col, val, nullptr, x, x_dt, elu_y, y, y_dt, batch, m, n, c, stream);
}

constexpr int kSpmmUvm = 1;
constexpr int kSpmmUvmRw = 4;
constexpr int kSpmmUrpt = 4;
extern "C" int cfsd_spmm_uniform(int k, const int32_t* col, const float* val, const void* x,
                                 int x_dt, const void* elu_y, void* y, int y_dt, int batch, int m,
                                 int n, int c, void* stream) {
  if (!col || !val || !x || !y) return set_error(CFSD_EINVAL, "spmm_uniform: null pointer");
  if (k < 1 || k > 4) return set_error(CFSD_EINVAL, "spmm_uniform: %d entries per row (1..4)", k);
  if (batch <= 0 || m <= 0 || n <= 0 || c <= 0 || (c % 4))
    return set_error(CFSD_EINVAL, "spmm_uniform: bad sizes batch=%d m=%d n=%d c=%d", batch, m, n, c);
  int xvm, yvm;
  if (!split_dt(x_dt, x_dt, xvm) || !split_dt(y_dt, y_dt, yvm)) return set_error(CFSD_EINVAL, "spmm_uniform: bad dtype");
  const long total = (long)batch * m * (c / 4);
  if (total >= (1L << 31) || (long)batch * n >= (1L << 31) || (long)m * k >= (1L << 31))
    return set_error(CFSD_EINVAL, "spmm_uniform: sizes >= 2^31 (32-bit indices)");
  if (kSpmmUvm && xvm && yvm && !elu_y && k == 3 && (batch * (c / 4)) % 64 == 0 &&
      (long)n * batch * c * 4 < 0x7ffff000L) {  // vertex-major: wave-uniform rows
    constexpr int RW = kSpmmUvmRw;
    const int rowq = batch * (c / 4), wpr = rowq / 64;
    const long waves = (long)((m + RW - 1) / RW) * wpr;
    const unsigned nb = (unsigned)((waves + 3) / 4);
    const hipStream_t st = (hipStream_t)stream;
#define SPUV(TX, TY)                                                                                \
  hipLaunchKernelGGL((spmm_uniform_vm_k<3, RW, TX, TY>), dim3(nb), dim3(256), 0, st, col, val, (const TX*)x, \
                     (TY*)y, m, n, rowq)
    if (x_dt == CFSD_DT_F32 && y_dt == CFSD_DT_F32) SPUV(float, float);
    else if (x_dt == CFSD_DT_F32) SPUV(float, bf16_t);
    else if (y_dt == CFSD_DT_F32) SPUV(bf16_t, float);
    else SPUV(bf16_t, bf16_t);
#undef SPUV
    return launch_status("spmm_uniform_vm");
  }
  constexpr int RPT = kSpmmUrpt;
  const long per_grp = (total + 7) / 8;
  const unsigned nblk = (unsigned)(8 * ((per_grp + 256 * RPT - 1) / (256 * RPT)));
  const hipStream_t st = (hipStream_t)stream;
#define SPMU(K_, TX, TY)                                                                          \
  hipLaunchKernelGGL((spmm_uniform_k<K_, RPT, TX, TY>), dim3(nblk), dim3(256), 0, st, col, val,    \
                     (const TX*)x, (const TY*)elu_y, (TY*)y, m, n, c / 4, total, batch, xvm, yvm)
#define SPMU_K(K_)                                                                                \
  if (k == K_) {                                                                                  \
    if (x_dt == CFSD_DT_F32 && y_dt == CFSD_DT_F32) SPMU(K_, float, float);                        \
    else if (x_dt == CFSD_DT_F32) SPMU(K_, float, bf16_t);                                         \
    else if (y_dt == CFSD_DT_F32) SPMU(K_, bf16_t, float);                                         \
    else SPMU(K_, bf16_t, bf16_t);                                                                 \
  }
  SPMU_K(1) SPMU_K(2) SPMU_K(3) SPMU_K(4)
#undef SPMU_K
#undef SPMU
  return launch_status("spmm_uniform");
}

extern "C" int cfsd_spmm_sched_csr(const int32_t* ptr_s, const int32_t* col_s, const float* val_s,
                                   const int32_t* rows_s, const void* x, int x_dt,
                                   const void* elu_y, void* y, int y_dt, int batch, int m, int n,
                                   int c, void* stream) {
  if (!ptr_s || !col_s || !val_s || !rows_s || !x || !y)
    return set_error(CFSD_EINVAL, "spmm_sched_csr: null pointer");
  if (batch <= 0 || m <= 0 || n <= 0 || c <= 0 || (c % 4))
    return set_error(CFSD_EINVAL, "spmm_sched_csr: bad sizes batch=%d m=%d n=%d c=%d", batch, m, n, c);
  int xvm, yvm;
  if (!split_dt(x_dt, x_dt, xvm) || !split_dt(y_dt, y_dt, yvm))
    return set_error(CFSD_EINVAL, "spmm_sched_csr: bad dtype");
  if ((long)batch * m * (c / 4) >= (1L << 31) || (long)batch * n >= (1L << 31))
    return set_error(CFSD_EINVAL, "spmm_sched_csr: batch x rows >= 2^31 (32-bit indices)");
  // batch-major x: XCD groups of whole meshes (their rows share an L2);
  // vertex-major x: one group, a slot's threads cover every mesh, so each
  // gathered vertex block is one contiguous load
  const int groups = (!xvm && batch % 8 == 0) ? 8 : 1, bpg = batch / groups;
  // bf16 x: 8 channels per thread (one 16-B load per entry; bf16 up0T 21.3 ->
  // see DESIGN) -- the same per-element folds
  const int V = (x_dt == CFSD_DT_BF16 && c % 8 == 0) ? 8 : 4;
  const int per = bpg * m * (c / V);
  const unsigned nb = (unsigned)(groups * ((per + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
  const bool uni = (bpg * (c / V)) % 64 == 0;
#define SPSC(TX, TY, V_)                                                                                       \
  if (uni)                                                                                                     \
    hipLaunchKernelGGL((spmm_sched_csr_k<TX, TY, V_, true>), dim3(nb), dim3(256), 0, st, ptr_s,                 \
                       col_s, val_s, rows_s, (const TX*)x, (const TY*)elu_y, (TY*)y, m, n, c / V_, groups, bpg, per, \
                       xvm, yvm, (int)nb);                                                                     \
  else                                                                                                         \
    hipLaunchKernelGGL((spmm_sched_csr_k<TX, TY, V_, false>), dim3(nb), dim3(256), 0, st, ptr_s,                \
                       col_s, val_s, rows_s, (const TX*)x, (const TY*)elu_y, (TY*)y, m, n, c / V_, groups, bpg, per, \
                       xvm, yvm, (int)nb)
  if (x_dt == CFSD_DT_F32 && y_dt == CFSD_DT_F32) {
    SPSC(float, float, 4);
  } else if (x_dt == CFSD_DT_F32) {
    SPSC(float, bf16_t, 4);
  } else if (V == 8 && y_dt == CFSD_DT_F32) {
    SPSC(bf16_t, float, 8);
  } else if (V == 8) {
    SPSC(bf16_t, bf16_t, 8);
  } else if (y_dt == CFSD_DT_F32) {
    SPSC(bf16_t, float, 4);
  } else {
    SPSC(bf16_t, bf16_t, 4);
  }
#undef SPSC
  return launch_status("spmm_sched_csr");
}

extern "C" int cfsd_cast(const void* src, int src_dt, void* dst, int dst_dt, size_t n, void* stream) {
  if (!src || !dst) return set_error(CFSD_EINVAL, "cast: null pointer");
  if (n == 0) return CFSD_OK;
  const dim3 grid((unsigned)((n / 4 + 1 + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
  if (src_dt == CFSD_DT_F32 && dst_dt == CFSD_DT_BF16)
    hipLaunchKernelGGL((cast_k<float, bf16_t>), grid, dim3(256), 0, st, (const float*)src, (bf16_t*)dst, (long)n);
  else if (src_dt == CFSD_DT_BF16 && dst_dt == CFSD_DT_F32)
    hipLaunchKernelGGL((cast_k<bf16_t, float>), grid, dim3(256), 0, st, (const bf16_t*)src, (float*)dst, (long)n);
  else
    return set_error(CFSD_EINVAL, "cast: unsupported dtypes %d -> %d", src_dt, dst_dt);
  return launch_status("cast");
}

extern "C" int cfsd_swap_features(const float* x, const int32_t* batch_idx,
                                  const uint8_t* region_mask, const int32_t* key, float* out,
                                  int bs, int nv, int c, int n_meshes, int n_regions,
                                  void* stream) {
  if (!x || !batch_idx || !region_mask || !key || !out)
    return set_error(CFSD_EINVAL, "swap_features: null pointer");
  if (bs <= 0 || nv <= 0 || c <= 0 || n_meshes <= 0 || n_regions <= 0)
    return set_error(CFSD_EINVAL, "swap_features: bad sizes");
  const long total = (long)bs * bs * nv;
  if (total >= (1L << 31)) return set_error(CFSD_EINVAL, "swap_features: bs^2 x nv >= 2^31");
  hipLaunchKernelGGL(swap_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, batch_idx, region_mask, key, out, bs, nv, c, n_meshes,
                     n_regions, total, 0);
  return launch_status("swap_features");
}

extern "C" int cfsd_swap_features_x(const float* x, const int32_t* batch_idx, const uint8_t* region_mask,
                                    const int32_t* key, float* out, int out_dt, int bs, int nv, int c,
                                    int n_meshes, int n_regions, void* stream) {
  if (!x || !batch_idx || !region_mask || !key || !out)
    return set_error(CFSD_EINVAL, "swap_features_x: null pointer");
  if (bs <= 0 || nv <= 0 || c <= 0 || n_meshes <= 0 || n_regions <= 0)
    return set_error(CFSD_EINVAL, "swap_features_x: bad sizes");
  if ((out_dt & ~CFSD_VM) != CFSD_DT_F32) return set_error(CFSD_EINVAL, "swap_features_x: bad dtype %d", out_dt);
  const long total = (long)bs * bs * nv;
  if (total >= (1L << 31)) return set_error(CFSD_EINVAL, "swap_features_x: bs^2 x nv >= 2^31");
  hipLaunchKernelGGL(swap_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, batch_idx, region_mask, key, out, bs, nv, c, n_meshes,
                     n_regions, total, (out_dt & CFSD_VM) != 0);
  return launch_status("swap_features_x");
}

extern "C" int cfsd_gather_meshes(const float* x, const int32_t* batch_idx, float* out, int out_dt, int bs,
                                  int nv, int c, int n_meshes, void* stream) {
  if (!x || !batch_idx || !out) return set_error(CFSD_EINVAL, "gather_meshes: null pointer");
  if (bs <= 0 || nv <= 0 || c <= 0 || n_meshes <= 0) return set_error(CFSD_EINVAL, "gather_meshes: bad sizes");
  if ((out_dt & ~CFSD_VM) != CFSD_DT_F32) return set_error(CFSD_EINVAL, "gather_meshes: bad dtype %d", out_dt);
  const long total = (long)bs * nv;
  if (total >= (1L << 31)) return set_error(CFSD_EINVAL, "gather_meshes: bs x nv >= 2^31");
  hipLaunchKernelGGL(gather_meshes_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                     batch_idx, out, bs, nv, c, n_meshes, total, (out_dt & CFSD_VM) != 0);
  return launch_status("gather_meshes");
}

extern "C" int cfsd_spectral_blend(const float* s1, const float* s2, const float* values, float* s4,
                                   int pairs, int k, int c, int n_blend, void* stream) {
  if (!s1 || !s2 || !values || !s4) return set_error(CFSD_EINVAL, "spectral_blend: null pointer");
  if (pairs <= 0 || k <= 0 || c <= 0 || n_blend < 0) return set_error(CFSD_EINVAL, "spectral_blend: bad sizes");
  const long total = (long)pairs * k * c;
  hipLaunchKernelGGL(spectral_blend_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, s1, s2, values, s4, k, c, n_blend, total);
  return launch_status("spectral_blend");
}

extern "C" int cfsd_normalize(const float* x, const float* mean, const float* std, float* out,
                              int n_meshes, int nv, int c, void* stream) {
  if (!x || !mean || !std || !out) return set_error(CFSD_EINVAL, "normalize: null pointer");
  if (n_meshes <= 0 || nv <= 0 || c <= 0) return set_error(CFSD_EINVAL, "normalize: bad sizes");
  const long total = (long)n_meshes * nv * c;
  hipLaunchKernelGGL(normalize_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, mean, std, out, nv * c, total);
  return launch_status("normalize");
}

extern "C" int cfsd_scale(float* y, size_t n, float alpha, void* stream) {
  if (!y) return set_error(CFSD_EINVAL, "scale: null pointer");
  if (n == 0) return CFSD_OK;
  hipLaunchKernelGGL(scale_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, y, (long)n, alpha);
  return launch_status("scale");
}

extern "C" int cfsd_elu_bwd(const float* dy, const float* y, float* dx, size_t n, void* stream) {
  if (!dy || !y || !dx) return set_error(CFSD_EINVAL, "elu_bwd: null pointer");
  if (n == 0) return CFSD_OK;
  hipLaunchKernelGGL(elu_bwd_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, dy, y, dx, (long)n);
  return launch_status("elu_bwd");
}
