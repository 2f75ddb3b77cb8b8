// Shared helpers for the CDNA4 (gfx950) kernels of the spiral mesh-VAE step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cfsd.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace cfsd {

constexpr int kSeq = 9;  // spiral length of every configuration (craniofacial/body/default.yaml)

// XCD-aware persistent tile schedule.  Blocks b and b+8 share an XCD (and
// its 4 MB L2) under the dispatcher's round-robin placement, so the blocks of
// group g = b % G sweep ONE contiguous 1/G of the tile range: neighbouring
// tiles gather neighbouring vertices, which then hit the same L2.  Placement
// only changes speed, never results.
constexpr long kContigTiles = 4096;  // persistent conv sweeps below this many tiles: contig
struct TileSweep {
  long begin, end, step;
};
// contig: each block walks its own contiguous sub-range of the group's
// tiles instead of the interleaved sweep (measured: level-1 32 -> 32 forward
// 27.8 -> 24.4 us and data gradient 35.4 -> 30.5 us; no gain at level 0,
// where a wave has ~2 tiles, and a loss for the dW slabs).
// (vb, nb: the block's index and count among the blocks sharing the sweep;
// a launch that pairs two bodies passes its virtual block numbering)
__device__ __forceinline__ TileSweep xcd_sweep_v(long n_tiles, int lanes_per_block, int lane_id, bool contig,
                                                 int vb, int nb) {
  const int G = nb < 8 ? nb : 8;
  const int grp = vb % G, lb = vb / G;
  const int nb_g = (nb - grp + G - 1) / G;  // blocks in this group
  const long per = (n_tiles + G - 1) / G;
  TileSweep t;
  if (contig) {
    const long chunk = (per + nb_g - 1) / nb_g;
    t.begin = grp * per + (long)lb * chunk + lane_id;
    t.end = min(n_tiles, min((grp + 1) * per, grp * per + (long)(lb + 1) * chunk));
    t.step = lanes_per_block;
    return t;
  }
  t.begin = grp * per + (long)lb * lanes_per_block + lane_id;
  t.end = min(n_tiles, (grp + 1) * per);
  t.step = (long)nb_g * lanes_per_block;
  return t;
}
__device__ __forceinline__ TileSweep xcd_sweep(long n_tiles, int lanes_per_block, int lane_id,
                                               bool contig = false) {
  return xcd_sweep_v(n_tiles, lanes_per_block, lane_id, contig, blockIdx.x, gridDim.x);
}

// Non-persistent grids: renumber workgroups so that XCD x (hardware
// dispatch is round-robin, x = blockIdx % 8) owns a CONTIGUOUS 1/8 of the
// block range -- its meshes' rows then stay in its own L2.  Bijective for any
// gridDim.
__device__ __forceinline__ int xcd_block_of(int bid, int nb) {
  if (nb < 8) return bid;
  const int g = bid & 7, lb = bid >> 3, q = nb >> 3, rem = nb & 7;
  return g * q + min(g, rem) + lb;
}
__device__ __forceinline__ int xcd_block() { return xcd_block_of(blockIdx.x, gridDim.x); }

// Records the last error text (thread-local) and returns its code.
int set_error(int code, const char* fmt, ...);

inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error((int)e, "%s: %s", what, hipGetErrorString(e));
  return CFSD_OK;
}

// ELU (alpha = 1, model.py's F.elu) with the hardware exp (v_exp_f32):
// x > 0 ? x : exp(x) - 1, branch-free (5 VALU).  |error| vs expm1 < ~1.2e-7
// absolute (one ulp of 1.0, near x = 0-), i.e. below the fp32 rounding of the
// conv sums feeding it.  The libm expm1f it replaces is a chain of divergent
// branches: 6.4 of the D3 forward's 60.5 us (kbench, ELU vs no activation,
// profiles/round5_d3_forward_diagnosis.txt).  Every fp32 and bf16 kernel uses
// this one function, so the layouts stay bit-identical to each other.
__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : __expf(x) - 1.f; }
__device__ __forceinline__ float elu_fast(float x) { return elu_f(x); }
// dELU/dx written from the ELU OUTPUT y (alpha = 1): 1 for y > 0, else y + 1 = exp(x).
__device__ __forceinline__ float elu_grad_from_out(float y) { return y > 0.f ? 1.f : y + 1.f; }

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// v_mfma_f32_32x32x2_f32: lane l holds A[l&31][l>>5], B[l>>5][l&31];
// D: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5).
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// v_mfma_f32_16x16x4_f32: lane l holds A[l&15][l>>4], B[l>>4][l&15];
// D: col = l&15, row = 4*(l>>4) + r.  32-cycle issue, 40-cycle dependent latency.
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// CS consecutive floats of one small-channel row (CS = 3: xyz) as ONE
// dwordx3 access: per-channel dword loads cost the texture path a cycle per
// cache line per instruction three times over.  Rows are only dword-aligned.
typedef float f32x3u __attribute__((ext_vector_type(3), aligned(4)));
template <int CS>
__device__ __forceinline__ void ld_row(const float* __restrict__ p, float* v) {
  if constexpr (CS == 3) {
    const f32x3u t = *reinterpret_cast<const f32x3u*>(p);
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
  } else {
#pragma unroll
    for (int q = 0; q < CS; ++q) v[q] = p[q];
  }
}
template <int CS>
__device__ __forceinline__ void st_row(float* __restrict__ p, const float* v) {
  if constexpr (CS == 3) {
    *reinterpret_cast<f32x3u*>(p) = (f32x3u){v[0], v[1], v[2]};
  } else {
#pragma unroll
    for (int q = 0; q < CS; ++q) p[q] = v[q];
  }
}

// torch.optim.Adam (non-amsgrad) update of one element.
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1,
                                          float b2, float eps, float wd, float step_size,
                                          float sqrt_bc2) {
  if (wd != 0.f) g = fmaf(wd, p, g);
  m = fmaf(b1, m, (1.f - b1) * g);
  v = fmaf(b2, v, (1.f - b2) * g * g);
  const float denom = sqrtf(v) / sqrt_bc2 + eps;
  p -= step_size * (m / denom);
}

constexpr int kMaxBatch = 1 << 20;

// ---------------------------------------------------------------- bf16 storage
// Activations of the bf16 path are stored as raw bfloat16 (uint16_t, the
// torch.bfloat16 bit layout) and always widened to fp32 for arithmetic;
// narrowing is round-to-nearest-even (v_cvt_pk_bf16_f32), as torch's casts.
typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint32_t h16) { return __uint_as_float(h16 << 16); }
__device__ __forceinline__ uint32_t f2bf(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) { return f2bf(lo) | (f2bf(hi) << 16); }
// element access of either storage type, arithmetic in fp32
__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ float ldf(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void stf(float* p, float v) { *p = v; }
__device__ __forceinline__ void stf(bf16_t* p, float v) { *p = (bf16_t)f2bf(v); }
// 4 consecutive elements as fp32 (16-B or 8-B load)
__device__ __forceinline__ f32x4 ld4f(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 ld4f(const bf16_t* p) {
  const u32x2 v = *reinterpret_cast<const u32x2*>(p);
  return (f32x4){__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                 __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
}
__device__ __forceinline__ void st4f(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void st4f(bf16_t* p, f32x4 v) {
  *reinterpret_cast<u32x2*>(p) = (u32x2){pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)};
}
// 8 consecutive elements as a packed bf16 MFMA fragment (fp32 sources are
// rounded to bf16 here)
__device__ __forceinline__ u32x4 ld8bf(const bf16_t* p) { return *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ u32x4 ld8bf(const float* p) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  return (u32x4){pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y), pack_bf2(b.z, b.w)};
}
// v_mfma_f32_16x16x32_bf16: lane l holds A[l&15][8(l>>4) + j], B[8(l>>4) + j][l&15]
// (j = 0..7); D: col = l&15, row = 4(l>>4) + r.
__device__ __forceinline__ f32x4 mfma_bf16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// Cooperative global -> LDS copy of n items: item e is loaded by ld(e) and
// stored by st(e, v), NB loads per thread issued before the first store.  (A
// load -> store loop waits out one memory latency per item; these copies open
// the persistent kernels, where every workgroup pays them at once.)
template <int NB, typename T, typename LD, typename ST>
__device__ __forceinline__ void coop_copy(int n, LD ld, ST st) {
  for (int e0 = threadIdx.x; e0 < n; e0 += NB * (int)blockDim.x) {
    T v[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int e = e0 + j * (int)blockDim.x;
      v[j] = ld(e < n ? e : n - 1);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int e = e0 + j * (int)blockDim.x;
      if (e < n) st(e, v[j]);
    }
  }
}

// Flattened row / element indices are < 2^31 (checked at every entry point),
// so per-thread index splits use 32-bit division: a 64-bit division is a
// ~100-instruction software sequence on CDNA, which showed up as VALU time
// in the gather-staging kernels (dW staging: 79 -> 73 us at level 0).
__device__ __forceinline__ void divmod32(long v, int d, int& q, int& r) {
  const int vi = (int)v;
  q = vi / d;
  r = vi - q * d;
}

// Row layout of a [batch, nv, c] activation (CFSD_VM storage flag, cfsd.h).
// BM (the reference's [B, V, C]): row (b, v) is b*nv + v.  VM (vertex-major):
// v*batch + b -- the rows of one vertex in every mesh of the batch form ONE
// contiguous block, so a spiral neighbour is gathered for all meshes by a
// single coalesced wave load (16 meshes x 32 bf16 channels = 1 KiB, 8 full
// cache lines) instead of 16 scattered 64-B rows.  Kernels iterate flat rows
// m in one operand's layout (split_row) and address the others with row_of.
struct Lay {
  int bs, vs;  // row index = b*bs + v*vs
};
__host__ __device__ inline Lay make_lay(bool vm, int batch, int nv) {
  return vm ? Lay{1, batch} : Lay{nv, 1};
}
__device__ __forceinline__ int row_of(const Lay& L, int b, int v) { return b * L.bs + v * L.vs; }
// flat row m of a tensor stored in layout (vm, batch, nv) -> (b, v)
__device__ __forceinline__ void split_row(long m, bool vm, int batch, int nv, int& b, int& v) {
  if (vm) divmod32(m, batch, v, b);
  else divmod32(m, nv, b, v);
}

// Workgroups of `kernel` that can be resident on the whole device at once
// (occupancy API x CU count).  Persistent grids are sized to this so no
// workgroup runs in a second, mostly idle, round.  Cached per kernel.
int resident_blocks(const void* kernel, int block_threads, size_t dyn_lds);
template <typename K>
inline int resident_blocks_of(K kernel, int block_threads, size_t dyn_lds) {
  return resident_blocks(reinterpret_cast<const void*>(kernel), block_threads, dyn_lds);
}

// The feature swap's source mesh of output mesh ob at vertex v
// (SwapFeatures, swap_batch_transform.py:13-42): ob = i * bs + j takes mesh
// batch_idx[j]'s vertex when i != j and v lies in region k's mask, else mesh
// batch_idx[i]'s.  Range-guarded: a key outside [0, n_regions) swaps nothing,
// a mesh index outside [0, n_meshes) is clamped (the host validates both).
struct SwapSrc {
  const float* data;  // resident set [n_meshes][nv][c], batch-major
  const int* batch_idx;
  const unsigned char* mask;  // [n_regions][nv]
  const int* key;
  int bs, n_meshes, n_regions;
};
__device__ __forceinline__ long swap_src_mesh(const SwapSrc& s, int k, int ob, int v, int nv) {
  const int i = ob / s.bs, j = ob % s.bs;
  // both candidates loaded up front: the mask load is the only one the
  // choice waits on (a gather through the swap is one load deeper, not two)
  const int bi = s.batch_idx[i], bj = s.batch_idx[j];
  const bool take = (i != j) && k >= 0 && k < s.n_regions && s.mask[(long)k * nv + v];
  return min(max(take ? bj : bi, 0), s.n_meshes - 1);
}

// CUs of the current device (cached).
int device_cus();
// Persistent grid with the SAME number of workgroups (bpc) on every CU,
// capped at one workgroup per `per_block` units: a grid that is not a multiple
// of the CU count leaves some CUs a third more waves than others, and those
// set the kernel's time.
inline unsigned cu_blocks(long units, int per_block, int bpc) {
  long need = (units + per_block - 1) / per_block;
  if (need < 1) need = 1;
  const long full = (long)bpc * device_cus();
  return (unsigned)(need < full ? need : full);
}

// Balanced persistent grid: `units` work items, `per_block` processed per
// block-iteration, at most `max_blocks` blocks.
inline unsigned balanced_blocks(long units, int per_block, long max_blocks) {
  long need = (units + per_block - 1) / per_block;
  if (need < 1) need = 1;
  if (need <= max_blocks) return (unsigned)need;
  const long iters = (need + max_blocks - 1) / max_blocks;
  return (unsigned)((need + iters - 1) / iters);
}

// Gather load hidden from hipcc's waitcnt bookkeeping (cdna_hip_programming.md
// §5.7 form (ii)): issue with gload4_async, then retire with a vm_wait4<N>
// naming the destinations before the first consumer.  Used where hipcc's own
// waitcnt placement would drain a prefetch one slot too early.
__device__ __forceinline__ void gload4_async(f32x4& d, const float* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}
// Store hidden from hipcc's waitcnt bookkeeping (counted like the loads).
template <int OFF>
__device__ __forceinline__ void gstore1_async(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off offset:%2" ::"v"(p), "v"(v), "n"(OFF) : "memory");
}
__device__ __forceinline__ void gload1_async(int& d, const int* p) {
  asm volatile("global_load_dword %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}
__device__ __forceinline__ void gload1f_async(float& d, const float* p) {
  asm volatile("global_load_dword %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}
// The same from a wave-uniform base (SGPR pair) + a 32-bit per-lane byte
// offset: no 64-bit address arithmetic per load.
__device__ __forceinline__ void gload1f_async_s(float& d, const float* base, int off) {
  asm volatile("global_load_dword %0, %1, %2" : "=v"(d) : "v"(off), "s"(base) : "memory");
}
// Retire counted loads and hand their 8 destinations back to the compiler.
template <int N, typename T>
__device__ __forceinline__ void vm_wait_arr8(T (&a)[8]) {
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),
                 "+v"(a[6]), "+v"(a[7])
               : "n"(N));
}
template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait4(f32x4& a, f32x4& b, f32x4& c, f32x4& d) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N));
}
template <int N>
__device__ __forceinline__ void vm_wait8(f32x4& a, f32x4& b, f32x4& c, f32x4& d, f32x4& e,
                                         f32x4& f, f32x4& g, f32x4& h) {
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
               : "n"(N));
}

}  // namespace cfsd
