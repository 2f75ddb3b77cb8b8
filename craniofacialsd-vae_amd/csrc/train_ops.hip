// Losses, latent bottleneck, dense layers and Adam for the mesh-VAE step (gfx950).
//
// Reference: ModelManager._do_iteration (model_manager.py:274-326) and the
// loss methods it calls (:333-393), Model.encode/decode's nn.Linear layers
// (model.py:114-124, 152-156, 167-168), Model._reparameterize (:184-188),
// torch.optim.Adam (:69-72, 316).  All reductions are fixed-order trees, so
// every kernel here is run-to-run deterministic.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>

#include "cfsd_common.h"

namespace cfsd {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int device_cus() {
  static thread_local int dev_cached = -1, cus_cached = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != dev_cached) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    dev_cached = dev;
    cus_cached = cus;
  }
  return cus_cached;
}

int resident_blocks(const void* kernel, int block_threads, size_t dyn_lds) {
  struct Key {
    const void* k;
    int t;
    size_t l;
    int v;
  };
  static thread_local Key cache[64];
  static thread_local int n_cache = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  for (int i = 0; i < n_cache; ++i)
    if (cache[i].k == kernel && cache[i].t == block_threads && cache[i].l == dyn_lds) return cache[i].v;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block_threads, dyn_lds) != hipSuccess ||
      per_cu <= 0)
    per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int v = per_cu * cus;
  if (n_cache < 64) cache[n_cache++] = Key{kernel, block_threads, dyn_lds, v};
  return v;
}

constexpr int kLapThreads = 256;

// Block-wide sum of two values in fixed order (wave shuffle tree + LDS).
__device__ __forceinline__ float2 block_sum2(float a, float b, float2* sh) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    a += __shfl_xor(a, d);
    b += __shfl_xor(b, d);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) sh[wave] = make_float2(a, b);
  __syncthreads();
  float2 r = make_float2(0.f, 0.f);
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      r.x += sh[w].x;
      r.y += sh[w].y;
    }
  return r;
}

// ----------------------------------------------------------- recon + Laplacian
// xb = the mesh's row of vertex 0, rs = floats between consecutive vertices'
// rows of one mesh (C batch-major, batch*C vertex-major)
template <int C>
__device__ __forceinline__ void lap_row_dot(int beg, int end, const int* __restrict__ col,
                                            const float* __restrict__ val,
                                            const float* __restrict__ xb, int rs, float (&acc)[C]) {
  constexpr int CK = 8;
  for (int e0 = beg; e0 < end; e0 += CK) {
    int cc[CK];
    float w[CK];
#pragma unroll
    for (int j = 0; j < CK; ++j) {
      const int e = e0 + j < end ? e0 + j : end - 1;
      cc[j] = col[e];
      w[j] = e0 + j < end ? val[e] : 0.f;
    }
    float xv[CK][C];
#pragma unroll
    for (int j = 0; j < CK; ++j) ld_row<C>(xb + (long)cc[j] * rs, xv[j]);
#pragma unroll
    for (int j = 0; j < CK; ++j)
#pragma unroll
      for (int q = 0; q < C; ++q) acc[q] = fmaf(w[j], xv[j][q], acc[q]);
  }
}

// Pass 1, one thread per (b, v): squared error, L.pred row, its norm and
// unit vector.  C <= 4.
template <int C>
__global__ __launch_bounds__(kLapThreads) void recon_lap_fwd_k(
    const float* __restrict__ pred, const float* __restrict__ gt, const int* __restrict__ l_ptr,
    const int* __restrict__ l_col, const float* __restrict__ l_val, float* __restrict__ unit,
    float* __restrict__ partials, int nv, long total, int batch, int vm) {
  __shared__ float2 sh[kLapThreads / 64];
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float sq = 0.f, nrm = 0.f;
  if (t < total) {
    // thread t = row t of the storage (vertex-major: the meshes of a vertex
    // are adjacent threads, each Laplacian neighbour one contiguous block)
    int b, v;
    split_row(t, vm, batch, nv, b, v);
    const Lay L = make_lay(vm, batch, nv);
    float lx[C];
#pragma unroll
    for (int q = 0; q < C; ++q) lx[q] = 0.f;
    lap_row_dot<C>(l_ptr[v], l_ptr[v + 1], l_col, l_val, pred + (long)b * L.bs * C, L.vs * C, lx);
    float n2 = 0.f, pv[C], gv[C];
    ld_row<C>(pred + t * C, pv);
    ld_row<C>(gt + t * C, gv);
#pragma unroll
    for (int q = 0; q < C; ++q) {
      const float d = pv[q] - gv[q];
      sq = fmaf(d, d, sq);
      n2 = fmaf(lx[q], lx[q], n2);
    }
    nrm = sqrtf(n2);
    const float inv = nrm > 0.f ? 1.f / nrm : 0.f;
    float un[C];
#pragma unroll
    for (int q = 0; q < C; ++q) un[q] = lx[q] * inv;
    st_row<C>(unit + t * C, un);
  }
  float2 r = block_sum2(sq, nrm, sh);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = r.x;
    partials[2 * blockIdx.x + 1] = r.y;
  }
}

// Loss finalisation: total = rec + w_kl*kl + w_lc*lc + w_lap*lap from the
// recon/Laplacian block partials and the latent terms (one workgroup).
struct LossFinalize {
  const float* partials;
  int nblocks;
  const float* terms;
  float* out;
  float* acc;
  float inv_n_rec, inv_lap, w_kl, w_lc, w_lap;
};

__device__ void loss_finalize_block(const LossFinalize& f, float2* sh) {
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < f.nblocks; i += blockDim.x) {
    a += f.partials[2 * i];
    b += f.partials[2 * i + 1];
  }
  float2 r = block_sum2(a, b, sh);
  if (threadIdx.x == 0) {
    const float rec = r.x * f.inv_n_rec, lap = r.y * f.inv_lap;
    const float kl = f.terms[0], lc = f.terms[1];
    const float tot = rec + f.w_kl * kl + f.w_lc * lc + f.w_lap * lap;
    const float v[5] = {rec, kl, lc, lap, tot};
    for (int q = 0; q < 5; ++q) {
      f.out[q] = v[q];
      if (f.acc) f.acc[q] += v[q];
    }
    if (f.acc) f.acc[5] += 1.f;
  }
}

// Pass 2, one thread per (b, u): d/dpred of w_rec*mse + w_lap*lap.  With
// fin.partials set, the LAST block also finalises the losses of pass 1
// (complete: pass 1 is the previous launch on the stream), saving a launch.
template <int C>
__global__ __launch_bounds__(256) void recon_lap_bwd_k(
    const float* __restrict__ pred, const float* __restrict__ gt, const float* __restrict__ unit,
    const int* __restrict__ lt_ptr, const int* __restrict__ lt_col,
    const float* __restrict__ lt_val, float* __restrict__ dpred, int nv, long total, float k_rec,
    float k_lap, const LossFinalize fin, int batch, int vm) {
  if (fin.partials && blockIdx.x == gridDim.x - 1) {
    __shared__ float2 sh[4];
    loss_finalize_block(fin, sh);
  }
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  int b, u;
  split_row(t, vm, batch, nv, b, u);
  const Lay L = make_lay(vm, batch, nv);
  float g[C];
#pragma unroll
  for (int q = 0; q < C; ++q) g[q] = 0.f;
  lap_row_dot<C>(lt_ptr[u], lt_ptr[u + 1], lt_col, lt_val, unit + (long)b * L.bs * C, L.vs * C, g);
  float pv[C], gv[C], dv[C];
  ld_row<C>(pred + t * C, pv);
  ld_row<C>(gt + t * C, gv);
#pragma unroll
  for (int q = 0; q < C; ++q) dv[q] = k_rec * (pv[q] - gv[q]) + k_lap * g[q];
  st_row<C>(dpred + t * C, dv);
}

// ----------------------------------------------------------- latent head
// Single workgroup.  mulv [B, 2L] = [logvar | mu] (rows of the stacked
// encoder Linear), z [B, L].  dlat [B, 3L] = {w_lc*dLC/dz | w_kl*dKL/dmu | w_kl*dKL/dlogvar}.
// terms[2] = {kl, lc}.
// 16 waves: the LC distance and gradient phases are chains of dependent LDS
// reads that one wave per SIMD cannot hide (256: 16.0 us, 512: 11.4,
// 1024: 9.8, same-box A/B in the step).
constexpr int kLatThreads = 1024;
struct LatentArgs {
  const float* mulv;
  const float* eps;
  const int* key;
  float* z;
  float* dlat;
  float* terms;
  int B, L, region_size, train, is_vae, sigmoid;
  float w_kl, w_lc, eta1, eta2;
  int bs;
};

// The latent head on one workgroup's LDS (zs [B][L], dist [4 npairs bs]).
// Every workgroup that runs it holds all of z and the LC distances; the
// `lead` one also writes z, the KL gradient pieces and terms[], and each
// writes the LC gradient elements [g0, g1) (one workgroup: [0, B L)).
// Each output element is the same expression whichever workgroup computes it.
__device__ __forceinline__ void latent_body(const LatentArgs& a, float* zs, float* dist, float2* red,
                                            bool lead, int g0, int g1) {
  const int B = a.B, L = a.L, bs = a.bs;
  const float w_lc = a.w_lc;
  const int tid = threadIdx.x;
  const int ldm = a.is_vae ? 2 * L : L;
  const int mu_off = a.is_vae ? L : 0;
  // z and KL pieces.  The inputs of up to 8 elements per thread are loaded
  // before any is used (mulv was just written by the encoder Linear, possibly
  // on another XCD: each dependent load round trip is ~1-2 us here).
  float kl_part = 0.f;
  constexpr int EPT = 8;
  for (int e0 = tid; e0 < B * L; e0 += EPT * blockDim.x) {
    float mu_r[EPT], lv_r[EPT], ep_r[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = e0 + k * blockDim.x;
      const int ec = e < B * L ? e : B * L - 1;
      const int i = ec / L, l = ec % L;
      mu_r[k] = a.mulv[i * ldm + mu_off + l];
      lv_r[k] = a.is_vae ? a.mulv[i * ldm + l] : 0.f;
      ep_r[k] = (a.is_vae && a.train) ? a.eps[ec] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = e0 + k * blockDim.x;
      if (e >= B * L) break;
      const int i = e / L, l = e % L;
      const float mu = mu_r[k];
      float zz = mu;
      if (a.is_vae) {
        const float lv = lv_r[k];
        const float ex = expf(lv);
        if (a.train) zz = mu + ep_r[k] * expf(0.5f * lv);
        kl_part += 1.f + lv - mu * mu - ex;
        if (lead) {
          a.dlat[i * 3 * L + L + l] = a.w_kl * mu / (float)B;
          a.dlat[i * 3 * L + 2 * L + l] = a.w_kl * (-0.5f) * (1.f - ex) / (float)B;
        }
      } else {
        if (a.sigmoid) zz = 1.f / (1.f + expf(-mu));
        if (lead) {
          a.dlat[i * 3 * L + L + l] = 0.f;
          a.dlat[i * 3 * L + 2 * L + l] = 0.f;
        }
      }
      if (lead) a.z[e] = zz;
      zs[e] = zz;
    }
  }
  __syncthreads();
  // latent consistency distances: kinds 0=lg 1=dg 2=dr 3=lr, pairs p<q, t.
  // Each of the 4*npairs*bs distances is summed by 8 lanes (l = j, j+8, ..)
  // and a 3-step shuffle tree (fixed order): 75-long serial loops were the
  // latency of this single-workgroup kernel.
  const int npairs = bs * (bs - 1) / 2;
  const int lo = a.region_size > 0 ? (*a.key) * a.region_size : 0;
  const int hi = lo + a.region_size;
  const int nd = 4 * npairs * bs;
  for (int e0 = 0; e0 < nd && w_lc != 0.f; e0 += blockDim.x / 8) {
    const int e = e0 + tid / 8, j = tid % 8;
    float d = 0.f;
    if (e < nd) {
      const int kind = e / (npairs * bs);
      const int pr = (e / bs) % npairs;
      const int t = e % bs;
      int p = 0, rem = pr;  // decode pair index in triu order
      while (rem >= bs - 1 - p) { rem -= bs - 1 - p; ++p; }
      const int q = p + 1 + rem;
      int ra, rb;
      if (kind == 0 || kind == 2) { ra = q * bs + t; rb = p * bs + t; }  // same donor t
      else { ra = t * bs + q; rb = t * bs + p; }                          // same base t
      const bool in_region = (kind <= 1);
      for (int l = j; l < L; l += 8) {
        const bool inr = (l >= lo && l < hi);
        const float df = inr == in_region ? zs[ra * L + l] - zs[rb * L + l] : 0.f;
        d = fmaf(df, df, d);
      }
    }
    d += __shfl_xor(d, 1);
    d += __shfl_xor(d, 2);
    d += __shfl_xor(d, 4);
    if (e < nd && j == 0) dist[e] = d;
  }
  __syncthreads();
  const float scale = 1.f / (float)(bs * bs * bs - bs * bs);
  float lc_part = 0.f;
  for (int e = tid; lead && e < npairs * bs && w_lc != 0.f; e += blockDim.x) {
    const float lg = dist[0 * npairs * bs + e], dg = dist[1 * npairs * bs + e];
    const float dr = dist[2 * npairs * bs + e], lr = dist[3 * npairs * bs + e];
    lc_part += fmaxf(0.f, lr - dr + a.eta2) + fmaxf(0.f, lg - dg + a.eta1);
  }
  // gradient of LC w.r.t. z: one thread per (row i, dim l).  Row i = (ii, jj)
  // (base ii, donor jj) appears in the hinge terms of the pairs that contain
  // ii (same-donor distances, t = jj) and of those that contain jj
  // (same-base distances, t = ii); the terms are added in a fixed order.
  const float k2 = 2.f * scale * w_lc;
  for (int e = g0 + tid; e < g1; e += blockDim.x) {
    const int i = e / L, l = e % L;
    float g = 0.f;
    if (w_lc != 0.f) {
      const bool inr = (l >= lo && l < hi);
      const float s1 = inr ? 1.f : -1.f;  // lg - dg  vs  lr - dr
      const int ii = i / bs, jj = i % bs;
      for (int pr = 0; pr < npairs; ++pr) {
        int p = 0, rem = pr;
        while (rem >= bs - 1 - p) { rem -= bs - 1 - p; ++p; }
        const int q = p + 1 + rem;
        // same-donor term (t = jj): rows a1 = q*bs + t, b1 = p*bs + t
        if (ii == q || ii == p) {
          const int de = pr * bs + jj;
          const bool act = inr ? (dist[0 * npairs * bs + de] - dist[1 * npairs * bs + de] + a.eta1) > 0.f
                               : (dist[3 * npairs * bs + de] - dist[2 * npairs * bs + de] + a.eta2) > 0.f;
          if (act) {
            const float d1 = zs[(q * bs + jj) * L + l] - zs[(p * bs + jj) * L + l];
            g += (ii == q ? 1.f : -1.f) * s1 * k2 * d1;
          }
        }
        // same-base term (t = ii): rows a2 = t*bs + q, b2 = t*bs + p
        if (jj == q || jj == p) {
          const int de = pr * bs + ii;
          const bool act = inr ? (dist[0 * npairs * bs + de] - dist[1 * npairs * bs + de] + a.eta1) > 0.f
                               : (dist[3 * npairs * bs + de] - dist[2 * npairs * bs + de] + a.eta2) > 0.f;
          if (act) {
            const float d2 = zs[(ii * bs + q) * L + l] - zs[(ii * bs + p) * L + l];
            g -= (jj == q ? 1.f : -1.f) * s1 * k2 * d2;
          }
        }
      }
    }
    a.dlat[i * 3 * L + l] = g;
  }
  if (lead) {
    float2 r = block_sum2(kl_part, lc_part, red);
    if (tid == 0) {
      a.terms[0] = a.is_vae ? -0.5f * r.x / (float)B : 0.f;
      a.terms[1] = w_lc != 0.f ? r.y * scale : 0.f;  // (no LC: bs = 1 and scale = 1/0)
    }
  }
}

// Single workgroup.  mulv [B, 2L] = [logvar | mu] (rows of the stacked
// encoder Linear), z [B, L].  dlat [B, 3L] = {w_lc*dLC/dz | w_kl*dKL/dmu | w_kl*dKL/dlogvar}.
// terms[2] = {kl, lc}.
// 16 waves: the LC distance and gradient phases are chains of dependent LDS
// reads that one wave per SIMD cannot hide (256: 16.0 us, 512: 11.4,
// 1024: 9.8, same-box A/B in the step).
__global__ __launch_bounds__(kLatThreads) void latent_fwd_k(const LatentArgs a) {
  // dynamic LDS: z [B][L], then the distances [kind][pair][t] (4 npairs bs)
  extern __shared__ float lat_lds[];
  __shared__ float2 red[kLatThreads / 64];
  latent_body(a, lat_lds, lat_lds + a.B * a.L, red, true, 0, a.B * a.L);
}

// Latent head + decoder Linear (model.py:184-188 then :167-168) in ONE
// launch: the Linear's input z is made in each workgroup's own LDS, so the
// kernel boundary between them (and the z round trip through memory) is gone.
// Workgroup g owns 32 columns of y = z W^T + b: its W slice ([32][k],
// contiguous) is loaded coalesced into registers before the latent phases
// and parked in LDS after them (lane stride k floats: k odd or 2 mod 4 keeps
// the reads conflict-free); thread (column, row pair) then runs the same
// fmaf chain per output as linear_fwd_nred (bit-identical y), z rows read as
// wave-uniform LDS broadcasts.  32-column slices: 134 workgroups at n = 4288
// (256-column slices with 8 outputs per thread left the Linear's chain of
// LDS reads as long as the latent head: 18.6 us vs 6.6 + 9.8 + 7.9 for the
// separate launches; 64 columns: 10.6-10.9 us, 32: 10.1-10.2, 128: 12.6).
// Every workgroup holds all of z and the LC distances in LDS and writes the
// LC gradient elements of its 1/grid slice; workgroup 0 also the KL pieces,
// z and terms with latent_fwd_k's thread mapping and sum tree (1024
// threads): z, dlat, terms and y all bit-identical to the two launches.
constexpr int kLatLinThreads = 1024;
constexpr int kLatLinCols = 32;
constexpr int kLatLinRows = kLatLinThreads / kLatLinCols;  // row groups (waves) of 2 rows
constexpr int kLatLinMaxK = 80;  // latent width (configs: 75, 33)
constexpr int kLatLinWPer = (kLatLinCols * kLatLinMaxK + kLatLinThreads - 1) / kLatLinThreads;
__global__ __launch_bounds__(kLatLinThreads) void latent_linear_fwd_k(const LatentArgs a,
                                                                      const float* __restrict__ w,
                                                                      const float* __restrict__ bias,
                                                                      float* __restrict__ y, int n,
                                                                      int lat_floats) {
  extern __shared__ float lat_lds[];
  __shared__ float2 red[kLatLinThreads / 64];
  const int m = a.B, k = a.L;
  const int c0 = blockIdx.x * kLatLinCols, nc = min(kLatLinCols, n - c0);
  const int nw = nc * k;
  const float* ws = w + (long)c0 * k;
  float wv[kLatLinWPer];
#pragma unroll
  for (int j = 0; j < kLatLinWPer; ++j) {
    const int e = j * kLatLinThreads + threadIdx.x;
    wv[j] = e < nw ? ws[e] : 0.f;
  }
  const int col = c0 + (int)(threadIdx.x % kLatLinCols);
  const float bv = (bias && col < n) ? bias[col] : 0.f;
  const int per = (m * k + gridDim.x - 1) / gridDim.x;
  const int g0 = min(m * k, (int)blockIdx.x * per), g1 = min(m * k, g0 + per);
  float* zs = lat_lds;
  float* wl = lat_lds + lat_floats;
  latent_body(a, zs, lat_lds + m * k, red, blockIdx.x == 0, g0, g1);
#pragma unroll
  for (int j = 0; j < kLatLinWPer; ++j) {
    const int e = j * kLatLinThreads + threadIdx.x;
    if (e < nw) wl[e] = wv[j];
  }
  __syncthreads();
  if (col >= n) return;
  const float* wr = wl + (col - c0) * k;
  for (int i0 = (threadIdx.x / kLatLinCols) * 2; i0 < m; i0 += 2 * kLatLinRows) {
    const int mr = min(2, m - i0);
    const float* z0 = zs + i0 * k;
    const float* z1 = zs + (i0 + mr - 1) * k;
    float a0 = 0.f, a1 = 0.f;
#pragma unroll 5
    for (int kk = 0; kk < k; ++kk) {
      const float wk = wr[kk];
      a0 = fmaf(z0[kk], wk, a0);
      a1 = fmaf(z1[kk], wk, a1);
    }
    y[(long)i0 * n + col] = a0 + bv;
    if (mr > 1) y[(long)(i0 + 1) * n + col] = a1 + bv;
  }
}

__global__ __launch_bounds__(256) void latent_bwd_k(const float* __restrict__ mulv,
                                                    const float* __restrict__ eps,
                                                    const float* __restrict__ dz_dec,
                                                    const float* __restrict__ dlat,
                                                    float* __restrict__ dmulv, int B, int L,
                                                    int train, int is_vae, int sigmoid,
                                                    const float* __restrict__ zval, int n_parts,
                                                    int n_main) {
  const int e = (int)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * L) return;
  const int i = e / L, l = e % L;
  float dzd = dz_dec[e];
  // decoder-Linear dx as split partial products: summed here in slice order,
  // 16 loads in flight per batch (a load-add chain per part was 4x slower)
  for (int p0 = 1; p0 < n_parts; p0 += 16) {
    float t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = dz_dec[(long)min(p0 + j, n_parts - 1) * B * L + e];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (p0 + j < n_parts) dzd += t[j];
  }
  const float dz = dzd + dlat[i * 3 * L + l];
  if (is_vae) {
    const float lv = mulv[i * 2 * L + l];
    const float dmu = dz + dlat[i * 3 * L + L + l];
    float dlv = dlat[i * 3 * L + 2 * L + l];
    if (train) dlv += dz * eps[e] * 0.5f * expf(0.5f * lv);
    dmulv[i * 2 * L + l] = dlv;
    dmulv[i * 2 * L + L + l] = dmu;
  } else {
    float dmu = dz;
    if (sigmoid) dmu *= zval[e] * (1.f - zval[e]);
    dmulv[i * L + l] = dmu;
  }
}

__global__ __launch_bounds__(256) void loss_finalize_k(const LossFinalize f) {
  __shared__ float2 sh[4];
  loss_finalize_block(f, sh);
}

// ----------------------------------------------------------- dense Linear
// The bottleneck Linears are [16 x 4288] x [4288 x 150] (encoder, stacked
// mu/logvar) and [16 x 75] x [75 x 4288] (decoder): tiny GEMMs whose cost is
// parallelism and latency, not FLOPs.  Each product is ONE launch: long
// reductions are spread over a 256-thread block and summed in fixed order
// (deterministic), short ones run thread-per-output with the small operand
// staged in LDS.
// Row-group width of the block-reduction kernels (one accumulator per row).
// Rows per block (blockIdx.y = row group).  The forward's 150 column blocks
// leave most CUs idle: 4-row groups quadruple its blocks (9.8 -> 6.7 us,
// same-box A/B); the decoder dx is bound by its strided W column reads, which
// every row group would repeat (16: 10.7 us, 4: 10.7-11.7, 2: 15, 1: 23.6).
// Each row's sum order is the same for any group width.
constexpr int kLinRGFwd = 4;
constexpr int kLinRGDx = 16;
constexpr int kLinRG = kLinRGDx > kLinRGFwd ? kLinRGDx : kLinRGFwd;  // LDS sizing
constexpr int kLinRedThreads = 512;   // block of the long-reduction kernels
constexpr int kLinUnroll = 9;         // reduction terms per thread issued together

// Sum kLinRG per-thread values over a kLinRedThreads block in fixed order
// (wave butterfly, then waves in index order); thread i < kLinRG gets row i.
// `sh` is [16 waves][kLinRG] LDS.
template <int RG>
__device__ __forceinline__ float block_rows_sum(float (&v)[RG], float* sh) {
  constexpr int kWaves = kLinRedThreads / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < RG; ++i) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v[i] += __shfl_xor(v[i], d);
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < RG; ++i) sh[wave * RG + i] = v[i];
  }
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x < RG) {
    r = sh[threadIdx.x];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) r += sh[w * RG + threadIdx.x];
  }
  __syncthreads();
  return r;
}

// Long k (encoder Linear: [16 x 4288] x [4288 x 150]): one 512-thread block
// per output column; each thread owns up to kLinUnroll k-terms per pass (all
// x / W loads issued before the FMAs), rows in groups of 16, fixed-order
// block sum.  One launch, no workspace, deterministic.
__global__ __launch_bounds__(kLinRedThreads) void linear_fwd_kred(const float* __restrict__ x,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ bias,
                                                                  float* __restrict__ y, int m,
                                                                  int k, int n) {
  __shared__ float sh[(kLinRedThreads / 64) * kLinRG];
  const int col = blockIdx.x;
  const float* wr = w + (long)col * k;
  for (int i0 = blockIdx.y * kLinRGFwd; i0 < m; i0 += kLinRGFwd * gridDim.y) {
    const int mr = min(kLinRGFwd, m - i0);
    float acc[kLinRGFwd];
#pragma unroll
    for (int i = 0; i < kLinRGFwd; ++i) acc[i] = 0.f;
    for (int k0 = 0; k0 < k; k0 += kLinRedThreads * kLinUnroll) {
      float wv[kLinUnroll];
#pragma unroll
      for (int u = 0; u < kLinUnroll; ++u) {
        const int kk = k0 + u * kLinRedThreads + threadIdx.x;
        wv[u] = kk < k ? wr[kk] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < kLinRGFwd; ++i) {
        const float* xr = x + (long)(i0 + min(i, mr - 1)) * k;
        float xv[kLinUnroll];
#pragma unroll
        for (int u = 0; u < kLinUnroll; ++u) {
          const int kk = k0 + u * kLinRedThreads + threadIdx.x;
          xv[u] = kk < k ? xr[kk] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kLinUnroll; ++u) acc[i] = fmaf(xv[u], wv[u], acc[i]);
      }
    }
    const float r = block_rows_sum<kLinRGFwd>(acc, sh);
    if (threadIdx.x < mr) y[(long)(i0 + threadIdx.x) * n + col] = r + (bias ? bias[col] : 0.f);
  }
}

// Short k (decoder Linear: [16 x 75] x [75 x 4288]): thread per (column,
// row quad); the quad's x rows are staged in LDS (broadcast reads), the
// thread's W row is read once for 4 outputs; y stores are coalesced.
constexpr int kLinSmallK = 512;
__global__ __launch_bounds__(256) void linear_fwd_nred(const float* __restrict__ x,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ y, int m, int k,
                                                       int n) {
  __shared__ float xs[4 * kLinSmallK];
  const int i0 = blockIdx.y * 4, mr = min(4, m - i0);
  for (int e = threadIdx.x; e < mr * k; e += 256) xs[e] = x[(long)i0 * k + e];
  __syncthreads();
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= n) return;
  const float* wr = w + (long)col * k;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 5
  for (int kk = 0; kk < k; ++kk) {
    const float wv = wr[kk];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = fmaf(xs[i * k + kk], wv, acc[i]);
  }
  const float bv = bias ? bias[col] : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < mr) y[(long)(i0 + i) * n + col] = acc[i] + bv;
}

// dx, short n (encoder Linear: dx [16 x 4288] = dy [16 x 150] . W [150 x 4288]):
// block = 64 k-columns x 4 waves; wave w sums the c-range w*n/4 .. for a row
// quad (blockIdx.y) with dy staged in LDS and W[c][k] coalesced (all of a
// wave's W loads in flight together); the 4 wave partials are added in order.
constexpr int kLinDxChunk = 40;  // c terms per wave and pass
__device__ __forceinline__ void linear_dx_nsmall_body(int bx, int by, const float* __restrict__ dy,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ elu_y,
                                                      float* __restrict__ dx, int m, int k, int n,
                                                      int accumulate) {
  __shared__ float ds[4 * kLinSmallK];
  __shared__ float part[4][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i0 = by * 4, mr = min(4, m - i0);
  for (int e = threadIdx.x; e < mr * n; e += 256) ds[e] = dy[(long)i0 * n + e];
  __syncthreads();
  const int kk = bx * 64 + lane;
  const int kc = kk < k ? kk : k - 1;
  const int per = (n + 3) / 4, c0 = wave * per, c1 = min(n, c0 + per);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int cb = c0; cb < c1; cb += kLinDxChunk) {
    float wv[kLinDxChunk];
#pragma unroll
    for (int u = 0; u < kLinDxChunk; ++u) wv[u] = cb + u < c1 ? w[(long)(cb + u) * k + kc] : 0.f;
#pragma unroll
    for (int u = 0; u < kLinDxChunk; ++u) {
      const int c = min(cb + u, n - 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = fmaf(ds[i * n + c], wv[u], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) part[wave][i][lane] = acc[i];
  __syncthreads();
  if (wave < mr && kk < k) {
    const int i = wave;
    float v = part[0][i][lane] + part[1][i][lane] + part[2][i][lane] + part[3][i][lane];
    const long o = (long)(i0 + i) * k + kk;
    if (elu_y) v *= elu_grad_from_out(elu_y[o]);
    dx[o] = accumulate ? dx[o] + v : v;
  }
}
__global__ __launch_bounds__(256) void linear_dx_nsmall(const float* __restrict__ dy,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ elu_y,
                                                        float* __restrict__ dx, int m, int k,
                                                        int n, int accumulate) {
  linear_dx_nsmall_body(blockIdx.x, blockIdx.y, dy, w, elu_y, dx, m, k, n, accumulate);
}

// dx, long n (decoder Linear: dz [16 x 75] = dh [16 x 4288] . W [4288 x 75]):
// one 512-thread block per k column, the n reduction spread over the block
// (kLinUnroll terms per thread in flight), fixed-order block sum.
__global__ __launch_bounds__(kLinRedThreads) void linear_dx_nred(const float* __restrict__ dy,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ elu_y,
                                                                 float* __restrict__ dx, int m,
                                                                 int k, int n, int accumulate) {
  __shared__ float sh[(kLinRedThreads / 64) * kLinRG];
  const int kk = blockIdx.x;
  for (int i0 = blockIdx.y * kLinRGDx; i0 < m; i0 += kLinRGDx * gridDim.y) {
    const int mr = min(kLinRGDx, m - i0);
    float acc[kLinRGDx];
#pragma unroll
    for (int i = 0; i < kLinRGDx; ++i) acc[i] = 0.f;
    for (int c0 = 0; c0 < n; c0 += kLinRedThreads * kLinUnroll) {
      float wv[kLinUnroll];
#pragma unroll
      for (int u = 0; u < kLinUnroll; ++u) {
        const int c = c0 + u * kLinRedThreads + threadIdx.x;
        wv[u] = c < n ? w[(long)c * k + kk] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < kLinRGDx; ++i) {
        const float* dr = dy + (long)(i0 + min(i, mr - 1)) * n;
        float dv[kLinUnroll];
#pragma unroll
        for (int u = 0; u < kLinUnroll; ++u) {
          const int c = c0 + u * kLinRedThreads + threadIdx.x;
          dv[u] = c < n ? dr[c] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kLinUnroll; ++u) acc[i] = fmaf(dv[u], wv[u], acc[i]);
      }
    }
    float r = block_rows_sum<kLinRGDx>(acc, sh);
    if (threadIdx.x < mr) {
      const long o = (long)(i0 + threadIdx.x) * k + kk;
      if (elu_y) r *= elu_grad_from_out(elu_y[o]);
      dx[o] = accumulate ? dx[o] + r : r;
    }
  }
}

// dw[n,k] = sum_i dy[i,n] x[i,k], db[n] = sum_i dy[i,n]: block row n =
// blockIdx.y (dy[., n] wave-uniform -> scalar loads), thread per k
// (coalesced x loads), the m terms unrolled by 16 so their loads overlap.
__device__ __forceinline__ void linear_dw_body(int bx, int nn, const float* __restrict__ x,
                                               const float* __restrict__ dy,
                                               float* __restrict__ dw, float* __restrict__ db,
                                               int m, int k, int n) {
  const int kk = bx * blockDim.x + threadIdx.x;
  if (dw && kk < k) {
    float s = 0.f;
    int i = 0;
    for (; i + 16 <= m; i += 16) {
      float xv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) xv[j] = x[(long)(i + j) * k + kk];
#pragma unroll
      for (int j = 0; j < 16; ++j) s = fmaf(dy[(long)(i + j) * n + nn], xv[j], s);
    }
    for (; i < m; ++i) s = fmaf(dy[(long)i * n + nn], x[(long)i * k + kk], s);
    dw[(long)nn * k + kk] = s;
  }
  if (db && bx == 0 && threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < m; ++i) s += dy[(long)i * n + nn];
    db[nn] = s;
  }
}
__global__ __launch_bounds__(256) void linear_dw_k(const float* __restrict__ x,
                                                   const float* __restrict__ dy,
                                                   float* __restrict__ dw,
                                                   float* __restrict__ db, int m, int k, int n) {
  linear_dw_body(blockIdx.x, blockIdx.y, x, dy, dw, db, m, k, n);
}

// dx and dW of one Linear in ONE launch (independent halves; the horizontal
// fusion saves a dependent kernel boundary): blocks [0, ndx) run the dx body
// (dx_nsmall), the rest the dW body.
constexpr int kLinSplitN = 64;   // rows of W per dx-partial block
constexpr int kLinSplitK = 128;  // max Linear input width of the split dx
constexpr int kLinSplitM = 16;   // max batch of the split dx
// Decoder-Linear backward, one launch of two block kinds:
//  * blocks [0, ndx): 64-row slices of W ([n][k] row-major, rows contiguous),
//    W slice + dy's columns staged in LDS with coalesced loads (the
//    column-per-block nred kernel read W in 4-B pieces at a k-float stride):
//    dx partial parts[p][i][kk] = sum_{c in slice p} dy[i][c] w[c][kk] (c ascending);
//  * the rest: 16 rows c of dW per block, dw[c][kk] = sum_i dy[i][c] x[i][kk],
//    db[c] = sum_i dy[i][c] (i ascending), dy's columns and x staged in LDS.
constexpr int kLinDwRows = 16;
// global -> LDS copy of n floats, 8 loads per thread in flight per batch (a
// load -> store loop exposes one memory latency per element)
__device__ __forceinline__ void stage_lds(const float* __restrict__ src, float* dst, int n) {
  constexpr int B = 8;
  for (int e0 = threadIdx.x; e0 < n; e0 += B * (int)blockDim.x) {
    float v[B];
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int e = e0 + j * (int)blockDim.x;
      v[j] = src[e < n ? e : n - 1];
    }
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int e = e0 + j * (int)blockDim.x;
      if (e < n) dst[e] = v[j];
    }
  }
}
__global__ __launch_bounds__(256) void linear_bwd_split_k(const float* __restrict__ x,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ dy,
                                                          float* __restrict__ parts,
                                                          float* __restrict__ dw,
                                                          float* __restrict__ db, int m, int k,
                                                          int n, int ndx) {
  __shared__ float wl[kLinSplitN * kLinSplitK];
  __shared__ float dl[kLinSplitM * kLinSplitN];
  const int bid = blockIdx.x;
  if (bid < ndx) {
    const int c0 = bid * kLinSplitN, nc = min(kLinSplitN, n - c0);
    stage_lds(w + (long)c0 * k, wl, nc * k);
    for (int e = threadIdx.x; e < m * kLinSplitN; e += blockDim.x) {
      const int i = e / kLinSplitN, c = e % kLinSplitN;
      dl[e] = c < nc ? dy[(long)i * n + c0 + c] : 0.f;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < m * k; e += blockDim.x) {
      const int i = e / k, kk = e % k;
      float acc = 0.f;
      for (int c = 0; c < nc; ++c) acc = fmaf(dl[i * kLinSplitN + c], wl[c * k + kk], acc);
      parts[(long)bid * m * k + e] = acc;
    }
    return;
  }
  float* xl = wl;  // [m][k]
  const int c0 = (bid - ndx) * kLinDwRows, nc = min(kLinDwRows, n - c0);
  stage_lds(x, xl, m * k);
  for (int e = threadIdx.x; e < m * kLinDwRows; e += blockDim.x) {
    const int i = e / kLinDwRows, c = e % kLinDwRows;
    dl[e] = c < nc ? dy[(long)i * n + c0 + c] : 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nc * k; e += blockDim.x) {
    const int c = e / k, kk = e % k;
    float acc = 0.f;
    for (int i = 0; i < m; ++i) acc = fmaf(dl[i * kLinDwRows + c], xl[i * k + kk], acc);
    dw[(long)c0 * k + e] = acc;
  }
  for (int c = threadIdx.x; c < nc; c += blockDim.x) {
    float acc = 0.f;
    for (int i = 0; i < m; ++i) acc += dl[i * kLinDwRows + c];
    db[c0 + c] = acc;
  }
}
__global__ __launch_bounds__(256) void linear_bwd_pair_k(const float* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ dy,
                                                         const float* __restrict__ elu_y,
                                                         float* __restrict__ dx,
                                                         float* __restrict__ dw,
                                                         float* __restrict__ db, int m, int k,
                                                         int n, int accumulate, int ndx_x,
                                                         int ndx, int ndw_x) {
  const int bid = blockIdx.x;
  if (bid < ndx) {
    linear_dx_nsmall_body(bid % ndx_x, bid / ndx_x, dy, w, elu_y, dx, m, k, n, accumulate);
  } else {
    const int j = bid - ndx;
    linear_dw_body(j % ndw_x, j / ndw_x, x, dy, dw, db, m, k, n);
  }
}

// ----------------------------------------------------------- bottleneck backward, one launch
// The step's bottleneck backward -- Pool(up)^T of the coarsest Deblock
// (model.py:172-173), the decoder Linear's dW/db/dz (:167-168), the latent
// head (:184-188) and the stacked encoder Linear's dx/dW/db (:158-160) -- as
// ONE launch of five workgroup roles instead of four launches (spmm_sched_csr,
// linear_bwd_split, latent_bwd, linear_bwd_pair):
//   A  [0, ndx_d)            decoder-Linear dz partials of one 64-row W slice;
//                             its dy slice (= one coarse vertex of dh) folded
//                             from the fine gradient on the fly (no dh round trip)
//   L  next nb_lat           latent head: waits for every A, then dmulv
//   D  next ndw_d            decoder-Linear dW/db rows (dy folded the same way)
//   E  next ndx_e + ndw_e    encoder-Linear dx / dW (8 rows per workgroup);
//                             each loads its W / x operands, then waits for L
// A waiting workgroup only waits for workgroups of LOWER index, which the
// dispatcher places first on every XCD, so the lowest unfinished workgroup can
// always run: no deadlock for any residency.  Writers arrive with an
// agent-scope release (L2 writeback: the partials / dmulv reach memory);
// waiters poll relaxed and then read with plain loads (see bn_ld); the last
// L workgroup raises one flag per E group and the E workgroups count
// themselves out in two levels, the last one zeroing every counter, so graph
// replays and eager calls start from zero.  A wait gives up after ~2^20 polls
// and raises a sticky bit in sync[kBnSyncErr] (the host checks it: a broken
// launch fails loudly instead of training on garbage, and never hangs the GPU).
// Exchanged values travel through `exchange` in LINE-EXCLUSIVE layout: every
// 128-B line of it is written by exactly one workgroup (A: its partials at a
// 32-float-aligned stride; L: whole dmulv rows at a 32-float-aligned stride),
// so no L2 ever holds a partial copy of a line another XCD writes, and a
// reader's L2 can only hold a line its own XCD wrote completely.  Every value
// is formed by the same per-element operations in the same order as the four
// launches: bit-identical (GPU-tested).  Per-workgroup timestamps (round 5):
// A 0-11.7 us, L 12.1-15.9, E 16.3-21.4; the four launches take ~29 us.
// Measured on the way (each fixed): acquiring polls 173 us, an acq_rel
// done-count 44 us, one shared done-counter 33 us, uncached exchanged loads
// ~29 us, one acquire per waiting workgroup ~20 us.
struct BneckArgs {
  const int* up_ptr;  // CSR of Pool(up)^T, rows = coarse vertices (plain per-row order)
  const int* up_col;
  const float* up_val;
  const float* g;  // fine-level gradient [m][n_up][cup], batch-major
  int n_up, cup;
  const float* z;  // decoder Linear: z [m][kd], W_d [nd][kd] (nd = coarse vertices x cup)
  const float* wd;
  float* parts;  // exchange: [ndx_d][pstride], pstride = m x kd rounded up to 32 floats
  float* dwd;
  float* dbd;
  int m, kd, nd, ndx_d, ndw_d;
  const float* mulv;  // latent head (latent_bwd_k's operands)
  const float* eps;
  const float* dlat;
  float* dmulv;
  const float* zval;
  int L, train, is_vae, sigmoid, nb_lat, lat_rows;  // L workgroup = lat_rows whole rows of dmulv
  float* xdmulv;  // exchange: [m][dstride], dstride = ne rounded up to 32 floats
  int pstride, dstride;
  const float* xe;  // encoder Linear: x_e [m][ke], W_e [ne][ke]
  const float* we;
  const float* elu_y;
  float* dxe;
  float* dwe;
  float* dbe;
  int ke, ne, accumulate, ndx_x, ndx_e, ndw_x, ndw_g;
  int* sync;  // kBnSyncInts counters, one 128-B line each: A done, L done, E groups done, E done per group
};
constexpr int kBnSyncLine = 32;  // ints per 128-B line
constexpr int kBnGroups = 8;
constexpr int kBnSyncA = 0, kBnSyncL = kBnSyncLine, kBnSyncTop = 2 * kBnSyncLine, kBnSyncSub = 3 * kBnSyncLine;
constexpr int kBnSyncFlag = kBnSyncSub + kBnGroups * kBnSyncLine;  // L-done flag per E group
constexpr int kBnSyncErr = kBnSyncTop + 1;  // sticky: bit r set when a role-r wait timed out (host-checked)
static_assert(kBnSyncFlag + kBnGroups * kBnSyncLine == 608, "cfsd.h documents 608 sync ints");
static_assert(kBnSyncErr == CFSD_BN_SYNC_ERR, "cfsd.h documents the error word");
constexpr int kBnDwRows = 4;  // encoder dW rows per E workgroup (x loaded once for all of them)
constexpr int kBnWPer = kLinSplitN * kLinSplitK / 256;  // W-slice floats per thread of an A workgroup
constexpr int kBnMaxParts = 80;                          // decoder-Linear partials (nd <= 80 x 64)
constexpr int kBnWT = kLinSplitN + 4;  // row stride of the A role's transposed W slice (16-B aligned rows)

__device__ __forceinline__ void bn_arrive(int* ctr) {
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
// relaxed polls (an acquiring poll invalidates the XCD's L2 every time: the
// waiting workgroups then evict the running ones' operands -- 173 vs ~20 us)
// A wait that gives up sets `code` in the sticky error word (never cleared by
// the kernel): the launch then returns wrong values, which the host refuses.
__device__ __forceinline__ void bn_wait(int* ctr, int target, int* err, int code) {
  if (threadIdx.x == 0) {
    bool seen = false;
    for (int it = 0; it < (1 << 20) && !seen; ++it) {
      seen = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
      if (!seen) __builtin_amdgcn_s_sleep(8);
    }
    if (!seen) __hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
}
// The exchanged values (dz partials, dmulv) are read with plain, L2-cached
// loads after the counter / flag is seen.  No line of them can be stale in a
// reader's L2: every dispatch starts with the caches invalidated, nothing
// reads them in this launch before the writers' release (an L2 writeback),
// each exchange line has ONE writer workgroup (no XCD holds a partial copy
// of a line another XCD writes), and the writer's own XCD keeps its written
// (then clean) lines.  Acquiring
// each wait instead (an L2 invalidate by each of ~600 workgroups) cost ~20
// us, and agent-scope atomic loads (uncached) of the 9.6-KB dmulv by every E
// workgroup put ~12k requests on a handful of lines (~15 us).
__device__ __forceinline__ float bn_ld(const float* p) { return *p; }

// dst[i * ds + c] = dh[i][c0 + c], c < nc (nc <= cup, inside one coarse vertex):
// the transposed Pool's sequential fold of spmm_fold_prefetch (acc = acc +
// x * v over the row's entries in order, contraction off).
// The row (one coarse vertex: workgroup-uniform) is read ONCE per wave -- lane
// e holds entry e's column / value (bn_fold_row, issued before the caller
// parks its own operands), read back by v_readlane -- so the x gathers of 16
// entries at a time depend on that one load only.  The per-8-entry
// column -> x round trips of the plain walk (up to 9 dependent trips for the
// 29-entry rows at level 3) were the A role's critical path.
constexpr int kBnFoldLanes = 64;  // longest row held in one wave's lanes (level 3: 29)
constexpr int kBnFoldBatch = 16;  // x gathers in flight per thread
struct BnRow {
  int beg, n, col;
  float val;
};
__device__ __forceinline__ BnRow bn_fold_row(const BneckArgs& a, int c0) {
  const int v = c0 / a.cup;
  BnRow r;
  r.beg = a.up_ptr[v];
  r.n = a.up_ptr[v + 1] - r.beg;
  const int lane = threadIdx.x & 63;
  const bool in = lane < r.n && r.n <= kBnFoldLanes;
  r.col = in ? a.up_col[r.beg + lane] : 0;
  r.val = in ? a.up_val[r.beg + lane] : 0.f;
  return r;
}
__device__ __forceinline__ void bn_fold_dh(const BneckArgs& a, const BnRow& r, int c0, int nc, float* dst, int ds) {
#pragma clang fp contract(off)
  const int v = c0 / a.cup, ch0 = c0 - v * a.cup, q4 = nc / 4;
  if (r.n <= kBnFoldLanes) {
    for (int t = threadIdx.x; t < a.m * q4; t += blockDim.x) {
      const int i = t / q4, q = t - i * q4;
      const float* xb = a.g + (long)i * a.n_up * a.cup + ch0 + 4 * q;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int e0 = 0; e0 < r.n; e0 += kBnFoldBatch) {  // uniform
        f32x4 xv[kBnFoldBatch];
#pragma unroll
        for (int j = 0; j < kBnFoldBatch; ++j) {
          const int e = min(e0 + j, r.n - 1);
          xv[j] = ld4(xb + (long)__builtin_amdgcn_readlane(r.col, e) * a.cup);
        }
#pragma unroll
        for (int j = 0; j < kBnFoldBatch; ++j) {
          if (e0 + j < r.n) {
            const float vv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, r.val), e0 + j));
            acc.x = acc.x + xv[j].x * vv;
            acc.y = acc.y + xv[j].y * vv;
            acc.z = acc.z + xv[j].z * vv;
            acc.w = acc.w + xv[j].w * vv;
          }
        }
      }
      st4(dst + i * ds + 4 * q, acc);
    }
    return;
  }
  const int beg = r.beg, end = r.beg + r.n;  // (rows longer than a wave: the plain walk)
  for (int t = threadIdx.x; t < a.m * q4; t += blockDim.x) {
    const int i = t / q4, q = t - i * q4;
    const float* xb = a.g + (long)i * a.n_up * a.cup + ch0 + 4 * q;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int e0 = beg; e0 < end; e0 += 8) {
      f32x4 xv[8];
      float vv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = min(e0 + j, end - 1);
        xv[j] = ld4(xb + (long)a.up_col[e] * a.cup);
        vv[j] = a.up_val[e];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (e0 + j < end) {
          acc.x = acc.x + xv[j].x * vv[j];
          acc.y = acc.y + xv[j].y * vv[j];
          acc.z = acc.z + xv[j].z * vv[j];
          acc.w = acc.w + xv[j].w * vv[j];
        }
      }
    }
    st4(dst + i * ds + 4 * q, acc);
  }
}

#ifdef CFSD_BN_STAMPS
// diagnostic build only (tools/kbench.py KB_BNSTAMPS): per-workgroup role,
// start, two phase marks and end times (wall_clock64, 100 MHz)
__device__ unsigned long long g_bn_stamps[4096 * 5];
#define BN_T0 const unsigned long long bn_t0 = wall_clock64(); unsigned long long bn_t1 = bn_t0, bn_t2 = 0;
#define BN_T1 bn_t1 = wall_clock64();
#define BN_T2 bn_t2 = wall_clock64();
#define BN_OUT(role) \
  if (threadIdx.x == 0 && bid < 4096) { \
    g_bn_stamps[5 * bid] = role; g_bn_stamps[5 * bid + 1] = bn_t0; g_bn_stamps[5 * bid + 2] = bn_t1; \
    g_bn_stamps[5 * bid + 3] = bn_t2 ? bn_t2 : bn_t1; g_bn_stamps[5 * bid + 4] = wall_clock64(); }
extern "C" int cfsd_debug_bn_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bn_stamps), sizeof(g_bn_stamps), 0, hipMemcpyDeviceToHost);
}
#else
#define BN_T0
#define BN_T1
#define BN_T2
#define BN_OUT(role)
#endif
__global__ __launch_bounds__(256) void bottleneck_bwd_k(const BneckArgs a) {
  extern __shared__ float bn_lds[];
  const int bid = blockIdx.x;
  BN_T0
  const int b_lat = a.ndx_d, b_dwd = b_lat + a.nb_lat, b_enc = b_dwd + a.ndw_d;
  const int n_enc = a.ndx_e + a.ndw_x * a.ndw_g;
  const int m = a.m;
  if (bid < b_lat) {  // A: parts[bid][i][kk] = sum_{c in slice} dy[i][c] W_d[c][kk]
    float* wt = bn_lds;                      // W slice transposed: [kd][kBnWT] (c contiguous)
    float* dl = bn_lds + kBnWT * a.kd;       // [m][64]
    const int c0 = bid * kLinSplitN, nc = kLinSplitN;  // (nd % 64 == 0: whole slices, host-checked)
    // the W slice's loads go out first and land while the dh fold's own
    // gathers are in flight (one memory round trip for both, not 3 + 2)
    const float* ws = a.wd + (long)c0 * a.kd;
    const int nw = nc * a.kd;
    float wv[kBnWPer];
#pragma unroll
    for (int j = 0; j < kBnWPer; ++j) {
      const int e = j * 256 + (int)threadIdx.x;
      wv[j] = e < nw ? ws[e] : 0.f;
    }
    const BnRow row = bn_fold_row(a, c0);
    // (the W slice is parked while the row's column / value loads land; its
    // registers are free again before the gathers)
#pragma unroll
    for (int j = 0; j < kBnWPer; ++j) {
      const int e = j * 256 + (int)threadIdx.x;
      if (e < nw) {
        const int c = e / a.kd;
        wt[(e - c * a.kd) * kBnWT + c] = wv[j];
      }
    }
    bn_fold_dh(a, row, c0, nc, dl, kLinSplitN);
    __syncthreads();
    BN_T1
    // register blocks of 4 meshes x 2 columns: per 4 terms c, four 16-B dl
    // reads and two 16-B W reads feed 32 fmaf (one 64-term LDS chain per
    // output with two 4-B reads per fmaf took ~5 us); per output the same
    // fmaf chain over c ascending as linear_bwd_split_k
    const int nkp = (a.kd + 1) / 2, nblk = ((m + 3) / 4) * nkp;
    for (int t = threadIdx.x; t < nblk; t += blockDim.x) {
      const int ib = t / nkp, kp = t - ib * nkp;
      const int i0 = ib * 4, k0 = 2 * kp, k1 = min(k0 + 1, a.kd - 1);
      float acc[4][2];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r][0] = acc[r][1] = 0.f;
#pragma unroll 2
      for (int c = 0; c < kLinSplitN; c += 4) {
        f32x4 d[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r] = ld4(dl + min(i0 + r, m - 1) * kLinSplitN + c);
        const f32x4 w0 = ld4(wt + k0 * kBnWT + c), w1 = ld4(wt + k1 * kBnWT + c);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc[r][0] = fmaf(d[r][q], w0[q], acc[r][0]);
            acc[r][1] = fmaf(d[r][q], w1[q], acc[r][1]);
          }
      }
      float* pp = a.parts + (long)bid * a.pstride;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (i0 + r < m) {
          pp[(i0 + r) * a.kd + k0] = acc[r][0];
          if (k0 + 1 < a.kd) pp[(i0 + r) * a.kd + k0 + 1] = acc[r][1];
        }
    }
    BN_T2
    bn_arrive(a.sync + kBnSyncA);
    BN_OUT(0)
    return;
  }
  if (bid < b_dwd) {  // L: latent_bwd_k's per-element arithmetic, lat_rows whole dmulv rows per workgroup
    bn_wait(a.sync + kBnSyncA, a.ndx_d, a.sync + kBnSyncErr, 1);
    BN_T1
    const int B = m, L = a.L;
    const int i = (bid - b_lat) * a.lat_rows + (int)threadIdx.x / L, l = (int)threadIdx.x % L;
    if ((int)threadIdx.x < a.lat_rows * L && i < B) {
      const int e = i * L + l;
      // every partial in flight at once (one round trip; 16-load batches were
      // 5 trips, 4.5 us), then summed in part order as latent_bwd_k
      float t[kBnMaxParts];
#pragma unroll
      for (int j = 0; j < kBnMaxParts; ++j) t[j] = bn_ld(a.parts + (long)min(j, a.ndx_d - 1) * a.pstride + e);
      float dzd = t[0];
#pragma unroll
      for (int j = 1; j < kBnMaxParts; ++j)
        if (j < a.ndx_d) dzd += t[j];
      const float dz = dzd + a.dlat[i * 3 * L + l];
      float* xr = a.xdmulv + (long)i * a.dstride;  // this workgroup's own lines
      if (a.is_vae) {
        const float lv = a.mulv[i * 2 * L + l];
        const float dmu = dz + a.dlat[i * 3 * L + L + l];
        float dlv = a.dlat[i * 3 * L + 2 * L + l];
        if (a.train) dlv += dz * a.eps[e] * 0.5f * expf(0.5f * lv);
        xr[l] = dlv;
        xr[L + l] = dmu;
        a.dmulv[i * 2 * L + l] = dlv;  // the caller's copy (not read in this launch)
        a.dmulv[i * 2 * L + L + l] = dmu;
      } else {
        float dmu = dz;
        if (a.sigmoid) dmu *= a.zval[e] * (1.f - a.zval[e]);
        xr[l] = dmu;
        a.dmulv[i * L + l] = dmu;
      }
    }
    // the last L workgroup raises one flag per E group (the E workgroups poll
    // their group's line, not one shared address)
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(a.sync + kBnSyncL, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) == a.nb_lat - 1) {
      // only groups with members: an empty group's flag would never be reset
      for (int g = 0; g < kBnGroups && g < n_enc; ++g)
        __hip_atomic_store(a.sync + kBnSyncFlag + kBnSyncLine * g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    BN_OUT(1)
    return;
  }
  if (bid < b_enc) {  // D: dW_d / db_d rows c0 .. c0 + 15 (linear_bwd_split_k's dW body)
    float* xl = bn_lds;              // [m][kd]
    float* dl = bn_lds + m * a.kd;   // [m][16]
    const int c0 = (bid - b_dwd) * kLinDwRows, nc = min(kLinDwRows, a.nd - c0);
    const BnRow row = bn_fold_row(a, c0);
    stage_lds(a.z, xl, m * a.kd);
    bn_fold_dh(a, row, c0, nc, dl, kLinDwRows);
    __syncthreads();
    BN_T1
    for (int e = threadIdx.x; e < nc * a.kd; e += blockDim.x) {
      const int c = e / a.kd, kk = e % a.kd;
      float acc = 0.f;
      for (int i = 0; i < m; ++i) acc = fmaf(dl[i * kLinDwRows + c], xl[i * a.kd + kk], acc);
      a.dwd[(long)c0 * a.kd + e] = acc;
    }
    for (int c = threadIdx.x; c < nc; c += blockDim.x) {
      float acc = 0.f;
      for (int i = 0; i < m; ++i) acc += dl[i * kLinDwRows + c];
      a.dbd[c0 + c] = acc;
    }
    BN_OUT(2)
    return;
  }
  // E: encoder Linear, operands loaded before the wait for dmulv
  const int ej = bid - b_enc;
  const int n = a.ne, k = a.ke;
  if (ej < a.ndx_e) {  // dx: linear_dx_nsmall_body (row quad by, 64 k-columns bx)
    const int bx = ej % a.ndx_x, by = ej / a.ndx_x;
    float* ds = bn_lds;                  // [4][n]
    float* part = bn_lds + 4 * n;        // [4 waves][4 rows][64]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i0 = by * 4, mr = min(4, m - i0);
    const int kk = bx * 64 + lane;
    const int kc = kk < k ? kk : k - 1;
    const int per = (n + 3) / 4, c0 = wave * per, c1 = min(n, c0 + per);
    // the wave's whole c-range is one kLinDxChunk chunk (n <= 4 x 40, checked
    // by the host): its W column loads are in flight while this workgroup waits
    float wv[kLinDxChunk];
#pragma unroll
    for (int u = 0; u < kLinDxChunk; ++u) wv[u] = c0 + u < c1 ? a.we[(long)(c0 + u) * k + kc] : 0.f;
    bn_wait(a.sync + kBnSyncFlag + kBnSyncLine * (ej % kBnGroups), 1, a.sync + kBnSyncErr, 2);
    BN_T1
    for (int e = threadIdx.x; e < mr * n; e += blockDim.x)
      ds[e] = bn_ld(a.xdmulv + (long)(i0 + e / n) * a.dstride + e % n);
    __syncthreads();
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < kLinDxChunk; ++u) {
      const int c = min(c0 + u, n - 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = fmaf(ds[i * n + c], wv[u], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) part[(wave * 4 + i) * 64 + lane] = acc[i];
    __syncthreads();
    if (wave < mr && kk < k) {
      const int i = wave;
      float v = part[(0 * 4 + i) * 64 + lane] + part[(1 * 4 + i) * 64 + lane] + part[(2 * 4 + i) * 64 + lane] +
                part[(3 * 4 + i) * 64 + lane];
      const long o = (long)(i0 + i) * k + kk;
      if (a.elu_y) v *= elu_grad_from_out(a.elu_y[o]);
      a.dxe[o] = a.accumulate ? a.dxe[o] + v : v;
    }
  } else {  // dW rows nn0 .. nn0 + 7 over the 256 k-columns bx (linear_dw_body per row), db by bx == 0
    const int j = ej - a.ndx_e, bx = j % a.ndw_x, nn0 = (j / a.ndw_x) * kBnDwRows;
    const int kk = bx * blockDim.x + threadIdx.x;
    const bool on = kk < k;
    float xv[kLinSplitM];
#pragma unroll
    for (int i = 0; i < kLinSplitM; ++i) xv[i] = (on && i < m) ? a.xe[(long)i * k + kk] : 0.f;
    bn_wait(a.sync + kBnSyncFlag + kBnSyncLine * (ej % kBnGroups), 1, a.sync + kBnSyncErr, 4);
    BN_T1
    // the block's dmulv columns [m][8] in ONE round of vector loads (per-row
    // scalar loads were 8 dependent trips to memory: 40 us for this phase)
    float* dl = bn_lds;  // [m][kBnDwRows]
    if ((int)threadIdx.x < m * kBnDwRows) {
      const int i = threadIdx.x / kBnDwRows, r = threadIdx.x % kBnDwRows;
      dl[threadIdx.x] = nn0 + r < n ? bn_ld(a.xdmulv + (long)i * a.dstride + nn0 + r) : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < kBnDwRows; ++r) {
      const int nn = nn0 + r;
      if (nn >= n) break;
      if (on) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < kLinSplitM; ++i)
          if (i < m) s = fmaf(dl[i * kBnDwRows + r], xv[i], s);
        a.dwe[(long)nn * k + kk] = s;
      }
      if (bx == 0 && threadIdx.x == 0) {
        float s = 0.f;
        for (int i = 0; i < m; ++i) s += dl[i * kBnDwRows + r];
        a.dbe[nn] = s;
      }
    }
  }
  BN_OUT(ej < a.ndx_e ? 3 : 4)
  // the last E workgroup resets the counters for the next launch.  Counted in
  // two levels (8 group counters on their own cache lines, then one top
  // counter): 591 RMWs on ONE address serialise at its memory channel (the E
  // stage cost ~17 us that way).  Relaxed: a counting RMW needs no cache
  // maintenance (acq_rel is an L2 writeback + invalidate per workgroup).
  __syncthreads();
  if (threadIdx.x == 0) {
    const int grp = ej % kBnGroups, n_grp = n_enc < kBnGroups ? n_enc : kBnGroups;
    const int quota = (n_enc - grp + kBnGroups - 1) / kBnGroups;
    int* sub = a.sync + kBnSyncSub + kBnSyncLine * grp;
    if (__hip_atomic_fetch_add(sub, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == quota - 1) {
      __hip_atomic_store(sub, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.sync + kBnSyncFlag + kBnSyncLine * grp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int* top = a.sync + kBnSyncTop;
      if (__hip_atomic_fetch_add(top, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_grp - 1) {
        __hip_atomic_store(a.sync + kBnSyncA, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.sync + kBnSyncL, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(top, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ----------------------------------------------------------- Adam
// Four elements per thread in 16-B accesses (the four state arrays are
// streamed once: 7 x 4 B per element of HBM traffic); the n % 4 tail goes to
// the last thread.  Same per-element arithmetic as a scalar loop.
// With `shadow` != NULL the updated parameters are also written as bf16 (the
// weights the bf16 kernels read: fp32 master + bf16 copy in one pass).
// SCALED (cfsd_adam_scaled, the data-parallel step): the gradient is first
// multiplied by gscale (1 / world after the all-reduce SUM) and written back,
// the same fp32 product cfsd_scale forms -- one launch instead of two.
template <bool SCALED>
__global__ __launch_bounds__(256) void adam_k(float* __restrict__ p, float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              const int* __restrict__ step, long n, float lr,
                                              float b1, float b2, float eps, float wd,
                                              bf16_t* __restrict__ shadow, float gscale) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x, n4 = n / 4;
  if (q > n4) return;
  const int t = *step;
  const float bc1 = 1.f - powf(b1, (float)t);
  const float sqrt_bc2 = sqrtf(1.f - powf(b2, (float)t));
  const float step_size = lr / bc1;
  if (q < n4) {
    const f32x4 pv = ld4(p + 4 * q), mv = ld4(m + 4 * q), vv = ld4(v + 4 * q), gv = ld4(g + 4 * q);
    float pa[4] = {pv.x, pv.y, pv.z, pv.w}, ma[4] = {mv.x, mv.y, mv.z, mv.w};
    float va[4] = {vv.x, vv.y, vv.z, vv.w};
    float ga[4] = {gv.x, gv.y, gv.z, gv.w};
    if constexpr (SCALED) {
#pragma unroll
      for (int j = 0; j < 4; ++j) ga[j] *= gscale;
      st4(g + 4 * q, f32x4{ga[0], ga[1], ga[2], ga[3]});
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) adam_elem(pa[j], ga[j], ma[j], va[j], b1, b2, eps, wd, step_size, sqrt_bc2);
    st4(p + 4 * q, f32x4{pa[0], pa[1], pa[2], pa[3]});
    if (shadow) st4f(shadow + 4 * q, f32x4{pa[0], pa[1], pa[2], pa[3]});
    st4(m + 4 * q, f32x4{ma[0], ma[1], ma[2], ma[3]});
    st4(v + 4 * q, f32x4{va[0], va[1], va[2], va[3]});
  } else {
    for (long i = 4 * n4; i < n; ++i) {
      float gi = g[i];
      if constexpr (SCALED) {
        gi *= gscale;
        g[i] = gi;
      }
      adam_elem(p[i], gi, m[i], v[i], b1, b2, eps, wd, step_size, sqrt_bc2);
      if (shadow) stf(shadow + i, p[i]);
    }
  }
}

// ----------------------------------------------------------- step bookkeeping
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

// Keyed permutation of [0, n): a 4-round Feistel network on the smallest
// even-bit power-of-two domain >= n, cycle-walked back into [0, n) (the
// orbit of an in-domain value re-enters the domain, so the walk ends).
// Replaces the host RandomSampler's torch.randperm of MeshLoader
// (data_loading.py:40-48, shuffle=True): every epoch gets a fresh order from
// (seed, epoch), drawn on the device so a graph replay needs no host input.
// Restated by oracle/cfsd_oracle.py:epoch_permutation (tests).
__device__ __forceinline__ uint32_t feistel_perm(uint32_t x, uint32_t n, uint64_t key) {
  int bits = 2;
  while ((1u << bits) < n) bits += 2;
  const int h = bits / 2;
  const uint32_t mask = (1u << h) - 1u;
  do {
    uint32_t l = x >> h, r = x & mask;
#pragma unroll
    for (int round = 0; round < 4; ++round) {
      const uint32_t f = mix32(key + 0x9E3779B97F4A7C15ULL * (uint64_t)(round + 1) + r) & mask;
      const uint32_t nl = r;
      r = l ^ f;
      l = nl;
    }
    x = (l << h) | r;
  } while (x >= n);
  return x;
}

__global__ void step_begin_k(int* __restrict__ counter, unsigned long long seed,
                             float* __restrict__ eps, int n_eps, int* __restrict__ key,
                             int n_regions, int* __restrict__ batch_idx, int bs, int n_batches,
                             const int* __restrict__ perm, int n_items, int shuffle,
                             int* __restrict__ adam_step) {
  __shared__ int t_sh;
  if (threadIdx.x == 0) {
    t_sh = *counter + 1;
  }
  __syncthreads();
  const int t = t_sh;
  const uint64_t base = seed * 0x9E3779B97F4A7C15ULL + (uint64_t)t * 0x100000001B3ULL;
  if (threadIdx.x == 0) {
    if (key) *key = (int)(mix32(base ^ 0xABCDEFULL) % (uint32_t)n_regions);
  }
  if (batch_idx && (int)threadIdx.x < bs) {
    const int bt = (t - 1) % n_batches, epoch = (t - 1) / n_batches;
    int slot = bt * bs + threadIdx.x;
    if (shuffle) {
      const uint64_t ek = (seed ^ 0x5DEECE66DULL) * 0xD6E8FEB86659FD93ULL + (uint64_t)epoch;
      slot = (int)feistel_perm((uint32_t)slot, (uint32_t)n_items, ek);
    }
    batch_idx[threadIdx.x] = perm ? perm[slot] : slot;
  }
  if (eps) {
    for (int i = threadIdx.x; i < n_eps; i += blockDim.x) {  // Box-Muller
      const uint32_t a = mix32(base + 2ULL * i + 1), b = mix32(base + 2ULL * i + 2);
      const float u1 = ((a >> 8) + 1) * (1.0f / 16777217.0f);
      const float u2 = (b >> 8) * (1.0f / 16777216.0f);
      eps[i] = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    *counter = t;
    if (adam_step) *adam_step += 1;
  }
}

}  // namespace cfsd

using namespace cfsd;

extern "C" int cfsd_version(void) { return (4 << 16) | 12; }  // 4.12: cfsd_bottleneck_bwd exchange workspace + sticky error word; 4.11: cfsd_spiral_conv_bwd_flat_pair_bf16, cfsd_spiral_conv_bwd_rowsub_pair_bf16; 4.10: cfsd_spiral_conv_bwd_flat_pair; 4.9: cfsd_spiral_conv_fwd_in_swap; 4.8: cfsd_bottleneck_bwd; 4.7: cfsd_adam_scaled; 4.6: cfsd_side_work (side work riding in host launches); 3.0: per-epoch shuffle, bf16 path; 3.1: row-subset backward; 3.2: uniform / visiting-order SpMM; 3.3: reduce + Adam; 4.0: CFSD_VM vertex-major operands (dx_dt / dpre_dt arguments); 4.1: fp32 vertex-major operands; 4.2: vertex-major swap / loss passes (_x); 4.3: cfsd_dw_slabs.fused == 3 (vertex-major fp32 dW slabs); 4.4: cfsd_gather_meshes
extern "C" const char* cfsd_last_error_string(void) { return g_err; }

extern "C" int cfsd_recon_lap_blocks(int batch, int nv) {
  const long total = (long)batch * nv;
  return (int)((total + kLapThreads - 1) / kLapThreads);
}

static int recon_lap_fwd_launch(const float* pred, const float* gt, const int32_t* l_ptr,
                                const int32_t* l_col, const float* l_val, float* unit_lx,
                                float* partials, int batch, int nv, int c, int vm, void* stream) {
  if (!pred || !gt || !l_ptr || !l_col || !l_val || !unit_lx || !partials)
    return set_error(CFSD_EINVAL, "recon_lap_fwd: null pointer");
  if (batch <= 0 || nv <= 0 || c <= 0 || c > 4) return set_error(CFSD_EINVAL, "recon_lap_fwd: bad sizes");
  if ((long)batch * nv * c >= (1L << 31)) return set_error(CFSD_EINVAL, "recon_lap_fwd: too large");
  const long total = (long)batch * nv;
  const dim3 grid(cfsd_recon_lap_blocks(batch, nv));
  const hipStream_t st = (hipStream_t)stream;
#define RLF(C)                                                                                  \
  case C:                                                                                       \
    hipLaunchKernelGGL(recon_lap_fwd_k<C>, grid, dim3(kLapThreads), 0, st, pred, gt, l_ptr, l_col, \
                       l_val, unit_lx, partials, nv, total, batch, vm);                         \
    break;
  switch (c) { RLF(1) RLF(2) RLF(3) RLF(4) }
#undef RLF
  return launch_status("recon_lap_fwd");
}

extern "C" int cfsd_recon_lap_fwd(const float* pred, const float* gt, const int32_t* l_ptr,
                                  const int32_t* l_col, const float* l_val, float* unit_lx,
                                  float* partials, int batch, int nv, int c, void* stream) {
  return recon_lap_fwd_launch(pred, gt, l_ptr, l_col, l_val, unit_lx, partials, batch, nv, c, 0, stream);
}

extern "C" int cfsd_recon_lap_fwd_x(const float* pred, const float* gt, const int32_t* l_ptr,
                                    const int32_t* l_col, const float* l_val, float* unit_lx,
                                    float* partials, int batch, int nv, int c, int dt, void* stream) {
  if ((dt & ~CFSD_VM) != CFSD_DT_F32) return set_error(CFSD_EINVAL, "recon_lap_fwd_x: bad dtype %d", dt);
  return recon_lap_fwd_launch(pred, gt, l_ptr, l_col, l_val, unit_lx, partials, batch, nv, c,
                              (dt & CFSD_VM) != 0, stream);
}

static int recon_lap_bwd_launch(const float* pred, const float* gt, const float* unit_lx,
                                const int32_t* lt_ptr, const int32_t* lt_col, const float* lt_val,
                                float* dpred, int batch, int nv, int c, float w_rec, float w_lap,
                                const LossFinalize& fin, int vm, void* stream) {
  if (!pred || !gt || !unit_lx || !lt_ptr || !lt_col || !lt_val || !dpred)
    return set_error(CFSD_EINVAL, "recon_lap_bwd: null pointer");
  if (batch <= 0 || nv <= 0 || c <= 0 || c > 4) return set_error(CFSD_EINVAL, "recon_lap_bwd: bad sizes");
  if ((long)batch * nv * c >= (1L << 31)) return set_error(CFSD_EINVAL, "recon_lap_bwd: too large");
  const long total = (long)batch * nv;
  const float k_rec = w_rec * 2.f / (float)(total * c);
  const float k_lap = w_lap / (float)((long)nv * batch);
  const dim3 grid((unsigned)((total + 255) / 256));
  const hipStream_t st = (hipStream_t)stream;
#define RLB(C)                                                                                   \
  case C:                                                                                        \
    hipLaunchKernelGGL(recon_lap_bwd_k<C>, grid, dim3(256), 0, st, pred, gt, unit_lx, lt_ptr,    \
                       lt_col, lt_val, dpred, nv, total, k_rec, k_lap, fin, batch, vm);         \
    break;
  switch (c) { RLB(1) RLB(2) RLB(3) RLB(4) }
#undef RLB
  return launch_status("recon_lap_bwd");
}

extern "C" int cfsd_recon_lap_bwd(const float* pred, const float* gt, const float* unit_lx,
                                  const int32_t* lt_ptr, const int32_t* lt_col,
                                  const float* lt_val, float* dpred, int batch, int nv, int c,
                                  float w_rec, float w_lap, void* stream) {
  const LossFinalize none{};  // losses finalised by cfsd_loss_finalize
  return recon_lap_bwd_launch(pred, gt, unit_lx, lt_ptr, lt_col, lt_val, dpred, batch, nv, c, w_rec,
                              w_lap, none, 0, stream);
}

extern "C" int cfsd_recon_lap_bwd_x(const float* pred, const float* gt, const float* unit_lx,
                                    const int32_t* lt_ptr, const int32_t* lt_col,
                                    const float* lt_val, float* dpred, int batch, int nv, int c,
                                    float w_rec, float w_lap, int dt, void* stream) {
  if ((dt & ~CFSD_VM) != CFSD_DT_F32) return set_error(CFSD_EINVAL, "recon_lap_bwd_x: bad dtype %d", dt);
  const LossFinalize none{};
  return recon_lap_bwd_launch(pred, gt, unit_lx, lt_ptr, lt_col, lt_val, dpred, batch, nv, c, w_rec,
                              w_lap, none, (dt & CFSD_VM) != 0, stream);
}

static int recon_lap_bwd_fin(const float* pred, const float* gt, const float* unit_lx, const int32_t* lt_ptr,
                             const int32_t* lt_col, const float* lt_val, float* dpred, int batch, int nv, int c,
                             float w_rec, float w_lap, const float* partials, int nblocks, const float* terms,
                             float* out, float* acc, float w_kl, float w_lc, int vm, void* stream) {
  if (!partials || !terms || !out) return set_error(CFSD_EINVAL, "recon_lap_bwd_finalize: null pointer");
  if (batch <= 0 || nv <= 0 || c <= 0) return set_error(CFSD_EINVAL, "recon_lap_bwd_finalize: bad sizes");
  const LossFinalize fin{partials, nblocks, terms, out, acc, 1.f / (float)((long)batch * nv * c),
                         1.f / (float)((long)nv * batch), w_kl, w_lc, w_lap};
  return recon_lap_bwd_launch(pred, gt, unit_lx, lt_ptr, lt_col, lt_val, dpred, batch, nv, c, w_rec,
                              w_lap, fin, vm, stream);
}

extern "C" int cfsd_recon_lap_bwd_finalize(const float* pred, const float* gt, const float* unit_lx,
                                           const int32_t* lt_ptr, const int32_t* lt_col,
                                           const float* lt_val, float* dpred, int batch, int nv,
                                           int c, float w_rec, float w_lap, const float* partials,
                                           int nblocks, const float* terms, float* out, float* acc,
                                           float w_kl, float w_lc, void* stream) {
  return recon_lap_bwd_fin(pred, gt, unit_lx, lt_ptr, lt_col, lt_val, dpred, batch, nv, c, w_rec, w_lap,
                           partials, nblocks, terms, out, acc, w_kl, w_lc, 0, stream);
}

extern "C" int cfsd_recon_lap_bwd_finalize_x(const float* pred, const float* gt, const float* unit_lx,
                                             const int32_t* lt_ptr, const int32_t* lt_col,
                                             const float* lt_val, float* dpred, int batch, int nv,
                                             int c, float w_rec, float w_lap, const float* partials,
                                             int nblocks, const float* terms, float* out, float* acc,
                                             float w_kl, float w_lc, int dt, void* stream) {
  if ((dt & ~CFSD_VM) != CFSD_DT_F32)
    return set_error(CFSD_EINVAL, "recon_lap_bwd_finalize_x: bad dtype %d", dt);
  return recon_lap_bwd_fin(pred, gt, unit_lx, lt_ptr, lt_col, lt_val, dpred, batch, nv, c, w_rec, w_lap,
                           partials, nblocks, terms, out, acc, w_kl, w_lc, (dt & CFSD_VM) != 0, stream);
}

// LDS floats of the latent head (z + pair distances) for one workgroup
static size_t latent_lds_floats(int batch, int latent, int bs) {
  return (size_t)batch * latent + (size_t)4 * (bs * (bs - 1) / 2) * bs;
}
constexpr size_t kLatLdsMax = 160 * 1024 - 1024;  // minus the static reduction array

// Checks the latent head's arguments and sizes its dynamic LDS (z and the
// pair distances of one workgroup, up to 160 KB: e.g. batch 256 = 16^2 at
// latent 75 takes 105 KB); raises the kernel's dynamic-LDS limit when needed.
static int latent_prepare(const char* name, const void* kernel, const float* mulv, const float* eps,
                          const int32_t* key, float* z, float* dlat, float* terms, int batch,
                          int latent, int region_size, int train, int is_vae, float w_lc,
                          size_t extra_lds, int& bs, size_t& lds) {
  if (!mulv || !z || !dlat || !terms) return set_error(CFSD_EINVAL, "%s: null pointer", name);
  if (is_vae && train && !eps) return set_error(CFSD_EINVAL, "%s: eps required", name);
  if (w_lc != 0.f && (!key || region_size <= 0)) return set_error(CFSD_EINVAL, "%s: key/region required", name);
  bs = (int)lrint(sqrt((double)batch));
  if (w_lc != 0.f && bs * bs != batch) return set_error(CFSD_EINVAL, "%s: batch %d is not bs^2", name, batch);
  if (w_lc == 0.f) bs = 1;
  if (batch <= 0 || latent <= 0) return set_error(CFSD_EINVAL, "%s: bad sizes", name);
  lds = latent_lds_floats(batch, latent, bs) * sizeof(float) + extra_lds;
  if (lds > kLatLdsMax)
    return set_error(CFSD_EINVAL, "%s: batch %d x latent %d needs %zu B of LDS (> %zu)", name, batch,
                     latent, lds, kLatLdsMax);
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLatLdsMax) != hipSuccess)
    return set_error(CFSD_EINVAL, "%s: cannot raise the dynamic LDS limit", name);
  return CFSD_OK;
}

extern "C" int cfsd_latent_fwd(const float* mulv, const float* eps, const int32_t* key, float* z,
                               float* dlat, float* terms, int batch, int latent, int region_size,
                               int train, int is_vae, int sigmoid, float w_kl, float w_lc,
                               float eta1, float eta2, void* stream) {
  int bs = 1;
  size_t lds = 0;
  const int rc = latent_prepare("latent_fwd", (const void*)latent_fwd_k, mulv, eps, key, z, dlat, terms,
                                batch, latent, region_size, train, is_vae, w_lc, 0, bs, lds);
  if (rc != CFSD_OK) return rc;
  const LatentArgs a{mulv, eps, key, z, dlat, terms, batch, latent, region_size, train, is_vae,
                     sigmoid, w_kl, w_lc, eta1, eta2, bs};
  hipLaunchKernelGGL(latent_fwd_k, dim3(1), dim3(kLatThreads), lds, (hipStream_t)stream, a);
  return launch_status("latent_fwd");
}

extern "C" int cfsd_latent_linear_fwd_supported(int batch, int latent, int n) {
  if (batch <= 0 || latent <= 0 || latent > kLatLinMaxK || n <= 0) return 0;
  const int bs = (int)lrint(sqrt((double)batch));  // LC sizing (the larger case)
  const size_t f = latent_lds_floats(batch, latent, bs * bs == batch ? bs : 1);
  return (f + (size_t)kLatLinCols * latent) * sizeof(float) <= kLatLdsMax;
}

extern "C" int cfsd_latent_linear_fwd(const float* mulv, const float* eps, const int32_t* key, float* z,
                                      float* dlat, float* terms, int batch, int latent,
                                      int region_size, int train, int is_vae, int sigmoid,
                                      float w_kl, float w_lc, float eta1, float eta2,
                                      const float* w, const float* bias, float* y, int n,
                                      void* stream) {
  if (!w || !y) return set_error(CFSD_EINVAL, "latent_linear_fwd: null pointer");
  if (!cfsd_latent_linear_fwd_supported(batch, latent, n))
    return set_error(CFSD_EINVAL, "latent_linear_fwd: latent %d (max %d) / n %d unsupported", latent,
                     kLatLinMaxK, n);
  int bs = 1;
  size_t lds = 0;
  const int rc = latent_prepare("latent_linear_fwd", (const void*)latent_linear_fwd_k, mulv, eps, key, z,
                                dlat, terms, batch, latent, region_size, train, is_vae, w_lc,
                                (size_t)kLatLinCols * latent * sizeof(float), bs, lds);
  if (rc != CFSD_OK) return rc;
  const LatentArgs a{mulv, eps, key, z, dlat, terms, batch, latent, region_size, train, is_vae,
                     sigmoid, w_kl, w_lc, eta1, eta2, bs};
  hipLaunchKernelGGL(latent_linear_fwd_k, dim3((n + kLatLinCols - 1) / kLatLinCols), dim3(kLatLinThreads),
                     lds, (hipStream_t)stream, a, w, bias, y, n, (int)latent_lds_floats(batch, latent, bs));
  return launch_status("latent_linear_fwd");
}

extern "C" int cfsd_latent_bwd(const float* mulv, const float* eps, const float* z,
                               const float* dz_dec, const float* dlat, float* dmulv, int batch,
                               int latent, int train, int is_vae, int sigmoid, void* stream) {
  if (!mulv || !dz_dec || !dlat || !dmulv) return set_error(CFSD_EINVAL, "latent_bwd: null pointer");
  if (is_vae && train && !eps) return set_error(CFSD_EINVAL, "latent_bwd: eps required");
  const int n = batch * latent, nb = (n + 255) / 256;
  hipLaunchKernelGGL(latent_bwd_k, dim3(nb), dim3(256), 0, (hipStream_t)stream, mulv, eps, dz_dec, dlat, dmulv,
                     batch, latent, train, is_vae, sigmoid, z, 1, nb);
  return launch_status("latent_bwd");
}

extern "C" int cfsd_latent_bwd_parts(const float* mulv, const float* eps, const float* z,
                                     const float* dz_parts, int n_parts, const float* dlat,
                                     float* dmulv, int batch, int latent, int train, int is_vae,
                                     int sigmoid, void* stream) {
  if (!mulv || !dz_parts || !dlat || !dmulv) return set_error(CFSD_EINVAL, "latent_bwd_parts: null pointer");
  if (n_parts <= 0) return set_error(CFSD_EINVAL, "latent_bwd_parts: n_parts %d", n_parts);
  if (is_vae && train && !eps) return set_error(CFSD_EINVAL, "latent_bwd_parts: eps required");
  const int n = batch * latent, nb = (n + 255) / 256;
  hipLaunchKernelGGL(latent_bwd_k, dim3(nb), dim3(256), 0, (hipStream_t)stream, mulv, eps, dz_parts,
                     dlat, dmulv, batch, latent, train, is_vae, sigmoid, z, n_parts, nb);
  return launch_status("latent_bwd_parts");
}

extern "C" int cfsd_loss_finalize(const float* partials, int nblocks, const float* terms,
                                  float* out, float* acc, int batch, int nv, int c, float w_kl,
                                  float w_lc, float w_lap, void* stream) {
  if (!partials || !terms || !out) return set_error(CFSD_EINVAL, "loss_finalize: null pointer");
  const float inv_n = 1.f / (float)((long)batch * nv * c);
  const float inv_lap = 1.f / (float)((long)nv * batch);
  const LossFinalize f{partials, nblocks, terms, out, acc, inv_n, inv_lap, w_kl, w_lc, w_lap};
  hipLaunchKernelGGL(loss_finalize_k, dim3(1), dim3(256), 0, (hipStream_t)stream, f);
  return launch_status("loss_finalize");
}

extern "C" size_t cfsd_linear_workspace(int m, int k, int n) {
  if (m <= 0 || k <= 0 || n <= 0) return 0;
  return 0;  // single-pass kernels; kept for ABI stability
}

extern "C" int cfsd_linear_fwd(const float* x, const float* w, const float* bias, float* y,
                               float* workspace, size_t workspace_bytes, int m, int k, int n,
                               void* stream) {
  if (!x || !w || !y) return set_error(CFSD_EINVAL, "linear_fwd: null pointer");
  if (m <= 0 || k <= 0 || n <= 0) return set_error(CFSD_EINVAL, "linear_fwd: bad sizes");
  (void)workspace;
  (void)workspace_bytes;
  hipStream_t st = (hipStream_t)stream;
  if (k > kLinSmallK) {
    hipLaunchKernelGGL(linear_fwd_kred, dim3(n, (m + kLinRGFwd - 1) / kLinRGFwd), dim3(kLinRedThreads), 0, st, x, w, bias, y, m, k,
                       n);
    return launch_status("linear_fwd_kred");
  }
  hipLaunchKernelGGL(linear_fwd_nred, dim3((n + 255) / 256, (m + 3) / 4), dim3(256), 0, st, x, w,
                     bias, y, m, k, n);
  return launch_status("linear_fwd_nred");
}

extern "C" int cfsd_linear_bwd(const float* x, const float* w, const float* dy, const float* elu_y,
                               float* dx, float* dw, float* db, float* workspace,
                               size_t workspace_bytes, int m, int k, int n, int accumulate,
                               void* stream) {
  if (!dy) return set_error(CFSD_EINVAL, "linear_bwd: null dy");
  if (m <= 0 || k <= 0 || n <= 0) return set_error(CFSD_EINVAL, "linear_bwd: bad sizes");
  (void)workspace;
  (void)workspace_bytes;
  hipStream_t st = (hipStream_t)stream;
  const int bt = k >= 256 ? 256 : ((k + 63) / 64) * 64;
  if (dx && dw && x && w && n <= kLinSmallK && bt == 256) {  // dx + dW in one launch
    const int ndx_x = (k + 63) / 64, ndx = ndx_x * ((m + 3) / 4), ndw_x = (k + 255) / 256;
    hipLaunchKernelGGL(linear_bwd_pair_k, dim3(ndx + ndw_x * n), dim3(256), 0, st, x, w, dy,
                       elu_y, dx, dw, db, m, k, n, accumulate, ndx_x, ndx, ndw_x);
    return launch_status("linear_bwd_pair");
  }
  if (dx) {
    if (!w) return set_error(CFSD_EINVAL, "linear_bwd: null w");
    int rc;
    if (n <= kLinSmallK) {
      hipLaunchKernelGGL(linear_dx_nsmall, dim3((k + 63) / 64, (m + 3) / 4), dim3(256), 0, st, dy,
                         w, elu_y, dx, m, k, n, accumulate);
      rc = launch_status("linear_dx_nsmall");
    } else {
      hipLaunchKernelGGL(linear_dx_nred, dim3(k, (m + kLinRGDx - 1) / kLinRGDx), dim3(kLinRedThreads), 0, st, dy, w, elu_y, dx, m,
                         k, n, accumulate);
      rc = launch_status("linear_dx_nred");
    }
    if (rc) return rc;
  }
  if (dw || db) {
    if (dw && !x) return set_error(CFSD_EINVAL, "linear_bwd: null x");
    hipLaunchKernelGGL(linear_dw_k, dim3((k + bt - 1) / bt, n), dim3(bt), 0, st, x, dy, dw, db, m,
                       k, n);
    return launch_status("linear_bwd_dw");
  }
  return CFSD_OK;
}

extern "C" int cfsd_linear_bwd_split_parts(int n) { return n > 0 ? (n + kLinSplitN - 1) / kLinSplitN : 0; }

extern "C" int cfsd_linear_bwd_split(const float* x, const float* w, const float* dy, float* dx_parts,
                                     float* dw, float* db, int m, int k, int n, void* stream) {
  if (!x || !w || !dy || !dx_parts || !dw || !db) return set_error(CFSD_EINVAL, "linear_bwd_split: null pointer");
  if (m <= 0 || k <= 0 || n <= 0 || m > kLinSplitM || k > kLinSplitK)
    return set_error(CFSD_EINVAL, "linear_bwd_split: sizes m=%d k=%d n=%d (m <= %d, k <= %d)", m, k, n,
                     kLinSplitM, kLinSplitK);
  const int ndx = cfsd_linear_bwd_split_parts(n), ndw = (n + kLinDwRows - 1) / kLinDwRows;
  hipLaunchKernelGGL(linear_bwd_split_k, dim3(ndx + ndw), dim3(256), 0, (hipStream_t)stream, x, w, dy,
                     dx_parts, dw, db, m, k, n, ndx);
  return launch_status("linear_bwd_split");
}

static inline int bn_round32(long n) { return (int)((n + 31) / 32 * 32); }

extern "C" size_t cfsd_bottleneck_bwd_exchange_floats(int batch, int latent, int nd, int ne) {
  if (batch <= 0 || latent <= 0 || nd <= 0 || ne <= 0) return 0;
  return (size_t)cfsd_linear_bwd_split_parts(nd) * bn_round32((long)batch * latent) +
         (size_t)batch * bn_round32(ne);
}

extern "C" int cfsd_bottleneck_bwd(const int32_t* up_ptr, const int32_t* up_col, const float* up_val,
                                   const float* g, int n_up, int cup, const float* z, const float* wd,
                                   float* exchange, float* dwd, float* dbd, int nd, const float* mulv,
                                   const float* eps, const float* dlat, float* dmulv, int train, int is_vae,
                                   int sigmoid, const float* xe, const float* we, const float* elu_y, float* dxe,
                                   float* dwe, float* dbe, int ke, int ne, int accumulate, int32_t* sync, int batch,
                                   int latent, void* stream) {
  if (!up_ptr || !up_col || !up_val || !g || !z || !wd || !exchange || !dwd || !dbd || !mulv || !dlat || !dmulv ||
      !xe || !we || !dxe || !dwe || !dbe || !sync)
    return set_error(CFSD_EINVAL, "bottleneck_bwd: null pointer");
  if (is_vae && train && !eps) return set_error(CFSD_EINVAL, "bottleneck_bwd: eps required");
  const int m = batch, kd = latent;
  if (m <= 0 || m > kLinSplitM || kd <= 0 || kd > kLinSplitK || cup <= 0 || cup % kLinSplitN || nd <= 0 ||
      nd % cup || nd > kBnMaxParts * kLinSplitN || n_up <= 0 || ke <= 0 || ne <= 0 || ne > 4 * kLinDxChunk ||
      ne != (is_vae ? 2 : 1) * latent)
    return set_error(CFSD_EINVAL,
                     "bottleneck_bwd: sizes batch=%d latent=%d cup=%d nd=%d ke=%d ne=%d (batch <= %d, latent <= %d, "
                     "cup a multiple of %d, ne <= %d)",
                     m, kd, cup, nd, ke, ne, kLinSplitM, kLinSplitK, kLinSplitN, 4 * kLinDxChunk);
  BneckArgs a{};
  a.up_ptr = up_ptr;
  a.up_col = up_col;
  a.up_val = up_val;
  a.g = g;
  a.n_up = n_up;
  a.cup = cup;
  a.z = z;
  a.wd = wd;
  a.pstride = bn_round32((long)m * kd);
  a.dstride = bn_round32(ne);
  a.parts = exchange;
  a.dwd = dwd;
  a.dbd = dbd;
  a.m = m;
  a.kd = kd;
  a.nd = nd;
  a.ndx_d = cfsd_linear_bwd_split_parts(nd);
  a.ndw_d = (nd + kLinDwRows - 1) / kLinDwRows;
  a.mulv = mulv;
  a.eps = eps;
  a.dlat = dlat;
  a.dmulv = dmulv;
  a.zval = z;
  a.L = latent;
  a.train = train;
  a.is_vae = is_vae;
  a.sigmoid = sigmoid;
  a.lat_rows = 256 / latent;  // >= 2 (latent <= 128)
  a.nb_lat = (m + a.lat_rows - 1) / a.lat_rows;
  a.xdmulv = exchange + (size_t)a.ndx_d * a.pstride;
  a.xe = xe;
  a.we = we;
  a.elu_y = elu_y;
  a.dxe = dxe;
  a.dwe = dwe;
  a.dbe = dbe;
  a.ke = ke;
  a.ne = ne;
  a.accumulate = accumulate;
  a.ndx_x = (ke + 63) / 64;
  a.ndx_e = a.ndx_x * ((m + 3) / 4);
  a.ndw_x = (ke + 255) / 256;
  a.ndw_g = (ne + kBnDwRows - 1) / kBnDwRows;
  a.sync = sync;
  const int nb = a.ndx_d + a.nb_lat + a.ndw_d + a.ndx_e + a.ndw_x * a.ndw_g;
  size_t lds = (size_t)kBnWT * kd + (size_t)m * kLinSplitN;
  lds = std::max(lds, (size_t)m * kd + (size_t)m * kLinDwRows);
  lds = std::max(lds, (size_t)4 * ne + 16 * 64);
  lds = std::max(lds, (size_t)m * kBnDwRows);
  hipLaunchKernelGGL(bottleneck_bwd_k, dim3(nb), dim3(256), lds * sizeof(float), (hipStream_t)stream, a);
  return launch_status("bottleneck_bwd");
}

extern "C" int cfsd_adam(float* param, const float* grad, float* m, float* v,
                         const int32_t* step, size_t n, float lr, float beta1, float beta2,
                         float eps, float weight_decay, uint16_t* param_bf16, void* stream) {
  if (!param || !grad || !m || !v || !step) return set_error(CFSD_EINVAL, "adam: null pointer");
  if (n == 0) return CFSD_OK;
  if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v | (uintptr_t)param_bf16 * 2) & 15)
    return set_error(CFSD_EINVAL, "adam: param/grad/m/v must be 16-B aligned");
  hipLaunchKernelGGL(adam_k<false>, dim3((unsigned)((n / 4 + 1 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     param, const_cast<float*>(grad), m, v, step, (long)n, lr, beta1, beta2, eps, weight_decay,
                     param_bf16, 1.f);
  return launch_status("adam");
}

extern "C" int cfsd_adam_scaled(float* param, float* grad, float* m, float* v, const int32_t* step, size_t n,
                                float grad_scale, float lr, float beta1, float beta2, float eps,
                                float weight_decay, uint16_t* param_bf16, void* stream) {
  if (!param || !grad || !m || !v || !step) return set_error(CFSD_EINVAL, "adam_scaled: null pointer");
  if (n == 0) return CFSD_OK;
  if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v | (uintptr_t)param_bf16 * 2) & 15)
    return set_error(CFSD_EINVAL, "adam_scaled: param/grad/m/v must be 16-B aligned");
  hipLaunchKernelGGL(adam_k<true>, dim3((unsigned)((n / 4 + 1 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     param, grad, m, v, step, (long)n, lr, beta1, beta2, eps, weight_decay, param_bf16,
                     grad_scale);
  return launch_status("adam_scaled");
}

extern "C" int cfsd_step_begin(int32_t* counter, unsigned long long seed, float* eps, int n_eps,
                               int32_t* key, int n_regions, int32_t* batch_idx, int bs,
                               int n_batches, const int32_t* perm, int n_items, int shuffle,
                               int32_t* adam_step, void* stream) {
  if (!counter) return set_error(CFSD_EINVAL, "step_begin: null counter");
  if (key && n_regions <= 0) return set_error(CFSD_EINVAL, "step_begin: n_regions");
  if (batch_idx) {
    if (bs <= 0 || bs > 256 || n_batches <= 0) return set_error(CFSD_EINVAL, "step_begin: bs/n_batches");
    if (n_items < (long)n_batches * bs)
      return set_error(CFSD_EINVAL, "step_begin: n_items %d < n_batches %d x bs %d", n_items, n_batches, bs);
  }
  hipLaunchKernelGGL(step_begin_k, dim3(1), dim3(256), 0, (hipStream_t)stream, counter, seed, eps,
                     n_eps, key, n_regions, batch_idx, bs, n_batches, perm, n_items, shuffle, adam_step);
  return launch_status("step_begin");
}
