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
// Pass 1, one thread per (b, v).  C <= 4.
__global__ __launch_bounds__(kLapThreads) void recon_lap_fwd_k(
    const float* __restrict__ pred, const float* __restrict__ gt, const int* __restrict__ l_ptr,
    const int* __restrict__ l_col, const float* __restrict__ l_val, float* __restrict__ unit,
    float* __restrict__ partials, int nv, int c, long total) {
  __shared__ float2 sh[kLapThreads / 64];
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  float sq = 0.f, nrm = 0.f;
  if (t < total) {
    const int v = (int)(t % nv);
    const long b = t / nv;
    const float* pb = pred + b * nv * c;
    float lx[4] = {0.f, 0.f, 0.f, 0.f};
    for (int e = l_ptr[v]; e < l_ptr[v + 1]; ++e) {
      const float w = l_val[e];
      const float* p = pb + (long)l_col[e] * c;
      for (int q = 0; q < c; ++q) lx[q] = fmaf(w, p[q], lx[q]);
    }
    float n2 = 0.f;
    for (int q = 0; q < c; ++q) {
      float d = pred[t * c + q] - gt[t * c + q];
      sq = fmaf(d, d, sq);
      n2 = fmaf(lx[q], lx[q], n2);
    }
    nrm = sqrtf(n2);
    const float inv = nrm > 0.f ? 1.f / nrm : 0.f;
    for (int q = 0; q < c; ++q) unit[t * c + q] = lx[q] * inv;
  }
  float2 r = block_sum2(sq, nrm, sh);
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = r.x;
    partials[2 * blockIdx.x + 1] = r.y;
  }
}

// Pass 2, one thread per (b, u): d/dpred of w_rec*mse + w_lap*lap.
__global__ __launch_bounds__(256) void recon_lap_bwd_k(
    const float* __restrict__ pred, const float* __restrict__ gt, const float* __restrict__ unit,
    const int* __restrict__ lt_ptr, const int* __restrict__ lt_col,
    const float* __restrict__ lt_val, float* __restrict__ dpred, int nv, int c, long total,
    float k_rec, float k_lap) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int u = (int)(t % nv);
  const long b = t / nv;
  const float* ub = unit + b * nv * c;
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  for (int e = lt_ptr[u]; e < lt_ptr[u + 1]; ++e) {
    const float w = lt_val[e];
    const float* p = ub + (long)lt_col[e] * c;
    for (int q = 0; q < c; ++q) g[q] = fmaf(w, p[q], g[q]);
  }
  for (int q = 0; q < c; ++q)
    dpred[t * c + q] = k_rec * (pred[t * c + q] - gt[t * c + q]) + k_lap * g[q];
}

// ----------------------------------------------------------- latent head
// Single workgroup.  mulv [B, 2L] = [logvar | mu] (rows of the stacked
// encoder Linear), z [B, L].  dlat [B, 3L] = {w_lc*dLC/dz | w_kl*dKL/dmu | w_kl*dKL/dlogvar}.
// terms[2] = {kl, lc}.
__global__ __launch_bounds__(256) void latent_fwd_k(const float* __restrict__ mulv,
                                                    const float* __restrict__ eps,
                                                    const int* __restrict__ key,
                                                    float* __restrict__ z,
                                                    float* __restrict__ dlat,
                                                    float* __restrict__ terms, int B, int L,
                                                    int region_size, int train, int is_vae,
                                                    int sigmoid, float w_kl, float w_lc,
                                                    float eta1, float eta2, int bs) {
  __shared__ float zs[64 * 256];
  __shared__ float dist[4 * 64 * 8];  // [kind][pair][t]
  __shared__ float2 red[4];
  const int tid = threadIdx.x;
  const int ldm = is_vae ? 2 * L : L;
  const int mu_off = is_vae ? L : 0;
  // z and KL pieces
  float kl_part = 0.f;
  for (int e = tid; e < B * L; e += blockDim.x) {
    const int i = e / L, l = e % L;
    const float mu = mulv[i * ldm + mu_off + l];
    float zz = mu;
    if (is_vae) {
      const float lv = mulv[i * ldm + l];
      const float ex = expf(lv);
      if (train) zz = mu + eps[e] * expf(0.5f * lv);
      kl_part += 1.f + lv - mu * mu - ex;
      dlat[i * 3 * L + L + l] = w_kl * mu / (float)B;
      dlat[i * 3 * L + 2 * L + l] = w_kl * (-0.5f) * (1.f - ex) / (float)B;
    } else {
      if (sigmoid) zz = 1.f / (1.f + expf(-mu));
      dlat[i * 3 * L + L + l] = 0.f;
      dlat[i * 3 * L + 2 * L + l] = 0.f;
    }
    z[e] = zz;
    zs[e] = zz;
  }
  __syncthreads();
  // latent consistency distances: kinds 0=lg 1=dg 2=dr 3=lr, pairs p<q, t
  const int npairs = bs * (bs - 1) / 2;
  const int lo = region_size > 0 ? (*key) * region_size : 0;
  const int hi = lo + region_size;
  const int nd = 4 * npairs * bs;
  for (int e = tid; e < nd && w_lc != 0.f; e += blockDim.x) {
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
    float d = 0.f;
    for (int l = 0; l < L; ++l) {
      const bool inr = (l >= lo && l < hi);
      if (inr != in_region) continue;
      const float df = zs[ra * L + l] - zs[rb * L + l];
      d = fmaf(df, df, d);
    }
    dist[e] = d;
  }
  __syncthreads();
  const float scale = 1.f / (float)(bs * bs * bs - bs * bs);
  float lc_part = 0.f;
  for (int e = tid; e < npairs * bs && w_lc != 0.f; e += blockDim.x) {
    const float lg = dist[0 * npairs * bs + e], dg = dist[1 * npairs * bs + e];
    const float dr = dist[2 * npairs * bs + e], lr = dist[3 * npairs * bs + e];
    lc_part += fmaxf(0.f, lr - dr + eta2) + fmaxf(0.f, lg - dg + eta1);
  }
  // gradient of LC w.r.t. z: thread per latent dim, fixed term order
  if (tid < L) {
    const int l = tid;
    const bool inr = (l >= lo && l < hi);
    float col[64];
    for (int i = 0; i < B; ++i) col[i] = 0.f;
    if (w_lc != 0.f) {
      for (int pr = 0; pr < npairs; ++pr) {
        int p = 0, rem = pr;
        while (rem >= bs - 1 - p) { rem -= bs - 1 - p; ++p; }
        const int q = p + 1 + rem;
        for (int t = 0; t < bs; ++t) {
          const int e = pr * bs + t;
          float act;
          if (inr) act = (dist[0 * npairs * bs + e] - dist[1 * npairs * bs + e] + eta1) > 0.f;
          else act = (dist[3 * npairs * bs + e] - dist[2 * npairs * bs + e] + eta2) > 0.f;
          if (act == 0.f) continue;
          const float k2 = 2.f * scale * w_lc;
          // same-donor distance (lg or dr): + for inr, - for the complement
          const int a1 = q * bs + t, b1 = p * bs + t;
          const int a2 = t * bs + q, b2 = t * bs + p;
          const float d1 = zs[a1 * L + l] - zs[b1 * L + l];
          const float d2 = zs[a2 * L + l] - zs[b2 * L + l];
          const float s1 = inr ? 1.f : -1.f;  // lg - dg  vs  lr - dr
          col[a1] += s1 * k2 * d1;
          col[b1] -= s1 * k2 * d1;
          col[a2] -= s1 * k2 * d2;
          col[b2] += s1 * k2 * d2;
        }
      }
    }
    for (int i = 0; i < B; ++i) dlat[i * 3 * L + l] = col[i];
  }
  float2 r = block_sum2(kl_part, lc_part, red);
  if (tid == 0) {
    terms[0] = is_vae ? -0.5f * r.x / (float)B : 0.f;
    terms[1] = r.y * scale;
  }
}

__global__ __launch_bounds__(256) void latent_bwd_k(const float* __restrict__ mulv,
                                                    const float* __restrict__ eps,
                                                    const float* __restrict__ dz_dec,
                                                    const float* __restrict__ dlat,
                                                    float* __restrict__ dmulv, int B, int L,
                                                    int train, int is_vae, int sigmoid,
                                                    const float* __restrict__ zval) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * L) return;
  const int i = e / L, l = e % L;
  const float dz = dz_dec[e] + dlat[i * 3 * L + l];
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

__global__ void loss_finalize_k(const float* __restrict__ partials, int nblocks,
                                const float* __restrict__ terms, float* __restrict__ out,
                                float* __restrict__ acc, float inv_n_rec, float inv_lap,
                                float w_kl, float w_lc, float w_lap) {
  __shared__ float2 sh[4];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < nblocks; i += blockDim.x) {
    a += partials[2 * i];
    b += partials[2 * i + 1];
  }
  float2 r = block_sum2(a, b, sh);
  if (threadIdx.x == 0) {
    const float rec = r.x * inv_n_rec, lap = r.y * inv_lap;
    const float kl = terms[0], lc = terms[1];
    const float tot = rec + w_kl * kl + w_lc * lc + w_lap * lap;
    const float v[5] = {rec, kl, lc, lap, tot};
    for (int q = 0; q < 5; ++q) {
      out[q] = v[q];
      if (acc) acc[q] += v[q];
    }
    if (acc) acc[5] += 1.f;
  }
}

// ----------------------------------------------------------- dense Linear
// The bottleneck Linears are [16 x 4288] x [4288 x 150] (encoder, stacked
// mu/logvar) and [16 x 75] x [75 x 4288] (decoder): tiny GEMMs whose cost is
// parallelism and latency, not FLOPs.  Long reductions are split across
// workgroups into a workspace and summed in a second fixed-order pass.
constexpr int kLinKC = 256;   // k per split-K workgroup (64 lanes x 4)
constexpr int kLinNC = 128;   // n per split-n chunk (dx of the decoder Linear)

// Split-K partials: block (col n, chunk ks), one wave; lane l owns k =
// ks*256 + 4l .. +3.  ws[(ks*m + i)*n + col].
__global__ __launch_bounds__(64) void linear_fwd_splitk(const float* __restrict__ x,
                                                        const float* __restrict__ w,
                                                        float* __restrict__ ws, int m, int k,
                                                        int n) {
  const int col = blockIdx.x, ks = blockIdx.y, lane = threadIdx.x;
  const int k0 = ks * kLinKC + 4 * lane;
  float wv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) wv[q] = (k0 + q < k) ? w[(long)col * k + k0 + q] : 0.f;
  for (int i0 = 0; i0 < m; i0 += 16) {
    float acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc[i] = 0.f;
      if (i0 + i < m) {
        const float* xr = x + (long)(i0 + i) * k;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (k0 + q < k) acc[i] = fmaf(xr[k0 + q], wv[q], acc[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float v = acc[i];
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
      if (lane == i && i0 + i < m) ws[((long)ks * m + i0 + i) * n + col] = v;
    }
  }
}

__global__ __launch_bounds__(256) void linear_fwd_reduce(const float* __restrict__ ws,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ y, int m, int n,
                                                         int nks) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)m * n) return;
  float s = 0.f;
  for (int q = 0; q < nks; ++q) s += ws[(long)q * m * n + e];
  y[e] = s + (bias ? bias[e % n] : 0.f);
}

// Short k: one thread per (i, n); 16 consecutive threads share n (broadcast W).
__global__ __launch_bounds__(256) void linear_fwd_smallk(const float* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ y, int m, int k,
                                                         int n) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int i = (int)(t % 16);
  const long col = t / 16;
  if (col >= n) return;
  const float* wr = w + col * k;
  for (int ii = i; ii < m; ii += 16) {
    const float* xr = x + (long)ii * k;
    float acc = 0.f;
    for (int kk = 0; kk < k; ++kk) acc = fmaf(xr[kk], wr[kk], acc);
    y[(long)ii * n + col] = acc + (bias ? bias[col] : 0.f);
  }
}

// dx for short n (encoder Linear, n = 150): block = one wave of 64 k's for
// row i = blockIdx.y (wave-uniform -> dy is read with scalar loads).
__global__ __launch_bounds__(64) void linear_dx_rows(const float* __restrict__ dy,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ elu_y,
                                                     float* __restrict__ dx, int m, int k, int n,
                                                     int accumulate) {
  const int kk = blockIdx.x * 64 + threadIdx.x;
  const int i = blockIdx.y;
  if (kk >= k) return;
  const float* dyr = dy + (long)i * n;
  float acc = 0.f;
#pragma unroll 8
  for (int nn = 0; nn < n; ++nn) acc = fmaf(dyr[nn], w[(long)nn * k + kk], acc);
  const long o = (long)i * k + kk;
  if (elu_y) acc *= elu_grad_from_out(elu_y[o]);
  dx[o] = accumulate ? dx[o] + acc : acc;
}

// dx for long n (decoder Linear, n = 4288): split-n partials, thread per
// (i, k) pair, ws[ns][i*k + kk].
__global__ __launch_bounds__(256) void linear_dx_splitn(const float* __restrict__ dy,
                                                        const float* __restrict__ w,
                                                        float* __restrict__ ws, int m, int k,
                                                        int n) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (long)m * k) return;
  const int i = (int)(p / k), kk = (int)(p % k);
  const int n0 = blockIdx.y * kLinNC, n1 = min(n, n0 + kLinNC);
  const float* dyr = dy + (long)i * n;
  float acc = 0.f;
#pragma unroll 8
  for (int nn = n0; nn < n1; ++nn) acc = fmaf(dyr[nn], w[(long)nn * k + kk], acc);
  ws[(long)blockIdx.y * m * k + p] = acc;
}

__global__ __launch_bounds__(256) void linear_dx_reduce(const float* __restrict__ ws,
                                                        const float* __restrict__ elu_y,
                                                        float* __restrict__ dx, long mk, int nns,
                                                        int accumulate) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= mk) return;
  float s = 0.f;
  for (int q = 0; q < nns; ++q) s += ws[(long)q * mk + p];
  if (elu_y) s *= elu_grad_from_out(elu_y[p]);
  dx[p] = accumulate ? dx[p] + s : s;
}

// dw[n,k] = sum_i dy[i,n] x[i,k] (thread per element), db[n] = sum_i dy[i,n].
__global__ __launch_bounds__(256) void linear_dw_k(const float* __restrict__ x,
                                                   const float* __restrict__ dy,
                                                   float* __restrict__ dw,
                                                   float* __restrict__ db, int m, int k, int n) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nk = (long)n * k;
  if (e < nk) {
    const int nn = (int)(e / k), kk = (int)(e % k);
    float s = 0.f;
    for (int i = 0; i < m; ++i) s = fmaf(dy[(long)i * n + nn], x[(long)i * k + kk], s);
    if (dw) dw[e] = s;
  } else if (e < nk + n) {
    const int nn = (int)(e - nk);
    float s = 0.f;
    for (int i = 0; i < m; ++i) s += dy[(long)i * n + nn];
    if (db) db[nn] = s;
  }
}

// ----------------------------------------------------------- Adam
__global__ __launch_bounds__(256) void adam_k(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              const int* __restrict__ step, long n, float lr,
                                              float b1, float b2, float eps, float wd) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = *step;
  const float bc1 = 1.f - powf(b1, (float)t);
  const float bc2 = 1.f - powf(b2, (float)t);
  float gi = g[i];
  if (wd != 0.f) gi = fmaf(wd, p[i], gi);
  const float mi = fmaf(b1, m[i], (1.f - b1) * gi);
  const float vi = fmaf(b2, v[i], (1.f - b2) * gi * gi);
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / sqrtf(bc2) + eps;
  p[i] -= (lr / bc1) * (mi / denom);
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

__global__ void step_begin_k(int* __restrict__ counter, unsigned long long seed,
                             float* __restrict__ eps, int n_eps, int* __restrict__ key,
                             int n_regions, int* __restrict__ batch_idx, int bs, int n_batches,
                             const int* __restrict__ perm) {
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
    const int bt = (t - 1) % n_batches;
    const int slot = bt * bs + threadIdx.x;
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
  if (threadIdx.x == 0) *counter = t;
}

}  // namespace cfsd

using namespace cfsd;

extern "C" int cfsd_version(void) { return (1 << 16) | 0; }
extern "C" const char* cfsd_last_error_string(void) { return g_err; }

extern "C" int cfsd_recon_lap_blocks(int batch, int nv) {
  const long total = (long)batch * nv;
  return (int)((total + kLapThreads - 1) / kLapThreads);
}

extern "C" int cfsd_recon_lap_fwd(const float* pred, const float* gt, const int32_t* l_ptr,
                                  const int32_t* l_col, const float* l_val, float* unit_lx,
                                  float* partials, int batch, int nv, int c, void* stream) {
  if (!pred || !gt || !l_ptr || !l_col || !l_val || !unit_lx || !partials)
    return set_error(CFSD_EINVAL, "recon_lap_fwd: null pointer");
  if (batch <= 0 || nv <= 0 || c <= 0 || c > 4) return set_error(CFSD_EINVAL, "recon_lap_fwd: bad sizes");
  const long total = (long)batch * nv;
  hipLaunchKernelGGL(recon_lap_fwd_k, dim3(cfsd_recon_lap_blocks(batch, nv)), dim3(kLapThreads), 0,
                     (hipStream_t)stream, pred, gt, l_ptr, l_col, l_val, unit_lx, partials, nv, c,
                     total);
  return launch_status("recon_lap_fwd");
}

extern "C" int cfsd_recon_lap_bwd(const float* pred, const float* gt, const float* unit_lx,
                                  const int32_t* lt_ptr, const int32_t* lt_col,
                                  const float* lt_val, float* dpred, int batch, int nv, int c,
                                  float w_rec, float w_lap, void* stream) {
  if (!pred || !gt || !unit_lx || !lt_ptr || !lt_col || !lt_val || !dpred)
    return set_error(CFSD_EINVAL, "recon_lap_bwd: null pointer");
  if (batch <= 0 || nv <= 0 || c <= 0 || c > 4) return set_error(CFSD_EINVAL, "recon_lap_bwd: bad sizes");
  const long total = (long)batch * nv;
  const float k_rec = w_rec * 2.f / (float)(total * c);
  const float k_lap = w_lap / (float)((long)nv * batch);
  hipLaunchKernelGGL(recon_lap_bwd_k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, pred, gt, unit_lx, lt_ptr, lt_col, lt_val, dpred, nv, c,
                     total, k_rec, k_lap);
  return launch_status("recon_lap_bwd");
}

extern "C" int cfsd_latent_fwd(const float* mulv, const float* eps, const int32_t* key, float* z,
                               float* dlat, float* terms, int batch, int latent, int region_size,
                               int train, int is_vae, int sigmoid, float w_kl, float w_lc,
                               float eta1, float eta2, void* stream) {
  if (!mulv || !z || !dlat || !terms) return set_error(CFSD_EINVAL, "latent_fwd: null pointer");
  if (is_vae && train && !eps) return set_error(CFSD_EINVAL, "latent_fwd: eps required");
  if (w_lc != 0.f && (!key || region_size <= 0)) return set_error(CFSD_EINVAL, "latent_fwd: key/region required");
  int bs = (int)lrint(sqrt((double)batch));
  if (w_lc != 0.f && bs * bs != batch) return set_error(CFSD_EINVAL, "latent_fwd: batch %d is not bs^2", batch);
  if (w_lc == 0.f) bs = 1;
  if (batch > 64 || latent > 256 || batch * latent > 64 * 256)
    return set_error(CFSD_EINVAL, "latent_fwd: batch %d / latent %d too large", batch, latent);
  hipLaunchKernelGGL(latent_fwd_k, dim3(1), dim3(256), 0, (hipStream_t)stream, mulv, eps, key, z,
                     dlat, terms, batch, latent, region_size, train, is_vae, sigmoid, w_kl, w_lc,
                     eta1, eta2, bs);
  return launch_status("latent_fwd");
}

extern "C" int cfsd_latent_bwd(const float* mulv, const float* eps, const float* z,
                               const float* dz_dec, const float* dlat, float* dmulv, int batch,
                               int latent, int train, int is_vae, int sigmoid, void* stream) {
  if (!mulv || !dz_dec || !dlat || !dmulv) return set_error(CFSD_EINVAL, "latent_bwd: null pointer");
  if (is_vae && train && !eps) return set_error(CFSD_EINVAL, "latent_bwd: eps required");
  const int n = batch * latent;
  hipLaunchKernelGGL(latent_bwd_k, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, mulv,
                     eps, dz_dec, dlat, dmulv, batch, latent, train, is_vae, sigmoid, z);
  return launch_status("latent_bwd");
}

extern "C" int cfsd_loss_finalize(const float* partials, int nblocks, const float* terms,
                                  float* out, float* acc, int batch, int nv, int c, float w_kl,
                                  float w_lc, float w_lap, void* stream) {
  if (!partials || !terms || !out) return set_error(CFSD_EINVAL, "loss_finalize: null pointer");
  const float inv_n = 1.f / (float)((long)batch * nv * c);
  const float inv_lap = 1.f / (float)((long)nv * batch);
  hipLaunchKernelGGL(loss_finalize_k, dim3(1), dim3(256), 0, (hipStream_t)stream, partials,
                     nblocks, terms, out, acc, inv_n, inv_lap, w_kl, w_lc, w_lap);
  return launch_status("loss_finalize");
}

static size_t linear_ws_floats(int m, int k, int n) {
  size_t f = 0;
  if (k >= 512) f = (size_t)((k + kLinKC - 1) / kLinKC) * m * n;
  if (n > 512) {
    const size_t g = (size_t)((n + kLinNC - 1) / kLinNC) * m * k;
    if (g > f) f = g;
  }
  return f;
}

extern "C" size_t cfsd_linear_workspace(int m, int k, int n) {
  if (m <= 0 || k <= 0 || n <= 0) return 0;
  return linear_ws_floats(m, k, n) * sizeof(float);
}

extern "C" int cfsd_linear_fwd(const float* x, const float* w, const float* bias, float* y,
                               float* workspace, size_t workspace_bytes, int m, int k, int n,
                               void* stream) {
  if (!x || !w || !y) return set_error(CFSD_EINVAL, "linear_fwd: null pointer");
  if (m <= 0 || k <= 0 || n <= 0) return set_error(CFSD_EINVAL, "linear_fwd: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (k >= 512) {
    const int nks = (k + kLinKC - 1) / kLinKC;
    if (!workspace || workspace_bytes < (size_t)nks * m * n * sizeof(float))
      return set_error(CFSD_EWORKSPACE, "linear_fwd: workspace too small");
    hipLaunchKernelGGL(linear_fwd_splitk, dim3(n, nks), dim3(64), 0, st, x, w, workspace, m, k, n);
    int rc = launch_status("linear_fwd_splitk");
    if (rc) return rc;
    const long mn = (long)m * n;
    hipLaunchKernelGGL(linear_fwd_reduce, dim3((unsigned)((mn + 255) / 256)), dim3(256), 0, st,
                       workspace, bias, y, m, n, nks);
    return launch_status("linear_fwd_reduce");
  }
  const long t = (long)n * 16;
  hipLaunchKernelGGL(linear_fwd_smallk, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, x, w,
                     bias, y, m, k, n);
  return launch_status("linear_fwd_smallk");
}

extern "C" int cfsd_linear_bwd(const float* x, const float* w, const float* dy, const float* elu_y,
                               float* dx, float* dw, float* db, float* workspace,
                               size_t workspace_bytes, int m, int k, int n, int accumulate,
                               void* stream) {
  if (!dy) return set_error(CFSD_EINVAL, "linear_bwd: null dy");
  if (m <= 0 || k <= 0 || n <= 0) return set_error(CFSD_EINVAL, "linear_bwd: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (dx) {
    if (!w) return set_error(CFSD_EINVAL, "linear_bwd: null w");
    int rc;
    if (n <= 512) {
      hipLaunchKernelGGL(linear_dx_rows, dim3((k + 63) / 64, m), dim3(64), 0, st, dy, w, elu_y, dx,
                         m, k, n, accumulate);
      rc = launch_status("linear_dx_rows");
    } else {
      const int nns = (n + kLinNC - 1) / kLinNC;
      const long mk = (long)m * k;
      if (!workspace || workspace_bytes < (size_t)nns * mk * sizeof(float))
        return set_error(CFSD_EWORKSPACE, "linear_bwd: workspace too small");
      hipLaunchKernelGGL(linear_dx_splitn, dim3((unsigned)((mk + 255) / 256), nns), dim3(256), 0,
                         st, dy, w, workspace, m, k, n);
      rc = launch_status("linear_dx_splitn");
      if (rc) return rc;
      hipLaunchKernelGGL(linear_dx_reduce, dim3((unsigned)((mk + 255) / 256)), dim3(256), 0, st,
                         workspace, elu_y, dx, mk, nns, accumulate);
      rc = launch_status("linear_dx_reduce");
    }
    if (rc) return rc;
  }
  if (dw || db) {
    if (dw && !x) return set_error(CFSD_EINVAL, "linear_bwd: null x");
    const long tot = (long)n * k + n;
    hipLaunchKernelGGL(linear_dw_k, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, x, dy,
                       dw, db, m, k, n);
    return launch_status("linear_bwd_dw");
  }
  return CFSD_OK;
}

extern "C" int cfsd_adam(float* param, const float* grad, float* m, float* v,
                         const int32_t* step, size_t n, float lr, float beta1, float beta2,
                         float eps, float weight_decay, void* stream) {
  if (!param || !grad || !m || !v || !step) return set_error(CFSD_EINVAL, "adam: null pointer");
  if (n == 0) return CFSD_OK;
  hipLaunchKernelGGL(adam_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     param, grad, m, v, step, (long)n, lr, beta1, beta2, eps, weight_decay);
  return launch_status("adam");
}

extern "C" int cfsd_step_begin(int32_t* counter, unsigned long long seed, float* eps, int n_eps,
                               int32_t* key, int n_regions, int32_t* batch_idx, int bs,
                               int n_batches, const int32_t* perm, void* stream) {
  if (!counter) return set_error(CFSD_EINVAL, "step_begin: null counter");
  if (key && n_regions <= 0) return set_error(CFSD_EINVAL, "step_begin: n_regions");
  if (batch_idx && (bs <= 0 || bs > 256 || n_batches <= 0))
    return set_error(CFSD_EINVAL, "step_begin: bs/n_batches");
  hipLaunchKernelGGL(step_begin_k, dim3(1), dim3(256), 0, (hipStream_t)stream, counter, seed, eps,
                     n_eps, key, n_regions, batch_idx, bs, n_batches, perm);
  return launch_status("step_begin");
}
