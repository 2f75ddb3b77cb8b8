// SpiralConv forward / backward kernels for gfx950 (CDNA4), fp32.
//
// Reference: SpiralConv.forward (model.py:27-41) = index_select of the
// spiral neighbourhood + nn.Linear(S*Cin -> Cout), and its autograd
// (index_add_ / addmm backward).  Here the gather is fused with the
// contraction: every 32-row output tile is one v_mfma_f32_32x32x2_f32
// accumulator chain whose A operand is gathered straight from HBM/L2 into
// VGPRs (each lane pair reads one 128-B neighbour row with 16-B loads) and
// whose B operand (the weights) is staged once per workgroup in LDS.
//
// K ordering inside one spiral slot is permuted (lane half h owns channels
// [h*C/2, h*C/2 + C/2)): MFMA step j sums A[i][h]*B[h][n] over h, so slot s's
// dot product is accumulated as pairs (j, j + C/2).  This is exact f32 (the
// f32 MFMA is a k-ordered fmaf chain), only the summation order differs from
// ATen's sgemm.
#include "cfsd_common.h"

namespace cfsd {

// --------------------------------------------------------------------------
// Forward, MFMA path: CIN in {32, 64}, COUT in {32, 64}.
// Block = 256 threads = 4 waves; wave w owns output rows [m0 + 32w, +32) of
// the flattened (b, r) row space and all COUT columns.
// W staged in LDS as [COUT][K + 4] (pad 4 floats: 16-lane ds_read_b128
// groups hit distinct 16-B slots for K = 288 and 576).
template <int CIN, int COUT, int ACT, bool W_LDS>
__global__ __launch_bounds__(256) void conv_fwd_mfma(const float* __restrict__ x,
                                                     const int* __restrict__ idx,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ bias,
                                                     float* __restrict__ y, int vsrc, int rows,
                                                     int seq, long total_rows) {
  constexpr int HALF = CIN / 2;   // channels per lane half
  constexpr int NT = COUT / 32;   // 32-wide output tiles
  extern __shared__ float lds_w[];
  const int K = seq * CIN;
  const int KP = K + 4;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;

  if (W_LDS) {
    for (int i = threadIdx.x; i < COUT * (K / 4); i += 256) {
      int n = i / (K / 4), k4 = i % (K / 4);
      st4(&lds_w[n * KP + 4 * k4], ld4(&w[(long)n * K + 4 * k4]));
    }
    __syncthreads();
  }

  const long m0 = (long)blockIdx.x * 128 + wave * 32;
  if (m0 >= total_rows) return;
  const int i = lane & 31, h = lane >> 5;
  long m = m0 + i;
  if (m >= total_rows) m = total_rows - 1;  // clamp loads, stores are masked
  const int b = (int)(m / rows), r = (int)(m % rows);
  const float* xb = x + (long)b * vsrc * CIN + h * HALF;
  const int* irow = idx + (long)r * seq;

  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = (f32x16){0.f};

  float a[HALF], an[HALF];
  {
    const float* src = xb + (long)irow[0] * CIN;
#pragma unroll
    for (int q = 0; q < HALF / 4; ++q) {
      f32x4 v = ld4(src + 4 * q);
      a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
    }
  }
  for (int s = 0; s < seq; ++s) {
    if (s + 1 < seq) {  // prefetch next slot's neighbour row
      const float* src = xb + (long)irow[s + 1] * CIN;
#pragma unroll
      for (int q = 0; q < HALF / 4; ++q) {
        f32x4 v = ld4(src + 4 * q);
        an[4 * q] = v.x; an[4 * q + 1] = v.y; an[4 * q + 2] = v.z; an[4 * q + 3] = v.w;
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = t * 32 + i;
      const float* wr = W_LDS ? &lds_w[n * KP + s * CIN + h * HALF]
                              : &w[(long)n * K + s * CIN + h * HALF];
#pragma unroll
      for (int q = 0; q < HALF / 4; ++q) {
        f32x4 bw = ld4(wr + 4 * q);
        acc[t] = mfma32(a[4 * q + 0], bw.x, acc[t]);
        acc[t] = mfma32(a[4 * q + 1], bw.y, acc[t]);
        acc[t] = mfma32(a[4 * q + 2], bw.z, acc[t]);
        acc[t] = mfma32(a[4 * q + 3], bw.w, acc[t]);
      }
    }
#pragma unroll
    for (int q = 0; q < HALF; ++q) a[q] = an[q];
  }

  // epilogue: bias + activation, lanes 0..31 / 32..63 each store one
  // 128-B row segment per register.
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = t * 32 + i;
    const float bn = bias ? bias[n] : 0.f;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      long mo = m0 + acc_row(rr, lane);
      if (mo < total_rows) {
        float v = acc[t][rr] + bn;
        if (ACT == CFSD_ACT_ELU) v = elu_f(v);
        y[mo * COUT + n] = v;
      }
    }
  }
}

// --------------------------------------------------------------------------
// Forward, VALU path for tiny channel counts (E0: CIN = 3; Dout: COUT = 3).
// One thread per output row; weights are read with wave-uniform addresses
// (scalar loads), neighbour rows with plain loads.
template <int CIN, int COUT, int ACT>
__global__ __launch_bounds__(256) void conv_fwd_small(const float* __restrict__ x,
                                                      const int* __restrict__ idx,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ bias,
                                                      float* __restrict__ y, int vsrc, int rows,
                                                      int seq, long total_rows) {
  long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= total_rows) return;
  const int b = (int)(m / rows), r = (int)(m % rows);
  const float* xb = x + (long)b * vsrc * CIN;
  const int K = seq * CIN;
  float acc[COUT];
#pragma unroll
  for (int o = 0; o < COUT; ++o) acc[o] = 0.f;
  for (int s = 0; s < seq; ++s) {
    const float* src = xb + (long)idx[(long)r * seq + s] * CIN;
    float xv[CIN];
    if (CIN % 4 == 0) {
#pragma unroll
      for (int q = 0; q < CIN / 4; ++q) {
        f32x4 v = ld4(src + 4 * q);
        xv[4 * q] = v.x; xv[4 * q + 1] = v.y; xv[4 * q + 2] = v.z; xv[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int c = 0; c < CIN; ++c) xv[c] = src[c];
    }
#pragma unroll
    for (int o = 0; o < COUT; ++o) {
      const float* wr = w + (long)o * K + s * CIN;
#pragma unroll
      for (int c = 0; c < CIN; ++c) acc[o] = fmaf(xv[c], wr[c], acc[o]);
    }
  }
#pragma unroll
  for (int o = 0; o < COUT; ++o) {
    float v = acc[o] + (bias ? bias[o] : 0.f);
    if (ACT == CFSD_ACT_ELU) v = elu_f(v);
    y[m * COUT + o] = v;
  }
}

// --------------------------------------------------------------------------
// Backward data, MFMA path.  dx rows are source vertices u (flattened with
// b).  For slot s the A operand is T_s[u, :] = sum_{r in inv(u,s)} dpre[r, :]
// (gather-sum through the inverse-spiral CSR, fixed order -> deterministic),
// the B operand is W_s^T staged in LDS as [s][c][COUT + 4].
template <int CIN, int COUT, bool W_LDS>
__global__ __launch_bounds__(256) void conv_dx_mfma(const float* __restrict__ dpre,
                                                    const int* __restrict__ inv_ptr,
                                                    const int* __restrict__ inv_row,
                                                    const float* __restrict__ w,
                                                    const float* __restrict__ elu_y,
                                                    float* __restrict__ dx, int vsrc, int rows,
                                                    int seq, long total_rows) {
  constexpr int HALF = COUT / 2;  // reduction channels (o) per lane half
  constexpr int NT = CIN / 32;    // output tiles over c
  constexpr int OP = COUT + 4;
  extern __shared__ float lds_wt[];
  const int K = seq * CIN;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;

  if (W_LDS) {
    // lds_wt[(s*CIN + c) * OP + o] = w[o, s*CIN + c]
    for (int e = threadIdx.x; e < COUT * K; e += 256) {
      int o = e / K, k = e % K;
      lds_wt[k * OP + o] = w[e];
    }
    __syncthreads();
  }

  const long m0 = (long)blockIdx.x * 128 + wave * 32;
  if (m0 >= total_rows) return;
  const int i = lane & 31, h = lane >> 5;
  long m = m0 + i;
  if (m >= total_rows) m = total_rows - 1;
  const int b = (int)(m / vsrc), u = (int)(m % vsrc);
  const float* db_ = dpre + (long)b * rows * COUT + h * HALF;
  const int* pu = inv_ptr + (long)u * seq;

  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = (f32x16){0.f};

  for (int s = 0; s < seq; ++s) {
    float a[HALF];
#pragma unroll
    for (int q = 0; q < HALF; ++q) a[q] = 0.f;
    const int beg = pu[s], end = pu[s + 1];
    for (int e = beg; e < end; ++e) {
      const float* src = db_ + (long)inv_row[e] * COUT;
#pragma unroll
      for (int q = 0; q < HALF / 4; ++q) {
        f32x4 v = ld4(src + 4 * q);
        a[4 * q] += v.x; a[4 * q + 1] += v.y; a[4 * q + 2] += v.z; a[4 * q + 3] += v.w;
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int c = t * 32 + i;
      if (W_LDS) {
        const float* wr = &lds_wt[(s * CIN + c) * OP + h * HALF];
#pragma unroll
        for (int q = 0; q < HALF / 4; ++q) {
          f32x4 bw = ld4(wr + 4 * q);
          acc[t] = mfma32(a[4 * q + 0], bw.x, acc[t]);
          acc[t] = mfma32(a[4 * q + 1], bw.y, acc[t]);
          acc[t] = mfma32(a[4 * q + 2], bw.z, acc[t]);
          acc[t] = mfma32(a[4 * q + 3], bw.w, acc[t]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < HALF; ++q)
          acc[t] = mfma32(a[q], w[(long)(h * HALF + q) * K + s * CIN + c], acc[t]);
      }
    }
  }

#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c = t * 32 + i;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      long mo = m0 + acc_row(rr, lane);
      if (mo < total_rows) {
        float v = acc[t][rr];
        if (elu_y) v *= elu_grad_from_out(elu_y[mo * CIN + c]);
        dx[mo * CIN + c] = v;
      }
    }
  }
}

// Backward data, VALU path for COUT = 3 (Dout): one thread per source row.
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv_dx_small(const float* __restrict__ dpre,
                                                     const int* __restrict__ inv_ptr,
                                                     const int* __restrict__ inv_row,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ elu_y,
                                                     float* __restrict__ dx, int vsrc, int rows,
                                                     int seq, long total_rows) {
  long m = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= total_rows) return;
  const int b = (int)(m / vsrc), u = (int)(m % vsrc);
  const int K = seq * CIN;
  const float* db_ = dpre + (long)b * rows * COUT;
  float acc[CIN];
#pragma unroll
  for (int c = 0; c < CIN; ++c) acc[c] = 0.f;
  for (int s = 0; s < seq; ++s) {
    float t[COUT];
#pragma unroll
    for (int o = 0; o < COUT; ++o) t[o] = 0.f;
    const int beg = inv_ptr[(long)u * seq + s], end = inv_ptr[(long)u * seq + s + 1];
    for (int e = beg; e < end; ++e) {
      const float* src = db_ + (long)inv_row[e] * COUT;
#pragma unroll
      for (int o = 0; o < COUT; ++o) t[o] += src[o];
    }
#pragma unroll
    for (int o = 0; o < COUT; ++o) {
      const float* wr = w + (long)o * K + s * CIN;
#pragma unroll
      for (int c = 0; c < CIN; ++c) acc[c] = fmaf(t[o], wr[c], acc[c]);
    }
  }
  float* out = dx + m * CIN;
  const float* ey = elu_y ? elu_y + m * CIN : nullptr;
#pragma unroll
  for (int c = 0; c < CIN; ++c) out[c] = ey ? acc[c] * elu_grad_from_out(ey[c]) : acc[c];
}

// --------------------------------------------------------------------------
// Backward weight, MFMA path.  Units u = (s, ot, ct): output tile
// dW[ot*32 .. +32][s*CIN + ct*32 .. +32].  Each wave owns UPW units and a
// strided set of 32-row blocks; lane half h takes rows j + 16h of a block
// (MFMA step j reduces the pair).  A = dpre^T (o on lanes), B = gathered x
// (c on lanes).  The block's 4 wave partials are summed through LDS in
// wave order and written as one slab: ws[(blockIdx.x * gridDim.y + y) * UPW * 1024].
// db partials (sum over rows of dpre) go to ws_db[blockIdx.x * COUT + o] from
// the y == 0 blocks.
template <int CIN, int COUT, int UPW>
__global__ __launch_bounds__(256) void conv_dw_mfma(const float* __restrict__ x,
                                                    const int* __restrict__ idx,
                                                    const float* __restrict__ dpre,
                                                    float* __restrict__ ws,
                                                    float* __restrict__ ws_db, int vsrc,
                                                    int rows, int seq, long total_rows) {
  constexpr int OT = COUT / 32, CT = CIN / 32;
  __shared__ float red[UPW * 1024];
  __shared__ float redb[COUT];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int n_units = seq * OT * CT;
  const int u0 = blockIdx.y * UPW;

  f32x16 acc[UPW];
#pragma unroll
  for (int q = 0; q < UPW; ++q) acc[q] = (f32x16){0.f};
  float dbs[OT];
#pragma unroll
  for (int t = 0; t < OT; ++t) dbs[t] = 0.f;

  const long nblk = (total_rows + 31) / 32;
  const long stride = (long)gridDim.x * 4;
  for (long blk = (long)blockIdx.x * 4 + wave; blk < nblk; blk += stride) {
    const long mbase = blk * 32;
    // this lane's row for the index broadcast: row mbase + i
    long mi = mbase + i;
    const bool mi_ok = mi < total_rows;
    if (!mi_ok) mi = total_rows - 1;
    const int bi = (int)(mi / rows), ri = (int)(mi % rows);
    // dpre fragments: rows mbase + 16h + j, column o = ot*32 + i
    float dp[OT][16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      long mj = mbase + 16 * h + j;
      bool ok = mj < total_rows;
      long mc = ok ? mj : total_rows - 1;
#pragma unroll
      for (int t = 0; t < OT; ++t) {
        float v = dpre[mc * COUT + t * 32 + i];
        dp[t][j] = ok ? v : 0.f;
      }
    }
    if (blockIdx.y == 0) {
#pragma unroll
      for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) dbs[t] += dp[t][j];
    }
#pragma unroll
    for (int q = 0; q < UPW; ++q) {
      const int un = u0 + q;
      if (un >= n_units) break;
      const int s = un / (OT * CT);
      const int ot = (un / CT) % OT;
      const int ct = un % CT;
      const int my_src = idx[(long)ri * seq + s];
      const long my_base = ((long)bi * vsrc + my_src) * CIN + ct * 32;
      float xv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        // row mbase + 16h + j lives in lane (16h + j) for the index broadcast
        long base = __shfl(my_base, 16 * h + j);
        xv[j] = x[base + i];
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[q] = mfma32(dp[ot][j], xv[j], acc[q]);
    }
  }

  // block reduction in fixed wave order (deterministic)
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int q = 0; q < UPW; ++q)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          int e = q * 1024 + acc_row(rr, lane) * 32 + i;  // [o][c]
          red[e] = (wv == 0) ? acc[q][rr] : red[e] + acc[q][rr];
        }
      if (blockIdx.y == 0) {
#pragma unroll
        for (int t = 0; t < OT; ++t) {
          float v = dbs[t] + __shfl_xor(dbs[t], 32);
          if (h == 0) redb[t * 32 + i] = (wv == 0) ? v : redb[t * 32 + i] + v;
        }
      }
    }
    __syncthreads();
  }
  float* slab = ws + ((long)blockIdx.x * gridDim.y + blockIdx.y) * (UPW * 1024);
  for (int e = threadIdx.x; e < UPW * 1024; e += 256) slab[e] = red[e];
  if (blockIdx.y == 0)
    for (int o = threadIdx.x; o < COUT; o += 256) ws_db[(long)blockIdx.x * COUT + o] = redb[o];
}

// Reduce the dw slabs: dw[o, s*CIN + ct*32 + c] = sum_p slab_p[unit][o%32][c].
// 16 threads per output element, each sums a strided subset of slabs, then a
// fixed-order xor-shuffle tree (deterministic).
template <int CIN, int COUT, int UPW>
__global__ __launch_bounds__(256) void conv_dw_reduce(const float* __restrict__ ws,
                                                      const float* __restrict__ ws_db,
                                                      float* __restrict__ dw,
                                                      float* __restrict__ db, int seq,
                                                      int n_slabs, int gy) {
  constexpr int OT = COUT / 32, CT = CIN / 32;
  const long n_out = (long)COUT * seq * CIN;
  long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long e = tid >> 4;
  const int sub = threadIdx.x & 15;
  const bool is_db = e >= n_out;
  if (e >= n_out + COUT) e = n_out + COUT - 1;  // keep lanes alive for the shuffle
  float sum = 0.f;
  if (!is_db) {
    const int o = (int)(e / (seq * CIN));
    const int k = (int)(e % (seq * CIN));
    const int s = k / CIN, cc = k % CIN;
    const int ot = o / 32, ct = cc / 32;
    const int un = (s * OT + ot) * CT + ct;
    const int y = un / UPW, q = un % UPW;
    const long off = (long)q * 1024 + (o % 32) * 32 + (cc % 32);
    for (int p = sub; p < n_slabs; p += 16) sum += ws[((long)p * gy + y) * (UPW * 1024) + off];
  } else {
    const int o = (int)(e - n_out);
    for (int p = sub; p < n_slabs; p += 16) sum += ws_db[(long)p * COUT + o];
  }
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1) sum += __shfl_xor(sum, d);
  if (sub == 0 && (tid >> 4) < n_out + COUT) {
    if (!is_db) dw[e] = sum;
    else db[e - n_out] = sum;
  }
}

// Backward weight, VALU path for tiny channels: one output weight column
// group per thread block.  Thread t of a block owns (o, k) pairs; rows are
// split across blocks and partial sums go to slabs [block][COUT*K + COUT].
template <int CIN, int COUT>
__global__ __launch_bounds__(256) void conv_dw_small(const float* __restrict__ x,
                                                     const int* __restrict__ idx,
                                                     const float* __restrict__ dpre,
                                                     float* __restrict__ ws, int vsrc, int rows,
                                                     int seq, long total_rows, int rows_per_blk) {
  // element e in [0, COUT*K + COUT): weights then biases
  const int K = seq * CIN;
  const int n_el = COUT * K + COUT;
  const long r0 = (long)blockIdx.x * rows_per_blk;
  const long r1 = min(total_rows, r0 + rows_per_blk);
  for (int e = threadIdx.x; e < n_el; e += blockDim.x) {
    float sum = 0.f;
    if (e < COUT * K) {
      const int o = e / K, k = e % K;
      const int s = k / CIN, c = k % CIN;
      for (long m = r0; m < r1; ++m) {
        const int b = (int)(m / rows), r = (int)(m % rows);
        const float xv = x[((long)b * vsrc + idx[(long)r * seq + s]) * CIN + c];
        sum = fmaf(dpre[m * COUT + o], xv, sum);
      }
    } else {
      const int o = e - COUT * K;
      for (long m = r0; m < r1; ++m) sum += dpre[m * COUT + o];
    }
    ws[(long)blockIdx.x * n_el + e] = sum;
  }
}

__global__ __launch_bounds__(256) void slab_reduce(const float* __restrict__ ws, int n_slabs,
                                                   int n_el, float* __restrict__ out_a, int n_a,
                                                   float* __restrict__ out_b) {
  long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long e = tid >> 4;
  const int sub = threadIdx.x & 15;
  const bool valid = e < n_el;
  if (!valid) e = n_el - 1;
  float sum = 0.f;
  for (int p = sub; p < n_slabs; p += 16) sum += ws[(long)p * n_el + e];
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1) sum += __shfl_xor(sum, d);
  if (sub == 0 && valid) {
    if (e < n_a) out_a[e] = sum;
    else out_b[e - n_a] = sum;
  }
}

// Materialising gather (roofline probe): g[m, s*CIN + c] = x[b, idx[r,s], c].
// One thread per 16-B chunk of the output.
__global__ __launch_bounds__(256) void spiral_gather_k(const float* __restrict__ x,
                                                       const int* __restrict__ idx,
                                                       float* __restrict__ g, int vsrc, int rows,
                                                       int seq, int cin, long total_chunks) {
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total_chunks) return;
  const int c4 = cin / 4;
  const int q = (int)(t % c4);
  long rs = t / c4;
  const int s = (int)(rs % seq);
  const long m = rs / seq;
  const int b = (int)(m / rows), r = (int)(m % rows);
  const float* src = x + ((long)b * vsrc + idx[(long)r * seq + s]) * cin + 4 * q;
  st4(g + t * 4, ld4(src));
}

}  // namespace cfsd

using namespace cfsd;

// ============================================================== C ABI
static int check_conv_args(const void* a, const void* b, const void* c, int batch, int vsrc,
                           int rows, int seq, int cin, int cout) {
  if (!a || !b || !c) return set_error(CFSD_EINVAL, "null pointer");
  if (batch <= 0 || vsrc <= 0 || rows <= 0 || seq <= 0 || cin <= 0 || cout <= 0)
    return set_error(CFSD_EINVAL, "non-positive size (batch=%d vsrc=%d rows=%d seq=%d cin=%d cout=%d)",
                     batch, vsrc, rows, seq, cin, cout);
  return CFSD_OK;
}

template <int CIN, int COUT, int ACT>
static int launch_fwd_mfma(const float* x, const int* idx, const float* w, const float* bias,
                           float* y, int vsrc, int rows, int seq, long M, hipStream_t st) {
  const size_t lds = (size_t)COUT * (seq * CIN + 4) * sizeof(float);
  dim3 grid((unsigned)((M + 127) / 128));
  if (lds <= 64 * 1024)
    hipLaunchKernelGGL((conv_fwd_mfma<CIN, COUT, ACT, true>), grid, dim3(256), lds, st, x, idx, w,
                       bias, y, vsrc, rows, seq, M);
  else
    hipLaunchKernelGGL((conv_fwd_mfma<CIN, COUT, ACT, false>), grid, dim3(256), 0, st, x, idx, w,
                       bias, y, vsrc, rows, seq, M);
  return launch_status("spiral_conv_fwd");
}

template <int CIN, int COUT, int ACT>
static int launch_fwd_small(const float* x, const int* idx, const float* w, const float* bias,
                            float* y, int vsrc, int rows, int seq, long M, hipStream_t st) {
  dim3 grid((unsigned)((M + 255) / 256));
  hipLaunchKernelGGL((conv_fwd_small<CIN, COUT, ACT>), grid, dim3(256), 0, st, x, idx, w, bias, y,
                     vsrc, rows, seq, M);
  return launch_status("spiral_conv_fwd_small");
}

#define CFSD_DISPATCH_MFMA(CIN_, COUT_, CALL) \
  if (cin == CIN_ && cout == COUT_) return CALL;

extern "C" int cfsd_spiral_conv_fwd(const float* x, const int32_t* idx, const float* w,
                                    const float* bias, float* y, int batch, int vsrc, int rows,
                                    int seq, int cin, int cout, int act, void* stream) {
  int rc = check_conv_args(x, idx, w, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!y) return set_error(CFSD_EINVAL, "null y");
  if (act != CFSD_ACT_NONE && act != CFSD_ACT_ELU) return set_error(CFSD_EINVAL, "bad act %d", act);
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * rows;
#define FWD(CIN_, COUT_)                                                                       \
  if (cin == CIN_ && cout == COUT_) {                                                          \
    return act == CFSD_ACT_ELU                                                                 \
               ? launch_fwd_mfma<CIN_, COUT_, CFSD_ACT_ELU>(x, idx, w, bias, y, vsrc, rows, seq, M, st) \
               : launch_fwd_mfma<CIN_, COUT_, CFSD_ACT_NONE>(x, idx, w, bias, y, vsrc, rows, seq, M, st); \
  }
  FWD(32, 32) FWD(32, 64) FWD(64, 32) FWD(64, 64)
#undef FWD
#define FWDS(CIN_, COUT_)                                                                      \
  if (cin == CIN_ && cout == COUT_) {                                                          \
    return act == CFSD_ACT_ELU                                                                 \
               ? launch_fwd_small<CIN_, COUT_, CFSD_ACT_ELU>(x, idx, w, bias, y, vsrc, rows, seq, M, st) \
               : launch_fwd_small<CIN_, COUT_, CFSD_ACT_NONE>(x, idx, w, bias, y, vsrc, rows, seq, M, st); \
  }
  FWDS(3, 32) FWDS(3, 64) FWDS(32, 3) FWDS(64, 3) FWDS(3, 16) FWDS(16, 3) FWDS(16, 16)
#undef FWDS
  return set_error(CFSD_EINVAL, "spiral_conv_fwd: unsupported channels %d -> %d", cin, cout);
}

extern "C" int cfsd_spiral_conv_bwd_data(const float* dpre, const int32_t* inv_ptr,
                                         const int32_t* inv_row, const float* w,
                                         const float* elu_y, float* dx, int batch, int vsrc,
                                         int rows, int seq, int cin, int cout, void* stream) {
  int rc = check_conv_args(dpre, inv_ptr, inv_row, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!w || !dx) return set_error(CFSD_EINVAL, "null w/dx");
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * vsrc;
#define DXM(CIN_, COUT_)                                                                         \
  if (cin == CIN_ && cout == COUT_) {                                                            \
    const size_t lds = (size_t)seq * CIN_ * (COUT_ + 4) * sizeof(float);                         \
    dim3 grid((unsigned)((M + 127) / 128));                                                      \
    if (lds <= 80 * 1024)                                                                        \
      hipLaunchKernelGGL((conv_dx_mfma<CIN_, COUT_, true>), grid, dim3(256), lds, st, dpre,      \
                         inv_ptr, inv_row, w, elu_y, dx, vsrc, rows, seq, M);                    \
    else                                                                                         \
      hipLaunchKernelGGL((conv_dx_mfma<CIN_, COUT_, false>), grid, dim3(256), 0, st, dpre,       \
                         inv_ptr, inv_row, w, elu_y, dx, vsrc, rows, seq, M);                    \
    return launch_status("spiral_conv_bwd_data");                                                \
  }
  DXM(32, 32) DXM(32, 64) DXM(64, 32) DXM(64, 64)
#undef DXM
#define DXS(CIN_, COUT_)                                                                        \
  if (cin == CIN_ && cout == COUT_) {                                                           \
    hipLaunchKernelGGL((conv_dx_small<CIN_, COUT_>), dim3((unsigned)((M + 255) / 256)),         \
                       dim3(256), 0, st, dpre, inv_ptr, inv_row, w, elu_y, dx, vsrc, rows, seq, M); \
    return launch_status("spiral_conv_bwd_data_small");                                        \
  }
  DXS(32, 3) DXS(64, 3) DXS(3, 32) DXS(3, 64) DXS(16, 3) DXS(3, 16) DXS(16, 16)
#undef DXS
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data: unsupported channels %d -> %d", cin, cout);
}

// ---- bwd weight: launch geometry shared by workspace query and launch
namespace {
struct DwGeom {
  bool mfma;
  int gx, gy, upw;
  long rows_per_blk;
  size_t ws_floats;
};

DwGeom dw_geom(int batch, int rows, int seq, int cin, int cout) {
  DwGeom g{};
  const long M = (long)batch * rows;
  const bool mfma = (cin % 32 == 0) && (cout % 32 == 0) && cin <= 64 && cout <= 64;
  g.mfma = mfma;
  if (mfma) {
    const int units = seq * (cout / 32) * (cin / 32);
    g.upw = 9;
    g.gy = (units + g.upw - 1) / g.upw;
    const long nblk = (M + 31) / 32;
    long gx = (nblk + 31) / 32;  // ~8 row-blocks per wave
    if (gx > 256) gx = 256;
    if (gx < 1) gx = 1;
    g.gx = (int)gx;
    g.ws_floats = (size_t)g.gx * g.gy * g.upw * 1024 + (size_t)g.gx * cout;
  } else {
    long per = 512;
    long gx = (M + per - 1) / per;
    if (gx > 512) {
      gx = 512;
      per = (M + gx - 1) / gx;
    }
    g.gx = (int)gx;
    g.gy = 1;
    g.rows_per_blk = per;
    g.ws_floats = (size_t)g.gx * ((size_t)cout * seq * cin + cout);
  }
  return g;
}
}  // namespace

extern "C" size_t cfsd_spiral_conv_bwd_weight_workspace(int batch, int rows, int seq, int cin,
                                                        int cout) {
  if (batch <= 0 || rows <= 0 || seq <= 0 || cin <= 0 || cout <= 0) return 0;
  return dw_geom(batch, rows, seq, cin, cout).ws_floats * sizeof(float);
}

extern "C" int cfsd_spiral_conv_bwd_weight(const float* x, const int32_t* idx, const float* dpre,
                                           float* dw, float* db, float* workspace,
                                           size_t workspace_bytes, int batch, int vsrc, int rows,
                                           int seq, int cin, int cout, void* stream) {
  int rc = check_conv_args(x, idx, dpre, batch, vsrc, rows, seq, cin, cout);
  if (rc) return rc;
  if (!dw || !db || !workspace) return set_error(CFSD_EINVAL, "null dw/db/workspace");
  DwGeom g = dw_geom(batch, rows, seq, cin, cout);
  if (workspace_bytes < g.ws_floats * sizeof(float))
    return set_error(CFSD_EWORKSPACE, "workspace %zu < %zu bytes", workspace_bytes,
                     g.ws_floats * sizeof(float));
  hipStream_t st = (hipStream_t)stream;
  const long M = (long)batch * rows;
  if (g.mfma) {
    float* ws_db = workspace + (size_t)g.gx * g.gy * g.upw * 1024;
    const long n_out = (long)cout * seq * cin + cout;
    dim3 rg((unsigned)((n_out * 16 + 255) / 256));
#define DWM(CIN_, COUT_)                                                                       \
  if (cin == CIN_ && cout == COUT_) {                                                          \
    hipLaunchKernelGGL((conv_dw_mfma<CIN_, COUT_, 9>), dim3(g.gx, g.gy), dim3(256), 0, st, x,  \
                       idx, dpre, workspace, ws_db, vsrc, rows, seq, M);                      \
    rc = launch_status("spiral_conv_bwd_weight");                                              \
    if (rc) return rc;                                                                         \
    hipLaunchKernelGGL((conv_dw_reduce<CIN_, COUT_, 9>), rg, dim3(256), 0, st, workspace,      \
                       ws_db, dw, db, seq, g.gx, g.gy);                                        \
    return launch_status("spiral_conv_bwd_weight_reduce");                                     \
  }
    DWM(32, 32) DWM(32, 64) DWM(64, 32) DWM(64, 64)
#undef DWM
  } else {
    const int n_el = cout * seq * cin + cout;
#define DWS(CIN_, COUT_)                                                                          \
  if (cin == CIN_ && cout == COUT_) {                                                             \
    hipLaunchKernelGGL((conv_dw_small<CIN_, COUT_>), dim3(g.gx), dim3(256), 0, st, x, idx, dpre,  \
                       workspace, vsrc, rows, seq, M, (int)g.rows_per_blk);                       \
    rc = launch_status("spiral_conv_bwd_weight_small");                                           \
    if (rc) return rc;                                                                            \
    hipLaunchKernelGGL(slab_reduce, dim3((unsigned)(((long)n_el * 16 + 255) / 256)), dim3(256), 0, \
                       st, workspace, g.gx, n_el, dw, cout * seq * cin, db);                      \
    return launch_status("spiral_conv_bwd_weight_small_reduce");                                  \
  }
    DWS(3, 32) DWS(3, 64) DWS(32, 3) DWS(64, 3) DWS(3, 16) DWS(16, 3) DWS(16, 16)
#undef DWS
  }
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight: unsupported channels %d -> %d", cin, cout);
}

extern "C" int cfsd_spiral_gather(const float* x, const int32_t* idx, float* g, int batch,
                                  int vsrc, int rows, int seq, int cin, void* stream) {
  int rc = check_conv_args(x, idx, g, batch, vsrc, rows, seq, cin, 1);
  if (rc) return rc;
  if (cin % 4) return set_error(CFSD_EINVAL, "spiral_gather: cin %% 4 != 0");
  const long chunks = (long)batch * rows * seq * (cin / 4);
  hipLaunchKernelGGL(spiral_gather_k, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, idx, g, vsrc, rows, seq, cin, chunks);
  return launch_status("spiral_gather");
}
