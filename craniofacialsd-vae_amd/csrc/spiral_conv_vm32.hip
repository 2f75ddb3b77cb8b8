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
#include "dx_flat_vm32.h"

namespace cfsd {
namespace vm32 {


// ------------------------------------------------------------------ forward
// Wave = tile of UPT units (vertex r, mesh group mg of 16) x all COUT
// columns.  Lane (j, g): mesh j, channel chunks g, g + 4 (16 B each) of every
// neighbour = the B operand X^T[k][mesh]; A = W rows from LDS (the batch-major
// kernel's B fragment, unchanged).  Slot s + PD's gathers are in flight while
// slot s runs its MFMAs.  y vertex-major (yvm) or batch-major (the Enblock
// evaluated at the kept rows writes the coarser, batch-major level).
constexpr int kVm32FwdOcc = 4;  // waves per SIMD (VGPR budget 128)
template <int CIN, int COUT, int ACT, int UPT, int PD>
__global__ __launch_bounds__(256, kVm32FwdOcc) void conv_fwd_vm32(const float* __restrict__ x,
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


template <int CIN, int COUT, int FW, typename TY = float>
__global__ __launch_bounds__(512, kVm32DxOcc) void conv_dx_flat_vm32(const float* __restrict__ dpre,
                                                         const int4* __restrict__ flat,
                                                         const float* __restrict__ w,
                                                         const TY* __restrict__ elu_y,
                                                         TY* __restrict__ dx, int vsrc, int rows,
                                                         int batch, int dpvm, int dxvm) {
  extern __shared__ float lwt[];
  dx_flat_body<CIN, COUT, FW, TY>(dpre, flat, w, elu_y, dx, vsrc, rows, batch, dpvm, dxvm, blockIdx.x, gridDim.x,
                                  lwt);
}

// The row-subset Enblock backward with vertex-major x / dx (the fp32 step's
// E1): the flat-list data gradient above (dpre batch-major) and the dW slabs
// of conv_dw_lat_body (eight waves per workgroup, one (unit, row chunk) task
// each) as the two halves of ONE launch, workgroups interleaved (no dG round
// trip, no gather launch, one kernel boundary).
struct DxFlatArgs {
  const float* dpre;
  const int4* flat;
  const float* w;
  const float* elu_y;
  float* dx;
  int vsrc, rows, batch, dpvm, dxvm, nb;
};
#ifdef CFSD_LAT_STAMPS
// diagnostic build only (tools/kbench.py KB_STAMPFN=cfsd_debug_flat_stamps): role, start, end
__device__ unsigned long long g_flat_stamps[4096 * 3];
extern "C" int cfsd_debug_flat_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_flat_stamps), sizeof(g_flat_stamps), 0, hipMemcpyDeviceToHost);
}
#endif
template <int CIN, int COUT, int FW>
__global__ __launch_bounds__(512) void conv_bwd_flat_pair(const DxFlatArgs a, const DwLatArgs d) {
  extern __shared__ float lwt[];
  // the data-gradient role first (see conv_bwd_lat_pair)
  const int bid = (int)blockIdx.x;
  const bool is_dx = bid < a.nb;
  const int vb = is_dx ? bid : bid - a.nb;
#ifdef CFSD_LAT_STAMPS
  const unsigned long long t0 = wall_clock64();
#endif
  if (is_dx)
    dx_flat_body<CIN, COUT, FW>(a.dpre, a.flat, a.w, a.elu_y, a.dx, a.vsrc, a.rows, a.batch, a.dpvm, a.dxvm, vb,
                                a.nb, lwt);
  else
    conv_dw_lat_body<CIN, COUT, 8>(vb, d.nb, d.x, d.idx, d.dpre, d.ws, d.ws_db, d.vsrc, d.rows, d.total_rows,
                                   d.rchunk, d.n_chunks, d.batch, d.xvm, d.dpvm, lwt);  // lwt >= lat_red_floats(8)
#ifdef CFSD_LAT_STAMPS
  __syncthreads();
  if (threadIdx.x == 0 && bid < 4096) {
    g_flat_stamps[3 * bid] = is_dx ? 1 : 2;
    g_flat_stamps[3 * bid + 1] = t0;
    g_flat_stamps[3 * bid + 2] = wall_clock64();
  }
#endif
}


// ------------------------------------------------------------------ weight gradient (32 -> 32)
// dW_s[o][c] = sum over (vertex v, mesh m) of dpre[v][m][o] x[idx[v][s]][m][c]
// (the Linear's weight gradient over the gathered rows, model.py:34, 40) for
// vertex-major x and dpre, batch % 16 == 0.  No LDS staging: a unit
// (vertex v, 16-mesh group) contributes K = 16 meshes to every slot, and in
// the v_mfma_f32_32x32x2_f32 lane map (A[o][k]: lane (o, h) ~ mesh 2j + h)
// both operands of step j are two consecutive 128-B rows of a contiguous
// 2-KiB block -- ONE coalesced 256-B dword load each.  A wave keeps all nine
// 32x32 slot accumulators (144 registers) for its whole contiguous unit
// range, so the MFMA pipe always has nine independent chains; dpre is loaded
// once per unit for the nine slots and the next unit's 80 loads are in
// flight while this unit runs its 72 MFMAs (one wave per SIMD: a workgroup
// of 4 waves per CU).  The 4 waves' accumulators are summed in LDS in fixed
// order into one conv_dw_mfma-layout slab ([9][32][32] + db[32]) per
// workgroup, reduced by conv_dw_reduce / dw_reduce_batch (kind 0).
constexpr int kDwvNs = 3;  // slots per wave (3: a slot group of three, 9: all nine)
constexpr int kDwvNr = 4;  // unit ranges per workgroup (waves = NR * 9 / NS)
constexpr int DWV_NS = kDwvNs, DWV_NR = kDwvNr, DWV_WAVES = DWV_NR * (kS / DWV_NS);
constexpr int DWV_THREADS = DWV_WAVES * 64;
constexpr int DWV_LDS = kS * 1024 + DWV_NR * 64;  // floats: the block's slab image + db partials
// PF: the next unit's operands loaded during this unit's MFMAs (the dW-only
// kernel, 125 VGPRs); PF = 0 keeps the body under 80 VGPRs so that two
// 12-wave workgroups share a CU (conv_bwd_vm_pair).  bid / nb: this
// workgroup's slab and the slab count; lds: DWV_LDS floats.
template <int PF>
__device__ __forceinline__ void dw_vm32_body(const float* __restrict__ x, const int* __restrict__ idx,
                                             const float* __restrict__ dpre, float* __restrict__ ws,
                                             float* __restrict__ ws_db, int vsrc, int rows, int batch, int bid,
                                             int nb, float* __restrict__ lds) {
  constexpr int C = 32, NEL = kS * 1024, NS = DWV_NS, NG = kS / NS;
  float* red = lds;
  float* dbl = lds + NEL;
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int sg = wave % NG, vg = wave / NG;  // slot group, unit range
  const int G16 = batch >> 4;
  const long n_units = (long)rows * G16;
  // XCD-contiguous unit ranges: blocks b, b + 8, ... (one XCD) split one 1/8
  const int G = nb < 8 ? nb : 8;
  const int grp = bid % G, lb = bid / G, nb_g = (nb - grp + G - 1) / G;
  const long per = (n_units + G - 1) / G;
  const long g0 = grp * per, g1 = min(n_units, g0 + per);
  const int nr = nb_g * DWV_NR, ri = lb * DWV_NR + vg;
  // the XCD's unit ranges interleaved (unit g0 + ri + k nr): its waves sweep
  // a narrow window of vertices together, so their neighbour blocks stay in
  // the XCD's L2 (contiguous ranges gathered the whole eighth at once: HBM
  // traffic 147 vs 93 MB per D3 launch at equal time)
  const long u0 = g0 + ri, u1 = g1, ustep = nr;
  const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, (int)((long)vsrc * batch * C * 4),
                                                    0x00020000);
  const auto rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dpre), 0, (int)((long)rows * batch * C * 4),
                                                    0x00020000);
  const int voff = lane * 4;  // + 256 j: rows 2j, 2j + 1 of the 16-mesh block
  f32x16 acc[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) acc[k] = (f32x16){0.f};
  float dbs = 0.f;
  float a[8], b[NS][8], an[8], bn[NS][8];
  auto load_unit = [&](long un, float (&da)[8], float (&db)[NS][8]) {
    const int uu = uni((int)un);
    const int v = uu / G16, mg = uu - v * G16;
    const int sd = (v * batch + mg * 16) * C * 4;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      da[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rd, voff + 256 * j, sd, 0));
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int sx = (uni(idx[v * kS + NS * sg + k]) * batch + mg * 16) * C * 4;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        db[k][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, voff + 256 * j, sx, 0));
    }
  };
  if (PF && u0 < u1) load_unit(u0, a, b);
  for (long un = u0; un < u1; un += ustep) {
    const bool more = PF && un + ustep < u1;  // uniform
    if (!PF) load_unit(un, a, b);
    if (more) load_unit(un + ustep, an, bn);
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int k = 0; k < NS; ++k) acc[k] = mfma32(a[j], b[k][j], acc[k]);
    if (sg == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dbs += a[j];
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] = an[j];
#pragma unroll
        for (int k = 0; k < NS; ++k) b[k][j] = bn[k][j];
      }
    }
  }
  // block combine in fixed unit-range order -> one slab [9][32 o][32 c] + db
  for (int g = 0; g < DWV_NR; ++g) {
    if (vg == g) {
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int e = (NS * sg + k) * 1024 + acc_row(rr, lane) * 32 + (lane & 31);
          red[e] = g == 0 ? acc[k][rr] : red[e] + acc[k][rr];
        }
      if (sg == 0) dbl[g * 64 + lane] = dbs;
    }
    __syncthreads();
  }
  float* slab = ws + (long)bid * NEL;
  for (int e = threadIdx.x; e < NEL / 4; e += DWV_THREADS) st4(slab + 4 * e, ld4(red + 4 * e));
  if (threadIdx.x < C) {  // lanes o and o + 32 of each range hold meshes 2j and 2j + 1
    float t = 0.f;
    for (int g = 0; g < DWV_NR; ++g) t += dbl[g * 64 + threadIdx.x] + dbl[g * 64 + 32 + threadIdx.x];
    ws_db[(long)bid * C + threadIdx.x] = t;
  }
}
__global__ __launch_bounds__(DWV_THREADS) void conv_dw_vm32(const float* __restrict__ x,
                                                            const int* __restrict__ idx,
                                                            const float* __restrict__ dpre,
                                                            float* __restrict__ ws, float* __restrict__ ws_db,
                                                            int vsrc, int rows, int batch) {
  __shared__ float lds[DWV_LDS];
  dw_vm32_body<1>(x, idx, dpre, ws, ws_db, vsrc, rows, batch, blockIdx.x, gridDim.x, lds);
}

// Both gradients of a vertex-major 32 -> 32 conv in ONE launch: data-gradient
// workgroups (dx_flat_body, 12 waves) and weight-gradient workgroups
// (dw_vm32_body without prefetch, one slab each), interleaved.  Both bodies
// fit 80 VGPRs, so a CU holds one workgroup of each (6 waves per SIMD) and the
// two latency-bound MFMA streams hide each other's memory waits.
struct DwVmArgs {
  const float* x;
  const int* idx;
  float* ws;
  float* ws_db;
  int nb;
};
#ifdef CFSD_LAT_STAMPS
// diagnostic build only (tools/kbench.py KB_STAMPFN=cfsd_debug_vmp_stamps): role, start, end
__device__ unsigned long long g_vmp_stamps[4096 * 3];
extern "C" int cfsd_debug_vmp_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_vmp_stamps), sizeof(g_vmp_stamps), 0, hipMemcpyDeviceToHost);
}
#endif
template <int FW>
__global__ __launch_bounds__(DWV_THREADS, 2 * DWV_WAVES / 4) void conv_bwd_vm_pair(const DxFlatArgs a,
                                                                                const DwVmArgs d) {
  extern __shared__ float lds[];
  const int bid = blockIdx.x, both = 2 * min(a.nb, d.nb);
  bool is_dx;
  int vb;
  if (bid < both) {
    is_dx = (bid & 1) == 0;
    vb = bid >> 1;
  } else {
    is_dx = a.nb > d.nb;
    vb = bid - both + both / 2;
  }
#ifdef CFSD_LAT_STAMPS
  const unsigned long long t0 = wall_clock64();
#endif
  if (is_dx)
    dx_flat_body<32, 32, FW, float, DWV_WAVES>(a.dpre, a.flat, a.w, a.elu_y, a.dx, a.vsrc, a.rows, a.batch, 1, 1,
                                               vb, a.nb, lds);
  else
    dw_vm32_body<0>(d.x, d.idx, a.dpre, d.ws, d.ws_db, a.vsrc, a.rows, a.batch, vb, d.nb, lds);
#ifdef CFSD_LAT_STAMPS
  __syncthreads();
  if (threadIdx.x == 0 && bid < 4096) {
    g_vmp_stamps[3 * bid] = is_dx ? 1 : 2;
    g_vmp_stamps[3 * bid + 1] = t0;
    g_vmp_stamps[3 * bid + 2] = wall_clock64();
  }
#endif
}


// ------------------------------------------------------------------ output conv backward (32 -> 3)
// dx and dW/db of the xyz output conv (model.py:172-173 and its autograd) for
// vertex-major x / elu_y / dx and a vertex-major dout, batch % 16 == 0.
// Wave = unit (source vertex u, mesh group mg):
//  (1) T[s][m][o] = sum over u's flat inverse list (ascending p = 9r + s) of
//      dout[r][m][o]: lane l < 48 owns (m = l / 3, o = l % 3), one dword of
//      the 192-B dout block per entry, all FW entries in flight at once
//      (absent entries out of range).  Per (s, m, o) the rows are added in
//      list order, as the batch-major kernel adds its head rows;
//  (2) dx^T[c][m] = sum_k W'[k][c] T[k][m] (k = 3s + o, 27 rows padded to 28):
//      16x16x4 MFMAs, A = W' from LDS, B = T from a per-wave LDS image;
//      elu'(elu_y) epilogue, 16-B stores;
//  (3) dW'[k][c] += sum_m T[k][m] x[m][c] (K = the 16 meshes), kept in
//      registers across the wave's units, summed over the block's waves in
//      fixed order into one plain slab [3*288 + 3] (slab_reduce /
//      dw_reduce_batch kind 1); db[o] = sum of T[0][m][o] (slot 0 of every
//      spiral is the vertex itself: each output row is in exactly one slot-0
//      list).
// The batch-major kernel (conv_bwd_out_mfma) runs 32-row tiles at one wave
// per SIMD with every memory latency exposed per tile; here a unit's
// memory traffic is one flat list, 9 contiguous dout blocks and the 2-KiB x /
// dx blocks.
constexpr int kBoWaves = 4;  // waves per workgroup (one workgroup = one dW slab)
template <typename TX, int FW>
__global__ __launch_bounds__(64 * kBoWaves, kBoWaves) void conv_bwd_out_vm(const float* __restrict__ dout,
                                                       const int4* __restrict__ flat,
                                                       const float* __restrict__ w,
                                                       const TX* __restrict__ elu_y,
                                                       const TX* __restrict__ x, TX* __restrict__ dx,
                                                       float* __restrict__ ws, int vsrc, int rows,
                                                       int batch) {
  constexpr int CIN = 32, CO = 3, KR = kS * CO, KP = 28, K = kS * CIN, NEL = CO * K + CO;
  constexpr int WS = 48;  // W' row stride: conflict-free A reads (lane (c, g) -> bank 16g + c)
  constexpr int TS = 17;  // T row stride: conflict-free A reads of the dW step
  constexpr int FQ = FW / 4;
  __shared__ float wl[KP * WS];
  __shared__ float tl_all[kBoWaves * 32 * TS];
  __shared__ float red[NEL];
  __shared__ float dbl[kBoWaves * 48];
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int i = lane & 15, g = lane >> 4;
  // W'[k][c] = W[o][s*CIN + c], k = 3s + o; row 27 (padding) zero
  for (int e = threadIdx.x; e < KP * CIN; e += blockDim.x) {
    const int k = e / CIN, c = e % CIN;
    wl[k * WS + c] = k < KR ? w[(k % CO) * K + (k / CO) * CIN + c] : 0.f;
  }
  float* tl = tl_all + wave * 32 * TS;
  for (int e = lane; e < 32 * TS; e += 64) tl[e] = 0.f;  // rows 27..31 stay zero
  __syncthreads();
  const int G16 = batch >> 4;
  const long n_units = (long)vsrc * G16;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dout), 0,
                                                    (int)((long)rows * batch * CO * 4), 0x00020000);
  const int rstride = batch * CO * 4;  // bytes between two vertices' dout blocks
  const int m3 = lane / 3, o3 = lane - 3 * m3;
  f32x4 dwacc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) dwacc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbs = 0.f;
  // Each unit issues its flat list, dout dwords, x and elu_y at its top and
  // waits for them: no cross-unit prefetch.  Prefetching the next unit's
  // list + dout (one or two units ahead, scalar or vector-loaded lists) was
  // 2-7 us SLOWER (kbench, round 4): four waves per SIMD already keep the
  // CU's vector-memory pipeline at its limit (TD busy ~60 %, most of it
  // stalled on the L1; SQ counters) and the prefetch registers cost
  // occupancy.  A per-slot head-row table that removes the list's slot decode
  // (~40 % fewer scalar instructions) did not help either (28.1 vs 26.4 us).
  const TileSweep sw = xcd_sweep(n_units, kBoWaves, wave);
  const int voffl = lane < 48 ? lane * 4 : kAbsent;
  auto load_list = [&](long unit, int (&pe)[FW]) {
    const int u = uni((int)unit) / G16;
#pragma unroll
    for (int q = 0; q < FQ; ++q) {
      const int4 f = flat[(long)u * FQ + q];
      pe[4 * q] = uni(f.x);
      pe[4 * q + 1] = uni(f.y);
      pe[4 * q + 2] = uni(f.z);
      pe[4 * q + 3] = uni(f.w);
    }
  };
  auto load_dout = [&](long unit, const int (&pe)[FW], float (&v)[FW]) {
    const int mg = uni((int)unit) % G16;
    const int voff = voffl + mg * 48 * 4;
#pragma unroll
    for (int e = 0; e < FW; ++e)
      v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           rs, voff, pe[e] >= 0 ? (pe[e] / kS) * rstride : kAbsent, 0));
  };
  for (long unit = sw.begin; unit < sw.end; unit += sw.step) {
    const int un = uni((int)unit);
    const int u = un / G16, mg = un - u * G16;
    const long row = (long)u * batch + mg * 16 + i;
    // x (dW operand, lane (g, c)) and elu_y (dx epilogue, lane (m, g)) early
    const TX* xb = x + ((long)u * batch + mg * 16) * CIN + i;
    float xv[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) xv[q][nt] = ldf(xb + (4 * q + g) * CIN + 16 * nt);
    f32x4 ey[2];
    if (elu_y) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) ey[ct] = ld4f(elu_y + row * CIN + 16 * ct + 4 * g);
    }
    int pe[FW];
    float v[FW];
    load_list(unit, pe);
    load_dout(unit, pe, v);
    float t[kS];
#pragma unroll
    for (int s = 0; s < kS; ++s) t[s] = 0.f;
#pragma unroll
    for (int e = 0; e < FW; ++e) {
      if (pe[e] < 0) break;  // uniform: padding from here on
      const int se = pe[e] % kS;
      switch (se) {  // uniform: one add per entry instead of 9 selects + 9 adds (t is never -0: same bits)
        case 0: t[0] += v[e]; break;
        case 1: t[1] += v[e]; break;
        case 2: t[2] += v[e]; break;
        case 3: t[3] += v[e]; break;
        case 4: t[4] += v[e]; break;
        case 5: t[5] += v[e]; break;
        case 6: t[6] += v[e]; break;
        case 7: t[7] += v[e]; break;
        default: t[8] += v[e]; break;
      }
    }
    dbs += t[0];
    if (lane < 48) {
#pragma unroll
      for (int s = 0; s < kS; ++s) tl[(CO * s + o3) * TS + m3] = t[s];
    }
    wave_sync_lds();
    // dx^T = W'^T . T  (2 column tiles x 7 k-steps)
    f32x4 acc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) {
      const float b = tl[(4 * q + g) * TS + i];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) acc[ct] = mfma16(wl[(4 * q + g) * WS + 16 * ct + i], b, acc[ct]);
    }
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      f32x4 vv = acc[ct];
      if (elu_y) {
        vv.x *= elu_grad_from_out(ey[ct].x);
        vv.y *= elu_grad_from_out(ey[ct].y);
        vv.z *= elu_grad_from_out(ey[ct].z);
        vv.w *= elu_grad_from_out(ey[ct].w);
      }
      if (dx) st4f(dx + row * CIN + 16 * ct + 4 * g, vv);
    }
    // dW' += T . x  (K = meshes: 4 steps; 2 k-row tiles x 2 column tiles)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const float a = tl[(16 * mt + i) * TS + 4 * q + g];
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) dwacc[mt][nt] = mfma16(a, xv[q][nt], dwacc[mt][nt]);
      }
    wave_sync_lds();  // T image free for the next unit
  }
  // block combine in fixed wave order -> one slab
  if (lane < 48) dbl[wave * 48 + lane] = dbs;
  for (int wv = 0; wv < kBoWaves; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int k = 16 * mt + 4 * g + rr, c = 16 * nt + i;
            if (k < KR) {
              const int e = (k % CO) * K + (k / CO) * CIN + c;
              red[e] = wv == 0 ? dwacc[mt][nt][rr] : red[e] + dwacc[mt][nt][rr];
            }
          }
    }
    __syncthreads();
  }
  if (threadIdx.x < CO) {
    float sdb = 0.f;
    for (int wv = 0; wv < kBoWaves; ++wv)
      for (int m = 0; m < 16; ++m) sdb += dbl[wv * 48 + m * CO + threadIdx.x];
    red[CO * K + threadIdx.x] = sdb;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NEL; e += 64 * kBoWaves) ws[(long)blockIdx.x * NEL + e] = red[e];
}


// ------------------------------------------------------------------ output conv forward (32 -> CO <= 3)
// The xyz output conv (model.py:172) for a vertex-major x, batch % 8 == 0.
// Lane (r8, q): row r8 of an 8-row group (8 meshes of one vertex: each
// neighbour load is ONE contiguous 1-KiB wave access), input channels
// 4q .. 4q + 3.  A wave runs U groups per step: the U x 9 neighbour loads
// are all in flight before the first FMA (spiral offsets wave-uniform, in
// SGPRs), and every W fragment read from LDS serves all U groups (the
// batch-major conv_fwd_out_small re-reads the 27 fragments per 8 rows).
// Per output the products are accumulated in conv_fwd_out_small's order
// (slot by slot, 4 channels by fmaf per lane, then the xor tree 4, 2, 1 over
// the 8 lanes of the row, then the bias), so both layouts give the same bits.
constexpr int kVmOutU = 1;
// output-conv forward: 6 workgroups on every CU (17.7 vs 18.9 us with the
// balanced-iteration grid, profiles/round5r_kprof_grid_bf16_out.txt)
constexpr int kVmOutFwdBpc = 6;
template <int CO, int ACT, int U, typename TX>
__global__ __launch_bounds__(256) void conv_fwd_out_vm(const TX* __restrict__ x, const int* __restrict__ idx,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       float* __restrict__ y, int vsrc, int rows, int batch,
                                                       int yvm) {
  constexpr int CIN = 32, K = kS * CIN, EB = (int)sizeof(TX);
  __shared__ f32x4 lw[CO * K / 4];
  for (int i = threadIdx.x; i < CO * K / 4; i += blockDim.x) lw[i] = ld4(w + 4 * i);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const int q = lane & 7, r8 = lane >> 3;
  float bo[CO];
#pragma unroll
  for (int o = 0; o < CO; ++o) bo[o] = bias ? bias[o] : 0.f;
  const long n_grp = (long)rows * (batch >> 3);
  const long n_it = (n_grp + U - 1) / U;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<TX*>(x), 0, (int)((long)vsrc * batch * CIN * EB),
                                                    0x00020000);
  const int vstride = batch * CIN * EB;  // bytes between two vertices' blocks
  const TileSweep sw = xcd_sweep(n_it, 4, wave);
  for (long it = sw.begin; it < sw.end; it += sw.step) {
    int vv[U], bb[U], voff[U], soff[U][kS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long gl = it * U + u;
      if (gl >= n_grp) gl = n_grp - 1;  // clamp loads, stores are skipped
      const int m0 = uni((int)gl) * 8;
      vv[u] = m0 / batch;
      bb[u] = m0 - vv[u] * batch + r8;
      voff[u] = (bb[u] * CIN + 4 * q) * EB;
#pragma unroll
      for (int s = 0; s < kS; ++s) soff[u][s] = uni(idx[vv[u] * kS + s]) * vstride;
    }
    f32x4 xv[U][kS];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 0; s < kS; ++s) {
        if constexpr (EB == 4) {
          xv[u][s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff[u], soff[u][s], 0));
        } else {
          const u32x2 h = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff[u], soff[u][s], 0));
          xv[u][s] = (f32x4){__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xffff0000u),
                             __uint_as_float(h.y << 16), __uint_as_float(h.y & 0xffff0000u)};
        }
      }
    float acc[U][CO];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int o = 0; o < CO; ++o) acc[u][o] = 0.f;
    int wq = q;
    asm volatile("" : "+v"(wq));  // opaque: the W fragments stay LDS reads (not hoisted into VGPRs)
#pragma unroll
    for (int s = 0; s < kS; ++s)
#pragma unroll
      for (int o = 0; o < CO; ++o) {
        const f32x4 wv = lw[(o * K + s * CIN) / 4 + wq];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          acc[u][o] = fmaf(xv[u][s].x, wv.x, acc[u][o]);
          acc[u][o] = fmaf(xv[u][s].y, wv.y, acc[u][o]);
          acc[u][o] = fmaf(xv[u][s].z, wv.z, acc[u][o]);
          acc[u][o] = fmaf(xv[u][s].w, wv.w, acc[u][o]);
        }
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int o = 0; o < CO; ++o)
#pragma unroll
        for (int d = 4; d >= 1; d >>= 1) acc[u][o] += __shfl_xor(acc[u][o], d);
      if (it * U + u >= n_grp) break;  // uniform
      if (q < CO) {  // lane q stores output channel q of its row: CO x 8 consecutive floats per group
        float v = acc[u][0] + bo[0];
#pragma unroll
        for (int o = 1; o < CO; ++o)
          if (q == o) v = acc[u][o] + bo[o];
        if (ACT == CFSD_ACT_ELU) v = elu_f(v);
        const long row = yvm ? (long)vv[u] * batch + bb[u] : (long)bb[u] * rows + vv[u];
        y[row * CO + q] = v;
      }
    }
  }
}


// ------------------------------------------------------------------ launchers
bool ok(int batch, int cin, int cout) { return batch % 16 == 0 && cin == 32 && (cout == 32 || cout == 64); }

template <typename Kern>
static int resident(Kern k, int threads, size_t lds) {
  const int r = resident_blocks_of(k, threads, lds);
  return r > 0 ? r : 1;
}

// Persistent grids of the D3 / D2 forward and data gradient: the same
// number of workgroups on every CU (cu_blocks) -- the balanced-iteration grid
// (710 / 533 workgroups for D3 / D2) left some CUs a third more waves.
// Same-box kbench (profiles/round5q_kprof_grid.txt): forward 4 per CU D3
// 57.4 vs 60.7 us, D2 19.9 vs 23.5; data gradient 2 per CU D3 54.3-55.3 vs
// 57.2, D2 20.6-20.8 vs 22.9.  (0 = the balanced-iteration grid.)
constexpr int kVm32FwdBpc = 4;
constexpr int kVm32DxBpc = 2;

template <int CIN, int COUT, int ACT, int UPT, int PD>
static int fwd_t(const float* x, const int* idx, const float* w, const float* bias, float* y, int yvm,
                 int vsrc, int rows, int batch, hipStream_t st) {
  constexpr size_t lds = (size_t)COUT * (kS * CIN + 8) * sizeof(float);
  auto kern = conv_fwd_vm32<CIN, COUT, ACT, UPT, PD>;
  const long tiles = ((long)rows * (batch / 16) + UPT - 1) / UPT;
  constexpr int bpc = kVm32FwdBpc;
  const unsigned grid = bpc > 0 ? cu_blocks(tiles, 4, bpc) : balanced_blocks(tiles, 4, resident(kern, 256, lds));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, x, idx, w, bias, y, vsrc, rows, batch, yvm);
  return launch_status("spiral_conv_fwd_vm32");
}

// Units (vertex x 16 meshes) below which a wave takes ONE unit with two slots
// in flight (the level-1 row subset of an Enblock: ~1k units), else two units
// (more MFMA work per gathered slot) with one slot in flight.
constexpr int kVm32Upt1Units = 8192;
constexpr int kVm32Pd2 = 1;  // slots in flight ahead with two units per tile

template <int COUT, int ACT>
static int fwd_pick(const float* x, const int* idx, const float* w, const float* bias, float* y, int yvm,
                    int vsrc, int rows, int batch, hipStream_t st) {
  if ((long)rows * (batch / 16) < kVm32Upt1Units)
    return fwd_t<32, COUT, ACT, 1, 2>(x, idx, w, bias, y, yvm, vsrc, rows, batch, st);
  return fwd_t<32, COUT, ACT, 2, kVm32Pd2>(x, idx, w, bias, y, yvm, vsrc, rows, batch, st);
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

template <int CIN, int COUT, int FW, typename TY = float>
static int dxf_t(const float* dpre, int dpvm, int dxvm, const int* flat, const float* w, const TY* elu_y,
                 TY* dx, int vsrc, int rows, int batch, hipStream_t st) {
  constexpr size_t lds = (size_t)kS * CIN * (COUT + 8) * sizeof(float);
  auto kern = conv_dx_flat_vm32<CIN, COUT, FW, TY>;
  const long tiles = (long)vsrc * (batch / 16);
  constexpr int bpc = kVm32DxBpc;
  const unsigned grid = bpc > 0 ? cu_blocks(tiles, 8, bpc) : balanced_blocks(tiles, 8, resident(kern, 512, lds));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, dpre, (const int4*)flat, w, elu_y, dx, vsrc, rows,
                     batch, dpvm, dxvm);
  return launch_status("spiral_conv_bwd_data_flat_vm32");
}

template <int CIN, int COUT, int FW>
static int pair_t(const float* dpre, int dpvm, const int* flat, const float* w, const float* elu_y, float* dx,
                  int dxvm, int vsrc, int rows, int batch, DwLatArgs d, long dw_tasks, hipStream_t st) {
  constexpr size_t lds = (size_t)kS * CIN * (COUT + 8) * sizeof(float);
  auto kern = conv_bwd_flat_pair<CIN, COUT, FW>;
  const long tiles = (long)vsrc * (batch / 16);
  d.nb = (int)((dw_tasks + 7) / 8);
  const int res = resident(kern, 512, lds);
  const DxFlatArgs a{dpre, (const int4*)flat, w, elu_y, dx, vsrc, rows, batch, dpvm, dxvm,
                     (int)balanced_blocks(tiles, 8, res - d.nb > res / 2 ? res - d.nb : res / 2)};
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.nb + d.nb)), dim3(512), lds, st, a, d);
  return launch_status("spiral_conv_bwd_flat_pair");
}

int launch_bwd_flat_pair(const float* dpre, const int* flat, int width, const float* w, const float* elu_y,
                         float* dx, int dxvm, int vsrc, int rows, int batch, int cin, int cout, const DwLatArgs& d,
                         long dw_tasks, hipStream_t st) {
  if (!ok(batch, cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub (vertex-major): batch %% 16 == 0 and 32 -> 32/64 only");
  if ((long)batch * rows * cout * 4 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub (vertex-major): dpre exceeds 32-bit buffer offsets");
#define BP(CO, FW_)                                                                                         \
  if (cout == CO && width == FW_)                                                                           \
    return pair_t<32, CO, FW_>(dpre, 0, flat, w, elu_y, dx, dxvm, vsrc, rows, batch, d, dw_tasks, st);
  BP(32, 8) BP(32, 12) BP(32, 16)
#undef BP
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_rowsub (vertex-major): unsupported channels %d -> %d / width %d",
                   cin, cout, width);
}

int launch_bwd_vm_pair(const float* dpre, const int* flat, int width, const float* w, const float* elu_y, float* dx,
                       const float* x, const int* idx, float* ws, float* ws_db, int n_slabs, int vsrc, int rows,
                       int batch, hipStream_t st) {
  if (batch % 16) return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair: batch %% 16 != 0");
  if ((long)vsrc * batch * 128 >= (long)kAbsent || (long)rows * batch * 128 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair: operands exceed 32-bit offsets");
  constexpr size_t lds_dx = (size_t)kS * 32 * (32 + 8) * sizeof(float);
  constexpr size_t lds = lds_dx > DWV_LDS * sizeof(float) ? lds_dx : DWV_LDS * sizeof(float);
  constexpr int dxb = 0;  // dx workgroups (0: one per CU)
  DxFlatArgs a{dpre, (const int4*)flat, w, elu_y, dx, vsrc, rows, batch, 1, 1, dxb > 0 ? dxb : device_cus()};
  const DwVmArgs d{x, idx, ws, ws_db, n_slabs};
#define BV(FW_)                                                                                              \
  if (width == FW_) {                                                                                        \
    hipLaunchKernelGGL((conv_bwd_vm_pair<FW_>), dim3((unsigned)(a.nb + d.nb)), dim3(DWV_THREADS), lds, st, a, d); \
    return launch_status("spiral_conv_bwd_vm_pair");                                                         \
  }
  BV(8) BV(12) BV(16) BV(20)
#undef BV
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_flat_pair: flat width %d", width);
}

int launch_dx_flat_b16(const float* dpre, const int* flat, int width, const float* w, const bf16_t* elu_y,
                       bf16_t* dx, int dxvm, int vsrc, int rows, int batch, int cin, int cout, hipStream_t st) {
  if (!(batch % 16 == 0 && cin == 32 && cout == 32))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (bf16 dx): batch %% 16 == 0 and 32 -> 32 only");
  if ((long)batch * rows * cout * 4 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (bf16 dx): dpre exceeds 32-bit buffer offsets");
  if (width == 4) return dxf_t<32, 32, 4, bf16_t>(dpre, 0, dxvm, flat, w, elu_y, dx, vsrc, rows, batch, st);
  if (width == 8) return dxf_t<32, 32, 8, bf16_t>(dpre, 0, dxvm, flat, w, elu_y, dx, vsrc, rows, batch, st);
  if (width == 12) return dxf_t<32, 32, 12, bf16_t>(dpre, 0, dxvm, flat, w, elu_y, dx, vsrc, rows, batch, st);
  if (width == 16) return dxf_t<32, 32, 16, bf16_t>(dpre, 0, dxvm, flat, w, elu_y, dx, vsrc, rows, batch, st);
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (bf16 dx): width %d", width);
}

int launch_dx_flat(const float* dpre, int dpvm, int dxvm, const int* flat, int width, const float* w,
                   const float* elu_y, float* dx, int vsrc, int rows, int batch, int cin, int cout, hipStream_t st) {
  if (!ok(batch, cin, cout))
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (fp32): batch %% 16 == 0 and 32 -> 32/64 only");
  if ((long)batch * rows * cout * 4 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (fp32): dpre exceeds 32-bit buffer offsets");
#define DF(CI, CO, FW_)                                                                                 \
  if (cin == CI && cout == CO && width == FW_)                                                          \
    return dxf_t<CI, CO, FW_>(dpre, dpvm, dxvm, flat, w, elu_y, dx, vsrc, rows, batch, st);
  DF(32, 32, 8) DF(32, 32, 12) DF(32, 32, 16) DF(32, 32, 20) DF(32, 64, 8) DF(32, 64, 12) DF(32, 64, 16)
  DF(32, 64, 20)
#undef DF
  return set_error(CFSD_EINVAL, "spiral_conv_bwd_data_flat (fp32): unsupported channels %d -> %d / width %d",
                   cin, cout, width);
}


template <int CO, int ACT, typename TX>
static int fwd_out_t(const TX* x, const int* idx, const float* w, const float* bias, float* y, int yvm, int vsrc,
                     int rows, int batch, hipStream_t st) {
  constexpr int U = kVmOutU;
  auto kern = conv_fwd_out_vm<CO, ACT, U, TX>;
  const long its = ((long)rows * (batch / 8) + U - 1) / U;
  constexpr int bpc = kVmOutFwdBpc;
  const unsigned grid = bpc > 0 ? cu_blocks(its, 4, bpc) : balanced_blocks(its, 4, resident(kern, 256, 0));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, x, idx, w, bias, y, vsrc, rows, batch, yvm);
  return launch_status("spiral_conv_fwd_out_vm");
}

int launch_fwd_out(const void* x, int x_bf16, const int* idx, const float* w, const float* bias, float* y, int yvm,
                   int vsrc, int rows, int batch, int cout, int act, hipStream_t st) {
  if (batch % 8 || cout < 1 || cout > 3)
    return set_error(CFSD_EINVAL, "spiral_conv_fwd (vertex-major output conv): batch %% 8 == 0, 32 -> 1..3 only");
  if ((long)vsrc * batch * 32 * 4 >= (long)kAbsent || (long)rows * batch * cout >= (1L << 31))
    return set_error(CFSD_EINVAL, "spiral_conv_fwd (vertex-major output conv): x exceeds 32-bit buffer offsets");
#define FO(CO_, TX)                                                                                          \
  if (cout == CO_)                                                                                          \
    return act == CFSD_ACT_ELU                                                                              \
               ? fwd_out_t<CO_, CFSD_ACT_ELU, TX>((const TX*)x, idx, w, bias, y, yvm, vsrc, rows, batch, st) \
               : fwd_out_t<CO_, CFSD_ACT_NONE, TX>((const TX*)x, idx, w, bias, y, yvm, vsrc, rows, batch, st);
  if (x_bf16) {
    FO(1, bf16_t) FO(2, bf16_t) FO(3, bf16_t)
  } else {
    FO(1, float) FO(2, float) FO(3, float)
  }
#undef FO
  return set_error(CFSD_EINVAL, "spiral_conv_fwd (vertex-major output conv): cout %d", cout);
}

int dw_slabs(int batch, int rows, int max_slabs) {
  long n = resident(conv_dw_vm32, DWV_THREADS, 0);
  const long units = (long)rows * (batch / 16);
  if (n > (units + DWV_NR - 1) / DWV_NR) n = (units + DWV_NR - 1) / DWV_NR;  // >= 1 unit per range
  if (n > max_slabs) n = max_slabs;
  return n < 1 ? 1 : (int)n;
}

int launch_dw(const float* x, const int* idx, const float* dpre, float* ws, float* ws_db, int n_slabs, int vsrc,
              int rows, int batch, hipStream_t st) {
  if (batch % 16) return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight (fp32 vertex-major): batch %% 16 != 0");
  if ((long)vsrc * batch * 128 >= (long)kAbsent || (long)rows * batch * 128 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd_weight (fp32 vertex-major): operands exceed 32-bit offsets");
  hipLaunchKernelGGL(conv_dw_vm32, dim3(n_slabs), dim3(DWV_THREADS), 0, st, x, idx, dpre, ws, ws_db, vsrc, rows,
                     batch);
  return launch_status("spiral_conv_bwd_weight_vm32");
}

template <typename TX, int FW>
static int bwd_out_t(const float* dout, const int* flat, const float* w, const TX* elu_y, const TX* x, TX* dx,
                     float* ws, int n_slabs, int vsrc, int rows, int batch, hipStream_t st) {
  hipLaunchKernelGGL((conv_bwd_out_vm<TX, FW>), dim3(n_slabs), dim3(64 * kBoWaves), 0, st, dout, (const int4*)flat, w,
                     elu_y, x, dx, ws, vsrc, rows, batch);
  return launch_status("spiral_conv_bwd_out_vm");
}

int launch_bwd_out(const float* dout, const int* flat, int width, const float* w, const void* elu_y, const void* x,
                   void* dx, int x_bf16, float* ws, int n_slabs, int vsrc, int rows, int batch, hipStream_t st) {
  if (batch % 16) return set_error(CFSD_EINVAL, "spiral_conv_bwd (vertex-major output conv): batch %% 16 != 0");
  if ((long)rows * batch * 12 >= (long)kAbsent)
    return set_error(CFSD_EINVAL, "spiral_conv_bwd (vertex-major output conv): dout exceeds 32-bit offsets");
#define BO(FW_)                                                                                           \
  if (width == FW_)                                                                                       \
    return x_bf16 ? bwd_out_t<bf16_t, FW_>(dout, flat, w, (const bf16_t*)elu_y, (const bf16_t*)x, (bf16_t*)dx, \
                                           ws, n_slabs, vsrc, rows, batch, st)                            \
                  : bwd_out_t<float, FW_>(dout, flat, w, (const float*)elu_y, (const float*)x, (float*)dx, ws, \
                                          n_slabs, vsrc, rows, batch, st);
  BO(8) BO(12) BO(16) BO(20)
#undef BO
  return set_error(CFSD_EINVAL, "spiral_conv_bwd (vertex-major output conv): flat width %d", width);
}


}  // namespace vm32
}  // namespace cfsd
