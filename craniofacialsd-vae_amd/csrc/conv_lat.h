// The coarse-level weight-gradient body (shared by the dW-only launch and the
// launches pairing it with a data gradient: spiral_conv.hip,
// spiral_conv_coarse.hip).
#pragma once
#include "cfsd_common.h"

namespace cfsd {

struct DwLatArgs {
  const float* x;
  const int* idx;
  const float* dpre;
  float* ws;
  float* ws_db;
  int vsrc, rows, total_rows, rchunk, n_chunks;
  int nb;
  int batch, xvm, dpvm;  // layouts of x / dpre (cfsd.h CFSD_VM)
};

// Row chunks per dW slab: the kLatGroup waves of a workgroup that own one
// unit's consecutive chunks sum their partials in LDS (fixed chunk order) and
// write ONE slab, so the slab traffic written here and re-read by the reduce
// is 1/kLatGroup of one slab per chunk.  Slab c holds chunks [4c, 4c + 4).
constexpr int kLatGroup = 4;
constexpr int kLatRed = 1024 + 32;  // LDS floats per wave: its 32x32 partial + db
__host__ __device__ constexpr int lat_slabs(int n_chunks) { return (n_chunks + kLatGroup - 1) / kLatGroup; }
// dW-role waves to launch (whole chunk groups; with 9-wave workgroups waves 0-7 work)
__host__ __device__ constexpr long lat_tasks(int n_chunks, int units) { return (long)lat_slabs(n_chunks) * kLatGroup * units; }
// LDS floats the body needs as `red` for WPB waves per workgroup
__host__ __device__ constexpr int lat_red_floats(int wpb) { return (wpb / kLatGroup) * kLatGroup * kLatRed; }

// Backward weight for layers with few rows.  conv_dw_mfma's 9/12-wave
// workgroups each need >= 4 row tiles, which leaves most CUs idle on the
// coarse levels; here a wave owns ONE 32x32 dW unit (s, ot, ct) and a chunk
// of R rows (the K dimension), so units x chunks waves run at once.
// v_mfma_f32_32x32x2_f32 straight from memory, no LDS: step j covers rows
// (2j, 2j+1) of the chunk; A[o][k] = dpre[row_k][ot*32 + o] (a 128-B
// coalesced dpre segment per half-wave), B[k][c] = x[b, idx[r_k][s],
// ct*32 + c] (a 128-B gathered row segment).  8 steps per batch with all
// loads issued first, two accumulators.  Output: slab[chunk group][U][32][32]
// + db[chunk group][COUT] (units with s == 0 && ct == 0 also sum dpre) -- the
// conv_dw_mfma slab layout, lat_slabs(n_chunks) slabs, reduced by
// conv_dw_reduce / dw_reduce_batch.  `red`: lat_red_floats(WPB) floats of LDS.
template <int CIN, int COUT, int WPB = 4>
__device__ __forceinline__ void conv_dw_lat_body(int vb, int vnb, const float* __restrict__ x,
                                                 const int* __restrict__ idx,
                                                 const float* __restrict__ dpre,
                                                 float* __restrict__ ws,
                                                 float* __restrict__ ws_db, int vsrc, int rows,
                                                 int total_rows, int rchunk, int n_chunks, int batch,
                                                 int xvm, int dpvm, float* __restrict__ red) {
  constexpr int OT = COUT / 32, CT = CIN / 32, U = kSeq * OT * CT, NB = 8;
  constexpr int GC = kLatGroup, NGB = WPB / GC;  // chunk groups per workgroup
  static_assert(NGB >= 1, "at least kLatGroup waves per workgroup");
  const int lane = threadIdx.x & 63, li = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), sub = wave % GC;
  const long grp = (long)xcd_block_of(vb, vnb) * NGB + wave / GC;  // (chunk group, unit)
  const bool in_grp = wave < NGB * GC && grp < (long)lat_slabs(n_chunks) * U;
  const int unit = in_grp ? (int)(grp % U) : 0, cg = in_grp ? (int)(grp / U) : 0;
  const bool act = in_grp && cg * GC + sub < n_chunks;  // wave-uniform
  // a wave without a chunk of its own (a group's missing tail chunks, the 9th
  // wave of a 9-wave workgroup) runs an empty row range: the gather loop below
  // stays straight-line code (its counted asm loads must not be wrapped in a
  // branch the compiler can copy values across)
  const int chunk = min(cg * GC + sub, n_chunks - 1);
  const int ct = unit % CT, ot = (unit / CT) % OT, sl = unit / (CT * OT);
  f32x16 acc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[q][e] = 0.f;
  float dbs = 0.f;
  const bool do_db = sl == 0 && ct == 0;
  {
    const int r0 = chunk * rchunk, r1 = min(total_rows, r0 + rchunk);
    const int rend = act ? r1 : r0;  // an inactive wave skips the loop
    // (b, r) of this lane's first row (flat dpre row m in dpre's layout:
    // minor index mi of extent E, major ma), advanced incrementally by 2 per
    // step; x rows are addressed in x's layout
    const Lay lx = make_lay(xvm, batch, vsrc);
    const int E = dpvm ? batch : rows;
    int m = r0 + h;
    int ma = m / E, mi = m - ma * E;
    const float* dp = dpre + ot * 32 + li;
    const float* xs = x + ct * 32 + li;
    int b_last, r_last;
    split_row(r1 - 1, dpvm, batch, rows, b_last, r_last);
    static_assert(NB == 8, "vm_wait_arr8");
    // Rows past the chunk are clamped to its last row (loads stay in bounds,
    // no branches) and weighted 0.  Pipelined one batch ahead: while batch i's
    // 8 dependent x gathers are in flight, batch i+1's 8 idx and 8 dpre loads
    // are issued, so a batch costs ~one memory latency instead of two.  The x
    // gathers are counted asm loads retired by an explicit vmcnt in the same
    // iteration (hipcc's own placement serialised them); the idx / dpre loads
    // are ordinary loads that hipcc waits for itself -- they cross the loop
    // back-edge, where an asm-hidden load could be copied before it landed.
    int srcrow[NB], bvs[NB];
    float okf[NB], av[NB];
    auto fetch = [&](int m0_, int (&sr)[NB], int (&bs)[NB], float (&ok_)[NB], float (&a_)[NB]) {
  #pragma unroll
      for (int j = 0; j < NB; ++j) {
        const bool ok = m < r1;
        const int b = dpvm ? mi : ma, r = dpvm ? ma : mi;
        ok_[j] = ok ? 1.f : 0.f;
        bs[j] = (ok ? b : b_last) * lx.bs;
        sr[j] = idx[(ok ? r : r_last) * kSeq + sl] * lx.vs;
        m += 2;
        mi += 2;
        bool wrap = mi >= E;
        mi = wrap ? mi - E : mi;
        ma = wrap ? ma + 1 : ma;
        wrap = mi >= E;  // extent 1
        mi = wrap ? mi - E : mi;
        ma = wrap ? ma + 1 : ma;
      }
  #pragma unroll
      for (int j = 0; j < NB; ++j) a_[j] = dp[(long)min(m0_ + h + 2 * j, r1 - 1) * COUT];
    };
    fetch(r0, srcrow, bvs, okf, av);
    for (int m0 = r0; m0 < rend; m0 += 2 * NB) {
      float bv[NB];
  #pragma unroll
      for (int j = 0; j < NB; ++j) gload1f_async(bv[j], xs + (long)(bvs[j] + srcrow[j]) * CIN);
      // the next batch's 16 idx / dpre loads are issued unconditionally (past
      // the chunk they are clamped in-bounds rows, weighted 0), so the gathers'
      // outputs flow straight into ONE counted wait: a branch here let hipcc
      // copy the gather registers ahead of the wait on one path (stale values)
      int srcrow_n[NB], bvs_n[NB];
      float okf_n[NB], av_n[NB];
      fetch(m0 + 2 * NB, srcrow_n, bvs_n, okf_n, av_n);
      vm_wait_arr8<2 * NB>(bv);  // x gathers retired, the next batch in flight
  #pragma unroll
      for (int j = 0; j < NB; ++j) {
        const float aj = av[j] * okf[j];
        acc[j & 1] = mfma32(aj, bv[j], acc[j & 1]);
        dbs += aj;
      }
  #pragma unroll
      for (int j = 0; j < NB; ++j) {
        srcrow[j] = srcrow_n[j];
        bvs[j] = bvs_n[j];
        okf[j] = okf_n[j];
        av[j] = av_n[j];
      }
    }
  }
  // every wave parks its partial in its own LDS slot; after one barrier the
  // group's first wave sums the kLatGroup chunks in chunk order and stores
  // the group's slab (coalesced)
  dbs += __shfl_xor(dbs, 32);
  float* rw = red + wave * kLatRed;
  if (act) {
#pragma unroll
    for (int e = 0; e < 16; ++e) rw[acc_row(e, lane) * 32 + li] = acc[0][e] + acc[1][e];
    if (do_db && h == 0) rw[1024 + li] = dbs;
  }
  __syncthreads();
  if (in_grp) {  // the group's waves each sum and store a quarter of the slab
    const int na = min(GC, n_chunks - cg * GC);  // chunks present in this group (>= 1)
    const float* r0p = red + (wave - sub) * kLatRed;  // the group's first wave's slot
    float* slab = ws + ((long)cg * U + unit) * 1024;
    constexpr int PER = 16 / GC;  // 64-float rows per wave
#pragma unroll
    for (int i = sub * PER; i < sub * PER + PER; ++i) {
      float v = r0p[i * 64 + lane];
      for (int q = 1; q < na; ++q) v += r0p[q * kLatRed + i * 64 + lane];
      slab[i * 64 + lane] = v;
    }
    if (sub == 0 && do_db && h == 0) {
      float v = r0p[1024 + li];
      for (int q = 1; q < na; ++q) v += r0p[q * kLatRed + 1024 + li];
      ws_db[(long)cg * COUT + ot * 32 + li] = v;
    }
  }
}

}  // namespace cfsd
