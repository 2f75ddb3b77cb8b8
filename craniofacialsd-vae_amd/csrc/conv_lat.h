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
// ct*32 + c] (a 128-B gathered row segment).  8 steps per batch of 16 rows
// with all loads issued first, two accumulators.  Output: slab[chunk group]
// [U][32][32] + db[chunk group][COUT] (units with s == 0 && ct == 0 also sum
// dpre) -- the conv_dw_mfma slab layout, lat_slabs(n_chunks) slabs, reduced
// by conv_dw_reduce / dw_reduce_batch.  `red`: lat_red_floats(WPB) floats of
// LDS.
//
// Address work per MFMA (round 6: the SQ counters put these roles at ~15
// VALU instructions per MFMA, the rows' index arithmetic serialised per lane):
// a batch's 16 row offsets are computed ONCE, lane-parallel (lane t holds row
// m0 + t), and handed to the half-wave that needs them with ds_bpermute; the
// dpre rows are buffer loads at a wave-uniform row offset (SGPR) plus a
// per-lane constant, and rows past the tensor (the last chunk's tail: chunks
// are whole 16-row batches) read 0 from the buffer's range check, so no row
// is masked.  Same products in the same order as before: bit-identical.
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
  const int lane = threadIdx.x & 63, li = lane & 31, h = lane >> 5, t16 = lane & 15;
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
    // lane t16's row m of the next batch to describe, (ma, mi) its split in
    // dpre's layout (minor index mi of extent E); rows past the tensor take
    // the last row's x (their dpre reads 0)
    const Lay lx = make_lay(xvm, batch, vsrc);
    const int E = dpvm ? batch : rows;
    int m = r0 + t16, ma, mi;
    divmod32(m, E, ma, mi);
    int b_last, r_last;
    split_row(total_rows - 1, dpvm, batch, rows, b_last, r_last);
    // one batch = 2 NB rows: (ma, mi) advance by (q16, e16) plus a carry
    const int q16 = (2 * NB) / E, e16 = (2 * NB) % E;
    const int* idx_s = idx + sl;
    // (plain value arithmetic, no lambda captures by reference: a select of
    // captured references compiled to a select of stack addresses -> scratch)
#define CFSD_LAT_META(BROW, IV)                                                 \
  {                                                                             \
    const bool ok_ = m < total_rows;                                            \
    const int bsel_ = dpvm ? mi : ma, rsel_ = dpvm ? ma : mi;                   \
    const int b_ = ok_ ? bsel_ : b_last, r_ = ok_ ? rsel_ : r_last;             \
    BROW = b_ * lx.bs;                                                          \
    IV = idx_s[r_ * kSeq];                                                      \
    m += 2 * NB;                                                                \
    mi += e16;                                                                  \
    ma += q16;                                                                  \
    const bool w_ = mi >= E;                                                    \
    mi = w_ ? mi - E : mi;                                                      \
    ma += w_ ? 1 : 0;                                                           \
  }
    // dpre: rows past the tensor are out of the buffer's range (read as 0);
    // a batch past the chunk (the second half of a pair, below) gets an
    // out-of-range row offset, so it reads 0 too
    const auto drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dpre + ot * 32), 0,
                                                       (int)(((long)total_rows * COUT - ot * 32) * 4), 0x00020000);
    const int dvo = (h * COUT + li) * 4;
    constexpr int kOutOfRange = 0x7ffff000;
#define CFSD_LAT_LOAD_A(M0, A)                                                                      \
  {                                                                                                 \
    const int so_ = (M0) < r1 ? (M0) * COUT * 4 : kOutOfRange;                                     \
    _Pragma("unroll") for (int j = 0; j < NB; ++j) A[j] = __builtin_bit_cast(                      \
        float, __builtin_amdgcn_raw_buffer_load_b32(drs, dvo + j * 2 * COUT * 4, so_, 0));          \
  }
    // a batch's 16 row offsets (bytes into x, lane t16 = row m0 + t16), handed
    // to the half-wave that gathers them: lane (li, h) takes row 2j + h
    const float* xs = x + ct * 32;  // wave-uniform base
    const int lo4 = li * 4;
#define CFSD_LAT_PREP(OFF, BROW, IV)                                                                \
  {                                                                                                 \
    const int go_ = ((BROW) + (IV) * lx.vs) * (CIN * 4);                                            \
    _Pragma("unroll") for (int j = 0; j < NB; ++j) OFF[j] =                                         \
        __builtin_amdgcn_ds_bpermute((2 * j + h) * 4, go_) + lo4;                                   \
  }
#define CFSD_LAT_HALF(OFF, A, A_NEXT, M_NEXT, BROW_N, IV_N)                                         \
  {                                                                                                 \
    float bv[NB];                                                                                   \
    _Pragma("unroll") for (int j = 0; j < NB; ++j) gload1f_async_s(bv[j], xs, OFF[j]);              \
    CFSD_LAT_META(BROW_N, IV_N)                                                                     \
    CFSD_LAT_LOAD_A(M_NEXT, A_NEXT)                                                                 \
    vm_wait_arr8<NB + 1>(bv); /* x gathers retired, the next batch's idx + dpre in flight */        \
    _Pragma("unroll") for (int j = 0; j < NB; ++j) {                                                \
      acc[j & 1] = mfma32(A[j], bv[j], acc[j & 1]);                                                 \
      dbs += A[j];                                                                                  \
    }                                                                                               \
    CFSD_LAT_PREP(OFF, BROW_N, IV_N)                                                                \
    /* keep the halves apart: hipcc otherwise hoists the next half's db adds */                   \
    /* (and their vmcnt waits on its dpre loads) into this one */                                  \
    __builtin_amdgcn_sched_barrier(0);                                                              \
  }
    static_assert(NB == 8, "vm_wait_arr8");
    // Software pipeline, two batches per trip with alternating register sets
    // (no copies across the back-edge): while batch i's 8 dependent x gathers
    // are in flight, batch i+1's idx load and 8 dpre loads are issued, and
    // batch i+1's gather offsets are formed right after batch i's MFMAs, so
    // the next gathers issue at once.  The x gathers are counted asm loads
    // retired by an explicit vmcnt in the same half (hipcc's own placement
    // serialised them); the idx / dpre loads are ordinary loads that hipcc
    // waits for itself -- they cross the back-edge, where an asm-hidden load
    // could be copied before it landed.
    int brow, iv, off[NB];
    float aA[NB], aB[NB];
    CFSD_LAT_META(brow, iv)
    CFSD_LAT_LOAD_A(r0, aA)
    CFSD_LAT_PREP(off, brow, iv)
    for (int m0 = r0; m0 < rend; m0 += 4 * NB) {
      CFSD_LAT_HALF(off, aA, aB, m0 + 2 * NB, brow, iv)
      CFSD_LAT_HALF(off, aB, aA, m0 + 4 * NB, brow, iv)
    }
#undef CFSD_LAT_HALF
#undef CFSD_LAT_PREP
#undef CFSD_LAT_LOAD_A
#undef CFSD_LAT_META
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
