// Launchers of the fp32 SpiralConv kernels for VERTEX-MAJOR operands
// (spiral_conv_vm32.hip), called by the C ABI in spiral_conv.hip.  A batch
// that is a multiple of 16 makes one 16-row MFMA tile = one vertex x 16
// meshes: every spiral index of the tile is wave-uniform and every gathered
// neighbour is one contiguous 2-KiB block (16 meshes x 32 fp32 channels).
#pragma once
#include "cfsd_common.h"
#include "conv_lat.h"

namespace cfsd {
namespace vm32 {

bool ok(int batch, int cin, int cout);
// y[(b, r), :] = act(bias + W . gather(x)); x vertex-major [vsrc][batch][cin],
// y vertex-major (yvm) or batch-major [batch][rows][cout].  Same products in
// the same order as conv_fwd_mfma (bit-identical results).
int launch_fwd(const float* x, const int* idx, const float* w, const float* bias, float* y, int yvm,
               int vsrc, int rows, int batch, int cin, int cout, int act, hipStream_t st);
// dx[u] = elu'(elu_y[u]) * sum over the flat inverse list of u (ascending
// spiral position p = 9r + s) of W_s^T dpre[r]; dpre, dx (and elu_y, in dx's
// layout) vertex-major (dpvm / dxvm) or batch-major; 32 -> 32/64.
int launch_dx_flat(const float* dpre, int dpvm, int dxvm, const int* flat, int width, const float* w,
                   const float* elu_y, float* dx, int vsrc, int rows, int batch, int cin, int cout, hipStream_t st);
// launch_dx_flat with batch-major fp32 dpre and bf16 dx / elu_y (32 -> 32):
// the bf16 step's E1 data gradient, the fp32 sum rounded once.
int launch_dx_flat_b16(const float* dpre, const int* flat, int width, const float* w, const bf16_t* elu_y,
                       bf16_t* dx, int dxvm, int vsrc, int rows, int batch, int cin, int cout, hipStream_t st);
// The row-subset (Enblock) backward, 32 -> 32, batch-major dpre at the kept rows:
// launch_dx_flat's data gradient (dx / elu_y vertex-major when dxvm, else
// batch-major) and the dW slabs described by `d` (its nb is set here;
// dw_tasks = chunks x units) in one launch.
int launch_bwd_flat_pair(const float* dpre, const int* flat, int width, const float* w, const float* elu_y,
                         float* dx, int dxvm, int vsrc, int rows, int batch, int cin, int cout, const DwLatArgs& d,
                         long dw_tasks, hipStream_t st);
// Both gradients of a full (not row-subset) 32 -> 32 conv with dpre, x, dx
// and elu_y all vertex-major fp32 (the fp32 D2 / D3) in ONE launch: the
// flat-list dx and the launch_dw slabs (n_slabs = dw_slabs(), same layout and
// values as launch_dw up to summation order within a slab: bit-identical).
int launch_bwd_vm_pair(const float* dpre, const int* flat, int width, const float* w, const float* elu_y, float* dx,
                       const float* x, const int* idx, float* ws, float* ws_db, int n_slabs, int vsrc, int rows,
                       int batch, hipStream_t st);
// dW/db slabs (conv_dw_mfma layout: [n_slabs][9][32][32], db [n_slabs][32] at
// ws_db) of a 32 -> 32 conv, x and dpre vertex-major, batch % 16 == 0.
// Workgroups (= slabs) launch_dw uses; max_slabs = the workspace's slab capacity.
int dw_slabs(int batch, int rows, int max_slabs);
int launch_dw(const float* x, const int* idx, const float* dpre, float* ws, float* ws_db, int n_slabs, int vsrc,
              int rows, int batch, hipStream_t st);
// The xyz output conv forward (32 -> cout <= 3), x vertex-major fp32 or bf16,
// batch % 8 == 0, y vertex-major (yvm) or batch-major; the same bits as the
// batch-major conv_fwd_out_small.
int launch_fwd_out(const void* x, int x_bf16, const int* idx, const float* w, const float* bias, float* y, int yvm,
                   int vsrc, int rows, int batch, int cout, int act, hipStream_t st);
// dx (x's storage, times elu'(elu_y)) and the dW/db slab of one block per
// n_slabs of the xyz output conv (32 -> 3); x / elu_y / dx / dout
// vertex-major, flat = u's inverse list (topology.spiral_flat).
int launch_bwd_out(const float* dout, const int* flat, int width, const float* w, const void* elu_y, const void* x,
                   void* dx, int x_bf16, float* ws, int n_slabs, int vsrc, int rows, int batch, hipStream_t st);

}  // namespace vm32
}  // namespace cfsd
