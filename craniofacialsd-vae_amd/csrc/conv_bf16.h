// Launchers of the bf16 MFMA SpiralConv kernels (spiral_conv_bf16.hip),
// called by the mixed-precision C ABI in spiral_conv.hip.  Activations and
// gradients are bf16 or fp32 per operand (the bf16 path keeps the coarse
// levels and the bottleneck in fp32), weights are the bf16 shadow of the fp32
// master parameters, every product accumulates in fp32.
#pragma once
#include "cfsd_common.h"

namespace cfsd {
namespace bf {

constexpr int DT_F32 = CFSD_DT_F32;
constexpr int DT_BF16 = CFSD_DT_BF16;

// Layouts: xvm / dxvm (0/1) and the CFSD_VM bit of y_dt / dpre_dt (cfsd.h).
// y[m, :] = act(bias + W . gather(x)), x bf16, y bf16 or fp32 (y_dt).
int launch_fwd(const bf16_t* x, int xvm, const int* idx, const bf16_t* w, const float* bias, void* y,
               int y_dt, int vsrc, int rows, long total_rows, int cin, int cout, int act,
               hipStream_t st);
// dx bf16 (times elu'(elu_y) when elu_y != NULL; elu_y in dx's layout), dpre
// bf16 or fp32.
int launch_dx(const void* dpre, int dpre_dt, const int* inv_ptr, const int* inv_row,
              const int* inv_head, const bf16_t* w, const bf16_t* elu_y, bf16_t* dx, int dxvm, int vsrc,
              int rows, long total_src_rows, int cin, int cout, hipStream_t st);
// dW / db partial slabs [n_slabs][cout*9*cin + cout] (plain layout), x bf16,
// dpre bf16 or fp32.
int dw_slabs(int batch, int rows, int cin, int cout);
int launch_dw(const bf16_t* x, int xvm, const int* idx, const void* dpre, int dpre_dt, float* ws, int vsrc,
              int rows, long total_rows, int cin, int cout, hipStream_t st);

// Vertex-major operands with batch % 16 == 0 (spiral_conv_vm16.hip): one
// 16-row MFMA tile = one vertex x 16 meshes.
bool vm16_ok(int batch, int cin, int cout);
constexpr int kDwVm16 = 1;
constexpr int kDwVm16F32dp = 1;
// bf16 32 -> 32 weight gradient with vertex-major bf16 x and a vertex-major
// bf16 (or batch-major fp32: an Enblock's kept rows) dpre: conv_dw_vm16,
// n_slabs plain slabs (the conv_dw_b16 layout and count, dw_slabs())
bool dw_vm16_ok(int batch, int cin, int cout, int xvm, int dpvm, int dpre_bf16);
int launch_dw_vm16(const bf16_t* x, const int* idx, const void* dpre, int dpre_bf16, float* ws, int n_slabs, int vsrc,
                   int rows, int batch, hipStream_t st);
// The bf16 vertex-major Deblock backward (32 -> 32, dpre / x / dx / elu_y bf16
// vertex-major) in ONE launch: launch_dx_flat_vm16's dx and launch_dw_vm16's
// n_slabs slabs (same values) as interleaved workgroup roles.
int launch_bwd_vm16_pair(const bf16_t* x, const int* idx, const bf16_t* dpre, const int* flat, int width,
                         const bf16_t* w, const bf16_t* elu_y, bf16_t* dx, float* ws, int n_slabs, int vsrc, int rows,
                         int batch, hipStream_t st);
// The bf16 step's Enblock E1 backward (fp32 batch-major dpre at the kept rows,
// bf16 vertex-major x / dx / elu_y, fp32 w) in ONE launch: the fp32-product
// flat dx and the conv_dw_vm16<float> slabs (same values as the two launches).
int launch_bwd_rowsub16_pair(const bf16_t* x, const int* idx, const float* dpre, const int* flat, int width,
                             const float* w, const bf16_t* elu_y, bf16_t* dx, float* ws, int n_slabs, int vsrc,
                             int rows, int batch, hipStream_t st);
int launch_fwd_vm16(const bf16_t* x, const int* idx, const bf16_t* w, const float* bias, void* y, int y_dt,
                    int vsrc, int rows, int batch, int cin, int cout, int act, hipStream_t st);
int launch_dx_vm16(const void* dpre, int dpre_dt, const int* inv_ptr, const int* inv_row, const int* inv_head,
                   const bf16_t* w, const bf16_t* elu_y, bf16_t* dx, int vsrc, int rows, int batch, int cin,
                   int cout, hipStream_t st);
int launch_dx_flat_vm16(const void* dpre, int dpre_dt, const int* flat, int width, const bf16_t* w,
                        const bf16_t* elu_y, bf16_t* dx, int vsrc, int rows, int batch, int cin, int cout,
                        hipStream_t st);

}  // namespace bf
}  // namespace cfsd
