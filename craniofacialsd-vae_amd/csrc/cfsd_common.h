// Shared helpers for the CDNA4 (gfx950) kernels of the spiral mesh-VAE step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cfsd.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace cfsd {

// Records the last error text (thread-local) and returns its code.
int set_error(int code, const char* fmt, ...);

inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error((int)e, "%s: %s", what, hipGetErrorString(e));
  return CFSD_OK;
}

__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }
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

constexpr int kMaxBatch = 1 << 20;

}  // namespace cfsd
