// Calibration probe: v_mfma_f32_16x16x4_f32 throughput against waves per SIMD
// (256-thread blocks: 4 waves, one per SIMD; blocks = 256 CUs x k gives k
// waves per SIMD) and independent accumulators per wave (NACC), operands in
// registers, the in-kernel clock from s_memtime / s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void probe(float* out, unsigned long long* clk, int iters) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  float a[4], b[4];
  for (int k = 0; k < 4; ++k) {
    a[k] = 1e-3f * ((t + k) & 7);
    b[k] = 1e-3f * ((t >> 3) + k & 7);
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  f32x4 acc[NACC];
  for (int k = 0; k < NACC; ++k) acc[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 32 / NACC; ++j)
#pragma unroll
      for (int k = 0; k < NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j & 3], b[k & 3], acc[k], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int k = 0; k < NACC; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[t] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int NACC>
void run(int wps, int iters) {
  const int blocks = 256 * wps;
  float* out; unsigned long long* clk;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&clk, blocks * 16);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<NACC>, dim3(blocks), dim3(256), 0, 0, out, clk, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<NACC>, dim3(blocks), dim3(256), 0, 0, out, clk, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  const double flops = 2048.0 * 32 * iters * blocks * 4;  // 32 MFMAs per wave-iteration
  printf("16x16x4 nacc=%d waves/SIMD=%d iters=%d: %.3f ms, %.1f TFLOP/s (%.2f of 157.3), clock %.2f GHz\n", NACC,
         wps, iters, ms, flops / ms / 1e9, flops / ms / 1e9 / 157.3, (double)h[0] / (double)h[1] * 0.1);
  hipFree(out); hipFree(clk);
}

int main() {
  for (int wps : {1, 2, 3, 4}) {
    run<4>(wps, 27);  // one D3 forward wave's MFMA count (864) per wave
    run<4>(wps, 400);
    run<8>(wps, 400);
    run<2>(wps, 400);
  }
  return 0;
}
