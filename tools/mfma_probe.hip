// Calibration probe: throughput of v_mfma_f32_32x32x2_f32 with 1 vs 2 vs 4
// independent accumulators per wave, operands in registers (no memory).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void probe(float* out, int iters) {
  f32x16 acc[NACC];
  for (int k = 0; k < NACC; ++k) acc[k] = (f32x16){0.f};
  float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int k = 0; k < NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[k], 0, 0, 0);
  }
  float s = 0.f;
  for (int k = 0; k < NACC; ++k) for (int r = 0; r < 16; ++r) s += acc[k][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
void run(int blocks, int iters) {
  float* out;
  hipMalloc(&out, blocks * 256 * 4);
  hipLaunchKernelGGL(probe<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double flops = 2.0 * 32 * 32 * 2 * 16.0 * iters * NACC * blocks * 4;
  printf("nacc=%d blocks=%d: %.3f ms, %.1f TFLOP/s\n", NACC, blocks, ms, flops / ms / 1e9);
  hipFree(out);
}

int main() {
  for (int blocks : {256, 1024, 2048}) {
    run<1>(blocks, 200);
    run<2>(blocks, 100);
    run<4>(blocks, 50);
  }
  return 0;
}
