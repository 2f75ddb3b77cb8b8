// Calibration probe: sustained f32 MFMA throughput with RANDOM operands (power
// / clock limited) vs tiny operands, 32x32x2 and 16x16x4, and the in-kernel
// clock (s_memtime / s_memrealtime @ 100 MHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ float hashf(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return (float)(x & 0xffffff) / 16777216.f - 0.5f;
}

template <int SHAPE>  // 0: 32x32x2, 1: 16x16x4
__global__ __launch_bounds__(256) void probe(float* out, unsigned long long* clk, int iters, int rnd) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  float a[4], b[4];
  for (int k = 0; k < 4; ++k) {
    a[k] = rnd ? hashf(t * 8 + k) : 1e-3f * (threadIdx.x & 3);
    b[k] = rnd ? hashf(t * 8 + 4 + k + 12345) : 1e-3f * (blockIdx.x & 3);
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  if (SHAPE == 0) {
    f32x16 acc[4];
    for (int k = 0; k < 4; ++k) acc[k] = (f32x16){0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[k], acc[k], 0, 0, 0);
    }
    for (int k = 0; k < 4; ++k) for (int r = 0; r < 16; ++r) s += acc[k][r];
  } else {
    f32x4 acc[4];
    for (int k = 0; k < 4; ++k) acc[k] = (f32x4){0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j & 3], b[k], acc[k], 0, 0, 0);
    }
    for (int k = 0; k < 4; ++k) for (int r = 0; r < 4; ++r) s += acc[k][r];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[t] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int SHAPE>
void run(int blocks, int iters, int rnd) {
  float* out; unsigned long long* clk;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&clk, blocks * 16);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<SHAPE>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, rnd);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<SHAPE>, dim3(blocks), dim3(256), 0, 0, out, clk, iters, rnd);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  // flops per wave-iteration: 16 MFMAs of 32x32x2 (4096 flop) or 32 of 16x16x4 (2048 flop)
  double flops = 2.0 * 32 * 32 * 2 * 16.0 * iters * blocks * 4;
  printf("%s rnd=%d blocks=%d: %.3f ms, %.1f TFLOP/s, clock %.2f GHz\n", SHAPE ? "16x16x4" : "32x32x2", rnd,
         blocks, ms, flops / ms / 1e9, (double)h[0] / (double)h[1] * 0.1);
  hipFree(out); hipFree(clk);
}

int main() {
  for (int rnd : {0, 1})
    for (int blocks : {1024, 4096}) {
      run<0>(blocks, 400, rnd);
      run<1>(blocks, 400, rnd);
    }
  return 0;
}
