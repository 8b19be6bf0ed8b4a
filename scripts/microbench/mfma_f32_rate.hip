// Microbenchmark: issue rate of v_mfma_f32_32x32x2_f32 with 1, 2, 4 independent accumulator
// chains, B operand from VGPRs (as in mlp_kernel).  Grid: 256 CUs x 4 waves (one per SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CHAINS>
__global__ void __launch_bounds__(256, 1) k(float* out, int iters, float a0, float b0) {
  f32x16 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x16{};
  float a = a0 + threadIdx.x * 1e-3f, b = b0 - threadIdx.x * 1e-3f;
  float bv[16];
  for (int i = 0; i < 16; ++i) bv[i] = b + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      acc[i % CHAINS] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv[i & 15], acc[i % CHAINS], 0, 0, 0);
    }
  }
  float s = 0;
  for (int c = 0; c < CHAINS; ++c) for (int e = 0; e < 16; ++e) s += acc[c][e];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int C>
double run(float* d, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(256), 0, 0, d, 2, 1.0f, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<C>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0f, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double flop = (double)blocks * 4 * iters * 64 * 4096.0;
  return flop / (ms * 1e-3) / 1e12;
}

int main() {
  float* d; hipMalloc(&d, 1 << 24);
  int blocks = 256, iters = 4000;
  printf("1 chain : %.1f TFLOP/s\n", run<1>(d, blocks, iters));
  printf("2 chains: %.1f TFLOP/s\n", run<2>(d, blocks, iters));
  printf("4 chains: %.1f TFLOP/s\n", run<4>(d, blocks, iters));
  printf("1 chain x2 blocks/CU-ish (512 blocks): %.1f TFLOP/s\n", run<1>(d, 512, iters));
  return 0;
}
