// Calibration: issue rate of v_mfma_f32_32x32x16_f16 on one wave per SIMD (every CU busy), alone
// and with NV independent VALU ops (v_fma_f32 / v_cvt_pk_f16_f32 mixes) interleaved per MFMA;
// memtime ticks per MFMA and wall-clock TFLOP/s.  Random operands (clock: DVFS).
//   hipcc --offload-arch=gfx950 -O3 -o scripts/microbench/mfma_f16_issue scripts/microbench/mfma_f16_issue.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));

template <int NV, int CHAINS>
__global__ void __launch_bounds__(256, 1) k(const h8* __restrict__ in, float* out, unsigned long long* ticks, int iters) {
  h8 a = in[threadIdx.x], b = in[threadIdx.x + 256];
  f16x acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f16x{};
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = (float)in[threadIdx.x][i];
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS * 4; ++c) {
      acc[c % CHAINS] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[c % CHAINS], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j % 8] = __builtin_fmaf(v[j % 8], 1.0001f, 0.5f);
    }
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0;
  for (int c = 0; c < CHAINS; ++c) for (int i = 0; i < 16; ++i) s += acc[c][i];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) ticks[blockIdx.x] = t1 - t0;
}

template <int NV, int CHAINS>
void run(const h8* in, float* out, unsigned long long* ticks, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k<NV, CHAINS><<<blocks, 256>>>(in, out, ticks, iters);
  hipEventRecord(e0);
  k<NV, CHAINS><<<blocks, 256>>>(in, out, ticks, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long t; hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost);
  const double mfmas = (double)iters * CHAINS * 4;
  const double flop = (double)blocks * 4 * mfmas * 32 * 32 * 16 * 2;
  printf("NV=%d chains=%d: %.1f ticks/MFMA, %.0f TFLOP/s f16, wall %.3f ms\n", NV, CHAINS, t / mfmas, flop / ms / 1e9, ms);
}

int main() {
  const int blocks = 256, iters = 4000;
  h8* in; float* out; unsigned long long* ticks;
  hipMalloc(&in, 512 * 16); hipMalloc(&out, blocks * 256 * 4); hipMalloc(&ticks, blocks * 8);
  _Float16 h[512 * 8];
  unsigned s = 1;
  for (int i = 0; i < 512 * 8; ++i) { s = s * 1103515245u + 12345u; h[i] = (_Float16)(((s >> 8) & 0xffff) / 65536.0f - 0.5f); }
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  run<0, 1>(in, out, ticks, blocks, iters);
  run<0, 4>(in, out, ticks, blocks, iters);
  run<2, 4>(in, out, ticks, blocks, iters);
  run<4, 4>(in, out, ticks, blocks, iters);
  run<5, 4>(in, out, ticks, blocks, iters);
  run<6, 4>(in, out, ticks, blocks, iters);
  run<8, 4>(in, out, ticks, blocks, iters);
  run<12, 4>(in, out, ticks, blocks, iters);
  return 0;
}
