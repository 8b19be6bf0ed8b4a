// Shape A/B for the MLP's trunk schedule: v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16 at
// the same work per "half-step" (12 x 32x32x16 = 24 x 16x16x32 = 393,216 FLOP per wave), A
// fragments re-read from LDS (8 ds_read_b128 per half-step, as mlp16's k-step), B operands in
// registers, one wave per SIMD (LDS sized so one workgroup fits a CU), NV independent VALU fmas
// per half-step spread over the MFMA gaps (the epilogue's side work), random operands.
// Prints wall-clock TFLOP/s after >= 2 s of back-to-back launches (DVFS settles) and memtime
// cycles per half-step.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_shape_side scripts/microbench/mfma_shape_side.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kLdsBytes = 120 * 1024;   // one workgroup per CU

template <int SHAPE, int NV>
__global__ void __launch_bounds__(256, 1) k(const h8* __restrict__ in, float* out, unsigned long long* ticks, int iters) {
  __shared__ h8 lds[kLdsBytes / 16];
  for (int i = threadIdx.x; i < kLdsBytes / 16; i += 256) lds[i] = in[(i * 7 + blockIdx.x) & 4095];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  h8 b[4][2];
  for (int j = 0; j < 4; ++j)
    for (int p = 0; p < 2; ++p) b[j][p] = in[(threadIdx.x + 256 * (2 * j + p)) & 4095];
  float v[12];
  for (int i = 0; i < 12; ++i) v[i] = (float)in[threadIdx.x & 4095][i & 7];
  f16v acc32[4];
  f4v acc16[4][2];
  for (int t = 0; t < 4; ++t) {
    acc32[t] = f16v{};
    acc16[t][0] = f4v{};
    acc16[t][1] = f4v{};
  }
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  h8 abuf[2][4][2];
  int off = lane;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int p = 0; p < 2; ++p) abuf[0][t][p] = lds[(off + 64 * (2 * t + p)) & (kLdsBytes / 16 - 1)];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int hs = 0; hs < 4; ++hs) {
      // fragments of this half-step were read during the previous one (double buffer, as mlp16)
      h8 (&a)[4][2] = abuf[hs & 1];
      h8 (&an)[4][2] = abuf[(hs + 1) & 1];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int p = 0; p < 2; ++p) an[t][p] = lds[(off + 64 * (2 * t + p + 8 * (hs + 1))) & (kLdsBytes / 16 - 1)];
      const h8& bh = b[hs][0];
      const h8& bl = b[hs][1];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if constexpr (SHAPE == 32) {
          acc32[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[t][1], bh, acc32[t], 0, 0, 0);
          acc32[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[t][0], bl, acc32[t], 0, 0, 0);
          acc32[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[t][0], bh, acc32[t], 0, 0, 0);
        } else {
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            acc16[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t][1], n ? bl : bh, acc16[t][n], 0, 0, 0);
            acc16[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t][0], n ? bh : bl, acc16[t][n], 0, 0, 0);
            acc16[t][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[t][0], n ? bl : bh, acc16[t][n], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j % 12] = __builtin_fmaf(v[j % 12], 1.0001f, v[(j + 5) % 12]);
      constexpr int nm = SHAPE == 32 ? 12 : 24;
      constexpr int vpg = (NV + nm - 2) / (nm - 1);
#pragma unroll
      for (int i = 0; i < nm; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (i >= 1 && i < 9) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (i >= 1 && vpg > 0) __builtin_amdgcn_sched_group_barrier(0x002, vpg, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    off += 17;
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0;
  for (int t = 0; t < 4; ++t) {
    for (int i = 0; i < 16; ++i) s += acc32[t][i];
    for (int i = 0; i < 4; ++i) s += acc16[t][0][i] + acc16[t][1][i];
  }
  for (int i = 0; i < 12; ++i) s += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) ticks[blockIdx.x] = t1 - t0;
}

template <int SHAPE, int NV>
void run(const h8* in, float* out, unsigned long long* ticks, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // warm: >= 2 s of back-to-back launches
  float ms = 0;
  int reps = 1;
  for (;;) {
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) k<SHAPE, NV><<<blocks, 256>>>(in, out, ticks, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    if (ms > 2000.0f) break;
    reps *= 2;
  }
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) k<SHAPE, NV><<<blocks, 256>>>(in, out, ticks, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long* h = (unsigned long long*)malloc(blocks * 8);
  hipMemcpy(h, ticks, blocks * 8, hipMemcpyDeviceToHost);
  double tk = 0;
  for (int i = 0; i < blocks; ++i) tk += h[i];
  tk /= blocks;
  const double flop = (double)reps * blocks * 4 /*waves*/ * iters * 4 /*half-steps*/ * 393216.0;
  printf("shape %2d NV %3d: %8.1f TFLOP/s  %7.1f cycles/half-step (floor 384)  clock~%.2f GHz\n", SHAPE, NV,
         flop / (ms * 1e-3) / 1e12, tk / (iters * 4.0), tk * (blocks / 256.0) / (ms * 1e-3 / reps) / 1e9);
  free(h);
}

int main() {
  const int blocks = 256 * 8, iters = 400;
  h8* in;
  float* out;
  unsigned long long* ticks;
  hipMalloc(&in, 4096 * 16);
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&ticks, blocks * 8);
  _Float16* hbuf = (_Float16*)malloc(4096 * 16);
  srand(1);
  for (int i = 0; i < 4096 * 8; ++i) hbuf[i] = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.01f);
  hipMemcpy(in, hbuf, 4096 * 16, hipMemcpyHostToDevice);
  run<32, 0>(in, out, ticks, blocks, iters);
  run<16, 0>(in, out, ticks, blocks, iters);
  run<32, 24>(in, out, ticks, blocks, iters);
  run<16, 24>(in, out, ticks, blocks, iters);
  run<32, 36>(in, out, ticks, blocks, iters);
  run<16, 36>(in, out, ticks, blocks, iters);
  run<32, 48>(in, out, ticks, blocks, iters);
  run<16, 48>(in, out, ticks, blocks, iters);
  run<32, 0>(in, out, ticks, blocks, iters);
  run<16, 0>(in, out, ticks, blocks, iters);
  return 0;
}
