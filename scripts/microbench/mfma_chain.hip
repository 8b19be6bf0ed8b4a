// Accumulator-chain A/B for the MLP's trunk schedule:
// a "chunk-step" of two 16-deep k-steps x 4 output tiles x 3 split-f16 products = 24
// v_mfma_f32_32x32x16_f16, in three orders:
//   ORDER 0 (mlp16's): per k-step, each tile's three products chained (srcC = the previous result),
//                       tiles one after another: the accumulator of a tile is read once per 3 MFMAs;
//   ORDER 1 (six-chain): per tile, both k-steps' six products chained back to back: read once per 6;
//   ORDER 2 (product-major, for reference): per k-step, the 4 tiles' lo.hi, then hi.lo, then hi.hi.
// A fragments for the next chunk-step read from LDS meanwhile (16 ds_read_b128, as mlp16's two
// half-steps), B operands in registers, NV independent VALU fmas per chunk-step in the MFMA gaps
// (the epilogue's side work), one wave per SIMD, random operands, >= 2 s of back-to-back launches
// before the timed ones (DVFS settles).  Prints wall TFLOP/s, memtime cycles per chunk-step and the
// clock.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_chain scripts/microbench/mfma_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kLdsBytes = 120 * 1024;   // one workgroup per CU
#define MF(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0)

template <int ORDER, int NV>
__global__ void __launch_bounds__(256, 1) k(const h8* __restrict__ in, float* out, unsigned long long* ticks, int iters) {
  __shared__ h8 lds[kLdsBytes / 16];
  for (int i = threadIdx.x; i < kLdsBytes / 16; i += 256) lds[i] = in[(i * 7 + blockIdx.x) & 4095];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  h8 b[2][2];
  for (int j = 0; j < 2; ++j)
    for (int p = 0; p < 2; ++p) b[j][p] = in[(threadIdx.x + 256 * (2 * j + p)) & 4095];
  float v[12];
  for (int i = 0; i < 12; ++i) v[i] = (float)in[threadIdx.x & 4095][i & 7];
  f16v acc[4];
  for (int t = 0; t < 4; ++t) acc[t] = f16v{};
  h8 abuf[2][2][4][2];   // [chunk parity][k-step][tile][hi, lo]
  int off = lane;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int p = 0; p < 2; ++p) abuf[0][ks][t][p] = lds[(off + 64 * (8 * ks + 2 * t + p)) & (kLdsBytes / 16 - 1)];
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int cs = 0; cs < 2; ++cs) {
      h8 (&a)[2][4][2] = abuf[cs];
      h8 (&an)[2][4][2] = abuf[cs ^ 1];
      // Issue order is pinned segment by segment: each segment holds its MFMAs (one tile's chain, so
      // their order is the dependency order), its share of the next fragments' DS reads and of the
      // VALU, interleaved MFMA / DS / VALU by sched_group_barrier, closed by a sched_barrier.
      auto seg = [&](auto nm_c, auto nd_c, auto body) __attribute__((always_inline)) {
        constexpr int nm = decltype(nm_c)::value, nd = decltype(nd_c)::value;
        constexpr int nvs = NV * nm / 24;          // this segment's share of the VALU
        constexpr int vpg = nm > 1 ? (nvs + nm - 2) / (nm - 1) : nvs;
        body();
#pragma unroll
        for (int j = 0; j < nvs; ++j) v[j % 12] = __builtin_fmaf(v[j % 12], 1.0001f, v[(j + 5) % 12]);
#pragma unroll
        for (int i = 0; i < nm; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (i < nd) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          if ((nm == 1 || i >= 1) && vpg > 0) __builtin_amdgcn_sched_group_barrier(0x002, vpg, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      using I2 = std::integral_constant<int, 2>;
      using I3 = std::integral_constant<int, 3>;
      using I4 = std::integral_constant<int, 4>;
      using I6 = std::integral_constant<int, 6>;
      auto rd = [&](int ks, int t) __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
          an[ks][t][p] = lds[(off + 64 * (8 * ks + 2 * t + p + 16 * (cs + 1))) & (kLdsBytes / 16 - 1)];
      };
      if constexpr (ORDER == 0) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            seg(I3{}, I2{}, [&]() __attribute__((always_inline)) {
              rd(ks, t);
              f16v c = MF(a[ks][t][1], b[ks][0], acc[t]);
              c = MF(a[ks][t][0], b[ks][1], c);
              acc[t] = MF(a[ks][t][0], b[ks][0], c);
            });
      } else if constexpr (ORDER == 1) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          seg(I6{}, I4{}, [&]() __attribute__((always_inline)) {
            rd(0, t);
            rd(1, t);
            f16v c = acc[t];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              c = MF(a[ks][t][1], b[ks][0], c);
              c = MF(a[ks][t][0], b[ks][1], c);
              c = MF(a[ks][t][0], b[ks][0], c);
            }
            acc[t] = c;
          });
      } else {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          seg(I4{}, I3{}, [&]() __attribute__((always_inline)) {
            rd(ks, 0);
            rd(ks, 1);
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = MF(a[ks][t][1], b[ks][0], acc[t]);
          });
          seg(I4{}, I3{}, [&]() __attribute__((always_inline)) {
            rd(ks, 2);
            rd(ks, 3);
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = MF(a[ks][t][0], b[ks][1], acc[t]);
          });
          seg(I4{}, I2{}, [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = MF(a[ks][t][0], b[ks][0], acc[t]);
          });
        }
      }
    }
    off += 17;
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0;
  for (int t = 0; t < 4; ++t)
    for (int i = 0; i < 16; ++i) s += acc[t][i];
  for (int i = 0; i < 12; ++i) s += v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) ticks[blockIdx.x] = t1 - t0;
}

template <int ORDER, int NV>
void run(const h8* in, float* out, unsigned long long* ticks, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  int reps = 1;
  for (;;) {   // >= 2 s of back-to-back launches first
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) k<ORDER, NV><<<blocks, 256>>>(in, out, ticks, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    if (ms > 2000.0f) break;
    reps *= 2;
  }
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) k<ORDER, NV><<<blocks, 256>>>(in, out, ticks, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long* h = (unsigned long long*)malloc(blocks * 8);
  hipMemcpy(h, ticks, blocks * 8, hipMemcpyDeviceToHost);
  double tk = 0;
  for (int i = 0; i < blocks; ++i) tk += h[i];
  tk /= blocks;
  const double flop = (double)reps * blocks * 4 /*waves*/ * iters * 2 /*chunk-steps*/ * 24 * 32768.0;
  printf("order %d NV %3d: %8.1f TFLOP/s  %7.1f cycles/chunk-step (floor 768)  clock~%.2f GHz\n", ORDER, NV,
         flop / (ms * 1e-3) / 1e12, tk / (iters * 2.0), tk * (blocks / 256.0) / (ms * 1e-3 / reps) / 1e9);
  free(h);
}

int main() {
  const int blocks = 256 * 8, iters = 200;
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
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 72>(in, out, ticks, blocks, iters);
    run<1, 72>(in, out, ticks, blocks, iters);
    run<2, 72>(in, out, ticks, blocks, iters);
    run<0, 0>(in, out, ticks, blocks, iters);
    run<1, 0>(in, out, ticks, blocks, iters);
  }
  return 0;
}
