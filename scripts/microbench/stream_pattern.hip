// Does the weight gradient's stage shape cost DRAM efficiency?  Streams the hidden-layer phase's
// operand bytes (7 layers x 128 chunks of 2,048 samples; per sample a 1 KiB slice of a tile-major
// 2,320-float gradient row and of a 2,400-float save row) with two stage shapes:
//   MODE 0: 16-sample stages, as wgrad_h16w_kernel: each stage reads 32 pieces of 512 B (one half of
//           every 1 KiB feature group of the 32-sample block), the other halves one stage later;
//   MODE 1: 32-sample stages: each stage reads the block's whole 32 KiB slice in 1 KiB pieces.
// Same bytes, same workgroups; GB/s from hipEvents over 10 launches.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/microbench/stream_pattern scripts/microbench/stream_pattern.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr long M = 262144;
constexpr int RA = 2320, RX = 2400, CLEN = 2048, CHUNKS = 128, LAYERS = 7;

template <int MODE>
__global__ void __launch_bounds__(256) k(const float* __restrict__ A, const float* __restrict__ X, float* out) {
  const int b = blockIdx.x, l = b / CHUNKS, ch = b % CHUNKS, t = threadIdx.x;
  const long m0 = (long)ch * CLEN;
  const float* a = A + (m0 / 32) * 32 * RA + 8192 * l;   // slice of layer l: feature group 32 l (tile_col(256 l))
  const float* x = X + (m0 / 32) * 32 * RX + 8192 * l;
  f4 s = {0, 0, 0, 0};
  if (MODE == 0) {
    for (int st = 0; st < CLEN / 16; ++st) {
      const long blk = st / 2, half = st % 2;
      const float* ab = a + blk * 32 * RA;
      const float* xb = x + blk * 32 * RX;
      f4 v[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int g = t / 32 + 8 * q;
        v[q] = *(const f4*)(ab + g * 256 + half * 128 + (t % 32) * 4);
        v[4 + q] = *(const f4*)(xb + g * 256 + half * 128 + (t % 32) * 4);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s += v[q];
    }
  } else {
    for (int st = 0; st < CLEN / 32; ++st) {
      const float* ab = a + (long)st * 32 * RA;
      const float* xb = x + (long)st * 32 * RX;
      f4 v[16];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int g = t / 64 + 4 * q;
        v[q] = *(const f4*)(ab + g * 256 + (t % 64) * 4);
        v[8 + q] = *(const f4*)(xb + g * 256 + (t % 64) * 4);
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) s += v[q];
    }
  }
  out[(long)b * 256 + t] = s[0] + s[1] + s[2] + s[3];
}

__global__ void fill(float* p, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = (float)(i % 977) * 1e-3f;
}

int main() {
  float *A, *X, *out;
  if (hipMalloc(&A, M * RA * 4) || hipMalloc(&X, M * RX * 4) || hipMalloc(&out, LAYERS * CHUNKS * 256 * 4)) return 1;
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, A, M * RA);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, X, M * RX);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = (double)LAYERS * CHUNKS * CLEN * 2 * 1024;
  for (int rep = 0; rep < 3; ++rep)
    for (int mode = 0; mode < 2; ++mode) {
      for (int w = 0; w < 2; ++w) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(LAYERS * CHUNKS), dim3(256), 0, 0, A, X, out);
        else hipLaunchKernelGGL(k<1>, dim3(LAYERS * CHUNKS), dim3(256), 0, 0, A, X, out);
      }
      hipEventRecord(e0, 0);
      for (int i = 0; i < 10; ++i) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(LAYERS * CHUNKS), dim3(256), 0, 0, A, X, out);
        else hipLaunchKernelGGL(k<1>, dim3(LAYERS * CHUNKS), dim3(256), 0, 0, A, X, out);
      }
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("mode %d (%s): %.1f us per launch, %.0f GB/s\n", mode, mode ? "32-sample stages" : "16-sample stages",
             ms * 100.0, bytes / (ms / 10 * 1e-3) / 1e9);
    }
  return hipDeviceSynchronize() != hipSuccess;
}
