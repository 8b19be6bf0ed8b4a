// Rounding of v_mfma_f32_32x32x16_f16 (f32 accumulation) and of the v_fma_mixlo_f16 split, against
// exact double arithmetic: is the accumulation round-to-nearest-even, and is it unbiased?
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_rounding scripts/microbench/mfma_rounding.hip
// Case 0: small integers (exact in f32: checks the operand/result layout).  Case 1: random operands
// of similar magnitude.  Case 2: |C| >> |A B| (the accumulator dominates: the lo*hi products of the
// f16x3 split added to a running sum).  Per case: mean and rms of (D - exact) in ulps of the exact
// value, and the fraction of results farther than 0.5 ulp from exact (not correctly rounded).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void mfma_k(const _Float16* A, const _Float16* B, const float* C, float* D) {
  // tile t: A 32x16 row-major, B 16x32 row-major, C/D 32x32 row-major
  const int t = blockIdx.x, l = threadIdx.x;
  const _Float16* a = A + (size_t)t * 512;
  const _Float16* b = B + (size_t)t * 512;
  const float* c = C + (size_t)t * 1024;
  float* d = D + (size_t)t * 1024;
  h8 av, bv;
  for (int j = 0; j < 8; ++j) {
    av[j] = a[(l % 32) * 16 + 8 * (l / 32) + j];
    bv[j] = b[(8 * (l / 32) + j) * 32 + l % 32];
  }
  f16v cv;
  for (int r = 0; r < 16; ++r) cv[r] = c[(8 * (r / 4) + 4 * (l / 32) + r % 4) * 32 + l % 32];
  f16v dv = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, cv, 0, 0, 0);
  for (int r = 0; r < 16; ++r) d[(8 * (r / 4) + 4 * (l / 32) + r % 4) * 32 + l % 32] = dv[r];
}

__global__ void mix_k(const float* x, _Float16* lo_mix, _Float16* lo_rne, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  const _Float16 hi = (_Float16)v;
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const h2 hh = {hi, hi};
  uint32_t hi2 = __builtin_bit_cast(uint32_t, hh), lo;
  asm volatile("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=&v"(lo) : "v"(hi2), "v"(v));
  lo_mix[i] = __builtin_bit_cast(_Float16, (uint16_t)(lo & 0xffff));
  lo_rne[i] = (_Float16)(v - (float)hi);
}

static double ulp_of(double v) {
  const float f = fabsf((float)v);
  return (double)nextafterf(f, INFINITY) - (double)f;
}

int main() {
  const int T = 4096;
  std::vector<_Float16> A((size_t)T * 512), B((size_t)T * 512);
  std::vector<float> C((size_t)T * 1024), D((size_t)T * 1024);
  _Float16 *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
  srand(1);
  auto U = [] { return 2.0 * rand() / RAND_MAX - 1.0; };
  for (int cs = 0; cs < 3; ++cs) {
    for (size_t i = 0; i < A.size(); ++i) {
      A[i] = (_Float16)(cs == 0 ? (double)(rand() % 7 - 3) : U());
      B[i] = (_Float16)(cs == 0 ? (double)(rand() % 7 - 3) : U());
    }
    for (size_t i = 0; i < C.size(); ++i) C[i] = (float)(cs == 0 ? (double)(rand() % 7 - 3) : (cs == 1 ? U() : 4096.0 * U()));
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    mfma_k<<<T, 64>>>(dA, dB, dC, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    double s = 0, s2 = 0, maxe = 0;
    long bad = 0, n = 0;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          double ex = C[(size_t)t * 1024 + i * 32 + j];
          for (int k = 0; k < 16; ++k)
            ex += (double)A[(size_t)t * 512 + i * 16 + k] * (double)B[(size_t)t * 512 + k * 32 + j];
          const double u = ulp_of(ex);
          if (u == 0) continue;
          const double e = ((double)D[(size_t)t * 1024 + i * 32 + j] - ex) / u;
          s += e; s2 += e * e; ++n;
          if (fabs(e) > 0.5 + 1e-9) ++bad;
          if (fabs(e) > maxe) maxe = fabs(e);
        }
    printf("mfma case %d: n=%ld mean err %+.4f ulp, rms %.4f ulp, max %.3f ulp, not correctly rounded %.4f\n", cs, n,
           s / n, sqrt(s2 / n), maxe, (double)bad / n);
  }
  const int N = 1 << 20;
  std::vector<float> X(N);
  for (int i = 0; i < N; ++i) X[i] = (float)(U() * pow(2.0, rand() % 20 - 10));
  float* dX;
  _Float16 *dm, *dr;
  hipMalloc(&dX, N * 4); hipMalloc(&dm, N * 2); hipMalloc(&dr, N * 2);
  hipMemcpy(dX, X.data(), N * 4, hipMemcpyHostToDevice);
  mix_k<<<N / 256, 256>>>(dX, dm, dr, N);
  std::vector<_Float16> m(N), r(N);
  hipMemcpy(m.data(), dm, N * 2, hipMemcpyDeviceToHost);
  hipMemcpy(r.data(), dr, N * 2, hipMemcpyDeviceToHost);
  long diff = 0;
  double bias = 0;
  for (int i = 0; i < N; ++i) {
    if ((float)m[i] != (float)r[i]) ++diff;
    bias += (double)(float)m[i] - (double)(float)r[i];
  }
  printf("v_fma_mixlo_f16 vs RNE convert: %ld of %d differ, summed difference %g\n", diff, N, bias);
  return 0;
}
