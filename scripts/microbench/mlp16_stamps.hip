// Diagnostic: per-wave segment durations (s_memtime) of mlp16_kernel (the f16x3 MLP) on the
// coarse pass of an 800x800 frame (640,000 rays x 64 samples), synthetic inputs.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNERF_MLP16_STAMPS \
//     -I depth-aware-shader-effects-for-nerf_amd/csrc -o scripts/microbench/mlp16_stamps scripts/microbench/mlp16_stamps.hip
// Stamps: 0 start | 1 prologue done (PE, first chunk) | 2 + L after trunk layer L (0..7; each
// layer's epilogue runs inside the next layer's MFMAs) | 10 after the colour layer | 11 end.
// (Round 6: launch_mlp16 without saves runs mlp16s_kernel, which has no stamps; this tool timed the
// round-5 render kernel and needs round 5's csrc/mlp16.hip, e.g. from `git show 5134bc2:...`.)
#include "../../depth-aware-shader-effects-for-nerf_amd/csrc/mlp16.hip"
#include <algorithm>
#include <stdarg.h>
#include <vector>
#include <stdlib.h>
int nerf::set_error(int code, const char* fmt, ...) { va_list ap; va_start(ap, fmt); vprintf(fmt, ap); va_end(ap); return code; }

int main() {
  const int64_t R = 640000, N = 64, M = R * N;
  std::vector<float> h(nerf::kPackedFloats);
  srand(1);
  for (auto& v : h) v = ((float)rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  for (int L = 0; L < nerf::kS16Layers; ++L) {
    h[nerf::kOffScale16 + nerf::kS16Sw + L] = 65536.f;
    h[nerf::kOffScale16 + nerf::kS16InvW + L] = 1.f / 65536.f;
    if (L < 8) { h[nerf::kOffScale16 + nerf::kS16R + L] = 8.f; h[nerf::kOffScale16 + nerf::kS16B + L] = 0.1f; }
  }
  float *packed, *o, *d, *z, *feat, *rgb, *sig;
  (void)hipMalloc(&packed, h.size() * 4);
  (void)hipMemcpy(packed, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  std::vector<float> od(R * 3);
  for (int64_t i = 0; i < R; ++i) { od[3*i] = 0; od[3*i+1] = 0.5f; od[3*i+2] = 4; }
  (void)hipMalloc(&o, R * 12); (void)hipMemcpy(o, od.data(), R * 12, hipMemcpyHostToDevice);
  for (int64_t i = 0; i < R; ++i) { od[3*i] = (i % 800 - 400) / 1111.f; od[3*i+1] = (i / 800 - 400) / 1111.f; od[3*i+2] = -1; }
  (void)hipMalloc(&d, R * 12); (void)hipMemcpy(d, od.data(), R * 12, hipMemcpyHostToDevice);
  std::vector<float> zz(M);
  for (int64_t i = 0; i < M; ++i) zz[i] = 2 + 4.f * (i % N) / (N - 1);
  (void)hipMalloc(&z, M * 4); (void)hipMemcpy(z, zz.data(), M * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&feat, R * 256 * 4); (void)hipMemset(feat, 0, R * 256 * 4);
  (void)hipMalloc(&rgb, M * 12); (void)hipMalloc(&sig, M * 4);
  // STAMP_REPS back-to-back launches (default 2): the last one is stamped and timed; with more
  // reps the per-launch times show the clock the chip settles at under sustained load.
  const int reps = getenv("STAMP_REPS") ? atoi(getenv("STAMP_REPS")) : 2;
  std::vector<hipEvent_t> ev(reps + 1);
  for (auto& e : ev) (void)hipEventCreate(&e);
  (void)hipEventRecord(ev[0], 0);
  for (int rep = 0; rep < reps; ++rep) {
    nerf::launch_mlp16(packed, o, d, z, R, N, feat, rgb, sig, nullptr, 0, 0);
    (void)hipEventRecord(ev[rep + 1], 0);
  }
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, ev[reps - 1], ev[reps]);
  if (reps > 2) {
    printf("per-launch ms:");
    for (int rep = 0; rep < reps; ++rep) {
      float t = 0;
      (void)hipEventElapsedTime(&t, ev[rep], ev[rep + 1]);
      printf(" %.1f", t);
    }
    printf("\n");
  }
  static unsigned long long st[65536][16];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(nerf::nerf16_stamps), sizeof(st));
  struct Seg { const char* name; int a, b; };
  std::vector<Seg> segs = {{"prologue", 0, 1}, {"L0", 1, 2}, {"L1", 2, 3}, {"L2", 3, 4}, {"L3", 4, 5}, {"L4", 5, 6},
                           {"L5", 6, 7}, {"L6", 7, 8}, {"L7", 8, 9}, {"colour", 9, 10}, {"heads", 10, 11}};
  double sum = 0;
  for (auto& sg : segs) {
    std::vector<double> v;
    for (int w = 0; w < 65536; ++w) v.push_back((double)(st[w][sg.b] - st[w][sg.a]));
    std::sort(v.begin(), v.end());
    printf("%-14s median %8.0f  p10 %8.0f  p90 %8.0f\n", sg.name, v[v.size() / 2], v[v.size() / 10], v[9 * v.size() / 10]);
    sum += v[v.size() / 2];
  }
  std::vector<double> tot;
  for (int w = 0; w < 65536; ++w) tot.push_back((double)(st[w][11] - st[w][0]));
  std::sort(tot.begin(), tot.end());
  printf("total median %.0f (sum of medians %.0f) memtime ticks; MFMA floor 98304 cycles per wave; kernel %.2f ms\n",
         tot[tot.size() / 2], sum, ms);
  return 0;
}
