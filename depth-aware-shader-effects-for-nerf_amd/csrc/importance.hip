// Inverse-CDF fine resampling with the H1 clamp, and the sorted merge with the coarse samples (R3).
//
// Reference: src/ray_utils.py:90-149.  One wave per ray:
//   w' = w + 1e-5;  pdf = w'/sum(w');  cdf = [0, cumsum(pdf)]            (:106-112)
//   u_j = linspace(0,1,Nf+1)[j] + rand_j/Nf                                (:115-119)
//   i = searchsorted(cdf, u) (left);  below = max(i-1,0), above = min(i,N)  (:122-124)
//   z_f = z[below'] + (u-cdf[below])/denom * (z[above']-z[below'])          (:127-139)
//     with denom = cdf[above]-cdf[below], 1 where < 1e-5, and below'/above' the z index
//     clamped to N-1 (H1: the reference gathers z[N] there and raises).
//   z_all = sort(cat[z, z_f]);  pts = o + d*z_all                           (:142-147)
// cumsum runs as a double-precision add scan (torch's CPU cumsum accumulates in double; the
// double partial sums of these floats are exact, so the association order does not matter).
// The merge computes every element's output slot by binary search in the other sorted list
// (merge path); if either list is not ascending (possible by one rounding step in
// degenerate bins) every slot is instead the element's full rank, so the output is always
// exactly sort(cat[z, z_f]).
//
// Coarse-evaluation reuse (optional outputs): the kernel also scatters the coarse pass's
// (rgb, sigma) into their merged slots and emits the fine samples with their slots, so the
// fine MLP pass evaluates only the Nf new samples.  Or (merged_src, nerf_render_rays) it records
// for each merged slot which sample sits there (index into cat[coarse, fine]) and emits the fine
// samples alone: the fine MLP then writes its results in sample order and the composite gathers
// through the map, so nothing is scattered.  The MLP is deterministic per sample and a
// coarse sample's point o + d*z is recomputed bit-identically, so this equals re-evaluating all
// N+Nf merged samples (tests/test_gpu_parity.py::test_coarse_reuse_is_bit_identical).
//
// Bound: HBM/latency.  Reads 8 B per coarse sample (+4 B per fine uniform), writes 4 B per
// merged sample (+12 B with pts).  LDS per wave: (N+1) + 2N + Nf floats.
#include "common.h"

namespace nerf {

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// first index i in [0, n] with a[i] >= v (n if none) over a[0..n-1]
__device__ __forceinline__ int lower_bound_lds(const float* a, int n, float v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}
// first index i with a[i] > v
__device__ __forceinline__ int upper_bound_lds(const float* a, int n, float v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(256)
importance_kernel(const float* __restrict__ o, const float* __restrict__ d, const float* __restrict__ zv,
                  const float* __restrict__ wv, int64_t B, int N, int Nf, const float* __restrict__ u_lin,
                  const float* __restrict__ u_rand, uint64_t seed, float* __restrict__ z_all,
                  float* __restrict__ pts_all, const float* __restrict__ rgb_c, const float* __restrict__ sigma_c,
                  float* __restrict__ rgb_all, float* __restrict__ sigma_all, float* __restrict__ z_fine,
                  int* __restrict__ fine_slot, uint16_t* __restrict__ merged_src) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * 4 + wid;
  const int per_wave = (N + 1) + N + Nf + N;
  float* cdf = lds + wid * per_wave;
  float* zc = cdf + (N + 1);
  float* zf = zc + N;
  float* wp = zf + Nf;
  const bool live = r < B;                     // dead waves still reach every barrier
  const int64_t rr = live ? r : 0;

  // pdf normaliser (:106-108), summed in the order torch's CPU sum reduces a contiguous float
  // row (aten SumKernel: 8-float vectors, 4 interleaved vector accumulators, then the scalar
  // tail and the 8 lanes left to right), so pdf and cdf come out bit-identical.
  for (int s = lane; s < N; s += 64) wp[s] = wv[rr * N + s] + 1e-5f;
  __syncthreads();
  const int nvec = N >> 3, ilp = nvec >> 2;
  float part = 0.0f;
  if (lane < 32) {
    const int k = lane >> 3, l = lane & 7;
    for (int i = 0; i < ilp; ++i) part += wp[(i * 4 + k) * 8 + l];
    if (k == 0)
      for (int i = ilp * 4; i < nvec; ++i) part += wp[i * 8 + l];
  }
  const float vsum = ((part + __shfl(part, lane + 8)) + __shfl(part, lane + 16)) + __shfl(part, lane + 24);
  float total = 0.0f;
  if (nvec > 0) {
    for (int s = nvec * 8; s < N; ++s) total += wp[s];
#pragma unroll
    for (int l = 0; l < 8; ++l) total += __shfl(vsum, l);
  } else {  // rows shorter than one vector: 4 interleaved scalar accumulators
    float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 0; i < (N >> 2); ++i)
      for (int k = 0; k < 4; ++k) p[k] += wp[4 * i + k];
    for (int s = (N >> 2) * 4; s < N; ++s) p[0] += wp[s];
    total = ((p[0] + p[1]) + p[2]) + p[3];
  }

  // cdf = [0, cumsum(pdf)] (:111-112), z to LDS
  double carry = 0.0;
  for (int c0 = 0; c0 < N; c0 += 64) {
    const int s = c0 + lane;
    double v = 0.0;
    if (s < N) {
      v = (double)(wp[s] / total);
      zc[s] = zv[rr * N + s];
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double up = __shfl_up(v, off);
      if (lane >= off) v += up;
    }
    if (s < N) cdf[s + 1] = (float)(carry + v);
    carry += __shfl(v, 63);
  }
  if (lane == 0) cdf[0] = 0.0f;
  __syncthreads();                             // every wave runs the same trip counts

  // inverse CDF (:115-139)
  const float nf = (float)Nf;
  for (int j = lane; j < Nf; j += 64) {
    const float ur = u_rand ? u_rand[rr * Nf + j] : hash_uniform(seed, (uint64_t)(rr * Nf + j));
    const float u = u_lin[j] + ur / nf;
    const int i = lower_bound_lds(cdf, N + 1, u);
    const int below = i - 1 > 0 ? i - 1 : 0;
    const int above = i < N ? i : N;
    const float c0 = cdf[below], c1 = cdf[above];
    const float z0 = zc[below < N - 1 ? below : N - 1];
    const float z1 = zc[above < N - 1 ? above : N - 1];
    float denom = c1 - c0;
    if (denom < 1e-5f) denom = 1.0f;
    const float t = (u - c0) / denom;
    zf[j] = z0 + t * (z1 - z0);
  }
  __syncthreads();

  // merge (:142-144)
  bool sorted_ok = true;
  for (int s = lane; s + 1 < N; s += 64) sorted_ok &= zc[s] <= zc[s + 1];
  for (int j = lane; j + 1 < Nf; j += 64) sorted_ok &= zf[j] <= zf[j + 1];
  sorted_ok = __all(sorted_ok);
  if (!live) return;
  const int T = N + Nf;
  float* zo = z_all + r * T;
  float3 orr, drr;
  if (pts_all) {
    orr = make_float3(o[3 * r], o[3 * r + 1], o[3 * r + 2]);
    drr = make_float3(d[3 * r], d[3 * r + 1], d[3 * r + 2]);
  }
  for (int e = lane; e < T; e += 64) {
    const bool coarse = e < N;
    const float v = coarse ? zc[e] : zf[e - N];
    int pos;
    if (sorted_ok) {
      pos = coarse ? e + lower_bound_lds(zf, Nf, v) : (e - N) + upper_bound_lds(zc, N, v);
    } else {
      // full rank with ties broken by position in cat[z, z_f]
      pos = 0;
      for (int k = 0; k < T; ++k) {
        const float w = k < N ? zc[k] : zf[k - N];
        pos += (w < v) || (w == v && k < e);
      }
    }
    zo[pos] = v;
    if (merged_src) merged_src[r * T + pos] = (uint16_t)e;
    if (coarse) {
      if (rgb_all) {                           // coarse evaluation reused at its merged slot
        const int64_t src = r * N + e, dst = r * T + pos;
        rgb_all[3 * dst] = rgb_c[3 * src];
        rgb_all[3 * dst + 1] = rgb_c[3 * src + 1];
        rgb_all[3 * dst + 2] = rgb_c[3 * src + 2];
        sigma_all[dst] = sigma_c[src];
      }
    } else if (z_fine) {                       // fine sample to evaluate, and where its result goes
      z_fine[r * Nf + (e - N)] = v;
      if (fine_slot) fine_slot[r * Nf + (e - N)] = pos;
    }
    if (pts_all) {
      float* p = pts_all + 3 * (r * T + pos);
      p[0] = orr.x + drr.x * v;
      p[1] = orr.y + drr.y * v;
      p[2] = orr.z + drr.z * v;
    }
  }
}

int launch_importance(const float* o, const float* d, const float* z, const float* w, int64_t B, int N, int Nf,
                      const float* u_lin, const float* u_rand, uint64_t seed, float* z_all, float* pts_all,
                      const float* rgb_c, const float* sigma_c, float* rgb_all, float* sigma_all, float* z_fine,
                      int* fine_slot, hipStream_t s, uint16_t* merged_src) {
  if (B == 0) return NERF_OK;
  const size_t lds = (size_t)4 * ((N + 1) + 2 * N + Nf) * sizeof(float);
  hipLaunchKernelGGL(importance_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), lds, s, o, d, z, w, B, N, Nf,
                     u_lin, u_rand, seed, z_all, pts_all, rgb_c, sigma_c, rgb_all, sigma_all, z_fine, fine_slot,
                     merged_src);
  return check_launch("importance_kernel");
}

}  // namespace nerf
