// Alpha compositing of volume_render (R7): 16 lanes per ray, 4 consecutive samples per lane.
//
// Reference: src/render.py:56-80.
//   dists = [z[s+1]-z[s], 1e-3]  alpha = 1 - exp(-sigma*dist)
//   T = exclusive cumprod(1 - alpha + 1e-10)   w = alpha*T
//   rgb_map = sum w*c     depth = sum w*z / (sum w + 1e-10)
// torch's CPU cumprod accumulates in double and rounds each prefix to float; the kernel
// computes the same prefixes as a double-precision product scan (below), the running product
// carried across 64-sample rounds.  Sums accumulate the reference's float products in double and
// round once.
//
// N == 1 reproduces the reference's degenerate case: z[1:]-z[:-1] is empty and so is the
// padded dists tensor (render.py:56-58 pads with ones_like of an empty slice), every
// per-sample tensor is empty and both maps are 0.
//
// Bound: HBM.  Reads 20 B/sample (rgb 12, sigma 4, z 4), writes 16 B/ray (+4 B/sample of
// weights when requested).
//
// Layout of the work: 16 lanes (one DPP row) per ray, 4 rays per wave.  A ray is taken in rounds
// of 64 samples; in a round lane k owns samples 4k .. 4k+3 (contiguous: 16-byte loads of z, sigma
// and the 48 bytes of rgb when the buffers allow, one 16-byte store of weights).  Per round: the
// lane's product of its 4 factors, an exclusive product scan over the row's 16 lanes in double
// (4 `row_shr` DPP steps, no LDS), each sample's T = carry * row prefix * lane prefix (products in
// double, rounded once to float), and the lane's running sums.  The row's last lane carries the
// product into the next round; the sums are added over the row by 4 DPP steps at the end.  (One
// wave per ray with 64-lane shuffle scans and reductions through ds_bpermute ran 0.50 / 0.88 ms for
// the 800^2 coarse / fine composite, 0.28 of HBM bandwidth: it was bound by the cross-lane traffic.)
#include "common.h"

namespace nerf {

// v from the lane `off` below in the same 16-lane row; lanes below off get `fill`
template <int OFF>
__device__ __forceinline__ double row_shr(double v, double fill) {
  const long long b = __builtin_bit_cast(long long, v), fb = __builtin_bit_cast(long long, fill);
  const int lo = __builtin_amdgcn_update_dpp((int)fb, (int)b, 0x110 + OFF, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(fb >> 32), (int)(b >> 32), 0x110 + OFF, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// inclusive product / sum over lanes 0..k of the row
__device__ __forceinline__ double row_scan_mul(double v) {
  v *= row_shr<1>(v, 1.0);
  v *= row_shr<2>(v, 1.0);
  v *= row_shr<4>(v, 1.0);
  v *= row_shr<8>(v, 1.0);
  return v;
}
__device__ __forceinline__ double row_scan_add(double v) {
  v += row_shr<1>(v, 0.0);
  v += row_shr<2>(v, 0.0);
  v += row_shr<4>(v, 0.0);
  v += row_shr<8>(v, 0.0);
  return v;
}

// MERGED (the fine composite of nerf_render_rays): sample s of ray r is sample src[r N + s] of
// cat[coarse, fine] (importance.hip's merged_src), gathered from the coarse pass's and the fine MLP's
// outputs, which both lie in sample order; z comes from the merged z row.  The same values in the
// same order as compositing rows the coarse results were scattered into: the same bits.
struct MergedSrc {
  const float* rgb_c;
  const float* sigma_c;
  const float* rgb_f;
  const float* sigma_f;
  const uint16_t* src;
  int nc, nf;
};

// VEC: every pointer 16-byte aligned and N % 4 == 0, so a lane's 4 samples load as one f32x4.
// STAGE (MERGED, T <= kStageT): 8 rays per block; their coarse and fine (rgb, sigma) are first copied
// into LDS as one (r, g, b, sigma) quad per cat index, with whole-row coalesced loads, and the
// composite gathers from there (gathering each sample's 16 bytes from global memory cost 1.14 ms
// for the 800^2 fine pass against 0.18 ms of staging).
constexpr int kStageT = 256;
template <bool VEC, bool MERGED, bool STAGE = false>
__global__ void __launch_bounds__(256)
composite_kernel(const float* __restrict__ rgb, const float* __restrict__ sigma, const float* __restrict__ zv,
                 int64_t B, int N, float* __restrict__ rgb_map, float* __restrict__ depth_map,
                 float* __restrict__ weights, MergedSrc ms) {
  extern __shared__ f32x4 quads[];   // STAGE: [8 rays][T]
  const int k = threadIdx.x & 15;
  const int rpb = (int)blockDim.x >> 4;                       // rays per block: 16, or 8 when STAGE
  const int64_t r = (int64_t)blockIdx.x * rpb + (threadIdx.x >> 4);
  const bool ray = r < B;          // rows past B run on with no samples (the DPP stays inside a row)
  const int64_t base = ray ? r * N : 0;
  if constexpr (STAGE) {           // every thread reaches the barrier
    const int64_t r0 = (int64_t)blockIdx.x * rpb;
    const int nr = (int)(B - r0 < rpb ? B - r0 : rpb);
    const int nc = ms.nc, nf = ms.nf;
    for (int i = threadIdx.x; i < nr * N; i += (int)blockDim.x) {   // quad i: ray i / T, cat index i % T
      const int rr = i / N, e = i - rr * N;
      const bool crs = e < nc;
      const int64_t at = crs ? (r0 + rr) * nc + e : (r0 + rr) * nf + (e - nc);
      const float* cs = crs ? ms.rgb_c : ms.rgb_f;
      quads[i] = f32x4{cs[3 * at], cs[3 * at + 1], cs[3 * at + 2], (crs ? ms.sigma_c : ms.sigma_f)[at]};
    }
    __syncthreads();
  }
  const f32x4* rq = quads + (threadIdx.x >> 4) * N;   // STAGE: this ray's quads
  if (ray && N == 1 && weights && k == 0) weights[base] = 0.0f;
  const int n_eff = ray && N > 1 ? N : 0;
  double carry = 1.0;
  double acc_r = 0.0, acc_g = 0.0, acc_b = 0.0, acc_wz = 0.0, acc_w = 0.0;
  for (int c0 = 0; c0 < n_eff; c0 += 64) {
    const int s0 = c0 + 4 * k;
    float z[5], sg[4], c[12];
    if constexpr (MERGED) {
      int e[4];
      if (VEC && s0 + 4 <= n_eff) {    // z and the 4 slots' sources as one 16- and one 8-byte load
        const f32x4 zq = *reinterpret_cast<const f32x4*>(zv + base + s0);
        const uint2 sq = *reinterpret_cast<const uint2*>(ms.src + base + s0);
#pragma unroll
        for (int j = 0; j < 4; ++j) z[j] = zq[j];
        e[0] = (int)(sq.x & 0xffffu), e[1] = (int)(sq.x >> 16), e[2] = (int)(sq.y & 0xffffu), e[3] = (int)(sq.y >> 16);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool v = s0 + j < n_eff;
          z[j] = v ? zv[base + s0 + j] : 0.0f;
          e[j] = v ? (int)ms.src[base + s0 + j] : -1;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool v = e[j] >= 0;
        f32x4 q = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (STAGE) {
          if (v) q = rq[e[j]];
        } else if (v) {
          const bool crs = e[j] < ms.nc;
          const int64_t at = crs ? r * ms.nc + e[j] : r * ms.nf + (e[j] - ms.nc);
          const float* cs = crs ? ms.rgb_c : ms.rgb_f;
          q = f32x4{cs[3 * at], cs[3 * at + 1], cs[3 * at + 2], (crs ? ms.sigma_c : ms.sigma_f)[at]};
        }
        sg[j] = q[3];
#pragma unroll
        for (int c3 = 0; c3 < 3; ++c3) c[3 * j + c3] = q[c3];
      }
    } else if (VEC && s0 + 4 <= n_eff) {
      const f32x4 zq = *reinterpret_cast<const f32x4*>(zv + base + s0);
      const f32x4 sq = *reinterpret_cast<const f32x4*>(sigma + base + s0);
#pragma unroll
      for (int j = 0; j < 4; ++j) z[j] = zq[j], sg[j] = sq[j];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const f32x4 cq = *reinterpret_cast<const f32x4*>(rgb + 3 * (base + s0) + 4 * q);
#pragma unroll
        for (int j = 0; j < 4; ++j) c[4 * q + j] = cq[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool v = s0 + j < n_eff;
        z[j] = v ? zv[base + s0 + j] : 0.0f;
        sg[j] = v ? sigma[base + s0 + j] : 0.0f;
#pragma unroll
        for (int q = 0; q < 3; ++q) c[3 * j + q] = v ? rgb[3 * (base + s0 + j) + q] : 0.0f;
      }
    }
    z[4] = s0 + 4 < n_eff ? zv[base + s0 + 4] : 0.0f;
    float alpha[4];
    double f[4], lane_prod = 1.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = s0 + j;
      alpha[j] = 0.0f;
      f[j] = 1.0;
      if (s < n_eff) {
        const float dist = (s + 1 < N) ? z[j + 1] - z[j] : 1e-3f;
        alpha[j] = 1.0f - expf_rn(-sg[j] * dist);
        f[j] = (double)((1.0f - alpha[j]) + 1e-10f);
      }
      lane_prod *= f[j];
    }
    const double incl = row_scan_mul(lane_prod);
    double pre = carry * row_shr<1>(incl, 1.0);      // product of every factor before this lane's first
    carry *= __shfl(incl, 15, 16);
    float w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w[j] = alpha[j] * (float)pre;                  // 0 past the ray's end (alpha = 0)
      pre *= f[j];
      acc_r += (double)(w[j] * c[3 * j]);
      acc_g += (double)(w[j] * c[3 * j + 1]);
      acc_b += (double)(w[j] * c[3 * j + 2]);
      acc_wz += (double)(w[j] * z[j]);
      acc_w += (double)w[j];
    }
    if (weights) {
      if (VEC && s0 + 4 <= n_eff) {
        *reinterpret_cast<f32x4*>(weights + base + s0) = f32x4{w[0], w[1], w[2], w[3]};
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (s0 + j < n_eff) weights[base + s0 + j] = w[j];
      }
    }
  }
  acc_r = row_scan_add(acc_r);
  acc_g = row_scan_add(acc_g);
  acc_b = row_scan_add(acc_b);
  acc_wz = row_scan_add(acc_wz);
  acc_w = row_scan_add(acc_w);
  if (ray && k == 15) {
    rgb_map[3 * r] = (float)acc_r;
    rgb_map[3 * r + 1] = (float)acc_g;
    rgb_map[3 * r + 2] = (float)acc_b;
    depth_map[r] = (float)acc_wz / ((float)acc_w + 1e-10f);
  }
}

int launch_composite(const float* rgb, const float* sigma, const float* z, int64_t B, int N, float* rgb_map,
                     float* depth, float* weights, hipStream_t s) {
  if (B == 0) return NERF_OK;
  const bool vec = N % 4 == 0 && (uintptr_t)rgb % 16 == 0 && (uintptr_t)sigma % 16 == 0 && (uintptr_t)z % 16 == 0 &&
                   (!weights || (uintptr_t)weights % 16 == 0);
  const dim3 grid((unsigned)((B + 15) / 16));
  const MergedSrc none{};
  if (vec)
    hipLaunchKernelGGL((composite_kernel<true, false>), grid, dim3(256), 0, s, rgb, sigma, z, B, N, rgb_map, depth,
                       weights, none);
  else
    hipLaunchKernelGGL((composite_kernel<false, false>), grid, dim3(256), 0, s, rgb, sigma, z, B, N, rgb_map, depth,
                       weights, none);
  return check_launch("composite_kernel");
}

int launch_composite_merged(const float* rgb_c, const float* sigma_c, const float* rgb_f, const float* sigma_f,
                            const uint16_t* src, const float* z_all, int64_t B, int N, int Nf, float* rgb_map,
                            float* depth, float* weights, hipStream_t s) {
  if (B == 0) return NERF_OK;
  const int T = N + Nf;
  const bool vec = T % 4 == 0 && (uintptr_t)z_all % 16 == 0 && (!weights || (uintptr_t)weights % 16 == 0);
  const dim3 grid((unsigned)((B + 15) / 16));
  const MergedSrc ms{rgb_c, sigma_c, rgb_f, sigma_f, src, N, Nf};
  if (T <= kStageT) {
    const size_t lds = (size_t)8 * T * sizeof(f32x4);
    const dim3 grid8((unsigned)((B + 7) / 8));
    if (vec)
      hipLaunchKernelGGL((composite_kernel<true, true, true>), grid8, dim3(128), lds, s, nullptr, nullptr, z_all, B, T,
                         rgb_map, depth, weights, ms);
    else
      hipLaunchKernelGGL((composite_kernel<false, true, true>), grid8, dim3(128), lds, s, nullptr, nullptr, z_all, B, T,
                         rgb_map, depth, weights, ms);
  } else if (vec)
    hipLaunchKernelGGL((composite_kernel<true, true>), grid, dim3(256), 0, s, nullptr, nullptr, z_all, B, T, rgb_map,
                       depth, weights, ms);
  else
    hipLaunchKernelGGL((composite_kernel<false, true>), grid, dim3(256), 0, s, nullptr, nullptr, z_all, B, T, rgb_map,
                       depth, weights, ms);
  return check_launch("composite_kernel (merged)");
}

}  // namespace nerf
