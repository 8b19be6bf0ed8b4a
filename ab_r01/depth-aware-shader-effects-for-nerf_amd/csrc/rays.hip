// Ray generation, direction normalisation and stratified sampling (R1, R2).
//
// HBM-bound elementwise kernels in ray-major layout.  Every expression keeps the
// reference's operation order and roundings: the library is built with
// -ffp-contract=off, so no multiply-add is fused unless written as fmaf().
#include "common.h"

namespace nerf {

// ---------------------------------------------------------------------------- get_rays
// src/ray_utils.py:4-50.  One thread per pixel.  x = (j - W*0.5)/f, y = -((i - H*0.5)/f),
// z = -1 (:26-28); dir_w[r] = x*R[r][0] + y*R[r][1] + z*R[r][2] summed left to right
// (:40-42); divided by torch.norm, which torch evaluates as sqrt(fma(z,z,fma(y,y,x*x)))
// (:45, measured bit-exact against torch CPU).
struct C2W { float m[12]; };

__global__ void __launch_bounds__(256) get_rays_kernel(int H, int W, float focal, C2W c2w,
                                                       int row0, int64_t npix, float* __restrict__ o,
                                                       float* __restrict__ d) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const float i = (float)(row0 + (int)(p / W));
  const float j = (float)(int)(p % W);
  const float x = (j - (float)W * 0.5f) / focal;
  const float y = -((i - (float)H * 0.5f) / focal);
  const float z = -1.0f;
  float v[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float* R = c2w.m + 4 * r;
    v[r] = (x * R[0] + y * R[1]) + z * R[2];
  }
  const float n = sqrtf(fmaf(v[2], v[2], fmaf(v[1], v[1], v[0] * v[0])));
#pragma unroll
  for (int r = 0; r < 3; ++r) d[3 * p + r] = v[r] / n;
  if (o) {
#pragma unroll
    for (int r = 0; r < 3; ++r) o[3 * p + r] = c2w.m[4 * r + 3];
  }
}

int launch_get_rays(int H, int W, float focal, const float* c2w, int row0, int nrows, float* o,
                    float* d, hipStream_t s) {
  C2W m;
  for (int k = 0; k < 12; ++k) m.m[k] = c2w[k];
  const int64_t npix = (int64_t)nrows * W;
  if (npix == 0) return NERF_OK;
  const int blocks = (int)((npix + 255) / 256);
  hipLaunchKernelGGL(get_rays_kernel, dim3(blocks), dim3(256), 0, s, H, W, focal, m, row0, npix, o, d);
  return check_launch("get_rays_kernel");
}

// --------------------------------------------------------------------------- normalize
// F.normalize(rays_d, dim=-1) (src/render.py:19): x / max(||x||, 1e-12).
__global__ void __launch_bounds__(256) normalize_kernel(const float* __restrict__ d, int64_t B,
                                                        float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  const float x = d[3 * r], y = d[3 * r + 1], z = d[3 * r + 2];
  const float n = fmaxf(sqrtf(fmaf(z, z, fmaf(y, y, x * x))), 1e-12f);
  out[3 * r] = x / n;
  out[3 * r + 1] = y / n;
  out[3 * r + 2] = z / n;
}

int launch_normalize(const float* d, int64_t B, float* out, hipStream_t s) {
  if (B == 0) return NERF_OK;
  hipLaunchKernelGGL(normalize_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, d, B, out);
  return check_launch("normalize_kernel");
}

// -------------------------------------------------------------------------- stratified
// src/ray_utils.py:52-88.  z = near + t*(far-near) (:70); with perturb, mids = 0.5*(z[s+1]+z[s]),
// upper = [mids, z[N-1]], lower = [z[0], mids], z = lower + (upper-lower)*u (:76-81);
// pts = o + d*z (:86).  One thread per sample; consecutive threads walk the samples of a ray,
// so z and pts stores are coalesced.
__global__ void __launch_bounds__(256) stratified_kernel(const float* __restrict__ o,
                                                         const float* __restrict__ d, int64_t total,
                                                         float near_f, float span_f, int N,
                                                         const float* __restrict__ t_vals, int perturb,
                                                         const float* __restrict__ t_rand, uint64_t seed,
                                                         float* __restrict__ z_out, float* __restrict__ pts) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int64_t r = idx / N;
  const int s = (int)(idx - r * N);
  float z = near_f + t_vals[s] * span_f;
  if (perturb) {
    const float zc = z;
    const float zn = (s + 1 < N) ? near_f + t_vals[s + 1] * span_f : zc;
    const float zp = (s > 0) ? near_f + t_vals[s - 1] * span_f : zc;
    const float upper = (s + 1 < N) ? 0.5f * (zn + zc) : zc;
    const float lower = (s > 0) ? 0.5f * (zc + zp) : zc;
    const float u = t_rand ? t_rand[idx] : hash_uniform(seed, (uint64_t)idx);
    z = lower + (upper - lower) * u;
  }
  z_out[idx] = z;
  if (pts) {
#pragma unroll
    for (int c = 0; c < 3; ++c) pts[3 * idx + c] = o[3 * r + c] + d[3 * r + c] * z;
  }
}

int launch_stratified(const float* o, const float* d, int64_t B, float near_f, float span_f, int N,
                      const float* t_vals, int perturb, const float* t_rand, uint64_t seed, float* z,
                      float* pts, hipStream_t s) {
  const int64_t total = B * (int64_t)N;
  if (total == 0) return NERF_OK;
  hipLaunchKernelGGL(stratified_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, o, d,
                     total, near_f, span_f, N, t_vals, perturb, t_rand, seed, z, pts);
  return check_launch("stratified_kernel");
}

// ----------------------------------------------------------------- positional encoding
// PositionalEncoding.__call__ (src/models.py:14-47): out = [x, sin(2^0 x), cos(2^0 x), ...,
// sin(2^(L-1) x), cos(2^(L-1) x)] along the last dim (x dropped when include_input is 0).
// One thread per output element.
__global__ void __launch_bounds__(256) pe_kernel(const float* __restrict__ x, int64_t M, int dims, int levels,
                                                 int include_input, float* __restrict__ out) {
  const int width = dims * (2 * levels + (include_input ? 1 : 0));
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * width) return;
  const int64_t m = idx / width;
  int f = (int)(idx - m * width);
  if (include_input) {
    if (f < dims) { out[idx] = x[m * dims + f]; return; }
    f -= dims;
  }
  const int i = f / (2 * dims), rem = f % (2 * dims);
  const float v = x[m * dims + rem % dims] * (float)(1 << i);
  out[idx] = rem < dims ? sinf(v) : cosf(v);
}

int launch_pe(const float* x, int64_t M, int dims, int levels, int include_input, float* out, hipStream_t s) {
  const int64_t total = M * (int64_t)dims * (2 * levels + (include_input ? 1 : 0));
  if (total == 0) return NERF_OK;
  hipLaunchKernelGGL(pe_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, M, dims, levels,
                     include_input, out);
  return check_launch("pe_kernel");
}

}  // namespace nerf
