// Depth-aware post effects of the reference's PostProcessor (src/post_processor.py) on the GPU,
// the two effects that read the depth map, Fog (:451-493) and Toon Shader
// (:64-117), plus the depth normalisation run.py applies before them (run.py:248).
//
// Images are the reference's uint8 HxWx3 RGB frames; depth is fp32 HxW (a channel stride lets a
// HxWxC depth use its first channel, as post_processor.py:474-475 does).  The arithmetic follows
// numpy's float32 semantics of the reference expressions (Python scalars cast to float32, one
// rounding per operation, astype(uint8) truncating after the clip).  The cv2 operations of Toon
// (bilateralFilter, Sobel, dilate, cvtColor, Laplacian) are restated from OpenCV 4's algorithms:
// cv2 is not installed here, so that part is pinned to oracle/post_oracle.py, not to cv2.
//
// Every pass is a per-pixel HBM-bound kernel on an 800x800 frame (a few MB): the work is in
// global reductions (max/min for the normalisations, ordered-integer atomics, exact in any order)
// and 3x3 / 9x9 stencils.
#include <math.h>
#include <float.h>

#include "common.h"

namespace nerf {

// Total order on floats as unsigned integers (max/min by atomics are then exact).
__device__ __forceinline__ unsigned f2ord(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }

// mm[0] = max, mm[1] = min (ordered) of x[i*stride], i < n.  mm preset to {0, ~0}.
__global__ void __launch_bounds__(256) minmax_kernel(const float* __restrict__ x, int64_t n, int64_t stride,
                                                      unsigned* __restrict__ mm) {
  unsigned mx = 0u, mn = 0xffffffffu;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned o = f2ord(x[i * stride]);
    mx = max(mx, o);
    mn = min(mn, o);
  }
  for (int off = 32; off > 0; off >>= 1) {
    mx = max(mx, (unsigned)__shfl_xor((int)mx, off));
    mn = min(mn, (unsigned)__shfl_xor((int)mn, off));
  }
  __shared__ unsigned smx[4], smn[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smx[w] = mx;
    smn[w] = mn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
      mx = max(mx, smx[i]);
      mn = min(mn, smn[i]);
    }
    atomicMax(&mm[0], mx);
    atomicMin(&mm[1], mn);
  }
}

// Presets mm = {0, ~0} on the stream (a kernel, not a host copy: stream-ordered without a host
// sync, and capturable into a graph).
__global__ void minmax_init_kernel(unsigned* __restrict__ mm) {
  if (threadIdx.x == 0) {
    mm[0] = 0u;
    mm[1] = 0xffffffffu;
  }
}

static int launch_minmax(const float* x, int64_t n, int64_t stride, unsigned* mm, hipStream_t s) {
  hipLaunchKernelGGL(minmax_init_kernel, dim3(1), dim3(64), 0, s, mm);
  if (int rc = check_launch("minmax_init_kernel")) return rc;
  const int64_t blocks = n > 0 ? (n + 255) / 256 : 1;
  hipLaunchKernelGGL(minmax_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), 0, s, x, n, stride, mm);
  return check_launch("minmax_kernel");
}

__device__ __forceinline__ uint8_t to_u8(float v) {      // np.clip(v, 0, 255).astype(np.uint8)
  return (uint8_t)(int)fminf(fmaxf(v, 0.0f), 255.0f);
}

// run.py:248  depth_norm = (d - min) / (max - min + 1e-6)   (float32 array, Python 1e-6 as float32)
__global__ void __launch_bounds__(256) depth_norm_kernel(const float* __restrict__ d, int64_t n,
                                                          const unsigned* __restrict__ mm, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float mx = ord2f(mm[0]), mn = ord2f(mm[1]);
  out[i] = (d[i] - mn) / ((mx - mn) + 1e-6f);
}

// a**3.0 rounded once to float: a*a is exact in double (48 significant bits), the second product
// rounds to double and then to float.  numpy's float32 power is its SIMD pow (SVML on AVX-512
// hosts, libm elsewhere), within 1 ulp of this and host-dependent; oracle/post_oracle.py's fog
// takes either cube (tests/test_post_effects.py compares both).
__device__ __forceinline__ float cube_rn(float a) {
  const double d = (double)a;
  return (float)((d * d) * d);
}

// post_processor.py:451-493 (Fog): fog colour pure white, fog_start from the parameters.
//   dn = depth (/ max when max > 1); a = clip(max(dn - start, 0) / (1 - start), 0, 1)**3 * 0.3
//   out = clip(img * a + 255 * (1 - a), 0, 255) as uint8; without depth: img * 0.05 + 255 * 0.95.
// start_f / denom_f are float32(fog_start) and float32(1.0 - fog_start) (numpy's weak scalars).
__device__ __forceinline__ void fog_pixel(const uint8_t (&img)[3], float dn, float dmax, float start_f, float denom_f,
                                          uint8_t* __restrict__ out) {
  if (dmax > 1.0f) dn = dn / dmax;
  float a = fmaxf(dn - start_f, 0.0f) / denom_f;
  a = fminf(fmaxf(a, 0.0f), 1.0f);
  a = cube_rn(a);
  a = a * 0.3f;
  const float keep = 1.0f - a;
#pragma unroll
  for (int c = 0; c < 3; ++c) out[c] = to_u8((float)img[c] * a + 255.0f * keep);
}

__global__ void __launch_bounds__(256) fog_kernel(const uint8_t* __restrict__ img, const float* __restrict__ depth,
                                                   int64_t dstride, int64_t P, const unsigned* __restrict__ mm,
                                                   float start_f, float denom_f, uint8_t* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  if (!depth) {
#pragma unroll
    for (int c = 0; c < 3; ++c) out[3 * p + c] = to_u8((float)img[3 * p + c] * 0.05f + 255.0f * 0.95f);
    return;
  }
  const uint8_t px[3] = {img[3 * p], img[3 * p + 1], img[3 * p + 2]};
  fog_pixel(px, depth[p * dstride], ord2f(mm[0]), start_f, denom_f, out + 3 * p);
}

// The CLI's Fog frame (run.py:233 -> :248 -> post_processor.py:451-493) from the render outputs in
// one pass after the depth reduction:
//   img = uint8(rgb * 255) (truncation), dn = (d - min) / (max - min + 1e-6), Fog(img, dn).
// Fog's own maximum of dn is the normalised maximum, exactly: the normalisation is two correctly
// rounded, non-decreasing operations, so max(norm(d)) = norm(max d); no second reduction.
__global__ void __launch_bounds__(256) frame_fog_kernel(const float* __restrict__ rgb, const float* __restrict__ depth,
                                                         int64_t P, const unsigned* __restrict__ mm, float start_f,
                                                         float denom_f, uint8_t* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const float mx = ord2f(mm[0]), mn = ord2f(mm[1]);
  const float range = (mx - mn) + 1e-6f;
  uint8_t px[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) px[c] = (uint8_t)(int)(rgb[3 * p + c] * 255.0f);   // rgb in [0, 1]
  fog_pixel(px, (depth[p] - mn) / range, (mx - mn) / range, start_f, denom_f, out + 3 * p);
}

// ---------------------------------------------------------------------------------- Toon
// cv2 BORDER_DEFAULT = BORDER_REFLECT_101: -1 -> 1, n -> n-2.
__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

constexpr int kBilRadius = 4;                       // bilateralFilter(d=9): radius d/2
constexpr int kBilNumBins = 1 << 12;                // OpenCV's kExpNumBinsPerChannel (one channel)

// Normalised depth (post_processor.py:76-78): d / max when max > 1.
__device__ __forceinline__ float toon_dn(const float* depth, int64_t i, int64_t dstride, float dmax) {
  const float v = depth[i * dstride];
  return dmax > 1.0f ? v / dmax : v;
}

// cv2.bilateralFilter(depth_norm, 9, 75, 75) on float32 (OpenCV 4 bilateralFilter_32f): value range
// [minv, maxv] of the image, a 4096-bin colour LUT exp(-0.5 (i/scale)^2 / sigma_c^2) linearly
// interpolated, spatial weights exp(-0.5 r^2 / sigma_s^2) on the radius-4 disk without the centre,
// which enters with weight 1; reflect-101 borders.  A constant image is copied.
__global__ void __launch_bounds__(256) bilateral_kernel(const float* __restrict__ depth, int64_t dstride, int H, int W,
                                                         const unsigned* __restrict__ mm, float* __restrict__ out) {
  __shared__ float lut[kBilNumBins + 2];
  __shared__ float sw[(2 * kBilRadius + 1) * (2 * kBilRadius + 1)];
  __shared__ int sdy[(2 * kBilRadius + 1) * (2 * kBilRadius + 1)], sdx[(2 * kBilRadius + 1) * (2 * kBilRadius + 1)];
  __shared__ int nk;
  const float dmax_raw = ord2f(mm[0]), dmin_raw = ord2f(mm[1]);
  const float maxv = dmax_raw > 1.0f ? dmax_raw / dmax_raw : dmax_raw;
  const float minv = dmax_raw > 1.0f ? dmin_raw / dmax_raw : dmin_raw;
  const double gcc = -0.5 / (75.0 * 75.0), gsc = -0.5 / (75.0 * 75.0);
  const float len = (float)((double)maxv - (double)minv);    // minMaxLoc's doubles, then float
  const float scale_index = (float)kBilNumBins / len;
  for (int i = threadIdx.x; i < kBilNumBins + 2; i += blockDim.x) {
    const double v = i / scale_index;
    lut[i] = (float)exp(v * v * gcc);   // stays > 0 over the table at sigma 75 (no zero tail)
  }
  if (threadIdx.x == 0) {
    int k = 0;
    for (int i = -kBilRadius; i <= kBilRadius; ++i)
      for (int j = -kBilRadius; j <= kBilRadius; ++j) {
        const double r = sqrt((double)i * i + (double)j * j);
        if (r > kBilRadius || (i == 0 && j == 0)) continue;
        sw[k] = (float)exp(r * r * gsc);
        sdy[k] = i;
        sdx[k] = j;
        ++k;
      }
    nk = k;
  }
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (int64_t)H * W) return;
  const int y = (int)(p / W), x = (int)(p % W);
  const float val0 = toon_dn(depth, p, dstride, dmax_raw);
  if (fabsf(maxv - minv) < FLT_EPSILON) {
    out[p] = val0;
    return;
  }
  float sum = 0.0f, wsum = 0.0f;
  for (int k = 0; k < nk; ++k) {
    const int yy = reflect101(y + sdy[k], H), xx = reflect101(x + sdx[k], W);
    const float val = toon_dn(depth, (int64_t)yy * W + xx, dstride, dmax_raw);
    float alpha = fabsf(val - val0) * scale_index;
    const int idx = (int)floorf(alpha);
    alpha -= (float)idx;
    const float w = sw[k] * (lut[idx] + alpha * (lut[idx + 1] - lut[idx]));
    wsum += w;
    sum += val * w;
  }
  out[p] = (sum + val0) / (wsum + 1.0f);
}

// cv2.Sobel(f, CV_32F, 1, 0, 3) and (0, 1): separable [-1 0 1] x [1 2 1] with reflect-101
// borders (row pass first: r = s[x+1] - s[x-1], column pass: 2 r[y] + (r[y-1] + r[y+1])),
// magnitude sqrt(gx^2 + gy^2) (post_processor.py:84-86); max into mm[0].
__device__ __forceinline__ float at101(const float* f, int y, int x, int H, int W) {
  return f[(int64_t)reflect101(y, H) * W + reflect101(x, W)];
}
__global__ void __launch_bounds__(256) sobel_kernel(const float* __restrict__ f, int H, int W, float* __restrict__ mag) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (int64_t)H * W) return;
  const int y = (int)(p / W), x = (int)(p % W);
  // gx: row pass [-1 0 1] on rows y-1, y, y+1, column pass [1 2 1]
  float rx[3];
#pragma unroll
  for (int k = -1; k <= 1; ++k) rx[k + 1] = at101(f, y + k, x + 1, H, W) - at101(f, y + k, x - 1, H, W);
  const float gx = rx[1] * 2.0f + (rx[0] + rx[2]);
  // gy: row pass [1 2 1] on rows y-1, y+1, column pass [-1 0 1]
  float hy[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int yy = y - 1 + 2 * k;
    hy[k] = at101(f, yy, x, H, W) * 2.0f + (at101(f, yy, x - 1, H, W) + at101(f, yy, x + 1, H, W));
  }
  const float gy = hy[1] - hy[0];
  mag[p] = sqrtf(gx * gx + gy * gy);
}

// No-depth fallback (post_processor.py:105-111): cv2.cvtColor(RGB2GRAY) in 14-bit fixed point,
// |cv2.Laplacian(gray, CV_32F)| (ksize 1: [0 1 0; 1 -4 1; 0 1 0], reflect-101).
__device__ __forceinline__ float gray_at(const uint8_t* img, int y, int x, int H, int W) {
  const int64_t q = (int64_t)reflect101(y, H) * W + reflect101(x, W);
  const int v = (img[3 * q] * 4899 + img[3 * q + 1] * 9617 + img[3 * q + 2] * 1868 + (1 << 13)) >> 14;
  return (float)v;
}
__global__ void __launch_bounds__(256) laplacian_kernel(const uint8_t* __restrict__ img, int H, int W,
                                                         float* __restrict__ mag) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (int64_t)H * W) return;
  const int y = (int)(p / W), x = (int)(p % W);
  const float c = gray_at(img, y, x, H, W);
  const float l = gray_at(img, y - 1, x, H, W) + gray_at(img, y, x - 1, H, W) + gray_at(img, y, x + 1, H, W) +
                  gray_at(img, y + 1, x, H, W) - 4.0f * c;
  mag[p] = fabsf(l);
}

// Quantised colours with the edge mask (post_processor.py:71-72, :88-100 / :108-115):
//   q = floor(img / 255 * levels) / levels * 255;  e = mag / max(mag) > thr (max > 0), dilated 3x3
//   for depth edges (cv2.dilate, border ignored);  out = clip(q * (1 - strength * e)) as uint8.
__global__ void __launch_bounds__(256) toon_combine_kernel(const uint8_t* __restrict__ img, const float* __restrict__ mag,
                                                            const unsigned* __restrict__ mm, int H, int W, float levels,
                                                            float strength, float thr, int dilate,
                                                            uint8_t* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= (int64_t)H * W) return;
  const int y = (int)(p / W), x = (int)(p % W);
  const float gmax = ord2f(mm[0]);
  auto edge_at = [&](int yy, int xx) {
    float g = mag[(int64_t)yy * W + xx];
    if (gmax > 0.0f) g = g / gmax;
    return g > thr;
  };
  bool e = false;
  if (dilate) {
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int yy = y + dy, xx = x + dx;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) e = e || edge_at(yy, xx);
      }
  } else {
    e = edge_at(y, x);
  }
  const float ef = e ? 1.0f : 0.0f;
  const float k = 1.0f - strength * ef;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = (float)img[3 * p + c];
    const float q = floorf(v / 255.0f * levels) / levels * 255.0f;
    out[3 * p + c] = to_u8(q * k);
  }
}

}  // namespace nerf

using namespace nerf;

#define EREQUIRE(cond, ...)                                          \
  do {                                                               \
    if (!(cond)) return set_error(NERF_ERR_BAD_ARG, __VA_ARGS__);    \
  } while (0)

extern "C" {

size_t nerf_effect_workspace_bytes(int H, int W) {
  if (H <= 0 || W <= 0) return 0;
  return 256 + 2 * (((size_t)H * W * sizeof(float) + 255) & ~(size_t)255);
}

int nerf_depth_normalize(const float* depth, int64_t n, float* out, void* workspace, size_t ws_bytes,
                         nerf_stream_t stream) {
  EREQUIRE(n >= 0, "nerf_depth_normalize: n=%lld", (long long)n);
  if (n == 0) return NERF_OK;
  EREQUIRE(depth && out && workspace && ws_bytes >= 256, "nerf_depth_normalize: null pointer or workspace < 256 B");
  hipStream_t s = (hipStream_t)stream;
  unsigned* mm = (unsigned*)workspace;
  if (int rc = launch_minmax(depth, n, 1, mm, s)) return rc;
  hipLaunchKernelGGL(depth_norm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, depth, n, mm, out);
  return check_launch("depth_norm_kernel");
}

int nerf_effect_fog(const uint8_t* image, const float* depth, int64_t depth_stride, int H, int W, double fog_start,
                    uint8_t* out, void* workspace, size_t ws_bytes, nerf_stream_t stream) {
  EREQUIRE(H > 0 && W > 0 && depth_stride >= 1, "nerf_effect_fog: H=%d W=%d stride=%lld", H, W,
           (long long)depth_stride);
  EREQUIRE(image && out && workspace && ws_bytes >= nerf_effect_workspace_bytes(H, W),
           "nerf_effect_fog: null pointer or workspace too small");
  EREQUIRE(fog_start < 1.0, "nerf_effect_fog: fog_start=%g must be < 1", fog_start);
  hipStream_t s = (hipStream_t)stream;
  const int64_t P = (int64_t)H * W;
  unsigned* mm = (unsigned*)workspace;
  if (depth)
    if (int rc = launch_minmax(depth, P, depth_stride, mm, s)) return rc;
  hipLaunchKernelGGL(fog_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, image, depth, depth_stride, P, mm,
                     (float)fog_start, (float)(1.0 - fog_start), out);
  return check_launch("fog_kernel");
}

int nerf_frame_fog(const float* rgb, const float* depth, int H, int W, double fog_start, uint8_t* out,
                   void* workspace, size_t ws_bytes, nerf_stream_t stream) {
  EREQUIRE(H > 0 && W > 0, "nerf_frame_fog: H=%d W=%d", H, W);
  EREQUIRE(rgb && depth && out && workspace && ws_bytes >= 256, "nerf_frame_fog: null pointer or workspace < 256 B");
  EREQUIRE(fog_start < 1.0, "nerf_frame_fog: fog_start=%g must be < 1", fog_start);
  hipStream_t s = (hipStream_t)stream;
  const int64_t P = (int64_t)H * W;
  unsigned* mm = (unsigned*)workspace;
  if (int rc = launch_minmax(depth, P, 1, mm, s)) return rc;
  hipLaunchKernelGGL(frame_fog_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, rgb, depth, P, mm,
                     (float)fog_start, (float)(1.0 - fog_start), out);
  return check_launch("frame_fog_kernel");
}

int nerf_effect_toon(const uint8_t* image, const float* depth, int64_t depth_stride, int H, int W, double levels,
                     double edge_strength, uint8_t* out, void* workspace, size_t ws_bytes, nerf_stream_t stream) {
  EREQUIRE(H > 0 && W > 0 && depth_stride >= 1 && levels > 0.0, "nerf_effect_toon: H=%d W=%d stride=%lld levels=%g",
           H, W, (long long)depth_stride, levels);
  EREQUIRE(image && out && workspace && ws_bytes >= nerf_effect_workspace_bytes(H, W),
           "nerf_effect_toon: null pointer or workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int64_t P = (int64_t)H * W;
  const unsigned blocks = (unsigned)((P + 255) / 256);
  unsigned* mm = (unsigned*)workspace;
  const size_t plane = ((size_t)P * sizeof(float) + 255) & ~(size_t)255;
  float* filt = (float*)((char*)workspace + 256);
  float* mag = (float*)((char*)workspace + 256 + plane);
  int rc;
  if (depth) {
    if ((rc = launch_minmax(depth, P, depth_stride, mm, s))) return rc;
    hipLaunchKernelGGL(bilateral_kernel, dim3(blocks), dim3(256), 0, s, depth, depth_stride, H, W, mm, filt);
    if ((rc = check_launch("bilateral_kernel"))) return rc;
    hipLaunchKernelGGL(sobel_kernel, dim3(blocks), dim3(256), 0, s, filt, H, W, mag);
    if ((rc = check_launch("sobel_kernel"))) return rc;
  } else {
    hipLaunchKernelGGL(laplacian_kernel, dim3(blocks), dim3(256), 0, s, image, H, W, mag);
    if ((rc = check_launch("laplacian_kernel"))) return rc;
  }
  if ((rc = launch_minmax(mag, P, 1, mm, s))) return rc;
  hipLaunchKernelGGL(toon_combine_kernel, dim3(blocks), dim3(256), 0, s, image, mag, mm, H, W, (float)levels,
                     (float)edge_strength, depth ? 0.05f : 0.1f, depth ? 1 : 0, out);
  return check_launch("toon_combine_kernel");
}

}  // extern "C"
