// C ABI of libnerfmi.so (include/nerfmi.h): argument checks, the weight packer and the
// whole-path orchestration.  Kernels live in rays.hip, mlp.hip, composite.hip and
// importance.hip; this file only validates, carves the workspace and launches them in
// stream order.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "common.h"

namespace nerf {

static thread_local char g_err[512] = "";
int g_mlp_arith = NERF_ARITH_F16X3;

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// ---------------------------------------------------------------------------- packing
// Weight of fragment matrix m (layout.h) at output row `row`, source column `col` (-1 = padding).
NERF_HD inline float frag_weight(const float* const* P, int m, int row, int col) {
  if (col < 0) return 0.0f;
  if (m == 8) return P[P_DIR_W][(size_t)row * (kHidden + kDirEnc) + col];
  const int layer = (m == kSkipPeMat) ? kSkipLayer : m;
  const int K = (layer == 0) ? kPosEnc : (layer == kSkipLayer ? kHidden + kPosEnc : kHidden);
  return P[2 * layer][(size_t)row * K + col];
}

// Value of packed element e < kF32Floats (the exact-f32 path) from the 24 state_dict tensors.
NERF_HD inline float pack_value(const float* const* P, size_t e) {
  if (e < kFragFloats) {
    int m = 0;
    while (m + 1 < kNumFragMats && e >= frag_offset(m + 1)) ++m;
    const size_t rel = e - frag_offset(m);
    const int j = (int)(rel & 3);
    const int lane = (int)((rel >> 2) & 63);
    const size_t blk = rel >> 8;
    const int ksq = frag_ksteps(m) / 4;
    const int nt = (int)(blk / ksq), kq = (int)(blk % ksq);
    return frag_weight(P, m, nt * 32 + (lane & 31), frag_source_col(m, 4 * kq + j, lane));
  }
  if (e < kOffSigmaW) {
    const size_t k = e - kOffBias;
    return P[2 * (k / kHidden) + 1][k % kHidden];
  }
  if (e < kOffSigmaB) return P[P_SIGMA_W][e - kOffSigmaW];
  if (e < kOffDirB) return e == kOffSigmaB ? P[P_SIGMA_B][0] : 0.0f;
  if (e < kOffDirWd) return P[P_DIR_B][e - kOffDirB];
  if (e < kOffAppW) {
    const size_t k = e - kOffDirWd;
    return P[P_DIR_W][(k / kDirEnc) * (kHidden + kDirEnc) + kHidden + k % kDirEnc];
  }
  if (e < kOffAppB) return P[P_APP_W][e - kOffAppW];
  if (e < kOffRgbW) return P[P_APP_B][e - kOffAppB];
  if (e < kOffRgbB) return P[P_RGB_W][e - kOffRgbW];
  return (e - kOffRgbB < 3) ? P[P_RGB_B][e - kOffRgbB] : 0.0f;
}

// ---- split-f16 stream (layout.h) -----------------------------------------------------------
// Layer L's weight matrix in natural (row, column) order: rows 256 (128 for the colour layer),
// columns 63 (layer 0), 319 (layer 4: [h, enc_x]), 256 otherwise (colour layer: its h part).
NERF_HD inline int layer_rows(int L) { return L == 8 ? kDirHidden : kHidden; }
NERF_HD inline int layer_cols(int L) { return L == 0 ? kPosEnc : (L == kSkipLayer ? kHidden + kPosEnc : kHidden); }
NERF_HD inline float layer_weight(const float* const* P, int L, int row, int col) {
  if (L == 8) return P[P_DIR_W][(size_t)row * (kHidden + kDirEnc) + col];
  return P[2 * L][(size_t)row * layer_cols(L) + col];
}

// Row statistics of layer L: max |W|, max_row sum |W| (R), max |b| (B).
NERF_HD inline void layer_row_stats(const float* const* P, int L, int row, float& mx, float& l1, float& bmax) {
  mx = 0.0f;
  l1 = 0.0f;
  for (int c = 0; c < layer_cols(L); ++c) {
    const float w = fabsf(layer_weight(P, L, row, c));
    mx = fmaxf(mx, w);
    l1 += w;
  }
  bmax = L < 8 ? fabsf(P[2 * L + 1][row]) : 0.0f;
}

NERF_HD inline void store_layer_consts(float* consts, int L, float mx, float l1, float bmax) {
  const int e = s16_exponent(mx);
  consts[kS16Sw + L] = ldexpf(1.0f, 14 - e);
  consts[kS16InvW + L] = ldexpf(1.0f, e - 14);
  if (L < 8) {
    consts[kS16R + L] = l1 * 1.0001f;     // rounding margin on the float sum: the bound must hold
    consts[kS16B + L] = bmax;
  }
}

// f16x3 word w (two halves) of the stream, given the layer constants.
NERF_HD inline uint32_t pack16_word(const float* const* P, const float* consts, size_t w) {
  const int c = (int)(w / kChunkFloats), r = (int)(w % kChunkFloats);
  int L = 0;
  while (c >= s16_chunk0(L + 1)) ++L;
  const int per_group = s16_layer_ks(L) / 2;
  const int local = c - s16_chunk0(L), g = local / per_group, i = local % per_group;
  const int piece = r / 256, lane = (r % 256) / 4, jj = r % 4;
  const int kk = piece / 8, ti = (piece / 2) % 4, part = piece % 2;
  const int ks = 2 * i + kk, t = 4 * g + ti;
  const int m = s16_matrix(L, ks), ksm = s16_matrix_ks(L, ks);
  uint32_t word = 0;
  for (int k = 0; k < 2; ++k) {
    const int j = 2 * jj + k;
    const float v =
        frag_weight(P, m, t * 32 + (lane & 31), s16_source_col(m, ksm, lane >> 5, j)) * consts[kS16Sw + L];
    const _Float16 hi = (_Float16)v;
    const _Float16 out = part == 0 ? hi : (_Float16)(v - (float)hi);
    uint16_t bits;
    memcpy(&bits, &out, 2);
    word |= (uint32_t)bits << (16 * k);
  }
  return word;
}

struct ParamPtrs { const float* p[P_COUNT]; };

// (the last block also zeroes the split stream's constant slots, which scale16_kernel's atomics fill)
__global__ void __launch_bounds__(256) pack_kernel(ParamPtrs P, float* __restrict__ packed) {
  if (blockIdx.x == gridDim.x - 1) {
    if (threadIdx.x < kS16Consts) packed[kOffScale16 + threadIdx.x] = 0.0f;
    return;
  }
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < kOff16) packed[e] = e < kF32Floats ? pack_value(P.p, e) : 0.0f;
}
static_assert(kS16Consts <= 256, "one block zeroes the constant slots");

// One block per layer: its scale, bound constants (layout.h).
// Layer statistics for the split scales: each wave reduces 8 rows (lanes over the row's columns,
// so the loads are coalesced) to the rows' max |W|, max L1 norm and max |bias|; the block's 4 waves
// combine in LDS and one thread per block merges them into the layer's slots by atomicMax on the
// float bits (non-negative floats order as unsigned integers: exact in any order).  8 blocks per
// layer: 8 atomics per slot (one atomic per wave and row serialised at L2: 47 us -> a few).  The raw
// maxima land in the constants' own slots (zeroed by pack_kernel) and the last block to finish turns
// them into the constants.
constexpr int kS16RowsPerWave = 8;
constexpr int kS16Counter = kS16Consts - 1;   // (an unused constant slot: scale16_kernel's block counter)
static_assert(kS16Counter >= kS16B + 8, "the counter slot is unused by the constants");
__global__ void __launch_bounds__(256) scale16_kernel(ParamPtrs P, float* __restrict__ packed) {
  __shared__ float red[3][4];
  __shared__ unsigned last;          // the block finished last (an integer flag: no float compare)
  const int L = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // the wave's 8 rows loaded first (one memory round trip, not one per row), then per row the lane's
  // column-order sum and the xor tree as before (zeros past a row's end add nothing)
  const int rows = layer_rows(L), cols = layer_cols(L);
  constexpr int kColSteps = (kHidden + kPosEnc + 63) / 64;
  float w[kS16RowsPerWave][kColSteps];
#pragma unroll
  for (int j = 0; j < kS16RowsPerWave; ++j)
#pragma unroll
    for (int q = 0; q < kColSteps; ++q) {
      const int row = (blockIdx.x * 4 + wave) * kS16RowsPerWave + j, c = lane + 64 * q;
      w[j][q] = row < rows && c < cols ? fabsf(layer_weight(P.p, L, row, c)) : 0.0f;
    }
  float mx = 0.0f, l1m = 0.0f, bm = 0.0f;
#pragma unroll
  for (int j = 0; j < kS16RowsPerWave; ++j) {
    const int row = (blockIdx.x * 4 + wave) * kS16RowsPerWave + j;
    float l1 = 0.0f;
#pragma unroll
    for (int q = 0; q < kColSteps; ++q) {
      mx = fmaxf(mx, w[j][q]);
      l1 += w[j][q];
    }
    for (int off = 32; off > 0; off >>= 1) l1 += __shfl_xor(l1, off);
    l1m = fmaxf(l1m, l1);
    if (L < 8 && row < rows) bm = fmaxf(bm, fabsf(P.p[2 * L + 1][row]));
  }
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  if (lane == 0) {
    red[0][wave] = mx;
    red[1][wave] = l1m;
    red[2][wave] = bm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      mx = fmaxf(mx, red[0][w]);
      l1m = fmaxf(l1m, red[1][w]);
      bm = fmaxf(bm, red[2][w]);
    }
    unsigned* cw = reinterpret_cast<unsigned*>(packed + kOffScale16);
    atomicMax(cw + kS16Sw + L, __float_as_uint(mx));
    if (L < 8) {
      atomicMax(cw + kS16R + L, __float_as_uint(l1m));
      atomicMax(cw + kS16B + L, __float_as_uint(bm));
    }
    // the last block to finish turns the maxima into the constants (scale16_finalize_kernel's work,
    // without its launch); the block counter sits in the last constant slot (zeroed by pack_kernel,
    // reset to 0 here, so the packed buffer ends as the host pack writes it)
    __threadfence();
    last = atomicAdd(cw + kS16Counter, 1u) == gridDim.x * gridDim.y - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (last == 0u) return;   // (uniform: the flag is the block's own)
  __threadfence();
  unsigned* cw = reinterpret_cast<unsigned*>(packed + kOffScale16);
  const int Lf = threadIdx.x;
  if (Lf < kS16Layers) {
    const float mxf = __uint_as_float(__hip_atomic_load(cw + kS16Sw + Lf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const float l1f = Lf < 8 ? __uint_as_float(__hip_atomic_load(cw + kS16R + Lf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                             : 0.0f;
    const float bmf = Lf < 8 ? __uint_as_float(__hip_atomic_load(cw + kS16B + Lf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                             : 0.0f;
    store_layer_consts(packed + kOffScale16, Lf, mxf, l1f, bmf);
  }
  if (threadIdx.x == 0) __hip_atomic_store(cw + kS16Counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(256) pack16_kernel(ParamPtrs P, float* __restrict__ packed) {
  const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < kFragFloats)
    reinterpret_cast<uint32_t*>(packed)[kOff16 + w] = pack16_word(P.p, packed + kOffScale16, w);
}

int launch_pack(const float* const* params, float* packed, hipStream_t s) {
  ParamPtrs P;
  for (int i = 0; i < P_COUNT; ++i) P.p[i] = params[i];
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((kOff16 + 255) / 256 + 1)), dim3(256), 0, s, P, packed);
  if (int rc = check_launch("pack_kernel")) return rc;
  hipLaunchKernelGGL(scale16_kernel, dim3(kHidden / (4 * kS16RowsPerWave), kS16Layers), dim3(256), 0, s, P, packed);
  if (int rc = check_launch("scale16_kernel")) return rc;
  hipLaunchKernelGGL(pack16_kernel, dim3((unsigned)((kFragFloats + 255) / 256)), dim3(256), 0, s, P, packed);
  return check_launch("pack16_kernel");
}

static void pack_host(const float* const* P, float* packed) {
  for (size_t e = 0; e < kOff16; ++e) packed[e] = e < kF32Floats ? pack_value(P, e) : 0.0f;
  float* consts = packed + kOffScale16;
  for (int i = 0; i < kS16Consts; ++i) consts[i] = 0.0f;
  for (int L = 0; L < kS16Layers; ++L) {
    float mx = 0.0f, l1 = 0.0f, bm = 0.0f;
    for (int row = 0; row < layer_rows(L); ++row) {
      float a, b, c;
      layer_row_stats(P, L, row, a, b, c);
      mx = fmaxf(mx, a);
      l1 = fmaxf(l1, b);
      bm = fmaxf(bm, c);
    }
    store_layer_consts(consts, L, mx, l1, bm);
  }
  uint32_t* words = reinterpret_cast<uint32_t*>(packed);
  for (size_t w = 0; w < kFragFloats; ++w) words[kOff16 + w] = pack16_word(P, consts, w);
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace nerf

using namespace nerf;

#define REQUIRE(cond, ...)                                   \
  do {                                                       \
    if (!(cond)) return set_error(NERF_ERR_BAD_ARG, __VA_ARGS__); \
  } while (0)

extern "C" {

const char* nerf_last_error(void) { return g_err; }
int nerf_abi_version(void) { return 11; }

int nerf_get_rays(int H, int W, float focal, const float* c2w_host, int row0, int nrows, float* rays_o,
                  float* rays_d, nerf_stream_t stream) {
  REQUIRE(H > 0 && W > 0, "nerf_get_rays: H=%d W=%d must be positive", H, W);
  REQUIRE(row0 >= 0 && nrows >= 0 && row0 + nrows <= H, "nerf_get_rays: rows [%d,%d) outside [0,%d)", row0,
          row0 + nrows, H);
  REQUIRE(c2w_host && rays_d, "nerf_get_rays: null pointer");
  return launch_get_rays(H, W, focal, c2w_host, row0, nrows, rays_o, rays_d, (hipStream_t)stream);
}

int nerf_normalize_dirs(const float* rays_d, int64_t B, float* out, nerf_stream_t stream) {
  REQUIRE(B >= 0, "nerf_normalize_dirs: B=%lld", (long long)B);
  REQUIRE(B == 0 || (rays_d && out), "nerf_normalize_dirs: null pointer");
  return launch_normalize(rays_d, B, out, (hipStream_t)stream);
}

int nerf_positional_encoding(const float* x, int64_t M, int dims, int levels, int include_input, float* out,
                             nerf_stream_t stream) {
  REQUIRE(M >= 0 && dims >= 1 && levels >= 0 && levels <= 30, "nerf_positional_encoding: M=%lld dims=%d levels=%d",
          (long long)M, dims, levels);
  REQUIRE(M == 0 || (x && out), "nerf_positional_encoding: null pointer");
  return launch_pe(x, M, dims, levels, include_input, out, (hipStream_t)stream);
}

int nerf_rng_uniforms(uint64_t seed, int64_t first, int64_t n, float* out, nerf_stream_t stream) {
  REQUIRE(first >= 0 && n >= 0, "nerf_rng_uniforms: first=%lld n=%lld", (long long)first, (long long)n);
  REQUIRE(n == 0 || out, "nerf_rng_uniforms: null pointer");
  return launch_rng_uniforms(seed, first, n, out, (hipStream_t)stream);
}

int nerf_sample_stratified(const float* rays_o, const float* rays_d, int64_t B, double near, double far, int N,
                           const float* t_vals, int perturb, const float* t_rand, uint64_t seed, float* z_vals,
                           float* pts, nerf_stream_t stream) {
  REQUIRE(B >= 0 && N >= 1, "nerf_sample_stratified: B=%lld N=%d", (long long)B, N);
  REQUIRE(B == 0 || (t_vals && z_vals), "nerf_sample_stratified: null pointer");
  REQUIRE(!pts || (rays_o && rays_d), "nerf_sample_stratified: pts requested without rays");
  return launch_stratified(rays_o, rays_d, B, (float)near, (float)(far - near), N, t_vals, perturb, t_rand, seed,
                           z_vals, pts, (hipStream_t)stream);
}

int nerf_sample_importance(const float* rays_o, const float* rays_d, const float* z_vals, const float* weights,
                           int64_t B, int N, int Nf, const float* u_lin, const float* u_rand, uint64_t seed,
                           float* z_all, float* pts_all, nerf_stream_t stream) {
  REQUIRE(B >= 0, "nerf_sample_importance: B=%lld", (long long)B);
  if (N < 1 || N > 256 || Nf < 1 || Nf > 1024)
    return set_error(NERF_ERR_UNSUPPORTED, "nerf_sample_importance: N=%d (1..256) Nf=%d (1..1024)", N, Nf);
  REQUIRE(B == 0 || (z_vals && weights && u_lin && z_all), "nerf_sample_importance: null pointer");
  REQUIRE(!pts_all || (rays_o && rays_d), "nerf_sample_importance: pts requested without rays");
  return launch_importance(rays_o, rays_d, z_vals, weights, B, N, Nf, u_lin, u_rand, seed, z_all, pts_all,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, (hipStream_t)stream);
}

int nerf_sample_importance_merge(const float* z_vals, const float* weights, const float* rgb_c,
                                 const float* sigma_c, int64_t B, int N, int Nf, const float* u_lin,
                                 const float* u_rand, uint64_t seed, float* z_all, float* rgb_all,
                                 float* sigma_all, float* z_fine, int32_t* fine_slot, nerf_stream_t stream) {
  REQUIRE(B >= 0, "nerf_sample_importance_merge: B=%lld", (long long)B);
  if (N < 1 || N > 256 || Nf < 1 || Nf > 1024)
    return set_error(NERF_ERR_UNSUPPORTED, "nerf_sample_importance_merge: N=%d (1..256) Nf=%d (1..1024)", N, Nf);
  REQUIRE(B == 0 || (z_vals && weights && rgb_c && sigma_c && u_lin && z_all && rgb_all && sigma_all && z_fine &&
                     fine_slot),
          "nerf_sample_importance_merge: null pointer");
  return launch_importance(nullptr, nullptr, z_vals, weights, B, N, Nf, u_lin, u_rand, seed, z_all, nullptr, rgb_c,
                           sigma_c, rgb_all, sigma_all, z_fine, fine_slot, (hipStream_t)stream);
}

size_t nerf_packed_weights_floats(void) { return kPackedFloats; }

int nerf_set_mlp_arith(int arith) {
  if (arith != NERF_ARITH_F32 && arith != NERF_ARITH_F16X3) {
    set_error(NERF_ERR_BAD_ARG, "nerf_set_mlp_arith: unknown arithmetic %d", arith);
    return -1;
  }
  const int prev = g_mlp_arith;
  g_mlp_arith = arith;
  return prev;
}

int nerf_get_mlp_arith(void) { return g_mlp_arith; }

int nerf_pack_weights(const float* const* params, float* packed, nerf_stream_t stream) {
  REQUIRE(params && packed, "nerf_pack_weights: null pointer");
  for (int i = 0; i < P_COUNT; ++i) REQUIRE(params[i], "nerf_pack_weights: parameter %d is null", i);
  return launch_pack(params, packed, (hipStream_t)stream);
}

int nerf_pack_weights_host(const float* const* params, float* packed) {
  REQUIRE(params && packed, "nerf_pack_weights_host: null pointer");
  for (int i = 0; i < P_COUNT; ++i) REQUIRE(params[i], "nerf_pack_weights_host: parameter %d is null", i);
  pack_host(params, packed);
  return NERF_OK;
}

int nerf_ray_features(const float* packed, const float* dirs, int64_t R, const float* app, int64_t app_rows,
                      float* feat, nerf_stream_t stream) {
  REQUIRE(R >= 0, "nerf_ray_features: R=%lld", (long long)R);
  REQUIRE(app_rows == 0 || app_rows == 1 || app_rows == R, "nerf_ray_features: app_rows=%lld with R=%lld",
          (long long)app_rows, (long long)R);
  REQUIRE(R == 0 || (packed && dirs && feat && (app_rows == 0 || app)), "nerf_ray_features: null pointer");
  return launch_ray_features(packed, dirs, R, app, app_rows, feat, (hipStream_t)stream);
}

// ------------------------------------------------------------------ MLP launch profiling
// bench.py's roofline leg: while on, every fused-MLP launch (nerf_render_rays' two, or
// nerf_mlp_forward's one) is bracketed by HIP events recorded on the launch's own stream, so the
// shipped single-call path is timed per launch with no change to what it runs.  One process-wide
// recorder (a diagnostic for one host thread).
namespace {
struct MlpProfile {
  std::vector<hipEvent_t> ev;
  std::vector<int64_t> samples;
  int n = 0;
  bool on = false;
};
MlpProfile g_prof;
}  // namespace

static int profiled_mlp(const float* packed, const float* origins, const float* dirs, const float* z, int64_t R,
                        int N, const float* feat, float* rgb, float* sigma, const int* slot, int T, hipStream_t s) {
  const bool rec = g_prof.on && g_prof.n < (int)g_prof.samples.size();
  if (rec && hipEventRecord(g_prof.ev[2 * g_prof.n], s) != hipSuccess)
    return set_error(NERF_ERR_HIP, "nerf profile: hipEventRecord failed");
  if (int rc = launch_mlp(packed, origins, dirs, z, R, N, feat, rgb, sigma, slot, T, s)) return rc;
  if (rec) {
    if (hipEventRecord(g_prof.ev[2 * g_prof.n + 1], s) != hipSuccess)
      return set_error(NERF_ERR_HIP, "nerf profile: hipEventRecord failed");
    g_prof.samples[g_prof.n++] = R * (int64_t)N;
  }
  return NERF_OK;
}

int nerf_profile_mlp_begin(int capacity) {
  REQUIRE(capacity >= 1 && capacity <= 1 << 20, "nerf_profile_mlp_begin: capacity=%d", capacity);
  for (hipEvent_t e : g_prof.ev) (void)hipEventDestroy(e);
  g_prof.ev.assign(2 * (size_t)capacity, nullptr);
  for (auto& e : g_prof.ev)
    if (hipEventCreate(&e) != hipSuccess) return set_error(NERF_ERR_HIP, "nerf_profile_mlp_begin: hipEventCreate failed");
  g_prof.samples.assign(capacity, 0);
  g_prof.n = 0;
  g_prof.on = true;
  return NERF_OK;
}

int nerf_profile_mlp_end(float* ms, int64_t* samples, int capacity, int* count) {
  REQUIRE(count && (capacity == 0 || (ms && samples)), "nerf_profile_mlp_end: null pointer");
  g_prof.on = false;
  const int n = g_prof.n < capacity ? g_prof.n : capacity;
  for (int i = 0; i < n; ++i) {
    if (hipEventSynchronize(g_prof.ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms[i], g_prof.ev[2 * i], g_prof.ev[2 * i + 1]) != hipSuccess)
      return set_error(NERF_ERR_HIP, "nerf_profile_mlp_end: event %d", i);
    samples[i] = g_prof.samples[i];
  }
  *count = g_prof.n;
  return NERF_OK;
}

// Launch-size limit.  A sample-parallel launch spans 2 threads per sample (the MLP: 256 per 128
// samples) and a grid holds < 2^32 work-items per dimension, so one launch takes at most
// 2^30 samples; larger calls run in ray chunks of nerf_render_chunk_rays rays
// (the reference's volume_render has no such limit, src/render.py:5-97; its callers chunk at
// config.chunk, run.py:209-231).
// NERFMI_MAX_LAUNCH_SAMPLES (read once; test hook, >= 4096) lowers the limit so the GPU tests can
// check a chunked call against the one-launch call at small sizes (tests/test_gpu_parity.py).
static int64_t max_launch_samples() {
  static const int64_t v = [] {
    const char* e = getenv("NERFMI_MAX_LAUNCH_SAMPLES");
    const long long x = e ? atoll(e) : 0;
    return x >= 4096 && x < ((int64_t)1 << 30) ? (int64_t)x : ((int64_t)1 << 30);
  }();
  return v;
}

int64_t nerf_render_chunk_rays(int N, int Nf) {
  const int per = N > Nf ? N : Nf;
  return per >= 1 ? max_launch_samples() / per : 0;
}

int nerf_mlp_forward(const float* packed, const float* origins, const float* dirs, const float* z_vals, int64_t R,
                     int N, const float* ray_feat, float* rgb, float* sigma, const int32_t* out_slot, int out_T,
                     nerf_stream_t stream) {
  REQUIRE(R >= 0 && N >= 1, "nerf_mlp_forward: R=%lld N=%d", (long long)R, N);
  REQUIRE(!out_slot || out_T >= N, "nerf_mlp_forward: out_T=%d < N=%d", out_T, N);
  REQUIRE(z_vals || N == 1, "nerf_mlp_forward: without z_vals the origins are the points and N must be 1");
  REQUIRE(R == 0 || (packed && origins && ray_feat && rgb && sigma && (!z_vals || dirs)),
          "nerf_mlp_forward: null pointer");
  const int64_t rc_rays = nerf_render_chunk_rays(N, 0);
  if (R > 0 && rc_rays < 1)   // one ray's N samples already exceed the per-launch sample limit
    return set_error(NERF_ERR_UNSUPPORTED, "nerf_mlp_forward: N=%d samples per ray exceed the launch limit %lld", N,
                     (long long)max_launch_samples());
  for (int64_t r0 = 0; r0 < R; r0 += rc_rays) {            // (one chunk unless R N > 2^30)
    const int64_t n = R - r0 < rc_rays ? R - r0 : rc_rays;
    const int64_t orow = out_slot ? (int64_t)out_T : (int64_t)N;   // output rows per ray
    if (int rc = profiled_mlp(packed, origins + 3 * r0, dirs ? dirs + 3 * r0 : nullptr, z_vals ? z_vals + r0 * N : nullptr,
                              n, N, ray_feat + r0 * kRayFeat, rgb + 3 * r0 * orow, sigma + r0 * orow,
                              out_slot ? out_slot + r0 * N : nullptr, out_T, (hipStream_t)stream))
      return rc;
  }
  return NERF_OK;
}

int nerf_composite(const float* rgb, const float* sigma, const float* z_vals, int64_t B, int N, float* rgb_map,
                   float* depth_map, float* weights, nerf_stream_t stream) {
  REQUIRE(B >= 0, "nerf_composite: B=%lld", (long long)B);
  if (N < 1 || N > 4096) return set_error(NERF_ERR_UNSUPPORTED, "nerf_composite: N=%d (1..4096)", N);
  REQUIRE(B == 0 || (rgb && sigma && z_vals && rgb_map && depth_map), "nerf_composite: null pointer");
  return launch_composite(rgb, sigma, z_vals, B, N, rgb_map, depth_map, weights, (hipStream_t)stream);
}

// Workspace carve of nerf_render_rays, in this order (each region 256-B aligned), T = N + Nf:
//   dirs (B,3) | z (B,N) | feat (B,256) | rgb_c (B,N,3) | sigma_c (B,N) | w_c (B,N) | z_all (B,T)
//   | z_fine (B,Nf) | merged_src (B,T) uint16 | rgb_f (B,Nf,3) | sigma_f (B,Nf) | maps (B,4)
enum { W_DIRS, W_Z, W_FEAT, W_RGBC, W_SIGC, W_WC, W_ZALL, W_ZF, W_SRC, W_RGBF, W_SIGF, W_MAPS, W_COUNT };

static size_t carve(int64_t B, int N, int Nf, size_t* off) {
  const size_t T = (size_t)N + Nf, b = (size_t)B;
  const size_t sizes[W_COUNT] = {b * 3, b * N, b * kRayFeat, b * N * 3, b * N, b * N, b * T,
                                 b * Nf, (b * T + 1) / 2, b * Nf * 3, b * Nf, b * 4};
  size_t at = 0;
  for (int i = 0; i < W_COUNT; ++i) {
    off[i] = at;
    at += align_up(sizes[i] * 4);
  }
  return at;
}

int64_t nerf_render_chunk_rays(int N, int Nf);

// (one chunk's worth: the chunks of a call past the launch-size limit reuse it in stream order)
size_t nerf_render_workspace_bytes(int64_t B, int N, int Nf) {
  if (B < 0 || N < 1 || Nf < 0) return 0;
  const int64_t chunk = nerf_render_chunk_rays(N, Nf);
  size_t off[W_COUNT];
  return carve(B < chunk ? B : chunk, N, Nf, off);
}

static int render_rays_chunk(const float* packed, const float* rays_o, const float* rays_d, int64_t B, double near,
                             double far, int N, int Nf, const float* t_vals, const float* u_lin, int perturb,
                             const float* t_rand, const float* u_rand, uint64_t seed, int64_t ray0, const float* app,
                             int64_t app_rows, float* rgb_map, float* depth_map, float* weights_out, float* z_out,
                             float* coarse_rgb, float* coarse_depth, void* workspace, size_t ws_bytes,
                             nerf_stream_t stream);

int nerf_render_rays(const float* packed, const float* rays_o, const float* rays_d, int64_t B, double near,
                     double far, int N, int Nf, const float* t_vals, const float* u_lin, int perturb,
                     const float* t_rand, const float* u_rand, uint64_t seed, int64_t ray0, const float* app,
                     int64_t app_rows, float* rgb_map, float* depth_map, float* weights_out, float* z_out,
                     float* coarse_rgb, float* coarse_depth, void* workspace, size_t ws_bytes,
                     nerf_stream_t stream) {
  REQUIRE(B >= 0 && ray0 >= 0, "nerf_render_rays: B=%lld ray0=%lld", (long long)B, (long long)ray0);
  if (N < 1 || N > 4096 || Nf < 0 || N + Nf > 4096 || (Nf > 0 && (N > 256 || Nf > 1024)))
    return set_error(NERF_ERR_UNSUPPORTED, "nerf_render_rays: N=%d Nf=%d outside the supported range", N, Nf);
  // calls past the launch-size limit run in ray chunks: every per-ray input and output advances by
  // the chunk's first ray, the in-kernel draws stay keyed by the global ray index (ray0 + c0), and
  // each chunk carves the caller's workspace for its own (smaller) B
  REQUIRE(app_rows == 0 || app_rows == 1 || app_rows == B, "nerf_render_rays: app_rows=%lld with B=%lld",
          (long long)app_rows, (long long)B);
  const int64_t chunk = nerf_render_chunk_rays(N, Nf);
  if (chunk < 1)   // (N + Nf <= 4096 <= the launch limit: unreachable, but never loop on a zero step)
    return set_error(NERF_ERR_UNSUPPORTED, "nerf_render_rays: N=%d Nf=%d exceed the launch limit", N, Nf);
  const int64_t T = Nf > 0 ? (int64_t)N + Nf : (int64_t)N;   // weights_out / z_out columns
  for (int64_t c0 = 0; c0 < B || (B == 0 && c0 == 0); c0 += chunk) {
    const int64_t n = B - c0 < chunk ? B - c0 : chunk;
    const bool per_ray_app = app_rows > 1;
    if (int rc = render_rays_chunk(packed, rays_o + 3 * c0, rays_d + 3 * c0, n, near, far, N, Nf, t_vals, u_lin, perturb,
                                   t_rand ? t_rand + c0 * N : nullptr, u_rand ? u_rand + c0 * Nf : nullptr, seed,
                                   ray0 + c0, per_ray_app ? app + c0 * kAppDim : app, per_ray_app ? n : app_rows,
                                   rgb_map + 3 * c0, depth_map + c0, weights_out ? weights_out + c0 * T : nullptr,
                                   z_out ? z_out + c0 * T : nullptr, coarse_rgb ? coarse_rgb + 3 * c0 : nullptr,
                                   coarse_depth ? coarse_depth + c0 : nullptr, workspace, ws_bytes, stream))
      return rc;
    if (B == 0) break;
  }
  return NERF_OK;
}

static int render_rays_chunk(const float* packed, const float* rays_o, const float* rays_d, int64_t B, double near,
                             double far, int N, int Nf, const float* t_vals, const float* u_lin, int perturb,
                             const float* t_rand, const float* u_rand, uint64_t seed, int64_t ray0, const float* app,
                             int64_t app_rows, float* rgb_map, float* depth_map, float* weights_out, float* z_out,
                             float* coarse_rgb, float* coarse_depth, void* workspace, size_t ws_bytes,
                             nerf_stream_t stream) {
  if (N < 1 || N > 4096 || Nf < 0 || N + Nf > 4096 || (Nf > 0 && (N > 256 || Nf > 1024)))
    return set_error(NERF_ERR_UNSUPPORTED, "nerf_render_rays: N=%d Nf=%d outside the supported range", N, Nf);
  if (B == 0) return NERF_OK;
  REQUIRE(packed && rays_o && rays_d && t_vals && rgb_map && depth_map && workspace, "nerf_render_rays: null pointer");
  REQUIRE(Nf == 0 || u_lin, "nerf_render_rays: u_lin required when Nf > 0");
  REQUIRE(app_rows == 0 || app_rows == 1 || app_rows == B, "nerf_render_rays: app_rows=%lld with B=%lld",
          (long long)app_rows, (long long)B);
  REQUIRE(app_rows == 0 || app, "nerf_render_rays: null appearance");
  size_t off[W_COUNT];
  const size_t need = carve(B, N, Nf, off);
  if (ws_bytes < need)
    return set_error(NERF_ERR_WORKSPACE, "nerf_render_rays: workspace %zu < %zu bytes", ws_bytes, need);
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  auto region = [&](int i) { return (float*)(ws + off[i]); };
  float* dn = region(W_DIRS);
  float* z = (Nf == 0 && z_out) ? z_out : region(W_Z);
  float* feat = region(W_FEAT);
  float* rgb_c = region(W_RGBC);
  float* sigma_c = region(W_SIGC);
  float* wc = (Nf == 0) ? weights_out : region(W_WC);
  float* z_all = z_out ? z_out : region(W_ZALL);
  float* maps = region(W_MAPS);
  // in-kernel draws keyed by the global ray index ray0 + r (nerf_rng_uniforms)
  const uint64_t seed_c = rng_key_at(seed, (uint64_t)ray0 * (uint64_t)N);
  const uint64_t seed_f = rng_key_at(seed ^ 0x5DEECE66Dull, (uint64_t)ray0 * (uint64_t)Nf);
  int rc;
  // render.py:19's normalisation in the ray-feature kernel (it writes dn)
  if ((rc = launch_ray_features(packed, rays_d, B, app, app_rows, feat, s, nullptr, dn))) return rc;
  if ((rc = launch_stratified(rays_o, dn, B, (float)near, (float)(far - near), N, t_vals, perturb, t_rand, seed_c,
                              z, nullptr, s)))
    return rc;                                                                                 // render.py:22
  if ((rc = profiled_mlp(packed, rays_o, dn, z, B, N, feat, rgb_c, sigma_c, nullptr, 0, s))) return rc;  // :49
  if (Nf == 0)
    return launch_composite(rgb_c, sigma_c, z, B, N, rgb_map, depth_map, wc, s);               // render.py:56-80
  float* crgb = coarse_rgb ? coarse_rgb : maps;
  float* cdepth = coarse_depth ? coarse_depth : maps + 3 * B;
  if ((rc = launch_composite(rgb_c, sigma_c, z, B, N, crgb, cdepth, wc, s))) return rc;
  // H1 fine pass: resample + merge (each merged slot records which coarse or fine sample it holds),
  // the MLP run on the Nf new samples only, in sample order, and the composite over all N+Nf merged
  // samples gathering the coarse evaluations and the fine ones through the map.  (Round 3 scattered
  // the coarse results into merged rows and the fine MLP wrote into its slots: 4.0 GB written by
  // the resample and 24 B per fine sample by the MLP, for the same bits.)
  float* z_fine = region(W_ZF);
  uint16_t* msrc = (uint16_t*)region(W_SRC);
  float* rgb_f = region(W_RGBF);
  float* sigma_f = region(W_SIGF);
  if ((rc = launch_importance(nullptr, nullptr, z, wc, B, N, Nf, u_lin, u_rand, seed_f, z_all, nullptr, nullptr,
                              nullptr, nullptr, nullptr, z_fine, nullptr, s, msrc)))
    return rc;
  if ((rc = profiled_mlp(packed, rays_o, dn, z_fine, B, Nf, feat, rgb_f, sigma_f, nullptr, 0, s))) return rc;
  return launch_composite_merged(rgb_c, sigma_c, rgb_f, sigma_f, msrc, z_all, B, N, Nf, rgb_map, depth_map,
                                 weights_out, s);
}

}  // extern "C"
