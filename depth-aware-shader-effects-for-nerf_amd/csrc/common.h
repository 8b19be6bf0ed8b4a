// Internal helpers shared by the HIP translation units of libnerfmi.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <utility>
#include "../../include/nerfmi_train.h"
#include "layout.h"

namespace nerf {

// Records the message of a failed call for nerf_last_error() and returns `code`.
int set_error(int code, const char* fmt, ...);

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(NERF_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return NERF_OK;
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Compile-time loop: f(std::integral_constant<int, i>) for i = 0..N-1, fully expanded by the
// front end (the loop unroller gives up on bodies this large and would leave the register
// arrays runtime-indexed, i.e. in scratch).
template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__host__ __device__ __forceinline__ int64_t imin64(int64_t a, int64_t b) { return a < b ? a : b; }

// expf rounded once: exp evaluated in double, then rounded to float.  The alpha of the
// composite, 1 - exp(-sigma*dist), cancels catastrophically for small sigma*dist, so the
// rounding of exp dominates the error of the coarse weights (and, through the ill-conditioned
// inverse CDF, of the fine pass); the device's single-precision expf is a 1-ulp function, torch's
// CPU exp is correctly rounded on almost every input.  This keeps the reference's fp32
// expression (one float exp, then the float subtraction) with the best-rounded exp.
// lo part of the f16 split x = hi + lo: f16(x - hi), through an fma with a -1.0f the compiler
// cannot fold, so it selects v_fma_mix (f16 hi, f32 x, one f16 rounding) instead of a convert
// back, a subtract and a convert.  x - hi is exact in f32, so the result is bit-identical.
__device__ __forceinline__ float opaque_neg_one() {
  float v = -1.0f;
  asm("" : "+s"(v));
  return v;
}
__device__ __forceinline__ _Float16 split_lo(float x, _Float16 hi) {
  return (_Float16)__builtin_fmaf((float)hi, opaque_neg_one(), x);
}

// lo parts of a split pair whose hi parts are packed in hi2: f16(x0 - hi.x) | f16(x1 - hi.y), one
// v_fma_mix each reading its hi half in place (op_sel).  x - hi is exact in f32, so this is
// bit-identical to split_lo; the compiler, given the same expression, converts both halves back to
// f32 and packs the residuals with a third convert (or SLP-packs them into v_pk_fma_f32).  Used by
// the training forward (mlp16.hip, issue-bound: 1.28 -> 1.19 ms, same-box A/B) and the data
// gradient's row split (train.hip); the render kernel measured -0.3 % with it and keeps its own.
__device__ __forceinline__ uint32_t split_lo_pair(uint32_t hi2, float x0, float x1) {
  uint32_t lo;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lo)
      : "v"(hi2), "v"(x0), "v"(x1));
  return lo;
}

// Cache policy (buffer instruction aux bits: 2 = nt, 1 = sc0, 16 = sc1) of the training kernels'
// activation / gradient row stores: 2.5 GB per step written once and read by a later kernel.  nt
// (streaming) keeps them from evicting the weight stream's L2 lines and retires them sooner: the
// forward with saves 0.99 -> 0.82 ms and the data gradient 0.87 -> 0.71 ms per 262K-sample step, the
// training step 1.13 -> 1.19 M rays/s (same-box A/B, profiles/r04/ab_train_store_policy.log; sc0 nt
// the same, sc1 slower).  kRowLoadAux: the weight-gradient GEMMs' once-read row loads.
constexpr int kRowStoreAux = 2;
constexpr int kRowLoadAux = 0;

// A 16-byte row store with its whole offset in the lane's VGPR `voff` (+ the instruction's offset
// field) and soffset the literal 0.  For a store of more than 8 bytes whose soffset is a register, the
// compiler's hazard model pads no wait states before an instruction that overwrites the store's data
// VGPRs, and a uniform or large constant soffset is always a register.  Measured on gfx950 (round 6,
// scripts/diag_train_det.py): in the training forward a `v_accvgpr_read` into the first data VGPR
// right behind a `buffer_store_dwordx4 ..., s60` that followed an LDS-DMA issue reached the register
// before the store read it; that activation (one float of the four, both lane halves) came out
// different from run to run.  With soffset 0 the compiler pads those wait states (and
// scripts/check_isa.py rejects a data VGPR written within two of them in the stream kernels).
typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
// PAD: two wait states right behind the store in an asm statement, which no memory instruction is
// scheduled across (a load whose destination is one of the data VGPRs; the compiler pads only VALU).
template <int AUX, bool PAD = false, typename V>
__device__ __forceinline__ void store16_rows(V v, __amdgpu_buffer_rsrc_t rows, uint32_t voff) {
  static_assert(sizeof(V) == 16, "16-byte stores");
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4s, v), rows, (int)voff, 0, AUX);
  if constexpr (PAD) asm volatile("s_nop 1");
}

__device__ __forceinline__ float expf_rn(float x) { return (float)exp((double)x); }

// Max over the wave of a non-negative v, uniform result: DPP within each 16-lane row (quad swaps,
// half-row and row mirrors), then the four rows' values by readlane.  No LDS, no branch.
__device__ __forceinline__ float wave_max_nn(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)));   // quad [1,0,3,2]
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false)));   // quad [2,3,0,1]
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false)));  // row_half_mirror
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false)));  // row_mirror
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// The block exponent record of layout.h for a block maximum m >= 0: -(kBlockExpBias + e), m < 2^e.
__device__ __forceinline__ float block_exp_record(float m) {
  int e;
  frexpf(m, &e);
  return -(float)(kBlockExpBias + (m > 0.0f ? e : kBlockExpZero));
}

// Counter-based uniform in [0,1) (splitmix64 finaliser), used when the caller
// passes no explicit uniforms; it is a device RNG for throughput runs only.
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// The key whose stream starts at index `first` of `seed`'s: hash_uniform(rng_key_at(seed, f), i) ==
// hash_uniform(seed, f + i) (mod 2^64).  A ray shard keys its draws by the global index of its
// first ray this way, so a sharded frame draws exactly the uniforms of the unsharded frame.
__host__ __device__ __forceinline__ uint64_t rng_key_at(uint64_t seed, uint64_t first) {
  return seed + 0x9E3779B97F4A7C15ull * first;
}

// Kernel launchers (one per translation unit); each returns a nerf_status.
int launch_get_rays(int H, int W, float focal, const float* c2w, int row0, int nrows,
                    float* o, float* d, hipStream_t s);
int launch_rng_uniforms(uint64_t seed, int64_t first, int64_t n, float* out, hipStream_t s);
int launch_pe(const float* x, int64_t M, int dims, int levels, int include_input, float* out, hipStream_t s);
int launch_normalize(const float* d, int64_t B, float* out, hipStream_t s);
int launch_stratified(const float* o, const float* d, int64_t B, float near_f, float span_f,
                      int N, const float* t_vals, int perturb, const float* t_rand,
                      uint64_t seed, float* z, float* pts, hipStream_t s);
int launch_importance(const float* o, const float* d, const float* z, const float* w,
                      int64_t B, int N, int Nf, const float* u_lin, const float* u_rand,
                      uint64_t seed, float* z_all, float* pts_all, const float* rgb_c, const float* sigma_c,
                      float* rgb_all, float* sigma_all, float* z_fine, int* fine_slot, hipStream_t s,
                      uint16_t* merged_src = nullptr);
int launch_pack(const float* const* params, float* packed, hipStream_t s);
int launch_ray_features(const float* packed, const float* dirs, int64_t R, const float* app,
                        int64_t app_rows, float* feat, hipStream_t s, float* encd = nullptr, float* dn_out = nullptr);
extern int g_mlp_arith;   // nerf_arith, set by nerf_set_mlp_arith
int launch_mlp16(const float* packed, const float* o, const float* d, const float* z, int64_t R, int N,
                 const float* feat, float* rgb, float* sigma, const int* out_slot, int out_T, hipStream_t s,
                 float* save = nullptr, const float* encd = nullptr, uint32_t* masks = nullptr);
// the render MLP on 16 x 16 x 32 tiles (mlp16s.hip): launch_mlp16 without saves
int launch_mlp16s(const float* packed, const float* o, const float* d, const float* z, int64_t R, int N,
                  const float* feat, float* rgb, float* sigma, const int* out_slot, int out_T, hipStream_t s);
int launch_mlp(const float* packed, const float* o, const float* d, const float* z, int64_t R,
               int N, const float* feat, float* rgb, float* sigma, const int* out_slot, int out_T,
               hipStream_t s, float* save = nullptr, const float* encd = nullptr, uint32_t* masks = nullptr);
int launch_composite(const float* rgb, const float* sigma, const float* z, int64_t B, int N,
                     float* rgb_map, float* depth, float* weights, hipStream_t s);
// The fine composite of nerf_render_rays: merged slot p of ray r holds sample src[r T + p] of
// cat[coarse (rgb_c, sigma_c: N per ray), fine (rgb_f, sigma_f: Nf per ray)], z_all its z.
int launch_composite_merged(const float* rgb_c, const float* sigma_c, const float* rgb_f, const float* sigma_f,
                            const uint16_t* src, const float* z_all, int64_t B, int N, int Nf, float* rgb_map,
                            float* depth, float* weights, hipStream_t s);

}  // namespace nerf
