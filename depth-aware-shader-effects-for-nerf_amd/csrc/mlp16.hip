// Fused positional encoding -> NeRF MLP forward on split-f16 MFMA ("f16x3"), the render
// path's default MLP arithmetic (R4-R6; reference src/models.py:105-162, :14-47).
//
// Arithmetic.  Every dense layer out^T = W . in^T runs on v_mfma_f32_32x32x16_f16 as
//     hi(W) hi(a) + hi(W) lo(a) + lo(W) hi(a)       (f32 accumulation)
// with x*s = hi + lo + O(2^-24 |x*s|), hi = f16(x*s), lo = f16(x*s - hi), and s a power of two:
// per matrix for W (packed, layout.h) and per SAMPLE for the activations (each sample's largest
// input maps just under 2^14).  A power-of-two scale of a column of B scales that column of the
// product exactly, so the accumulator holds s_w * s_j * (W a) and one multiply by the exact
// inverse recovers it.  The dropped lo*lo term and the split residual are both O(2^-24): the
// result has fp32-level error (tests/test_gpu_parity.py measures it against float64 next to
// the exact-f32 kernel in mlp.hip), at 3 x 32 MFMA cycles per 16-deep k-step instead of the
// f32 instruction's 8 x 64.
//
// Work decomposition.  One wave owns 32 samples and runs the whole network for them, as in
// mlp.hip: a layer's 8 accumulator tiles are the next layer's B operands in place (layout.h,
// "split-f16 fragments"), so activations never leave registers.  At 5.3x the f32 rate one wave
// would need ~21 B/clk of weights from L2, so the 4 waves of a workgroup share the weight
// stream: each 16-deep k-step ("chunk": NT tiles x {hi, lo} x 1 KiB) is loaded once per
// workgroup, a quarter by each wave, one step ahead into registers, published into a 2-slot LDS
// ring, and read back by all four waves with ds_read_b128 (one barrier per k-step).
//
// Epilogue of a layer (VALU): y = acc * (1/(s_w s_j)) + bias (the true pre-activation), the
// per-sample max of ReLU(y) over the 256 neurons (both lane halves), the next scale s, and the
// f16 hi/lo split of ReLU(y) * s into the next layer's operands.  The heads (sigma, rgb) run in
// f32 on the unscaled activations, as in mlp.hip.
#include "common.h"

namespace nerf {

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

constexpr int kW16Waves = 4;           // waves per workgroup, one per SIMD; they share the weight stream

#ifdef NERF_MLP16_STAMPS   // diagnostic build (scripts/microbench/mlp16_stamps.hip): per-wave segment clocks
__device__ unsigned long long nerf16_stamps[65536][24];
#define STAMP16(i)                                                                          \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long t_;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    const int64_t w_ = (int64_t)blockIdx.x * kW16Waves + wave;                              \
    if (w_ < 65536 && lane == 0) nerf16_stamps[w_][i] = t_;                                 \
  } while (0)
#else
#define STAMP16(i) do {} while (0)
#endif

struct Operand {                       // B operand of one 16-deep k-step, split
  h16x8 hi, lo;
};

__device__ __forceinline__ f32x16 mfma16(h16x8 a, h16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// Per-sample power-of-two scale for values bounded by m: s = 2^(14-e) with m < 2^e.
__device__ __forceinline__ float pow2_scale(float m, float& inv) {
  int e;
  frexpf(m, &e);                       // m = f 2^e, f in [0.5, 1); m = 0 gives e = 0
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  inv = ldexpf(1.0f, e - 14);
  return ldexpf(1.0f, 14 - e);
}

__device__ __forceinline__ void split_into(float x, Operand& op, int j) {
  const _Float16 h = (_Float16)x;
  op.hi[j] = h;
  op.lo[j] = (_Float16)(x - (float)h);
}

// ---- the shared weight stream ------------------------------------------------------------
// LDS (one __shared__ array: a second object can make hipcc drain the DMA before every ds_read):
//   [ring: 4 slots x 16 KiB][PE: 4 waves x 32 x 64 floats]
//   [trunk biases 8 x 256 | density_head weight 256, bias 4 | 1/s_w of the 10 matrices, pad 16]
// (every small vector the layers read sits in LDS: an ordinary global load used while a DMA is in
// flight makes hipcc wait vmcnt(0), draining the stream)
constexpr int kSlotFloats = 4096;
constexpr int kLdsPe = 4 * kSlotFloats;
constexpr int kLdsBias = kLdsPe + kW16Waves * kPeSteps * 64;
constexpr int kLdsSigmaW = kLdsBias + 8 * kHidden;
constexpr int kLdsVecFloats = 8 * kHidden + kHidden + 4;    // kOffBias .. kOffSigmaB + 4, contiguous in `packed`
constexpr int kLdsScaleInv = kLdsBias + kLdsVecFloats;
constexpr int kLdsFloats = kLdsScaleInv + 16;               // 105 KiB
static_assert(kOffSigmaW == kOffBias + 8 * kHidden && kOffSigmaB == kOffSigmaW + kHidden, "packed vector order");

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// A chunk (one 16-deep k-step of NT tiles) is 2*NT pieces of 256 floats (64 lanes x 16 B); wave w
// moves pieces w, w+4, ... straight into its LDS slot with global_load_lds_dwordx4 (no registers).
template <int NT>
__device__ __forceinline__ void chunk_dma(const float* __restrict__ chunk, float* slot, int wave, int lane) {
#ifdef NERF16_T_NODMA
  return;
#endif
#pragma unroll
  for (int i = 0; i < 2 * NT / kW16Waves; ++i) {
    const int p = wave + kW16Waves * i;
    __builtin_amdgcn_global_load_lds((gptr_t)(chunk + p * 256 + lane * 4), (lptr_t)(slot + p * 256), 16, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// A fragments of half a chunk (tiles HALF*NT/2 ..), hi and lo per tile.
template <int NT, int HALF>
__device__ __forceinline__ void read_half(const float* slot, h16x8 (&a)[4][2], int lane) {
#ifdef NERF16_T_NOREAD
#pragma unroll
  for (int i = 0; i < NT / 2; ++i) asm volatile("" : "+v"(a[i][0]), "+v"(a[i][1]));
  return;
#endif
#pragma unroll
  for (int i = 0; i < NT / 2; ++i) {
    const int t = HALF * (NT / 2) + i;
    a[i][0] = __builtin_bit_cast(h16x8, *reinterpret_cast<const f32x4*>(slot + (2 * t) * 256 + lane * 4));
    a[i][1] = __builtin_bit_cast(h16x8, *reinterpret_cast<const f32x4*>(slot + (2 * t + 1) * 256 + lane * 4));
  }
}

template <int NT, int HALF, bool FIRST>
__device__ __forceinline__ void mfma_half(const h16x8 (&a)[4][2], const Operand& b, f32x16 (&acc)[8]) {
#ifdef NERF16_T_NOMFMA   // timing-only builds (scripts/microbench/mlp16_stamps.hip); wrong results
#pragma unroll
  for (int i = 0; i < NT / 2; ++i)
    asm volatile("" : "+v"(acc[HALF * (NT / 2) + i]) : "v"(a[i][0]), "v"(a[i][1]), "v"(b.hi), "v"(b.lo));
  return;
#endif
  static_for<NT / 2>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    constexpr int t = HALF * (NT / 2) + i;
    f32x16 c;
    if constexpr (FIRST) c = mfma16(a[i][1], b.hi, f32x16{});
    else c = mfma16(a[i][1], b.hi, acc[t]);
    c = mfma16(a[i][0], b.lo, c);
    acc[t] = mfma16(a[i][0], b.hi, c);
  });
}

// DMA instructions one wave issues for chunk j of a layer with KS chunks of NT tiles followed by
// a matrix of NEXT_NT tiles (0: the stream ends).
template <int NT, int KS, int NEXT_NT>
__device__ __forceinline__ constexpr int dma_per_wave(int j) {
  return j < KS ? 2 * NT / kW16Waves : 2 * NEXT_NT / kW16Waves;
}

// Half a k-step: the MFMAs of tiles HALF*NT/2 .. from the fragments in `am`, interleaved with
// the reads of the next half's fragments into `ar` (RT tiles' worth, from `slot_r`; 0 = none):
// 2 ds_read_b128 between consecutive tiles' 3 MFMAs, so the LDS latency hides under them.
template <int NT, int HALF, bool FIRST, int RT, int RHALF>
__device__ __forceinline__ void half_step(const h16x8 (&am)[4][2], const Operand& b, f32x16 (&acc)[8],
                                          const float* slot_r, h16x8 (&ar)[4][2], int lane) {
  if constexpr (RT > 0) read_half<RT, RHALF>(slot_r, ar, lane);
  mfma_half<NT, HALF, FIRST>(am, b, acc);
  static_for<NT / 2>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    if constexpr (i < RT / 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // 2 DS reads
    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);                            // 3 MFMAs
  });
  __builtin_amdgcn_sched_barrier(0);
}

// One dense layer: NT output tiles, KS_ACT activation k-steps from `in` then KS_PE PE k-steps
// from `pe`, weights at `wm` (stream order; layer 4's PE part follows its activation part).
// Pipeline per k-step ks (chunk ks sits in LDS slot ks&3):
//   MFMA half 0, reading half 1's A | wait own DMA of chunk ks+1, barrier | DMA chunk ks+3 into
//   the slot chunk ks-1 used | MFMA half 1, reading chunk ks+1's half-0 A
// On entry chunk 0 is published, chunks 1-2 are in flight and a0 holds chunk 0's half 0; on exit
// the same holds for `next` (NEXT_NT tiles; 0 = last matrix).
template <int NT, int KS_ACT, int KS_PE, int NEXT_NT>
__device__ __forceinline__ void dense16(const float* __restrict__ wm, const float* __restrict__ next, float* lds,
                                        h16x8 (&a0)[4][2], h16x8 (&a1)[4][2], const Operand (&in)[16],
                                        const Operand (&pe)[4], f32x16 (&acc)[8], int wave, int lane) {
  constexpr int KS = KS_ACT + KS_PE;
  static_assert(KS % 4 == 0, "every matrix starts on LDS slot 0");
  static_for<KS>([&](auto kc) __attribute__((always_inline)) {
    constexpr int ks = decltype(kc)::value;
    const Operand& b = [&]() -> const Operand& {
      if constexpr (ks < KS_ACT) return in[ks];
      else return pe[ks - KS_ACT];
    }();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): a0's reads (interleaved in the last half-step) are in
    half_step<NT, 0, ks == 0, NT, 1>(a0, b, acc, lds + (ks & 3) * kSlotFloats, a1, lane);
    constexpr bool has1 = ks + 1 < KS || NEXT_NT > 0;
    constexpr bool has2 = ks + 2 < KS || NEXT_NT > 0;
    constexpr bool has3 = ks + 3 < KS || NEXT_NT > 0;
#ifndef NERF16_T_NOBARRIER
    if constexpr (has1) {
      wait_vmcnt<has2 ? dma_per_wave<NT, KS, NEXT_NT>(ks + 2) : 0>();
      __builtin_amdgcn_s_barrier();
    }
#endif
    if constexpr (ks + 3 < KS) chunk_dma<NT>(wm + (size_t)(ks + 3) * NT * 512, lds + ((ks + 3) & 3) * kSlotFloats, wave, lane);
    else if constexpr (has3)
      chunk_dma<NEXT_NT>(next + (size_t)(ks + 3 - KS) * NEXT_NT * 512, lds + ((ks + 3) & 3) * kSlotFloats, wave, lane);
    __builtin_amdgcn_s_waitcnt(0xC07F);   // a1's reads are in
    constexpr int RT = ks + 1 < KS ? NT : NEXT_NT;
    half_step<NT, 1, ks == 0, RT, 0>(a1, b, acc, lds + ((ks + 1) & 3) * kSlotFloats, a0, lane);
  });
}

// acc[t] <- y = acc * inv + vec[neuron] for the NT tiles (vec: biases, or a per-ray row);
// returns the sample's max of ReLU(y) (lane halves combined).
template <int NT>
__device__ __forceinline__ float unscale(f32x16 (&acc)[8], float inv, const float* __restrict__ vec, int h) {
  float m = 0.0f;
  static_for<NT>([&](auto tc) __attribute__((always_inline)) {
    constexpr int t = decltype(tc)::value;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(vec + t * 32 + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = fmaf(acc[t][4 * q + e], inv, b[e]);
        acc[t][4 * q + e] = y;
        m = fmaxf(m, y);
      }
    }
  });
  return fmaxf(m, __shfl_xor(m, 32));
}

// The next layer's operands: split(ReLU(acc) * s) in the k-step order of layout.h.
__device__ __forceinline__ void to_operands(const f32x16 (&acc)[8], float s, Operand (&in)[16]) {
  static_for<8>([&](auto tc) __attribute__((always_inline)) {
    constexpr int t = decltype(tc)::value;
#pragma unroll
    for (int sh = 0; sh < 2; ++sh)
#pragma unroll
      for (int j = 0; j < 8; ++j) split_into(fmaxf(acc[t][8 * sh + j], 0.0f) * s, in[2 * t + sh], j);
  });
}

__device__ __forceinline__ void pe_operands(const float (&pe)[kPeSteps], float s, Operand (&op)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) split_into(pe[8 * q + j] * s, op[q], j);
}

__global__ void __launch_bounds__(64 * kW16Waves, 1)
mlp16_kernel(const float* __restrict__ packed, const float* __restrict__ orig, const float* __restrict__ dirs,
             const float* __restrict__ zv, int64_t M, int N, const float* __restrict__ feat,
             float* __restrict__ rgb, float* __restrict__ sigma, const int* __restrict__ out_slot, int out_T) {
  __shared__ __attribute__((aligned(16))) float lds[kLdsFloats];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, h = lane >> 5;

  STAMP16(0);
  const int64_t s0 = ((int64_t)blockIdx.x * kW16Waves + wave) * 32;
  // every wave runs to the end (the weight stream has barriers); tail lanes repeat sample M-1
  const bool valid = s0 + (lane & 31) < M;
  const int64_t s = imin64(s0 + (lane & 31), M - 1);
  const int64_t r = s / N;

  // Sample position: pts = o + d*z with separate roundings (ray_utils.py:86).
  float x[3];
  if (zv) {
    const float z = zv[s];
#pragma unroll
    for (int c = 0; c < 3; ++c) x[c] = orig[3 * r + c] + dirs[3 * r + c] * z;
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c) x[c] = orig[3 * s + c];
  }
  // small vectors into LDS, then the weight stream starts: chunks 0-2 of layer 0 in flight while
  // the PE is computed (every ordinary load retired first: hipcc waits vmcnt(0) at the use of an
  // ordinary load while a DMA is in flight)
  for (int i = threadIdx.x; i < kLdsVecFloats / 4; i += 64 * kW16Waves)
    reinterpret_cast<f32x4*>(lds + kLdsBias)[i] = reinterpret_cast<const f32x4*>(packed + kOffBias)[i];
  if (threadIdx.x < kNumFragMats) lds[kLdsScaleInv + threadIdx.x] = packed[kOffScale16 + kNumFragMats + threadIdx.x];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  const float* w0 = packed + s16_offset(0);
  chunk_dma<8>(w0, lds, wave, lane);
  chunk_dma<8>(w0 + 8 * 512, lds + kSlotFloats, wave, lane);
  chunk_dma<8>(w0 + 2 * 8 * 512, lds + 2 * kSlotFloats, wave, lane);
  // PE in layout.h::pe_feature order (models.py:36-44): sin on lane half 0, cos on half 1.
  float pe[kPeSteps];
#pragma unroll
  for (int i = 0; i < kPosLevels; ++i)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float sn, cs;
      sincosf(x[c] * (float)(1 << i), &sn, &cs);
      pe[3 * i + c] = h ? cs : sn;
    }
  pe[30] = h ? x[1] : x[0];
  pe[31] = h ? 0.0f : x[2];
  float* pe_mine = lds + kLdsPe + wave * kPeSteps * 64;
#pragma unroll
  for (int p = 0; p < kPeSteps; ++p) pe_mine[p * 64 + lane] = pe[p];
  const float m_pe = fmaxf(1.0f, fmaxf(fabsf(x[0]), fmaxf(fabsf(x[1]), fabsf(x[2]))));   // bounds |PE|

  const float* scale_inv = lds + kLdsScaleInv;                     // 1/s_w per matrix
  const float* bias = lds + kLdsBias;
  float inv_s;
  float sc = pow2_scale(m_pe, inv_s);
  Operand pe_op[4];
  pe_operands(pe, sc, pe_op);
  float inv = inv_s * scale_inv[0];

  wait_vmcnt<2 * 2 * 8 / kW16Waves>();     // this wave's part of chunk 0 landed (chunks 1-2 in flight)
  __builtin_amdgcn_s_barrier();
  h16x8 a0[4][2], a1[4][2];
  read_half<8, 0>(lds, a0, lane);

  f32x16 acc[8];
  Operand in[16];
  STAMP16(1);
  // layer 0: PE(63) -> 256
  dense16<8, 0, 4, 8>(w0, packed + s16_offset(1), lds, a0, a1, in, pe_op, acc, wave, lane);
  STAMP16(2);
  float m = unscale<8>(acc, inv, bias, h);
  // layers 1..7; layer 4 reads [h3, enc_x] (models.py:128-134), its PE re-split at h3's scale
#pragma unroll 1
  for (int L = 1; L < 8; ++L) {
    if (L == kSkipLayer) m = fmaxf(m, m_pe);
    sc = pow2_scale(m, inv_s);
    to_operands(acc, sc, in);
    inv = inv_s * scale_inv[L];
    const float* wl = packed + s16_offset(L);
    STAMP16(1 + 2 * L);
    if (L == kSkipLayer) {
      float pe2[kPeSteps];
#pragma unroll
      for (int p = 0; p < kPeSteps; ++p) pe2[p] = pe_mine[p * 64 + lane];
      pe_operands(pe2, sc, pe_op);
      dense16<8, 16, 4, 8>(wl, packed + s16_offset(L + 1), lds, a0, a1, in, pe_op, acc, wave, lane);
    } else if (L == 7) {
      dense16<8, 16, 0, 4>(wl, packed + s16_offset(8), lds, a0, a1, in, pe_op, acc, wave, lane);
    } else {
      dense16<8, 16, 0, 8>(wl, packed + s16_offset(L + 1), lds, a0, a1, in, pe_op, acc, wave, lane);
    }
    STAMP16(2 + 2 * L);
    m = unscale<8>(acc, inv, bias + L * kHidden, h);
  }

  // density head: sigma = ReLU(density_head(ReLU(h7))) (models.py:137-138), f32.
  const float* ws = lds + kLdsSigmaW;
  float part = 0.0f;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(ws + t * 32 + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) part = fmaf(w[e], fmaxf(acc[t][4 * q + e], 0.0f), part);
    }
  const float sig = fmaxf(part + __shfl_xor(part, 32) + ws[kHidden], 0.0f);

  // colour branch: h_dir = ReLU(W_dh ReLU(h7) + [b_dir + W_dd PE(d)]) + appearance
  // (models.py:141-156); the bracket and the appearance part come per ray in `feat`.
  sc = pow2_scale(m, inv_s);
  to_operands(acc, sc, in);
  inv = inv_s * scale_inv[8];
  STAMP16(17);
  dense16<4, 16, 0, 0>(packed + s16_offset(8), nullptr, lds, a0, a1, in, pe_op, acc, wave, lane);
  STAMP16(18);
  const float* fr = feat + r * kRayFeat;
  const float* wr = packed + kOffRgbW;
  float pr[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 fd = *reinterpret_cast<const f32x4*>(fr + t * 32 + 8 * q + 4 * h);
      const f32x4 ap = *reinterpret_cast<const f32x4*>(fr + kDirHidden + t * 32 + 8 * q + 4 * h);
      float hd[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) hd[e] = fmaxf(fmaf(acc[t][4 * q + e], inv, fd[e]), 0.0f) + ap[e];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(wr + c * kDirHidden + t * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) pr[c] = fmaf(w[e], hd[e], pr[c]);
      }
    }
  float out[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = pr[c] + __shfl_xor(pr[c], 32) + packed[kOffRgbB + c];
    out[c] = 1.0f / (1.0f + expf(-v));                           // sigmoid (models.py:159-160)
  }
  if (h == 0 && valid) {
    const int64_t o_s = out_slot ? r * out_T + out_slot[s] : s;
    sigma[o_s] = sig;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[3 * o_s + c] = out[c];
  }
  STAMP16(19);
}

int launch_mlp16(const float* packed, const float* o, const float* d, const float* z, int64_t R, int N,
                 const float* feat, float* rgb, float* sigma, const int* out_slot, int out_T, hipStream_t s) {
  const int64_t M = R * (int64_t)N;
  if (M == 0) return NERF_OK;
  constexpr int per_block = 32 * kW16Waves;
  const int64_t blocks = (M + per_block - 1) / per_block;
  hipLaunchKernelGGL(mlp16_kernel, dim3((unsigned)blocks), dim3(64 * kW16Waves), 0, s, packed, o, d, z, M, N, feat,
                     rgb, sigma, out_slot, out_T);
  return check_launch("mlp16_kernel");
}

}  // namespace nerf
