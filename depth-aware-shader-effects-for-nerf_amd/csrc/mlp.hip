// Fused positional encoding -> NeRF MLP forward on fp32 MFMA (R4, R5, R6), and the per-ray
// colour-branch features it consumes.
//
// Reference: src/models.py:105-162 (NeRF.forward), :14-47 (PositionalEncoding).
//
// Work decomposition: one wave owns 32 consecutive samples and runs the whole network for
// them; a 256-thread workgroup is 4 independent waves (one per SIMD).  Every dense layer is
//     out^T[n][m] = sum_k W[n][k] in^T[k][m]
// on v_mfma_f32_32x32x2_f32 (A = 32 weight rows x 2 inputs, B = 2 inputs x 32 samples,
// exact f32: a k-ordered fmaf chain).  A layer's accumulators (8 tiles x 16 registers) are
// the next layer's B operands as they stand (layout.h), so activations never leave
// registers: the kernel reads only the samples' (o, d, z), the 2 MiB packed weights
// (L2-resident on every XCD) and writes 16 B per sample.
//
// Bound: MFMA.  1,048,832 algorithmic FLOP per sample; the kernel
// issues 8,192 MFMAs of 4,096 FLOP per 32 samples (63->64 and 319->320 input padding).
#include <utility>

#include "common.h"

namespace nerf {

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Accumulator initialised from a per-neuron vector: register 4q+e of lane half h holds
// neuron nt*32 + 8q + 4h + e, so each group of 4 registers is one 16-byte load.
__device__ __forceinline__ f32x16 load_rows(const float* __restrict__ v, int nt, int h) {
  f32x16 out;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(v + nt * 32 + 8 * q + 4 * h);
    out[4 * q + 0] = t[0];
    out[4 * q + 1] = t[1];
    out[4 * q + 2] = t[2];
    out[4 * q + 3] = t[3];
  }
  return out;
}

__device__ __forceinline__ void relu16(f32x16& v) {
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = fmaxf(v[e], 0.0f);
}

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

#ifndef NERF_MLP_SPLIT
#define NERF_MLP_SPLIT 2      // independent accumulation chains per output tile
#endif
#ifndef NERF_MLP_WAVES
#define NERF_MLP_WAVES 4      // waves per workgroup (each wave is independent: no barriers, own LDS slice)
#endif
#ifndef NERF_MLP_DEPTH
#define NERF_MLP_DEPTH 8      // weight-fragment blocks in flight per wave
#endif

// One dense layer: NT output tiles of 32 neurons, KS_ACT activation k-steps read from the `in`
// registers and KS_PE positional-encoding k-steps read from `pe`.  BIAS: the tile starts at zero
// and the per-neuron vector `init` (a bias, or the per-ray colour feature) is added after the
// last k-step — its loads are issued at the tile's first k-step and land long before they are
// needed.  Without BIAS the layer is a further K-slice accumulated onto `out` (the skip layer's
// PE inputs).  Each tile is accumulated in SPLIT chains taking alternate k-steps, summed at the
// end: consecutive MFMAs are independent, and each chain is SPLIT times shorter (less rounding
// growth than one K-long chain).  Weight fragments stream from L2 through a register ring
// DEPTH blocks deep (1 KiB per block per wave) that runs across layers: on entry `ring` holds
// this matrix's first DEPTH blocks, and the last DEPTH steps load the first DEPTH blocks of
// `next` (the last matrix passes any valid fragment array and the loads go unused), so no
// layer starts on an L2 round trip.
constexpr int kDepth = NERF_MLP_DEPTH;

__device__ __forceinline__ void ring_fill(f32x4 (&ring)[kDepth], const float* __restrict__ wmat, int lane) {
  const f32x4* __restrict__ wf = reinterpret_cast<const f32x4*>(wmat) + lane;
#pragma unroll
  for (int p = 0; p < kDepth; ++p) ring[p] = wf[p * 64];
}

#ifndef NERF_MLP_OVERLAP
#define NERF_MLP_OVERLAP 0   // 1: overlapped epilogues (spills at this register budget)
#endif

#if NERF_MLP_OVERLAP
// Tile epilogues overlapped with the next tile's MFMAs.  Tile nt accumulates in acc[nt & 1]
// (one chain: the 32x32x2 f32 MFMA's dependent latency equals its issue interval).  With
// BIAS (a per-neuron vector shared by all samples) the chain starts with one extra MFMA,
// A = init[nt*32 + (lane&31)], B = 1 on lane half 0 and 0 on half 1, C = 0, which writes
// the bias into every column exactly; the epilogue is then just ReLU and the copy to `out`,
// and it runs inside the first two k-quads of tile nt+1, interleaved one MFMA to ~6 VALU by
// sched_group_barrier, so it issues in the MFMA shadow instead of draining the matrix pipe.
// The bias value of tile nt+1 is loaded during tile nt.  PERLANE_INIT (the colour branch's
// per-ray feature, a different vector per sample) is added by VALU in the epilogue instead.
// The last tile's epilogue stays at the end of the layer.
template <int NT, int KS_ACT, int KS_PE, bool BIAS, bool RELU, bool PERLANE_INIT = false>
__device__ __forceinline__ void dense(const float* __restrict__ wmat, const float* __restrict__ next,
                                      f32x4 (&ring)[kDepth], const float* __restrict__ init,
                                      const f32x16 (&in)[8], const float (&pe)[kPeSteps],
                                      f32x16 (&out)[8], int lane) {
  constexpr int KS = KS_ACT + KS_PE;
  constexpr int KSQ = KS / 4;
  constexpr int G = NT * KSQ;
  constexpr int DEPTH = kDepth;
  static_assert(G >= DEPTH && G % DEPTH == 0, "the ring hands over whole DEPTH-block windows");
  static_assert(KSQ >= 2, "the epilogue spans two k-quads");
  const int h = lane >> 5;
  const f32x4* __restrict__ wf = reinterpret_cast<const f32x4*>(wmat) + lane;
  const f32x4* __restrict__ nf = reinterpret_cast<const f32x4*>(next) + lane;
  const float one_h0 = h ? 0.0f : 1.0f;
  f32x16 acc[2];
  f32x4 bv[4];
  float bnext = 0.0f;
  if constexpr (BIAS && !PERLANE_INIT) bnext = init[lane & 31];
  auto epilogue = [&](auto ntc) __attribute__((always_inline)) {
    constexpr int t = decltype(ntc)::value;
    f32x16 a = acc[t & 1];
    if constexpr (PERLANE_INIT) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) a[4 * q + e] += bv[q][e];
    }
    if constexpr (RELU) relu16(a);
    out[t] = a;
  };
  static_for<G>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    constexpr int nt = g / KSQ, kq = g % KSQ;
    const f32x4 w = ring[g % DEPTH];
#ifndef NERF_MLP_NOLOAD
    if constexpr (g + DEPTH < G) {
      ring[g % DEPTH] = wf[(g + DEPTH) * 64];
    } else {
      ring[g % DEPTH] = nf[(g + DEPTH - G) * 64];
    }
#else   // timing-only build: the weight stream removed (wrong results)
    asm volatile("" : "+v"(ring[g % DEPTH]));
#endif
    if constexpr (kq == 0) {
      if constexpr (!BIAS) acc[nt & 1] = out[nt];
      else if constexpr (PERLANE_INIT) acc[nt & 1] = f32x16{};
      else acc[nt & 1] = mfma32(bnext, one_h0, f32x16{});
    }
    static_for<4>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      constexpr int ks = 4 * kq + j;
      float b;
      if constexpr (ks < KS_ACT) b = in[ks >> 4][ks & 15];
      else b = pe[ks - KS_ACT];
      acc[nt & 1] = mfma32(w[j], b, acc[nt & 1]);
    });
    if constexpr (kq == 0 && nt > 0) epilogue(std::integral_constant<int, nt - 1>{});
    if constexpr (kq == 1 && BIAS) {
      if constexpr (PERLANE_INIT) {
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[q] = *reinterpret_cast<const f32x4*>(init + nt * 32 + 8 * q + 4 * h);
      } else if constexpr (nt + 1 < NT) {
        bnext = init[(nt + 1) * 32 + (lane & 31)];
      }
    }
    if constexpr (kq == 1 && nt > 0) {
      // region = k-quads 0 and 1 of tile nt: 8 (9) MFMAs with the previous tile's epilogue between them
      static_for<9>([&](auto) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);   // up to 6 VALU
      });
    }
    if constexpr (kq != 0 || nt == 0) {
      // keep the ring's issue order: without this the scheduler hoists the whole layer's
      // weight loads and spills
      __builtin_amdgcn_sched_barrier(0);
    }
  });
  epilogue(std::integral_constant<int, NT - 1>{});
}
#else
template <int NT, int KS_ACT, int KS_PE, bool BIAS, bool RELU>
__device__ __forceinline__ void dense(const float* __restrict__ wmat, const float* __restrict__ next,
                                      f32x4 (&ring)[kDepth], const float* __restrict__ init,
                                      const f32x16 (&in)[8], const float (&pe)[kPeSteps],
                                      f32x16 (&out)[8], int lane) {
  constexpr int KS = KS_ACT + KS_PE;
  constexpr int KSQ = KS / 4;
  constexpr int G = NT * KSQ;
  constexpr int DEPTH = kDepth;
  constexpr int SPLIT = NERF_MLP_SPLIT;
  static_assert(G >= DEPTH && G % DEPTH == 0, "the ring hands over whole DEPTH-block windows");
  static_assert(SPLIT == 1 || SPLIT == 2 || SPLIT == 4, "SPLIT must divide a k-quad");
  const int h = lane >> 5;
  const f32x4* __restrict__ wf = reinterpret_cast<const f32x4*>(wmat) + lane;
  const f32x4* __restrict__ nf = reinterpret_cast<const f32x4*>(next) + lane;
  f32x16 part[SPLIT];
  f32x4 bv[4];
  static_for<G>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value;
    constexpr int nt = g / KSQ, kq = g % KSQ;
    const f32x4 w = ring[g % DEPTH];
#ifndef NERF_MLP_NOLOAD
    if constexpr (g + DEPTH < G) {
      ring[g % DEPTH] = wf[(g + DEPTH) * 64];
    } else {
      ring[g % DEPTH] = nf[(g + DEPTH - G) * 64];
    }
#else   // timing-only build: the weight stream removed (wrong results)
    asm volatile("" : "+v"(ring[g % DEPTH]));
#endif
    if constexpr (kq == 0) {
      if constexpr (BIAS) {
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[q] = *reinterpret_cast<const f32x4*>(init + nt * 32 + 8 * q + 4 * h);
        part[0] = f32x16{};
      } else {
        part[0] = out[nt];
      }
#pragma unroll
      for (int c = 1; c < SPLIT; ++c) part[c] = f32x16{};
    }
    static_for<4>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      constexpr int ks = 4 * kq + j;
      float b;
      if constexpr (ks < KS_ACT) b = in[ks >> 4][ks & 15];
      else b = pe[ks - KS_ACT];
      part[j % SPLIT] = mfma32(w[j], b, part[j % SPLIT]);
    });
    if constexpr (kq == KSQ - 1) {
      f32x16 acc = part[0];
#pragma unroll
      for (int c = 1; c < SPLIT; ++c) acc += part[c];
      if constexpr (BIAS) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[4 * q + e] += bv[q][e];
      }
      if constexpr (RELU) relu16(acc);
      out[nt] = acc;
    }
    // keep the ring's issue order: without this the scheduler hoists the whole layer's
    // weight loads and spills
    __builtin_amdgcn_sched_barrier(0);
  });
}

#endif  // NERF_MLP_OVERLAP

__global__ void __launch_bounds__(64 * NERF_MLP_WAVES, 1)
mlp_kernel(const float* __restrict__ packed, const float* __restrict__ orig, const float* __restrict__ dirs,
           const float* __restrict__ zv, int64_t M, int N, const float* __restrict__ feat,
           float* __restrict__ rgb, float* __restrict__ sigma, const int* __restrict__ out_slot, int out_T) {
  const int lane = threadIdx.x & 63;
  const int64_t s0 = ((int64_t)blockIdx.x * NERF_MLP_WAVES + (threadIdx.x >> 6)) * 32;
  if (s0 >= M) return;
  const int h = lane >> 5;
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

  // Positional encoding in the k order of layout.h::pe_feature: sin(2^i x_c) on lane half 0,
  // cos on half 1 (models.py:36-44; 2^i x is exact, sin/cos fully range-reduced).  Layer 0
  // reads it from registers; the skip layer reads it back from this wave's LDS slice
  // (32 floats x 64 lanes), so it does not occupy 32 registers through layers 1..3.
  __shared__ float pe_lds[NERF_MLP_WAVES][kPeSteps][64];
  float (*pe_mine)[64] = pe_lds[threadIdx.x >> 6];
  float pe[kPeSteps];
#pragma unroll
  for (int i = 0; i < kPosLevels; ++i) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float sn, cs;
#ifndef NERF_MLP_NOPE
      sincosf(x[c] * (float)(1 << i), &sn, &cs);
#else   // timing-only build: PE without the transcendental (wrong results)
      sn = x[c] * (float)(1 << i);
      cs = sn + 1.0f;
#endif
      pe[3 * i + c] = h ? cs : sn;
    }
  }
  pe[30] = h ? x[1] : x[0];
  pe[31] = h ? 0.0f : x[2];
#pragma unroll
  for (int p = 0; p < kPeSteps; ++p) pe_mine[p][lane] = pe[p];

  const float* bias = packed + kOffBias;
  const float* wtrunk = packed + frag_offset(1);                 // layers 1..7, frag_floats(1) apart
  auto wlayer = [&](int m) { return wtrunk + (size_t)(m - 1) * frag_floats(1); };
  const float* wskip = packed + frag_offset(kSkipPeMat);
  f32x4 ring[kDepth];
  ring_fill(ring, packed + frag_offset(0), lane);
  f32x16 A[8], B[8];
  // layer 0: PE(63) -> 256
  dense<8, 0, kPeSteps, true, true>(packed + frag_offset(0), wlayer(1), ring, bias, A, pe, A, lane);
  // layers 1..6 as three A->B->A pairs; the skip layer 4 adds its PE slice before its ReLU.
#pragma unroll 1
  for (int p = 0; p < 3; ++p) {
    const int m1 = 1 + 2 * p, m2 = 2 + 2 * p;
    dense<8, kActSteps, 0, true, true>(wlayer(m1), wlayer(m2), ring, bias + m1 * kHidden, A, pe, B, lane);
    dense<8, kActSteps, 0, true, false>(wlayer(m2), m2 == kSkipLayer ? wskip : wlayer(m2 + 1), ring,
                                        bias + m2 * kHidden, B, pe, A, lane);
    if (m2 == kSkipLayer) {
      float pe2[kPeSteps];
#pragma unroll
      for (int q = 0; q < kPeSteps; ++q) pe2[q] = pe_mine[q][lane];
      dense<8, 0, kPeSteps, false, false>(wskip, wlayer(m2 + 1), ring, bias, A, pe2, A, lane);
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) relu16(A[t]);
  }
  // layer 7: A -> B
  dense<8, kActSteps, 0, true, true>(wlayer(7), packed + frag_offset(8), ring, bias + 7 * kHidden, A, pe, B, lane);

  // density head: sigma = ReLU(density_head(h)) (models.py:137-138), h = B.
  const float* ws = packed + kOffSigmaW;
  float part = 0.0f;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(ws + t * 32 + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) part = fmaf(w[e], B[t][4 * q + e], part);
    }
  const float sig = fmaxf(part + __shfl_xor(part, 32) + packed[kOffSigmaB], 0.0f);

  // colour branch: h_dir = ReLU(W_dh h + [b_dir + W_dd PE(d)]) + appearance (models.py:141-156),
  // the bracket and the appearance part precomputed per ray in `feat`.
  const float* fr = feat + r * kRayFeat;
#if NERF_MLP_OVERLAP
  dense<4, kActSteps, 0, true, true, true>(packed + frag_offset(8), packed, ring, fr, B, pe, A, lane);
#else
  dense<4, kActSteps, 0, true, true>(packed + frag_offset(8), packed, ring, fr, B, pe, A, lane);
#endif
  float pr[3] = {0.0f, 0.0f, 0.0f};
  const float* wr = packed + kOffRgbW;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 app = load_rows(fr + kDirHidden, t, h);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(wr + c * kDirHidden + t * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) pr[c] = fmaf(w[e], A[t][4 * q + e] + app[4 * q + e], pr[c]);
      }
    }
  }
  float out[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = pr[c] + __shfl_xor(pr[c], 32) + packed[kOffRgbB + c];
    out[c] = 1.0f / (1.0f + expf(-v));                           // sigmoid (models.py:159-160)
  }
  if (h == 0 && s0 + (lane & 31) < M) {
    const int64_t o_s = out_slot ? r * out_T + out_slot[s] : s;
    sigma[o_s] = sig;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[3 * o_s + c] = out[c];
  }
}

int launch_mlp(const float* packed, const float* o, const float* d, const float* z, int64_t R, int N,
               const float* feat, float* rgb, float* sigma, const int* out_slot, int out_T, hipStream_t s) {
  const int64_t M = R * (int64_t)N;
  if (M == 0) return NERF_OK;
  constexpr int per_block = 32 * NERF_MLP_WAVES;
  const int64_t blocks = (M + per_block - 1) / per_block;
  hipLaunchKernelGGL(mlp_kernel, dim3((unsigned)blocks), dim3(64 * NERF_MLP_WAVES), 0, s, packed, o, d, z, M, N, feat, rgb,
                     sigma, out_slot, out_T);
  return check_launch("mlp_kernel");
}

// -------------------------------------------------------------------------- ray features
// Per ray: feat[0:128] = dir_linear.bias + dir_linear.weight[:,256:283] . PE_4(d)
//          feat[128:256] = appearance_projection(app) or 0.
// A block handles 16 rays: the 16x27 direction encodings and 16x32 appearance rows are
// staged in LDS, then thread n computes output n for all 16 rays (coalesced stores).
constexpr int kFeatRays = 16;

__global__ void __launch_bounds__(256)
ray_features_kernel(const float* __restrict__ packed, const float* __restrict__ dirs, int64_t R,
                    const float* __restrict__ app, int64_t app_rows, float* __restrict__ feat) {
  __shared__ float enc[kFeatRays][kDirEnc + 1];
  __shared__ float apps[kFeatRays][kAppDim];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kFeatRays;
  for (int q = tid; q < kFeatRays * 3 * kDirLevels; q += 256) {
    const int ray = q / (3 * kDirLevels), ic = q % (3 * kDirLevels);
    const int i = ic / 3, c = ic % 3;
    const int64_t r = imin64(r0 + ray, R - 1);
    float sn, cs;
    sincosf(dirs[3 * r + c] * (float)(1 << i), &sn, &cs);
    enc[ray][3 + 6 * i + c] = sn;
    enc[ray][6 + 6 * i + c] = cs;
  }
  if (tid < kFeatRays * 3) {
    const int ray = tid / 3, c = tid % 3;
    enc[ray][c] = dirs[3 * imin64(r0 + ray, R - 1) + c];
  }
  if (app_rows > 0) {
    for (int q = tid; q < kFeatRays * kAppDim; q += 256) {
      const int ray = q / kAppDim, k = q % kAppDim;
      const int64_t row = app_rows == 1 ? 0 : imin64(r0 + ray, R - 1);
      apps[ray][k] = app[row * kAppDim + k];
    }
  }
  __syncthreads();
  const int n = tid;
  float acc[kFeatRays];
  if (n < kDirHidden) {
    const float* w = packed + kOffDirWd + n * kDirEnc;
    const float b = packed[kOffDirB + n];
#pragma unroll
    for (int ray = 0; ray < kFeatRays; ++ray) acc[ray] = b;
    for (int k = 0; k < kDirEnc; ++k) {
      const float wk = w[k];
#pragma unroll
      for (int ray = 0; ray < kFeatRays; ++ray) acc[ray] = fmaf(wk, enc[ray][k], acc[ray]);
    }
  } else {
    const int m = n - kDirHidden;
    const float* w = packed + kOffAppW + m * kAppDim;
    const float b = app_rows > 0 ? packed[kOffAppB + m] : 0.0f;
#pragma unroll
    for (int ray = 0; ray < kFeatRays; ++ray) acc[ray] = b;
    if (app_rows > 0) {
      for (int k = 0; k < kAppDim; ++k) {
        const float wk = w[k];
#pragma unroll
        for (int ray = 0; ray < kFeatRays; ++ray) acc[ray] = fmaf(wk, apps[ray][k], acc[ray]);
      }
    }
  }
#pragma unroll
  for (int ray = 0; ray < kFeatRays; ++ray)
    if (r0 + ray < R) feat[(r0 + ray) * kRayFeat + n] = acc[ray];
}

int launch_ray_features(const float* packed, const float* dirs, int64_t R, const float* app,
                        int64_t app_rows, float* feat, hipStream_t s) {
  if (R == 0) return NERF_OK;
  hipLaunchKernelGGL(ray_features_kernel, dim3((unsigned)((R + kFeatRays - 1) / kFeatRays)), dim3(256), 0, s,
                     packed, dirs, R, app, app_rows, feat);
  return check_launch("ray_features_kernel");
}

}  // namespace nerf
