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
// No tile epilogue: each output tile starts with one MFMA that writes its bias into every
// column (A = bias, B = 1 on lane half 0 / 0 on half 1, C = 0: exact), then accumulates its
// k-steps in place; ReLU is applied by the CONSUMER when it reads a register as a B operand
// (one v_max per k-step, shared by the MFMAs of four tiles, issued in the MFMA shadow).  Four
// output tiles are accumulated together, their MFMAs interleaved, so consecutive MFMAs are
// independent (one dependent 32x32x2 f32 chain issues at ~90 % of peak, four at ~98 %:
// profiles/r01_mfma_f32_rate_microbench.log).
//
// Bound: MFMA.  1,048,832 algorithmic FLOP per sample; the kernel
// issues 8,192 MFMAs of 4,096 FLOP per 32 samples (63->64 and 319->320 input padding).
#include "common.h"

namespace nerf {

#ifdef NERF_MLP_STAMPS   // diagnostic build (scripts/microbench/mlp_stamps.hip): per-wave segment clocks
__device__ unsigned long long nerf_stamps[65536][12];
#define NERF_STAMP(i)                                                                       \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long t_;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    const int64_t w_ = (int64_t)blockIdx.x * kMlpWaves + (threadIdx.x >> 6);           \
    if (w_ < 65536 && (threadIdx.x & 63) == 0) nerf_stamps[w_][i] = t_;                     \
  } while (0)
#else
#define NERF_STAMP(i) do {} while (0)
#endif

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

constexpr int kMlpWaves = 4;   // waves per workgroup (each wave is independent: no barriers, own LDS slice)

// One dense layer: NT output tiles of 32 neurons in groups of four, KS_ACT activation k-steps
// read from `in` (ReLU applied on read when RELU_IN) and KS_PE positional-encoding k-steps
// read from `pe`.  INIT: kBias = bias via one MFMA per tile, kPerLane = a per-sample vector
// loaded into the accumulator (the colour branch's per-ray feature), kAccum = accumulate onto
// `out` (the skip layer's PE slice).  Outputs are pre-activations.  Weight fragments stream
// from L2 through a register ring DEPTH blocks deep (1 KiB per block per wave), in the order
// they are consumed (tile group, k-quad, tile), and the ring runs across layers: on entry it
// holds this matrix's first DEPTH blocks of that order, and the last DEPTH loads fetch the
// first blocks of `next` (the last matrix passes any valid fragment array; those loads go
// unused; next_ksq is its k-quad count), so no layer starts on an L2 round trip.
constexpr int kDepth = 8;   // weight-fragment blocks in flight per wave
enum Init { kBias, kPerLane, kAccum };

// packed block index (layout.h frag_elem / 256) of the g-th block of the consumption order
template <int NT, int KSQ>
__device__ __forceinline__ constexpr int stream_block(int g) {
  return ((g / (4 * KSQ)) * 4 + g % 4) * KSQ + (g / 4) % KSQ;
}

template <int NT, int KSQ>
__device__ __forceinline__ void ring_fill(f32x4 (&ring)[kDepth], const float* __restrict__ wmat, int lane) {
  const f32x4* __restrict__ wf = reinterpret_cast<const f32x4*>(wmat) + lane;
#pragma unroll
  for (int p = 0; p < kDepth; ++p) ring[p] = wf[stream_block<NT, KSQ>(p) * 64];
}

template <int NT, int KS_ACT, int KS_PE, int INIT, bool RELU_IN>
__device__ __forceinline__ void dense(const float* __restrict__ wmat, const float* __restrict__ next, int next_ksq,
                                      f32x4 (&ring)[kDepth], const float* __restrict__ init,
                                      const f32x16 (&in)[8], const float (&pe)[kPeSteps],
                                      f32x16 (&out)[8], int lane) {
  constexpr int KS = KS_ACT + KS_PE;
  constexpr int KSQ = KS / 4;
  constexpr int G = NT * KSQ;
  constexpr int DEPTH = kDepth;
  static_assert(NT % 4 == 0 && G >= DEPTH && DEPTH % 4 == 0, "ring/tile-group geometry");
  const int h = lane >> 5;
  const f32x4* __restrict__ wf = reinterpret_cast<const f32x4*>(wmat) + lane;
  const f32x4* __restrict__ nf = reinterpret_cast<const f32x4*>(next) + lane;
  const float one_h0 = h ? 0.0f : 1.0f;
  float bias_v[4];
  if constexpr (INIT == kBias) {
#pragma unroll
    for (int i = 0; i < 4; ++i) bias_v[i] = init[i * 32 + (lane & 31)];
  }
  static_for<G / 4>([&](auto sc) __attribute__((always_inline)) {
    constexpr int st = decltype(sc)::value;          // one k-quad of one tile group: 4 blocks
    constexpr int grp = st / KSQ, kq = st % KSQ;
    if constexpr (kq == 0) {
      static_for<4>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        constexpr int t = 4 * grp + i;
        if constexpr (INIT == kBias) out[t] = mfma32(bias_v[i], one_h0, f32x16{});
        else if constexpr (INIT == kPerLane) out[t] = load_rows(init, t, h);
      });
      if constexpr (INIT == kBias && grp + 1 < NT / 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) bias_v[i] = init[(4 * (grp + 1) + i) * 32 + (lane & 31)];
      }
    }
    static_for<4>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      constexpr int ks = 4 * kq + j;
      float b;
      if constexpr (ks < KS_ACT) {
        b = in[ks >> 4][ks & 15];
        if constexpr (RELU_IN) b = fmaxf(b, 0.0f);
      } else {
        b = pe[ks - KS_ACT];
      }
      static_for<4>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        out[4 * grp + i] = mfma32(ring[(4 * st + i) % DEPTH][j], b, out[4 * grp + i]);
      });
    });
    // refill the four slots just consumed
    static_for<4>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      constexpr int g = 4 * st + i;
      if constexpr (g + DEPTH < G) ring[g % DEPTH] = wf[stream_block<NT, KSQ>(g + DEPTH) * 64];
      else ring[g % DEPTH] = nf[(((g + DEPTH - G) % 4) * next_ksq + (g + DEPTH - G) / 4) * 64];
    });
    // keep the ring's issue order: without this the scheduler hoists the layer's weight
    // loads and runs out of registers
    __builtin_amdgcn_sched_barrier(0);
  });
}

// Training: store ReLU(tile) of an 8-tile activation set into the sample's save row at `off`
// (row: the sample's place in its tile-major block, layout.h).
__device__ __forceinline__ void save_tiles(float* __restrict__ row, int off, const f32x16 (&t8)[8], int ntiles,
                                           int h, bool valid) {
  if (!valid) return;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    if (t >= ntiles) break;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(t8[t][4 * q + e], 0.0f);
      *reinterpret_cast<f32x4*>(row + tile_col(off + t * 32 + 8 * q) + 4 * h) = v;
    }
  }
}

// SAVE = the training forward: also writes the per-sample activation row (layout.h kSave*) to
// `save` (M x kSaveRow); encd (R x 32) holds each ray's PE_4(d) from nerf_ray_features.
template <bool SAVE>
__global__ void __launch_bounds__(64 * kMlpWaves, 1)
mlp_kernel(const float* __restrict__ packed, const float* __restrict__ orig, const float* __restrict__ dirs,
           const float* __restrict__ zv, int64_t M, int N, const float* __restrict__ feat,
           float* __restrict__ rgb, float* __restrict__ sigma, const int* __restrict__ out_slot, int out_T,
           float* __restrict__ save, const float* __restrict__ encd) {
  const int lane = threadIdx.x & 63;
  const int64_t s0 = ((int64_t)blockIdx.x * kMlpWaves + (threadIdx.x >> 6)) * 32;
  if (s0 >= M) return;
  const int h = lane >> 5;
  const int64_t s = imin64(s0 + (lane & 31), M - 1);
  const int64_t r = s / N;
  NERF_STAMP(0);

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
  __shared__ float pe_lds[kMlpWaves][kPeSteps][64];
  float (*pe_mine)[64] = pe_lds[threadIdx.x >> 6];
  float pe[kPeSteps];
#pragma unroll
  for (int i = 0; i < kPosLevels; ++i) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float sn, cs;
      sincosf(x[c] * (float)(1 << i), &sn, &cs);
      pe[3 * i + c] = h ? cs : sn;
    }
  }
  pe[30] = h ? x[1] : x[0];
  pe[31] = h ? 0.0f : x[2];
#pragma unroll
  for (int p = 0; p < kPeSteps; ++p) pe_mine[p][lane] = pe[p];
  const bool valid = s0 + (lane & 31) < M;
  float* srow = SAVE ? save + (s / 32) * 32 * kSaveRow + (s % 32) * 8 : nullptr;   // tile-major (layout.h)
  if constexpr (SAVE) {
    if (valid) {
#pragma unroll
      for (int p = 0; p < kPeSteps; ++p) {
        const int f = pe_feature(p, h);
        const int F = kSaveEncX + (f < 0 ? kPosEnc : f);
        srow[tile_col(F) + F % 8] = f < 0 ? 0.0f : pe[p];
      }
      if (N < kEncDPerRayMinN || s == r * N) {   // enc_d: per ray (layout.h kEncDPerRayMinN)
        const f32x4* ed = reinterpret_cast<const f32x4*>(encd + r * 32 + 16 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int F = kSaveEncD + 16 * h + 4 * q;
          *reinterpret_cast<f32x4*>(srow + tile_col(F) + F % 8) = ed[q];
        }
      }
    }
  }

  NERF_STAMP(1);
  const float* bias = packed + kOffBias;
  const float* wtrunk = packed + frag_offset(1);                 // layers 1..7, frag_floats(1) apart
  auto wlayer = [&](int m) { return wtrunk + (size_t)(m - 1) * frag_floats(1); };
  const float* wskip = packed + frag_offset(kSkipPeMat);
  constexpr int Q_ACT = kActSteps / 4, Q_PE = kPeSteps / 4;
  f32x4 ring[kDepth];
  ring_fill<8, Q_PE>(ring, packed + frag_offset(0), lane);
  f32x16 A[8], B[8];
  // layer 0: PE(63) -> 256 (pre-activations in A)
  dense<8, 0, kPeSteps, kBias, false>(packed + frag_offset(0), wlayer(1), Q_ACT, ring, bias, A, pe, A, lane);
  if constexpr (SAVE) save_tiles(srow, save_h(0), A, 8, h, valid);
  NERF_STAMP(2);
  // layers 1..6 as three A->B->A pairs; the skip layer 4 accumulates its PE slice onto its
  // pre-activations (models.py:130-131).  Every layer reads ReLU(previous) as its input.
#pragma unroll 1
  for (int p = 0; p < 3; ++p) {
    const int m1 = 1 + 2 * p, m2 = 2 + 2 * p;
    const bool skip = m2 == kSkipLayer;
    dense<8, kActSteps, 0, kBias, true>(wlayer(m1), wlayer(m2), Q_ACT, ring, bias + m1 * kHidden, A, pe, B, lane);
    if constexpr (SAVE) save_tiles(srow, save_h(m1), B, 8, h, valid);
    NERF_STAMP(3 + 2 * p);
    dense<8, kActSteps, 0, kBias, true>(wlayer(m2), skip ? wskip : wlayer(m2 + 1), skip ? Q_PE : Q_ACT, ring,
                                        bias + m2 * kHidden, B, pe, A, lane);
    if (skip) {
      float pe2[kPeSteps];
#pragma unroll
      for (int q = 0; q < kPeSteps; ++q) pe2[q] = pe_mine[q][lane];
      dense<8, 0, kPeSteps, kAccum, false>(wskip, wlayer(m2 + 1), Q_ACT, ring, bias, A, pe2, A, lane);
    }
    if constexpr (SAVE) save_tiles(srow, save_h(m2), A, 8, h, valid);
    NERF_STAMP(4 + 2 * p);
  }
  // layer 7: A -> B; B holds h7's pre-activations
  dense<8, kActSteps, 0, kBias, true>(wlayer(7), packed + frag_offset(8), Q_ACT, ring, bias + 7 * kHidden, A, pe, B,
                                      lane);
  if constexpr (SAVE) save_tiles(srow, save_h(7), B, 8, h, valid);
  NERF_STAMP(9);

  // density head: sigma = ReLU(density_head(ReLU(h7))) (models.py:137-138).
  const float* ws = packed + kOffSigmaW;
  float part = 0.0f;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(ws + t * 32 + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) part = fmaf(w[e], fmaxf(B[t][4 * q + e], 0.0f), part);
    }
  const float sig = fmaxf(part + __shfl_xor(part, 32) + packed[kOffSigmaB], 0.0f);

  // colour branch: h_dir = ReLU(W_dh ReLU(h7) + [b_dir + W_dd PE(d)]) + appearance
  // (models.py:141-156), the bracket and the appearance part precomputed per ray in `feat`.
  const float* fr = feat + r * kRayFeat;
  dense<4, kActSteps, 0, kPerLane, true>(packed + frag_offset(8), packed + frag_offset(8), Q_ACT, ring, fr, B, pe, A,
                                         lane);
  NERF_STAMP(10);
  if constexpr (SAVE) save_tiles(srow, kSaveRDir, A, 4, h, valid);
  float pr[3] = {0.0f, 0.0f, 0.0f};
  const float* wr = packed + kOffRgbW;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f32x16 app = load_rows(fr + kDirHidden, t, h);
    if constexpr (SAVE) {
      if (valid) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(A[t][4 * q + e], 0.0f) + app[4 * q + e];
          *reinterpret_cast<f32x4*>(srow + tile_col(kSaveHd + t * 32 + 8 * q) + 4 * h) = v;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const f32x4 w = *reinterpret_cast<const f32x4*>(wr + c * kDirHidden + t * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) pr[c] = fmaf(w[e], fmaxf(A[t][4 * q + e], 0.0f) + app[4 * q + e], pr[c]);
      }
    }
  }
  float out[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = pr[c] + __shfl_xor(pr[c], 32) + packed[kOffRgbB + c];
    out[c] = 1.0f / (1.0f + expf_rn(-v));                           // sigmoid (models.py:159-160)
  }
  if (h == 0 && s0 + (lane & 31) < M) {
    const int64_t o_s = out_slot ? r * out_T + out_slot[s] : s;
    sigma[o_s] = sig;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[3 * o_s + c] = out[c];
  }
  NERF_STAMP(11);
}

int launch_mlp(const float* packed, const float* o, const float* d, const float* z, int64_t R, int N,
               const float* feat, float* rgb, float* sigma, const int* out_slot, int out_T, hipStream_t s,
               float* save, const float* encd, uint32_t* masks) {
  const int64_t M = R * (int64_t)N;
  if (M == 0) return NERF_OK;
  if (g_mlp_arith == NERF_ARITH_F16X3)
    return launch_mlp16(packed, o, d, z, R, N, feat, rgb, sigma, out_slot, out_T, s, save, encd, masks);
  constexpr int per_block = 32 * kMlpWaves;
  const int64_t blocks = (M + per_block - 1) / per_block;
  // tile-major save rows: the last block's rows past M are zeros (layout.h)
  if (save && M % 32 && hipMemsetAsync(save + (M / 32) * 32 * kSaveRow, 0, (size_t)32 * kSaveRow * 4, s) != hipSuccess)
    return set_error(NERF_ERR_HIP, "mlp training forward: hipMemsetAsync failed");
  if (save)
    hipLaunchKernelGGL(mlp_kernel<true>, dim3((unsigned)blocks), dim3(64 * kMlpWaves), 0, s, packed, o, d, z, M, N,
                       feat, rgb, sigma, out_slot, out_T, save, encd);
  else
    hipLaunchKernelGGL(mlp_kernel<false>, dim3((unsigned)blocks), dim3(64 * kMlpWaves), 0, s, packed, o, d, z, M,
                       N, feat, rgb, sigma, out_slot, out_T, nullptr, nullptr);
  return check_launch("mlp_kernel");
}

// -------------------------------------------------------------------------- ray features
// Per ray: feat[0:128] = dir_linear.bias + dir_linear.weight[:,256:283] . PE_4(d)
//          feat[128:256] = appearance_projection(app) or 0.
// A block handles kFeatRays = 64 rays: the 64x27 direction encodings and 64x32 appearance rows
// are staged in LDS, then thread n holds row n of its weight matrix in registers and computes
// output n for all 64 rays (LDS broadcast reads, coalesced 1 KiB stores per ray).  (16 rays per
// block re-read the weight rows, strided across threads, every 16 rays: 0.38 ms for the 800^2
// frame's 640,000 rays, 1.7 TB/s.)  A small batch (the training step's 4,096 rays: 64 blocks, each
// thread's 64-ray chain latency-bound, 23 us) runs 16 rays per block instead: 4x the blocks, a
// quarter of the chain, the same fmaf order per output (bit-identical).
constexpr int kFeatRays = 64;
constexpr int kFeatRaysSmall = 16;
constexpr int64_t kFeatSmallMaxRays = 65536;   // up to 4,096 blocks of 16 rays

// dn_out (nullable): the input directions are raw and normalised here first (render.py:19, the
// expression of normalize_kernel), written to dn_out for the MLP: one launch fewer per call.
template <int RAYS>
__global__ void __launch_bounds__(256)
ray_features_kernel(const float* __restrict__ packed, const float* __restrict__ dirs, int64_t R,
                    const float* __restrict__ app, int64_t app_rows, float* __restrict__ feat,
                    float* __restrict__ encd, float* __restrict__ dn_out) {
  __shared__ float enc[RAYS][kDirEnc + 1];
  __shared__ float apps[RAYS][kAppDim];
  __shared__ float dsh[RAYS][3];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * RAYS;
  if (tid < RAYS) {
    const int64_t r = imin64(r0 + tid, R - 1);
    float x = dirs[3 * r], y = dirs[3 * r + 1], z = dirs[3 * r + 2];
    if (dn_out) {
      const float n = fmaxf(sqrtf(fmaf(z, z, fmaf(y, y, x * x))), 1e-12f);
      x = x / n;
      y = y / n;
      z = z / n;
      if (r0 + tid < R) {
        dn_out[3 * r] = x;
        dn_out[3 * r + 1] = y;
        dn_out[3 * r + 2] = z;
      }
    }
    dsh[tid][0] = x;
    dsh[tid][1] = y;
    dsh[tid][2] = z;
  }
  __syncthreads();
  for (int q = tid; q < RAYS * 3 * kDirLevels; q += 256) {
    const int ray = q / (3 * kDirLevels), ic = q % (3 * kDirLevels);
    const int i = ic / 3, c = ic % 3;
    float sn, cs;
    sincosf(dsh[ray][c] * (float)(1 << i), &sn, &cs);
    enc[ray][3 + 6 * i + c] = sn;
    enc[ray][6 + 6 * i + c] = cs;
  }
  if (tid < RAYS * 3) {
    const int ray = tid / 3, c = tid % 3;
    enc[ray][c] = dsh[ray][c];
  }
  if (app_rows > 0) {
    for (int q = tid; q < RAYS * kAppDim; q += 256) {
      const int ray = q / kAppDim, k = q % kAppDim;
      const int64_t row = app_rows == 1 ? 0 : imin64(r0 + ray, R - 1);
      apps[ray][k] = app[row * kAppDim + k];
    }
  }
  __syncthreads();
  if (encd) {   // training: each ray's PE_4(d), padded to 32
    for (int q = tid; q < RAYS * 32; q += 256) {
      const int ray = q / 32, k = q % 32;
      if (r0 + ray < R) encd[(r0 + ray) * 32 + k] = k < kDirEnc ? enc[ray][k] : 0.0f;
    }
  }
  const int n = tid;
  const int nr = (int)imin64(RAYS, R - r0);
  // the same fmaf chain per output as before: b, then k = 0, 1, ... in order
  if (n < kDirHidden) {
    float w[kDirEnc];
#pragma unroll
    for (int k = 0; k < kDirEnc; ++k) w[k] = packed[kOffDirWd + n * kDirEnc + k];
    const float b = packed[kOffDirB + n];
    for (int ray = 0; ray < RAYS; ray += 4) {   // 4 independent chains (rows past R: garbage, not stored)
      float acc[4] = {b, b, b, b};
#pragma unroll
      for (int k = 0; k < kDirEnc; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = fmaf(w[k], enc[ray + i][k], acc[i]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (ray + i < nr) feat[(r0 + ray + i) * kRayFeat + n] = acc[i];
    }
  } else {
    const int m = n - kDirHidden;
    const float b = app_rows > 0 ? packed[kOffAppB + m] : 0.0f;
    if (app_rows > 0) {
      float w[kAppDim];
#pragma unroll
      for (int k = 0; k < kAppDim; ++k) w[k] = packed[kOffAppW + m * kAppDim + k];
      for (int ray = 0; ray < RAYS; ray += 4) {
        float acc[4] = {b, b, b, b};
#pragma unroll
        for (int k = 0; k < kAppDim; ++k)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = fmaf(w[k], apps[ray + i][k], acc[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (ray + i < nr) feat[(r0 + ray + i) * kRayFeat + n] = acc[i];
      }
    } else {
      for (int ray = 0; ray < nr; ++ray) feat[(r0 + ray) * kRayFeat + n] = b;
    }
  }
}

int launch_ray_features(const float* packed, const float* dirs, int64_t R, const float* app,
                        int64_t app_rows, float* feat, hipStream_t s, float* encd, float* dn_out) {
  if (R == 0) return NERF_OK;
  if (R <= kFeatSmallMaxRays)
    hipLaunchKernelGGL(ray_features_kernel<kFeatRaysSmall>, dim3((unsigned)((R + kFeatRaysSmall - 1) / kFeatRaysSmall)),
                       dim3(256), 0, s, packed, dirs, R, app, app_rows, feat, encd, dn_out);
  else
    hipLaunchKernelGGL(ray_features_kernel<kFeatRays>, dim3((unsigned)((R + kFeatRays - 1) / kFeatRays)), dim3(256), 0,
                       s, packed, dirs, R, app, app_rows, feat, encd, dn_out);
  return check_launch("ray_features_kernel");
}

}  // namespace nerf
