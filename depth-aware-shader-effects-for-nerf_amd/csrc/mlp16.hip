// Fused positional encoding -> NeRF MLP forward on split-f16 MFMA ("f16x3") with the training saves
// (R4-R6 + §8f-2; reference src/models.py:105-162, :14-47): the forward of nerf_mlp_forward_train /
// nerf_train_forward.  Since round 6 the render calls run mlp16s_kernel (mlp16s.hip: the same
// arithmetic and weight stream on v_mfma_f32_16x16x32_f16), so this kernel is instantiated with
// SAVE = true only; its SAVE = false branches (the round-5 render kernel) are not compiled into the
// library, and the DESIGN §4 measurements of that kernel come from the round-5 sources (git history).
//
// Arithmetic.  Every dense layer out^T = W . in^T runs on v_mfma_f32_32x32x16_f16 as
//     hi(W) hi(a) + hi(W) lo(a) + lo(W) hi(a)       (f32 accumulation)
// with x*s = hi + lo + O(2^-24 |x*s|), hi = f16(x*s), lo = f16(x*s - hi), and s a power of two:
// per layer for W (packed, layout.h) and per SAMPLE for the activations.  A power-of-two scale
// of a column of B scales that column of the product exactly, so the accumulator holds
// s_w * s_j * (W a) and one multiply by the exact inverse recovers it.  The dropped lo*lo term
// and the split residual are both O(2^-24): the result has fp32-level error
// (tests/test_gpu_parity.py::test_forward_accuracy_vs_float64 measures it against float64 next
// to the exact-f32 kernel in mlp.hip), at 3 x 32 MFMA cycles per 16-deep k-step instead of the
// f32 instruction's 8 x 64.
//
// Scales from a bound, not a max.  Layer L+1's inputs y_L are split at s = 2^(14-e) with
// R_L max|a_L| + B_L < 2^e, where max|a_L| is the sample's largest input of layer L and R_L
// (max row L1 norm of W_L) and B_L (max |bias|) are pack-time constants: |y_L| <= R_L max|a_L|
// + B_L rigorously, so nothing overflows f16, and the scale is known before y_L exists.  (A
// loose bound only moves the split's absolute error floor, 2^-25 of the scaled unit, further
// below the sample's largest value.)  That lets outputs be converted tile by tile while MFMAs run:
//
// Schedule.  One wave owns 32 samples and runs the whole network for them; a layer's output
// tiles are the next layer's B operands in place (layout.h), so activations never leave
// registers.  A trunk layer's 8 tiles run as two groups of 4 over all k-steps.  The VALU
// epilogue of group A's outputs (unscale + bias, ReLU, split into the next layer's operands
// 0..7) runs in the MFMA shadow of group B's last 8 k-steps (operands 0..7 are dead by then);
// group B's epilogue (operands 8..15) runs in the shadow of the next layer's group A first 8
// k-steps, which read operands 0..7.  Only the prologue (PE) and the colour head stay exposed.
//
// Weight stream.  At 5.3x the f32 rate one wave would need ~21 B/clk of weights from L2, so the
// 4 waves of a workgroup share the stream: each 16 KiB chunk (2 k-steps x 4 tiles x {hi, lo}) is
// DMA'd once per workgroup (global_load_lds_dwordx4, a quarter by each wave) into a 4-slot LDS
// ring three chunks ahead, published by a counted vmcnt wait + barrier, and read back by all
// four waves with ds_read_b128 interleaved between the MFMAs.
#include "common.h"
#include "pe_sin.h"
#include "stream16.h"

namespace nerf {

#ifdef NERF_MLP16_STAMPS   // diagnostic build (scripts/microbench/mlp16_stamps.hip): per-wave segment clocks
__device__ unsigned long long nerf16_stamps[65536][16];
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

// ---- LDS: one __shared__ array (a second object can make hipcc drain the DMA before every
// ds_read).  [ring: 4 x 16 KiB][PE: 4 waves x 32 x 64][biases 8 x 256 | density_head w 256, b 4]
// [layer constants].  Every small vector the layers read sits here: an ordinary global load used
// while a DMA is in flight makes hipcc wait vmcnt(0), draining the stream.
constexpr int kLdsPe = 4 * kChunkFloats;
constexpr int kLdsBias = kLdsPe + kW16Waves * kPeSteps * 64;
constexpr int kLdsSigmaW = kLdsBias + 8 * kHidden;
constexpr int kLdsVecFloats = 8 * kHidden + kHidden + 4;    // kOffBias .. kOffSigmaB + 4, contiguous in `packed`
constexpr int kLdsConsts = kLdsBias + kLdsVecFloats;
constexpr int kLdsRgb = kLdsConsts + kS16Consts;             // rgb_linear weight (3 x 128) + bias (4)
constexpr int kLdsRgbFloats = 3 * kDirHidden + 4;
constexpr int kLdsFeat = kLdsRgb + kLdsRgbFloats;             // per wave: its ray's features (256)
constexpr int kLdsFloats = kLdsFeat + kW16Waves * kRayFeat;   // 111 KiB
// Training forward only: each wave's 32 ReLU-mask rows (layout.h kMaskRow words, 272 B per
// sample), accumulated by ds_or from the epilogue quarters and copied out at the end.
constexpr int kMaskWords = kMaskRow;                          // 68
constexpr int kLdsMask = kLdsFloats;
constexpr int kLdsFloatsSave = kLdsMask + kW16Waves * 32 * kMaskWords;   // 145 KiB
static_assert(kOffRgbB == kOffRgbW + 3 * kDirHidden && kLdsRgb % 4 == 0 && kLdsFeat % 4 == 0, "LDS vector layout");
static_assert(kOffSigmaW == kOffBias + 8 * kHidden && kOffSigmaB == kOffSigmaW + kHidden, "packed vector order");


// ---- epilogue pieces (the side work) ----------------------------------------------------------
// Quarter QG (0..15) of a 4-tile group = registers 4q..4q+3 (q = QG % 4) of output tile T0 + QG / 4
// -> elements 4(q & 1) .. +3 of the next layer's operand in[OP0 + QG / 2]:
//   y = acc*inv + bias, r = ReLU(y), op = split(r*s); m tracks max r; SIGMA adds ws . r to part.
// Phase 0 (load4) reads the quarter's bias (and density weights) from LDS into `qv`; phase 1
// (convert4) computes.
struct QuarterVec {
  f32x4 b, w;
};
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
struct SaveAt {      // training forward: where a layer's activations go (see convert4)
  __amdgpu_buffer_rsrc_t rows;   // the wave's 32 activation rows
  uint32_t loff;                 // this lane's byte offset in the wave's tile-major block: ((lane & 31) 8 + 4h) 4
  int hoff;                      // the layer's slice (floats), uniform
  bool valid;
  unsigned* mrow;                // this lane's mask words in LDS: the sample's row + 4h (words)
  int mlay;                      // the layer's words in the row: 8 * layer, uniform
};
// ReLU-mask bits of tile T (quarter q, element e -> bit 4q + e: neuron 32T + 8q + 4h + e) go to
// bits 16 (T % 2) of word T / 2 of the lane's 4-word (16-byte) slot of the layer: exactly the
// 128-bit mask the backward folds from the activations (train.hip dgrad16), so it loads one slot.
// One ds_or per quarter: no register lives across quarters.
__device__ __forceinline__ void mask_or(const SaveAt& sv, int T, uint32_t bits) {
  __hip_atomic_fetch_or(sv.mrow + sv.mlay + T / 2, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
// 16 bytes at byte offset voff + 4 * (hoff + c) of the wave's rows: a buffer store, so the lane's
// address stays one VGPR (store16_rows, common.h: the whole offset in the VGPR, soffset 0).
// (tile-major rows, layout.h: feature group c / 8 of the slice at hoff; c and hoff multiples of 8, so
// one store instruction writes the wave's 32 samples x 8 features, 1 KiB, contiguously)
__device__ __forceinline__ void save_store(const SaveAt& sv, int c, f32x4 v) {
  store16_rows<kRowStoreAux>(v, sv.rows, sv.loff + 4u * (uint32_t)tile_col(sv.hoff) + 4u * (uint32_t)tile_col(c));
}
template <int T0, int QG, bool SIGMA>
__device__ __forceinline__ void load4(const float* bias, const float* ws, int h, QuarterVec& qv) {
  constexpr int T = T0 + QG / 4, q = QG % 4;
  qv.b = *reinterpret_cast<const f32x4*>(bias + 32 * T + 8 * q + 4 * h);
  if constexpr (SIGMA) qv.w = *reinterpret_cast<const f32x4*>(ws + 32 * T + 8 * q + 4 * h);
}
// SV (training forward): also store ReLU(y) to the sample's activation row (SaveAt): neuron
// 32T + 8q + 4h + e of the layer's slice, the layout.h save order.
template <int T0, int OP0, int QG, bool SIGMA, bool SV>
__device__ __forceinline__ void convert4(const f32x16 (&acc)[8], float inv, const QuarterVec& qv, float s,
                                         Operand (&in)[16], float& m, float& part, const SaveAt& sv) {
  constexpr int T = T0 + QG / 4, q = QG % 4;
  constexpr int SH = 16 * (T % 2) + 4 * q;
  f32x4 rv;
  float xs[4];
  uint32_t bits = 0u;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float r = fmaxf(fmaf(acc[T][4 * q + e], inv, qv.b[e]), 0.0f);
    rv[e] = r;
    m = fmaxf(m, r);
    if constexpr (SIGMA) part = fmaf(qv.w[e], r, part);
    xs[e] = r * s;
    if constexpr (SV) bits |= (r > 0.0f ? 1u : 0u) << (SH + e);
    else split_into(xs[e], in[OP0 + QG / 2], 4 * (q & 1) + e);
  }
  if constexpr (SV) {   // split: hi pairs by v_cvt_pk_f16_f32, lo pairs by split_lo_pair
    Operand& op = in[OP0 + QG / 2];
    typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const h16x2 hi2 = {(_Float16)xs[2 * p], (_Float16)xs[2 * p + 1]};
      const h16x2 lo2 =
          __builtin_bit_cast(h16x2, split_lo_pair(__builtin_bit_cast(uint32_t, hi2), xs[2 * p], xs[2 * p + 1]));
      const int j = 4 * (q & 1) + 2 * p;
      op.hi[j] = hi2[0];
      op.hi[j + 1] = hi2[1];
      op.lo[j] = lo2[0];
      op.lo[j + 1] = lo2[1];
    }
  }
  if constexpr (SV) {
    save_store(sv, 32 * T + 8 * q, rv);     // tail lanes: offset past the buffer, dropped
    mask_or(sv, T, bits);
  }
}
// Phase PH of quarter QG (slot J of this half-step's quarter vectors).
template <int PH, int T0, int OP0, int QG, bool SIGMA, bool SV>
__device__ __forceinline__ void quarter(const f32x16 (&acc)[8], float inv, const float* bias, const float* ws, int h,
                                        float s, Operand (&in)[16], float& m, float& part, QuarterVec& qv,
                                        const SaveAt& sv) {
  if constexpr (PH == 0) load4<T0, QG, SIGMA>(bias, ws, h, qv);
  else convert4<T0, OP0, QG, SIGMA, SV>(acc, inv, qv, s, in, m, part, sv);
}

// PE operand Q split at scale s from this wave's LDS copy (layer 4 reads [h3, enc_x]): phase 0
// reads the 8 values into `v`, phase 1 splits them.
template <int PH, int Q>
__device__ __forceinline__ void pe_operand(const float* pe_mine, float s, Operand& op, float (&v)[8], int lane) {
  if constexpr (PH == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = pe_mine[(8 * Q + j) * 64 + lane];
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) split_into(v[j] * s, op, j);
  }
}


// SAVE = the training forward (nerf_mlp_forward_train): also writes each sample's activation row
// (layout.h kSave*: h_0..h_7 from the epilogue quarters, enc_x, enc_d, r_dir, hd from the heads)
// to `save` (M x kSaveRow); encd (R x 32) holds each ray's PE_4(d) from nerf_ray_features.
template <bool SAVE>
__global__ void __launch_bounds__(64 * kW16Waves, 1)
mlp16_kernel(const float* __restrict__ packed, const float* __restrict__ orig, const float* __restrict__ dirs,
             const float* __restrict__ zv, int64_t M, int N, const float* __restrict__ feat,
             float* __restrict__ rgb, float* __restrict__ sigma, const int* __restrict__ out_slot, int out_T,
             float* __restrict__ save, const float* __restrict__ encd, uint32_t* __restrict__ masks) {
  __shared__ __attribute__((aligned(16))) float lds[SAVE ? kLdsFloatsSave : kLdsFloats];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, h = lane >> 5;
  STAMP16(0);
  const int64_t s0 = ((int64_t)blockIdx.x * kW16Waves + wave) * 32;
  // every wave runs to the end (the weight stream has barriers); tail lanes repeat sample M-1
  const bool valid = s0 + (lane & 31) < M;
  const int64_t s = imin64(s0 + (lane & 31), M - 1);
  const int64_t r = s / N;
  // training: the wave's activation rows (uniform) and this lane's offset into them
  __amdgpu_buffer_rsrc_t wrows;
  if constexpr (SAVE)
    wrows = __builtin_amdgcn_make_buffer_rsrc(save + s0 * kSaveRow, (short)0, 32 * kSaveRow * 4, 0x00020000);
  // a tail lane's offset lies past the rows' buffer range, so its stores are dropped (no branch
  // inside the MFMA schedule)
  const uint32_t loff = valid ? ((uint32_t)(lane & 31) * 8 + 4 * h) * 4 : 0x40000000u;
  // training: this wave's mask rows in LDS, zeroed before the quarters OR their bits in
  unsigned* mwave = reinterpret_cast<unsigned*>(lds + kLdsMask) + wave * 32 * kMaskWords;
  unsigned* mrow = mwave + (lane & 31) * kMaskWords + 4 * h;
  if constexpr (SAVE) {
    for (int i = lane; i < 32 * kMaskWords; i += 64) mwave[i] = 0u;
  }

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
  // Small vectors into LDS, then the weight stream starts: chunks 0-2 in flight while the PE is
  // computed (every ordinary load retired first, see the LDS note).
  for (int i = threadIdx.x; i < kLdsVecFloats / 4; i += 64 * kW16Waves)
    reinterpret_cast<f32x4*>(lds + kLdsBias)[i] = reinterpret_cast<const f32x4*>(packed + kOffBias)[i];
  if (threadIdx.x < kS16Consts) lds[kLdsConsts + threadIdx.x] = packed[kOffScale16 + threadIdx.x];
  if (threadIdx.x < kLdsRgbFloats / 4)
    reinterpret_cast<f32x4*>(lds + kLdsRgb)[threadIdx.x] = reinterpret_cast<const f32x4*>(packed + kOffRgbW)[threadIdx.x];
  const int slot = out_slot && valid ? out_slot[s] : 0;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  const float* stream = packed + kOff16;
  const uint32_t lds_dma = (uint32_t)(uintptr_t)(lptr_t)lds + 1024u * wave;   // this wave's first piece
  const uint32_t voff = 16u * lane + 1024u * wave;
  chunk_dma<0>(stream, 0, lds_dma, voff);
  chunk_dma<1>(stream, 1, lds_dma, voff);
  chunk_dma<2>(stream, 2, lds_dma, voff);

  // PE in layout.h::pe_feature order (models.py:36-44): sin on lane half 0, cos on half 1.
  // pe_sin.h: one reduction + both polynomials per value; a wave with a coordinate beyond its
  // range (|x| 2^9 > kPeSinMax) takes the library sincosf.
  float pe[kPeSteps];
  const float ax = fmaxf(fabsf(x[0]), fmaxf(fabsf(x[1]), fabsf(x[2])));
  if (__any(ax * (float)(1 << (kPosLevels - 1)) > kPeSinMax)) {
#pragma unroll
    for (int i = 0; i < kPosLevels; ++i)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float sn, cs;
        sincosf(x[c] * (float)(1 << i), &sn, &cs);
        pe[3 * i + c] = h ? cs : sn;
      }
  } else {
#pragma unroll
    for (int i = 0; i < kPosLevels; ++i)
#pragma unroll
      for (int c = 0; c < 3; ++c) pe[3 * i + c] = pe_sin_reduced(x[c] * (float)(1 << i), h);
  }
  pe[30] = h ? x[1] : x[0];
  pe[31] = h ? 0.0f : x[2];
  float* pe_mine = lds + kLdsPe + wave * kPeSteps * 64;
#pragma unroll
  for (int p = 0; p < kPeSteps; ++p) pe_mine[p * 64 + lane] = pe[p];
  const float m_pe = fmaxf(1.0f, fmaxf(fabsf(x[0]), fmaxf(fabsf(x[1]), fabsf(x[2]))));   // bounds |PE|
  float rec_encx = 0.0f;    // training: the block exponent record of enc_x (entry 8, layout.h)
  if constexpr (SAVE) {
    float mx = 0.0f;
#pragma unroll
    for (int p = 0; p < kPeSteps; ++p) mx = fmaxf(mx, fabsf(pe[p]));
    rec_encx = block_exp_record(wave_max_nn(sample_max(mx)));
  }

  const float* bias = lds + kLdsBias;
  const float* ws = lds + kLdsSigmaW;
  const float* cst = lds + kLdsConsts;
  // s_cur: scale of the current layer's inputs; inv_cur unscales its accumulators; s_nxt: scale
  // of the next layer's inputs (from the bound on this layer's outputs).
  float s_cur = pow2_scale(m_pe);
  Operand pe_op[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) split_into(pe[8 * q + j] * s_cur, pe_op[q], j);

  wait_vmcnt<8>();                                          // this wave's part of chunk 0 (chunks 1-2 in flight)
  __builtin_amdgcn_s_barrier();
  h16x8 a0[4][2], a1[4][2];
  Operand in[16];
  read_kstep<0>(lds, a0, lane);

  f32x16 acc[8];
  float m = 0.0f, part = 0.0f;
  // training: lane j < 8 gathers the block exponent record of h_j, lane 8 holds enc_x's (layout.h)
  float bexp = (lane & 31) == 8 ? rec_encx : 0.0f;
  float inv_cur = cst[kS16InvW + 0] / s_cur;                // exact: powers of two
  float s_nxt = pow2_scale(cst[kS16R + 0] * m_pe + cst[kS16B + 0]);
  STAMP16(1);

  // ---- layer 0: PE(63) -> 256, 2 chunk-steps per group ----
  auto pe_operand_of = [&](auto i, auto kk) -> const Operand& { return pe_op[kstep_of(i, kk)]; };
  run_group<0, 2, 0, 3, kSideNone, SAVE>(stream, 0, lds, lds_dma, voff, a0, a1, acc, lane, pe_operand_of, NoSide{});
  // group B converts group A's outputs (tiles 0-3) into operands 0..7 (free: layer 0 reads the PE),
  // 4 quarters per half-step
  QuarterVec qv[4];
  float pe_v[8];
  SaveAt sv_prev{wrows, loff, save_h(0), valid, mrow, 0};   // training: save slices of y_{L-1}, y_L
  SaveAt sv_cur = sv_prev;
  run_group<1, 2, 2, 3, kSideL0, SAVE>(stream, 2, lds, lds_dma, voff, a0, a1, acc, lane, pe_operand_of,
                                       [&](auto i, auto kk, auto ph) __attribute__((always_inline)) {
                                         constexpr int hs = kstep_of(i, kk);
                                         static_for<4>([&](auto qc) __attribute__((always_inline)) {
                                           constexpr int j = decltype(qc)::value;
                                           quarter<decltype(ph)::value, 0, 0, 4 * hs + j, false, SAVE>(
                                               acc, inv_cur, bias, ws, h, s_nxt, in, m, part, qv[j], sv_cur);
                                         });
                                       });
  STAMP16(2);

  // ---- layers 1..7 ----
  // On entry to layer L: operands 0..7 hold y_{L-1} tiles 0-3 split at s_cur, y_{L-1} tiles 4-7
  // wait in acc[4..7], m holds the max of ReLU(y_{L-1}) tiles 0-3.
  //
  // Side-work schedule, by half-step hs of a group (one k-step), in quarter tiles (4 registers of a
  // tile, ~40 VALU instructions, spread over the half-step's 12 MFMA gaps):
  //  * group A converts y_{L-1} tiles 4-7 into operands 8..15: quarters 0, 1 at hs 0, quarter
  //    hs + 1 at hs 1..14.  Operand 8+j (quarters 2j, 2j+1) is complete at hs 2j and first read at
  //    hs 8+j; acc[4..7] is free again before group B;
  //  * group B converts this layer's y_L tiles 0-3 into operands 0..7: quarter hs - 1 at hs 1..14,
  //    quarters 14, 15 at hs 15.  Operand j was last read at hs j, and is next read at the next
  //    layer's hs j.
  float inv_prev = inv_cur;
  const float* bias_prev = bias;
  s_cur = s_nxt;
  auto act_operand = [&](auto i, auto kk) -> const Operand& { return in[kstep_of(i, kk)]; };
  auto op4 = [&](auto i, auto kk) -> const Operand& {
    constexpr int ks = kstep_of(i, kk);
    if constexpr (ks < 16) return in[ks];
    else return pe_op[ks - 16];
  };
  // group A's side: y_{L-1} tiles 4-7 (SIGMA: also the density head's dot product)
  auto side_prev = [&](auto i, auto kk, auto ph, auto sigma_tag) __attribute__((always_inline)) {
    constexpr int hs = kstep_of(i, kk), P = decltype(ph)::value;
    constexpr bool sg = decltype(sigma_tag)::value;
    if constexpr (hs == 0) {
      quarter<P, 4, 8, 0, sg, SAVE>(acc, inv_prev, bias_prev, ws, h, s_cur, in, m, part, qv[0], sv_prev);
      quarter<P, 4, 8, 1, sg, SAVE>(acc, inv_prev, bias_prev, ws, h, s_cur, in, m, part, qv[1], sv_prev);
    } else if constexpr (hs <= 14) {
      quarter<P, 4, 8, hs + 1, sg, SAVE>(acc, inv_prev, bias_prev, ws, h, s_cur, in, m, part, qv[0], sv_prev);
    }
  };
  // group B's side: this layer's y_L tiles 0-3
  auto side_cur = [&](auto i, auto kk, auto ph, const float* bias_l, auto sigma_tag) __attribute__((always_inline)) {
    constexpr int hs = kstep_of(i, kk), P = decltype(ph)::value;
    constexpr bool sg = decltype(sigma_tag)::value;
    if constexpr (hs >= 1 && hs <= 14) {
      quarter<P, 0, 0, hs - 1, sg, SAVE>(acc, inv_cur, bias_l, ws, h, s_nxt, in, m, part, qv[0], sv_cur);
    } else if constexpr (hs == 15) {
      quarter<P, 0, 0, 14, sg, SAVE>(acc, inv_cur, bias_l, ws, h, s_nxt, in, m, part, qv[0], sv_cur);
      quarter<P, 0, 0, 15, sg, SAVE>(acc, inv_cur, bias_l, ws, h, s_nxt, in, m, part, qv[1], sv_cur);
    }
  };
  using NoSigma = std::false_type;
  using Sigma = std::true_type;
  // One trunk layer (SKIP: layer 4 reads [h3, enc_x], 10 chunk-steps per group; SG: layer 7 starts
  // the density head).  Layers 1-3 and 5-6 run as loops of the plain body, layers 4 and 7 on their
  // own: one body with the variants behind runtime branches spilled 16 VGPRs in the training forward
  // (the register allocator serves every variant's live ranges at the loop's back edge).
  auto layer = [&](int L, auto skip_tag, auto sg_tag) __attribute__((always_inline)) {
    constexpr bool SKIP = decltype(skip_tag)::value;
    inv_cur = cst[kS16InvW + L] / s_cur;
    const float* bias_l = bias + L * kHidden;
    const int c0 = s16_chunk0(1) + (L - 1) * 16 + (L > kSkipLayer ? 4 : 0);
    if constexpr (SAVE) {
      sv_prev.hoff = save_h(L - 1);
      sv_cur.hoff = save_h(L);
      sv_prev.mlay = (kMaskLayerBytes / 4) * (L - 1);
      sv_cur.mlay = (kMaskLayerBytes / 4) * L;
    }
    // group A (k-steps 0..15, + PE 16..19 at layer 4)
    if constexpr (SKIP) {
      // layer 4 reads [h3, enc_x]: its PE operands are split at s_cur at hs 15..18 (PE operand q is
      // read at hs 16 + q)
      run_group<0, 10, 0, 3, kSideSkipPrev, SAVE>(stream, c0, lds, lds_dma, voff, a0, a1, acc, lane, op4,
                                            [&](auto i, auto kk, auto ph) __attribute__((always_inline)) {
                                              constexpr int hs = kstep_of(i, kk);
                                              side_prev(i, kk, ph, NoSigma{});
                                              if constexpr (hs >= 15 && hs < 19)
                                                pe_operand<decltype(ph)::value, hs - 15>(pe_mine, s_cur, pe_op[hs - 15],
                                                                                         pe_v, lane);
                                            });
    } else {
      run_group<0, 8, 0, 3, kSidePrev, SAVE>(stream, c0, lds, lds_dma, voff, a0, a1, acc, lane, act_operand,
                            [&](auto i, auto kk, auto ph) __attribute__((always_inline)) { side_prev(i, kk, ph, NoSigma{}); });
    }
    // the inputs of layer L are all known: the scale of layer L+1's inputs from the bound on y_L
    m = sample_max(m);
    if constexpr (SAVE) {   // m = the sample's max of h_{L-1}: the wave's block exponent (uniform)
      const float rec = block_exp_record(wave_max_nn(m));
      bexp = (lane & 31) == L - 1 ? rec : bexp;
    }
    float bound = cst[kS16R + L] * (SKIP ? fmaxf(m, m_pe) : m) + cst[kS16B + L];
    if (L + 1 == kSkipLayer) bound = fmaxf(bound, m_pe);    // layer 4 splits the PE at the same scale
    s_nxt = pow2_scale(bound);
    m = 0.0f;
    // group B (layer 7 also starts the density head)
    if constexpr (SKIP) {
      run_group<1, 10, 2, 3, kSideCur, SAVE>(stream, c0 + 10, lds, lds_dma, voff, a0, a1, acc, lane, op4,
                             [&](auto i, auto kk, auto ph) __attribute__((always_inline)) { side_cur(i, kk, ph, bias_l, NoSigma{}); });
    } else {
      run_group<1, 8, 0, 3, kSideCur, SAVE>(stream, c0 + 8, lds, lds_dma, voff, a0, a1, acc, lane, act_operand,
                            [&](auto i, auto kk, auto ph) __attribute__((always_inline)) { side_cur(i, kk, ph, bias_l, sg_tag); });
    }
    inv_prev = inv_cur;
    bias_prev = bias_l;
    s_cur = s_nxt;
    STAMP16(2 + L);
  };
#pragma unroll 1
  for (int L = 1; L < kSkipLayer; ++L) layer(L, NoSigma{}, NoSigma{});
  layer(kSkipLayer, std::true_type{}, NoSigma{});
#pragma unroll 1
  for (int L = kSkipLayer + 1; L < 7; ++L) layer(L, NoSigma{}, NoSigma{});
  layer(7, NoSigma{}, Sigma{});

  // ---- colour layer: h7 -> 128 (one group, 8 chunk-steps); its side converts y_7 tiles 4-7 into
  // operands 8..15 and finishes the density head ----
  // When N is a multiple of 32 the wave's 32 samples lie on one ray: its 1 KiB of ray features
  // (b_dir + W_dd PE(d) | appearance) is DMA'd into this wave's LDS area while the colour layer
  // runs (the stream's last vmcnt(0) covers it), so the heads read LDS, not HBM.
  const bool one_ray = (N & 31) == 0;
  float* feat_mine = lds + kLdsFeat + wave * kRayFeat;
  if (one_ray) {
    const char* src = reinterpret_cast<const char*>(feat + (imin64(s0, M - 1) / N) * kRayFeat);   // tail waves: last ray
    const uint32_t dst = (uint32_t)(uintptr_t)(lptr_t)feat_mine;
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(16u * lane), "s"(src), "s"(dst)
        : "memory");
  }
  inv_cur = cst[kS16InvW + 8] / s_cur;
  if constexpr (SAVE) {
    sv_prev.hoff = save_h(7);
    sv_prev.mlay = (kMaskLayerBytes / 4) * 7;
  }
  run_group<0, 8, 0, 0, kSidePrev, SAVE>(stream, s16_chunk0(8), lds, lds_dma, voff, a0, a1, acc, lane, act_operand,
                        [&](auto i, auto kk, auto ph) __attribute__((always_inline)) { side_prev(i, kk, ph, Sigma{}); });
  STAMP16(10);
  if constexpr (SAVE) {     // h_7 (m: y_7 tiles 0-3 from layer 7's group B, tiles 4-7 from the colour layer's)
    const float rec = block_exp_record(wave_max_nn(sample_max(m)));
    bexp = (lane & 31) == 7 ? rec : bexp;
  }

  // density head: sigma = ReLU(density_head(ReLU(h7))) (models.py:137-138), f32.
  const float sig = fmaxf(part + __shfl_xor(part, 32) + ws[kHidden], 0.0f);
  // colour branch: h_dir = ReLU(W_dh ReLU(h7) + [b_dir + W_dd PE(d)]) + appearance
  // (models.py:141-156); the bracket and the appearance part come per ray in `feat`.
  const float* wr = lds + kLdsRgb;
  float pr[3] = {0.0f, 0.0f, 0.0f};
  auto colour_head = [&](const float* fr) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 fd = *reinterpret_cast<const f32x4*>(fr + t * 32 + 8 * q + 4 * h);
        const f32x4 ap = *reinterpret_cast<const f32x4*>(fr + kDirHidden + t * 32 + 8 * q + 4 * h);
        f32x4 rd, hd;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          rd[e] = fmaxf(fmaf(acc[t][4 * q + e], inv_cur, fd[e]), 0.0f);
          hd[e] = rd[e] + ap[e];
        }
        if constexpr (SAVE) {
          const SaveAt at{wrows, loff, 0, true, mrow, 0};
          save_store(at, kSaveRDir + t * 32 + 8 * q, rd);
          save_store(at, kSaveHd + t * 32 + 8 * q, hd);
          uint32_t bits = 0u;
#pragma unroll
          for (int e = 0; e < 4; ++e) bits |= (rd[e] > 0.0f ? 1u : 0u) << (16 * (t % 2) + 4 * q + e);
          // r_dir: 8 bytes per lane half at byte 256 + 8h of the row (mrow holds + 4h words)
          __hip_atomic_fetch_or(mrow - 2 * h + kMaskRDirByte / 4 + t / 2, bits, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(wr + c * kDirHidden + t * 32 + 8 * q + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) pr[c] = fmaf(w[e], hd[e], pr[c]);
        }
      }
  };
  if (one_ray) {
    wait_vmcnt<0>();
    colour_head(feat_mine);
  } else {
    colour_head(feat + r * kRayFeat);
  }
  if constexpr (SAVE) {   // the wave's 32 mask rows: 8,704 contiguous bytes in LDS and in `masks`
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int n16 = (int)imin64(M - s0, 32) * (kMaskWords / 4);
    u32x4v* dst = reinterpret_cast<u32x4v*>(masks + s0 * kMaskWords);
    for (int i = lane; i < n16; i += 64) dst[i] = reinterpret_cast<const u32x4v*>(mwave)[i];
  }
  float out[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = pr[c] + __shfl_xor(pr[c], 32) + wr[3 * kDirHidden + c];
    out[c] = 1.0f / (1.0f + expf_rn(-v));                           // sigmoid (models.py:159-160)
  }
  if constexpr (SAVE) {
    if (valid) {   // enc_x in the reference order (pe_feature; slot 63: the block exponents, layout.h), enc_d
      const float pad = (lane & 31) < 9 ? bexp : 0.0f;
#pragma unroll
      for (int p = 0; p < kPeSteps; ++p) {
        const int f = pe_feature(p, h);
        const int F = kSaveEncX + (f < 0 ? kPosEnc : f);
        static_assert(kSaveEncX + kPosEnc == kMetaSaveF, "enc_x's pad slot holds the block exponents");
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(f < 0 ? pad : pe_mine[p * 64 + lane]), wrows,
                                              (int)loff - 16 * h + 4 * (int)(tile_col(F) + F % 8), 0, 0);
      }
      if (N < kEncDPerRayMinN || s == r * N) {   // enc_d: per ray (layout.h kEncDPerRayMinN)
        const f32x4* ed = reinterpret_cast<const f32x4*>(encd + r * 32 + 16 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {   // features kSaveEncD + 16h + 4q .. +3 of the sample (tile-major: group, then 4 of its 8)
          const int F = kSaveEncD + 16 * h + 4 * q;
          store16_rows<0>(ed[q], wrows, loff - 16u * h + 4u * (uint32_t)(tile_col(F) + F % 8));
        }
      }
    }
  }
  if (h == 0 && valid) {
    const int64_t o_s = out_slot ? r * out_T + slot : s;
    sigma[o_s] = sig;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[3 * o_s + c] = out[c];
  }
  STAMP16(11);
}

int launch_mlp16(const float* packed, const float* o, const float* d, const float* z, int64_t R, int N,
                 const float* feat, float* rgb, float* sigma, const int* out_slot, int out_T, hipStream_t s,
                 float* save, const float* encd, uint32_t* masks) {
  const int64_t M = R * (int64_t)N;
  if (M == 0) return NERF_OK;
  constexpr int per_block = 32 * kW16Waves;
  const int64_t blocks = (M + per_block - 1) / per_block;
  if (save && !masks) return set_error(NERF_ERR_BAD_ARG, "mlp16 training forward: mask rows required");
  // tile-major save rows: the last block's rows past M are zeros (layout.h), its tail lanes store nothing
  if (save && M % 32 && hipMemsetAsync(save + (M / 32) * 32 * kSaveRow, 0, (size_t)32 * kSaveRow * 4, s) != hipSuccess)
    return set_error(NERF_ERR_HIP, "mlp16 training forward: hipMemsetAsync failed");
  if (!save) return launch_mlp16s(packed, o, d, z, R, N, feat, rgb, sigma, out_slot, out_T, s);
  hipLaunchKernelGGL(mlp16_kernel<true>, dim3((unsigned)blocks), dim3(64 * kW16Waves), 0, s, packed, o, d, z, M, N,
                     feat, rgb, sigma, out_slot, out_T, save, encd, masks);
  return check_launch("mlp16_kernel");
}

}  // namespace nerf
