// The render path's fused PE -> NeRF MLP forward (R4-R6; reference src/models.py:105-162, :14-47)
// on v_mfma_f32_16x16x32_f16: mlp16_kernel's split-f16 arithmetic ("f16x3", mlp16.hip) and weight
// stream (stream16.h, the same packed chunks), with 16 x 16 output tiles instead of 32 x 32.
//
// Why.  The MLP runs against the part's power limit, not its issue rate: mlp16_kernel
// holds 1.78-1.85 GHz.  The 16x16x32 instruction does the same FLOP in the same cycles per SIMD, but
// under that limit the chip holds it at a higher clock (MI355X_MICROARCH "DVFS give-back" 7; on the
// trunk's half-step with its side work, scripts/microbench/mfma_shape_side.hip measured +2-5 %,
// profiles/r02_mfma_shape_side.log).  This kernel serves the render calls (nerf_render_rays,
// nerf_mlp_forward); the training forward with saves and the data-gradient kernels keep the 32 x 32
// shape (their mask and save layouts follow it).
//
// Layout.  A wave still owns 32 samples and runs the whole network for them, as two sample tiles
// st = 0, 1 (samples 16 st + (lane & 15)).  Lane l sits in lane group g = l >> 4; per MFMA it supplies
// row / column l & 15 and the 8 k values 8g .. 8g+7 of a 32-deep k-step.
//  * Weights (A): a k-step of 32 is one stream chunk's two 16-deep k-steps.  mlp16's 1 KiB piece
//    (tile T of 32 rows, old k-step kk, hi or lo part) holds W[32T + (p & 31)][k-group p >> 5] in
//    lane p; the 16 x 32 fragment of row half r reads, in lane l, piece kk = g >> 1's lane
//    R_r(l & 15) + 32 (g & 1), with R_r(i) = (i & 7) + 8r + 16 (i >> 3): a per-lane LDS address, the
//    packed stream unchanged.
//  * Outputs: the 16 x 16 tile (T, r, st) holds neuron 32T + R_r(4g + e) of sample 16 st + (l & 15)
//    in lane l, register e: neuron 32T + 8r + 4 (g & 1) + 16 (g >> 1) + e.
//  * Activations (B): the next layer's 32-deep k-step T reads in lane l (sample tile st) elements
//    4r + e = tile (T, r, st)'s register e as it stands: exactly the input order mlp16's packed k
//    order gives the 16-deep k-steps 2T, 2T+1 (layout.h s16_source_col), so the operands are built
//    in place, as in mlp16.
//  * PE: lane group g = 2s + h supplies PE slot 8 (2t + s) + j of k-step t (sin for h = 0, cos for
//    h = 1, layout.h pe_feature): 16 of the sample's slots per lane, for each of its 2 samples.
// Each lane holds two samples: scales, maxima, the density dot product and the colour head are kept
// per sample tile, and a sample's maximum / sums run over its 4 lane groups (xor 16, xor 32).
//
// Weight stream (per 16 KiB chunk = one 32-deep k-step of a 4-tile group): 4 tile segments of 12
// MFMAs (2 row halves x 2 sample tiles x 3 products).  A tile's fragments (4: row half x hi/lo) are
// read into its own 16 registers one chunk ahead: tile 3's at the chunk's segment 0, tiles 0-2 of the
// next chunk in segments 1-3, each right after the registers' last MFMAs; the next chunk is published
// (counted vmcnt + barrier, as stream16.h) after segment 0 and the chunk three ahead is DMA'd in
// segments 1-3.  The previous layer's epilogue (the side work) runs a quarter (one 16 x 16 tile of one
// sample tile: 4 values) per segment in the MFMA shadow, on mlp16's group schedule.
#include "common.h"
#include "pe_sin.h"
#include "stream16.h"

namespace nerf {

__device__ __forceinline__ f32x4 mfma16s(h16x8 a, h16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// LDS: [ring 4 x 16 KiB][PE: 4 waves x 2 samples x 16 slots x 64 lanes][biases | density_head w, b]
// [layer constants][rgb_linear][per-wave ray features] (mlp16.hip's layout)
constexpr int kSLdsPe = 4 * kChunkFloats;
constexpr int kSLdsBias = kSLdsPe + kW16Waves * kPeSteps * 64;
constexpr int kSLdsSigmaW = kSLdsBias + 8 * kHidden;
constexpr int kSLdsVecFloats = 8 * kHidden + kHidden + 4;
constexpr int kSLdsConsts = kSLdsBias + kSLdsVecFloats;
constexpr int kSLdsRgb = kSLdsConsts + kS16Consts;
constexpr int kSLdsRgbFloats = 3 * kDirHidden + 4;
constexpr int kSLdsFeat = kSLdsRgb + kSLdsRgbFloats;
constexpr int kSLdsFloats = kSLdsFeat + kW16Waves * kRayFeat;
static_assert(kSLdsRgb % 4 == 0 && kSLdsFeat % 4 == 0, "LDS vector layout");

typedef h16x8 STile[2][2];   // a tile's fragments: [row half][hi, lo]
typedef f32x4 SAcc[8][2][2]; // [tile][row half][sample tile]

// Tile TI's 4 fragments of the chunk in `slot`: off[r] = the lane's float offset of row half r
template <int TI>
__device__ __forceinline__ void sread_tile(const float* slot, const uint32_t (&off)[2], STile& a) {
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int part = 0; part < 2; ++part)
      a[r][part] = __builtin_bit_cast(h16x8, *reinterpret_cast<const f32x4*>(slot + off[r] + TI * 512 + part * 256));
}

// Tile TI's 12 MFMAs: per (row half, sample tile) lo(W)hi(a), hi(W)lo(a), hi(W)hi(a) chained.
// hook(j) after chain j (the DMA pieces).
template <int G, int TI, bool FIRST, typename Hook>
__device__ __forceinline__ void smfma_tile(const STile& a, const Operand& b0, const Operand& b1, SAcc& acc,
                                           Hook&& hook) {
  static_for<4>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value, r = j >> 1, st = j & 1;
    const Operand& b = st ? b1 : b0;
    f32x4 c;
    if constexpr (FIRST) c = mfma16s(a[r][1], b.hi, f32x4{});
    else c = mfma16s(a[r][1], b.hi, acc[4 * G + TI][r][st]);
    c = mfma16s(a[r][0], b.lo, c);
    acc[4 * G + TI][r][st] = mfma16s(a[r][0], b.hi, c);
    hook(jc);
  });
}

// One tile segment: side work phase 0 (its LDS reads first), the fragment reads (NRD tiles' worth,
// `reads`), tile TI's MFMAs (+ hook), side phase 1, interleaved: per MFMA gap one MFMA, one DS read
// (gaps 1..4 per tile read), VPG VALU from gap kSValuGap0 on.  The side's VALU waits for its LDS reads
// (biases, density weights), issued at the segment's start; a 16x16x32 MFMA issues in half the cycles
// of a 32x32x16 one, so mlp16's gap 1 left them ~2 MFMAs of cover and the in-order wave stalled
// there with the MFMA pipe drained.  From gap 5 (7 gaps of VALU): +2.2-2.9 % frame rate, same box
// (gap 3 +1.9 %, 4 and 6 within 0.2 % of 5, 7 the same, 9 +1.2-2.5 %; profiles/r06/ab_render_vgap*.log).
constexpr int kSValuGap0 = 5;
template <int G, int TI, bool FIRST, int NRD, int VPG, typename Reads, typename Side, typename Hook>
__device__ __forceinline__ void ssegment(const STile& a, const Operand& b0, const Operand& b1, SAcc& acc, Reads&& reads,
                                         Side&& side, Hook&& hook) {
  side(std::integral_constant<int, 0>{});
  __builtin_amdgcn_sched_barrier(0);
  reads();
  smfma_tile<G, TI, FIRST>(a, b0, b1, acc, hook);
  side(std::integral_constant<int, 1>{});
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                        // 1 MFMA
    if (i >= 1 && i <= 4 * NRD) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
    if (VPG > 0 && i >= kSValuGap0) __builtin_amdgcn_sched_group_barrier(0x002, VPG, 0);   // VALU
  }
  __builtin_amdgcn_sched_barrier(0);
}

// Side-work schedules, by (chunk i of the group, segment): which quarter (or PE operand) runs there.
enum SSide { kSNone, kSPrev, kSCur, kSL0, kSSkipPrev, kSSkipCur };
// The skip layer's PE operands (k-steps 8, 9; two sample tiles each) are split from the wave's LDS
// copy just before each group reads them: k-step 8's in chunk 7 (segments 0, 2), 9's in chunk 8
// (segments 0, 2), so they hold registers only while read (the rest of the layer needs all of in[]).
__device__ __forceinline__ constexpr int spe_at(int i, int seg) {
  return (i == 7 || i == 8) && (seg == 0 || seg == 2) ? 2 * (i - 7) + seg / 2 : -1;   // operand 2 t + st
}
// group A's side (the previous layer's tiles 4-7, quarters 0..15): 3, 3, 2, 2, 2, 2, 2 per chunk
// (chunks 0..6; tile 4+j's quarters are done before chunk 4+j reads them).  Segments: three
// quarters in segments 1-3, two in 1 and 3.
__device__ __forceinline__ constexpr int sq_prev(int i, int seg) {
  constexpr int base[7] = {0, 3, 6, 8, 10, 12, 14};
  if (i >= 7) return -1;
  const int n = i < 2 ? 3 : 2;
  if (n == 3) return seg >= 1 ? base[i] + seg - 1 : -1;
  return seg == 1 ? base[i] : (seg == 3 ? base[i] + 1 : -1);
}
// group B's side (this layer's tiles 0-3, quarters 0..15): 0, 2, 2, 2, 2, 3, 3, 2 per chunk (tile T's
// quarters only after chunk T has read its operands)
__device__ __forceinline__ constexpr int sq_cur(int i, int seg) {
  constexpr int base[8] = {0, 0, 2, 4, 6, 8, 11, 14};
  constexpr int cnt[8] = {0, 2, 2, 2, 2, 3, 3, 2};
  if (i >= 8 || cnt[i] == 0) return -1;
  if (cnt[i] == 3) return seg >= 1 ? base[i] + seg - 1 : -1;
  return seg == 1 ? base[i] : (seg == 3 ? base[i] + 1 : -1);
}
template <int KIND>
__device__ __forceinline__ constexpr int side_count(int i, int seg) {
  if constexpr (KIND == kSPrev) return sq_prev(i, seg) >= 0;
  if constexpr (KIND == kSSkipPrev) return (sq_prev(i, seg) >= 0) + (spe_at(i, seg) >= 0);
  if constexpr (KIND == kSCur) return sq_cur(i, seg) >= 0;
  if constexpr (KIND == kSSkipCur) return (sq_cur(i, seg) >= 0) + (spe_at(i, seg) >= 0);
  if constexpr (KIND == kSL0) return 2;
  return 0;
}
template <int KIND>
__device__ __forceinline__ constexpr int svpg(int i, int seg) {
  const int n = side_count<KIND>(i, seg);
  return n == 0 ? 0 : (n * 40 + 11 - kSValuGap0) / (12 - kSValuGap0);   // ~40 VALU per quarter
}

// One chunk-step: chunk c (global index, ring slot SLOT) = k-step i of group G; b0 / b1 its sample
// tiles' operands.  On entry chunk c is published and tiles 0-2 of its fragments are in a[0..2].
// TAIL = chunks left after c (capped at 3).
template <int G, int SLOT, bool FIRST, int TAIL, int KIND, int I, typename Side>
__device__ __forceinline__ void schunk(const float* __restrict__ stream, int c, float* lds, uint32_t lds_dma,
                                       uint32_t voff, const uint32_t (&off)[2], STile (&a)[4], const Operand& b0,
                                       const Operand& b1, SAcc& acc, Side&& side) {
  const float* cur = lds + SLOT * kChunkFloats;
  const float* nxt = lds + ((SLOT + 1) & 3) * kChunkFloats;
  auto none = [](auto) {};
  auto sd = [&side](auto seg_c) __attribute__((always_inline)) {
    return [&side, seg_c](auto ph) __attribute__((always_inline)) { side(std::integral_constant<int, I>{}, seg_c, ph); };
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  using S3 = std::integral_constant<int, 3>;
  // segment 0: this chunk's tile 3 fragments (their registers' last MFMAs were the previous chunk's)
  ssegment<G, 0, FIRST, 1, svpg<KIND>(I, 0)>(a[0], b0, b1, acc, [&]() __attribute__((always_inline)) {
    sread_tile<3>(cur, off, a[3]);
  }, sd(S0{}), none);
  // publish chunk c+1: own DMA pieces landed (younger: chunk c+2's 4), barrier
  if constexpr (TAIL >= 1) {
    wait_vmcnt<TAIL >= 2 ? 4 : 0>();
    __builtin_amdgcn_s_barrier();
  }
  // DMA of chunk c+3 into the slot chunk c-1 used (every wave's reads of it fed MFMAs issued before
  // the barrier): pieces 0, 1 in segment 1, 2 and 3 in segments 2, 3, after a chain's MFMAs
  auto dma = [&](auto pc) __attribute__((always_inline)) {
    if constexpr (TAIL >= 3) chunk_dma_piece<(SLOT + 3) & 3, decltype(pc)::value>(stream, c + 3, lds_dma, voff);
  };
  ssegment<G, 1, FIRST, (TAIL >= 1), svpg<KIND>(I, 1)>(a[1], b0, b1, acc, [&]() __attribute__((always_inline)) {
    if constexpr (TAIL >= 1) sread_tile<0>(nxt, off, a[0]);
  }, sd(S1{}), [&](auto jc) __attribute__((always_inline)) {
    if constexpr (decltype(jc)::value == 0) dma(S0{});
    if constexpr (decltype(jc)::value == 2) dma(S1{});
  });
  ssegment<G, 2, FIRST, (TAIL >= 1), svpg<KIND>(I, 2)>(a[2], b0, b1, acc, [&]() __attribute__((always_inline)) {
    if constexpr (TAIL >= 1) sread_tile<1>(nxt, off, a[1]);
  }, sd(S2{}), [&](auto jc) __attribute__((always_inline)) {
    if constexpr (decltype(jc)::value == 0) dma(S2{});
  });
  ssegment<G, 3, FIRST, (TAIL >= 1), svpg<KIND>(I, 3)>(a[3], b0, b1, acc, [&]() __attribute__((always_inline)) {
    if constexpr (TAIL >= 1) sread_tile<2>(nxt, off, a[2]);
  }, sd(S3{}), [&](auto jc) __attribute__((always_inline)) {
    if constexpr (decltype(jc)::value == 0) dma(S3{});
  });
}

// A group of NSTEP chunk-steps from global chunk c0 (ring slot SLOT0); operand(i, st) gives k-step
// i's B operand of sample tile st.  TAIL_END = chunks after this group (capped at 3).
template <int G, int NSTEP, int SLOT0, int TAIL_END, int KIND, typename Opnd, typename Side>
__device__ __forceinline__ void sgroup(const float* __restrict__ stream, int c0, float* lds, uint32_t lds_dma,
                                       uint32_t voff, const uint32_t (&off)[2], STile (&a)[4], SAcc& acc,
                                       Opnd&& operand, Side&& side) {
  static_for<NSTEP>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    constexpr int left = NSTEP - 1 - i + TAIL_END;
    schunk<G, (SLOT0 + i) & 3, i == 0, (left < 3 ? left : 3), KIND, i>(
        stream, c0 + i, lds, lds_dma, voff, off, a, operand(ic, std::integral_constant<int, 0>{}),
        operand(ic, std::integral_constant<int, 1>{}), acc, side);
  });
}

// The sample's value over its 4 lane groups
__device__ __forceinline__ float smax4(float m) {
  m = fmaxf(m, __shfl_xor(m, 16));
  return fmaxf(m, __shfl_xor(m, 32));
}
__device__ __forceinline__ float ssum4(float v) {
  v = v + __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}

struct SQuarter {
  f32x4 b, w;
};

// Quarter QG (0..15) of the 4-tile group from tile T0: tile T = T0 + QG / 4, row half r and sample
// tile st = (QG % 4) >> 1, QG % 2 -> elements 4r .. 4r+3 of operand in[2T + st].  Phase 0 reads the
// bias (and density weights) from LDS, phase 1 converts: y = ReLU(acc inv + b), max, (SIGMA) density
// dot, split at the sample's scale.
template <int PH, int T0, int QG, bool SIGMA>
__device__ __forceinline__ void squarter(const SAcc& acc, const float (&inv)[2], const float* bias, const float* ws,
                                         int nlane, const float (&sc)[2], Operand (&in)[16], float (&m)[2],
                                         float (&part)[2], SQuarter& qv) {
  constexpr int T = T0 + QG / 4, r = (QG % 4) >> 1, st = QG & 1;
  const int n0 = 32 * T + 8 * r + nlane;
  if constexpr (PH == 0) {
    qv.b = *reinterpret_cast<const f32x4*>(bias + n0);
    if constexpr (SIGMA) qv.w = *reinterpret_cast<const f32x4*>(ws + n0);
  } else {
    float xs[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float y = fmaxf(fmaf(acc[T][r][st][e], inv[st], qv.b[e]), 0.0f);
      m[st] = fmaxf(m[st], y);
      if constexpr (SIGMA) part[st] = fmaf(qv.w[e], y, part[st]);
      xs[e] = y * sc[st];
    }
    Operand& op = in[2 * T + st];
    typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const h16x2 hi2 = {(_Float16)xs[2 * p], (_Float16)xs[2 * p + 1]};
      const h16x2 lo2 = __builtin_bit_cast(h16x2, split_lo_pair(__builtin_bit_cast(uint32_t, hi2), xs[2 * p], xs[2 * p + 1]));
      const int j = 4 * r + 2 * p;
      op.hi[j] = hi2[0];
      op.hi[j + 1] = hi2[1];
      op.lo[j] = lo2[0];
      op.lo[j + 1] = lo2[1];
    }
  }
}

// PE operand of k-step t, sample tile st, split at sc[st] from this wave's LDS copy: phase 0 reads the
// 8 values into v, phase 1 splits.
template <int PH, int t, int st>
__device__ __forceinline__ void spe_operand(const float* pe_mine, const float (&sc)[2], Operand& op, float (&v)[8],
                                            int lane) {
  if constexpr (PH == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = pe_mine[((st * 2 + t) * 8 + j) * 64 + lane];
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) split_into(v[j] * sc[st], op, j);
  }
}

__global__ void __launch_bounds__(64 * kW16Waves, 1)
mlp16s_kernel(const float* __restrict__ packed, const float* __restrict__ orig, const float* __restrict__ dirs,
              const float* __restrict__ zv, int64_t M, int N, const float* __restrict__ feat,
              float* __restrict__ rgb, float* __restrict__ sigma, const int* __restrict__ out_slot, int out_T) {
  __shared__ __attribute__((aligned(16))) float lds[kSLdsFloats];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int g = lane >> 4, li = lane & 15;
  const int64_t s0 = ((int64_t)blockIdx.x * kW16Waves + wave) * 32;
  // every wave runs to the end (the weight stream has barriers); tail lanes repeat sample M-1.  A
  // launch spans < 2^31 samples (capi.hip max_launch_samples): 32-bit sample and ray indices.
  const int mlast = (int)(M - 1);
  auto sample_of = [&](int st) { return imin64(s0 + 16 * st + li, (int64_t)mlast); };
  float x[2][3];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const int sm = (int)sample_of(st), ry = sm / N;
    if (zv) {   // pts = o + d*z with separate roundings (ray_utils.py:86)
      const float z = zv[sm];
#pragma unroll
      for (int c = 0; c < 3; ++c) x[st][c] = orig[3 * ry + c] + dirs[3 * ry + c] * z;
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) x[st][c] = orig[3 * sm + c];
    }
  }
  for (int i = threadIdx.x; i < kSLdsVecFloats / 4; i += 64 * kW16Waves)
    reinterpret_cast<f32x4*>(lds + kSLdsBias)[i] = reinterpret_cast<const f32x4*>(packed + kOffBias)[i];
  if (threadIdx.x < kS16Consts) lds[kSLdsConsts + threadIdx.x] = packed[kOffScale16 + threadIdx.x];
  if (threadIdx.x < kSLdsRgbFloats / 4)
    reinterpret_cast<f32x4*>(lds + kSLdsRgb)[threadIdx.x] = reinterpret_cast<const f32x4*>(packed + kOffRgbW)[threadIdx.x];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  const float* stream = packed + kOff16;
  const uint32_t lds_dma = (uint32_t)(uintptr_t)(lptr_t)lds + 1024u * wave;
  const uint32_t voff = 16u * lane + 1024u * wave;
  chunk_dma<0>(stream, 0, lds_dma, voff);
  chunk_dma<1>(stream, 1, lds_dma, voff);
  chunk_dma<2>(stream, 2, lds_dma, voff);

  // PE: lane group g = 2s + h computes slots 8 (2t + s) + j (t = 0, 1) of both its samples, sin for
  // h = 0 and cos for h = 1 (pe_feature; slot 30: x0 | x1, 31: x2 | 0).  Slot p < 30 is frequency
  // p / 3 of coordinate p % 3.  A wave with a coordinate beyond pe_sin.h's range takes sincosf.
  const int hh = g & 1, ss = g >> 1;
  float pe[2][2][8];
  float ax = 0.0f;
#pragma unroll
  for (int st = 0; st < 2; ++st) ax = fmaxf(ax, fmaxf(fabsf(x[st][0]), fmaxf(fabsf(x[st][1]), fabsf(x[st][2]))));
  auto pe_arg = [&](int st, int p) __attribute__((always_inline)) {
    const int fi = p / 3, fc = p - 3 * fi;
    const float xc = fc == 0 ? x[st][0] : (fc == 1 ? x[st][1] : x[st][2]);
    return xc * __int_as_float((127 + (fi < kPosLevels ? fi : 0)) << 23);   // x 2^fi, exact
  };
  auto pe_tail = [&](int st, int p, float v) __attribute__((always_inline)) {
    return p < 3 * kPosLevels ? v : (p == 30 ? (hh ? x[st][1] : x[st][0]) : (hh ? 0.0f : x[st][2]));
  };
  if (__any(ax * (float)(1 << (kPosLevels - 1)) > kPeSinMax)) {
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int p = 8 * (2 * t + ss) + j;
          float sn, cs;
          sincosf(pe_arg(st, p), &sn, &cs);
          pe[st][t][j] = pe_tail(st, p, hh ? cs : sn);
        }
  } else {
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int p = 8 * (2 * t + ss) + j;
          pe[st][t][j] = pe_tail(st, p, pe_sin_reduced(pe_arg(st, p), hh));
        }
  }
  float* pe_mine = lds + kSLdsPe + wave * kPeSteps * 64;
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) pe_mine[((st * 2 + t) * 8 + j) * 64 + lane] = pe[st][t][j];
  float m_pe[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) m_pe[st] = fmaxf(1.0f, fmaxf(fabsf(x[st][0]), fmaxf(fabsf(x[st][1]), fabsf(x[st][2]))));

  const float* bias = lds + kSLdsBias;
  const float* ws = lds + kSLdsSigmaW;
  const float* cst = lds + kSLdsConsts;
  float s_cur[2], inv_cur[2], s_nxt[2], inv_prev[2], m[2] = {0.0f, 0.0f}, part[2] = {0.0f, 0.0f};
  Operand pe_op[4];   // [t][st] -> 2 t + st
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    s_cur[st] = pow2_scale(m_pe[st]);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) split_into(pe[st][t][j] * s_cur[st], pe_op[2 * t + st], j);
  }
  // fragment offsets: row half r, lane l reads piece (g >> 1) lane R_r(l & 15) + 32 (g & 1)
  uint32_t off[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) off[r] = (uint32_t)(ss * 2048 + 4 * ((li & 7) + 8 * r + 16 * (li >> 3) + 32 * hh));
  const int nlane = 4 * hh + 16 * ss;   // this lane's neuron offset in a 16 x 16 output tile (+ 8r + e)

  wait_vmcnt<8>();                                          // this wave's part of chunk 0 (chunks 1-2 in flight)
  __builtin_amdgcn_s_barrier();
  STile a[4];
  sread_tile<0>(lds, off, a[0]);
  sread_tile<1>(lds, off, a[1]);
  sread_tile<2>(lds, off, a[2]);
  SAcc acc;
  Operand in[16];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    inv_cur[st] = cst[kS16InvW + 0] / s_cur[st];
    s_nxt[st] = pow2_scale(cst[kS16R + 0] * m_pe[st] + cst[kS16B + 0]);
  }
  SQuarter qv[2];
  float pe_v[8];
  auto pe_operand_of = [&](auto i, auto st) -> const Operand& {
    return pe_op[2 * decltype(i)::value + decltype(st)::value];
  };

  // ---- layer 0: PE (2 k-steps of 32) -> 256; group B converts group A's tiles 0-3 into in[0..7],
  // two quarters per segment
  sgroup<0, 2, 0, 3, kSNone>(stream, 0, lds, lds_dma, voff, off, a, acc, pe_operand_of,
                             [](auto, auto, auto) {});
  sgroup<1, 2, 2, 3, kSL0>(stream, 2, lds, lds_dma, voff, off, a, acc, pe_operand_of,
                           [&](auto i, auto seg, auto ph) __attribute__((always_inline)) {
                             constexpr int q0 = 8 * decltype(i)::value + 2 * decltype(seg)::value;
                             squarter<decltype(ph)::value, 0, q0, false>(acc, inv_cur, bias, ws, nlane, s_nxt, in, m,
                                                                         part, qv[0]);
                             squarter<decltype(ph)::value, 0, q0 + 1, false>(acc, inv_cur, bias, ws, nlane, s_nxt, in,
                                                                             m, part, qv[1]);
                           });

  // ---- layers 1..7 (mlp16's schedule; on entry in[0..7] hold y_{L-1} tiles 0-3 at s_cur, its tiles
  // 4-7 wait in acc[4..7], m the sample tiles' maxima of y_{L-1} tiles 0-3)
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    inv_prev[st] = inv_cur[st];
    s_cur[st] = s_nxt[st];
  }
  const float* bias_prev = bias;
  auto act_operand = [&](auto i, auto st) -> const Operand& { return in[2 * decltype(i)::value + decltype(st)::value]; };
  auto op4 = [&](auto i, auto st) -> const Operand& {
    constexpr int k = decltype(i)::value, t = decltype(st)::value;
    if constexpr (k < 8) return in[2 * k + t];
    else return pe_op[2 * (k - 8) + t];
  };
  auto side_prev = [&](auto i, auto seg, auto ph, auto sigma_tag) __attribute__((always_inline)) {
    constexpr int q = sq_prev(decltype(i)::value, decltype(seg)::value);
    if constexpr (q >= 0)
      squarter<decltype(ph)::value, 4, q, decltype(sigma_tag)::value>(acc, inv_prev, bias_prev, ws, nlane, s_cur, in, m,
                                                                       part, qv[0]);
  };
  auto side_cur = [&](auto i, auto seg, auto ph, const float* bias_l, auto sigma_tag) __attribute__((always_inline)) {
    constexpr int q = sq_cur(decltype(i)::value, decltype(seg)::value);
    if constexpr (q >= 0)
      squarter<decltype(ph)::value, 0, q, decltype(sigma_tag)::value>(acc, inv_cur, bias_l, ws, nlane, s_nxt, in, m,
                                                                      part, qv[1]);
  };
  // the skip layer's PE operands at layer 4's input scale (s_cur in group A, which group B keeps)
  float s_pe[2] = {0.0f, 0.0f};
  auto side_pe = [&](auto i, auto seg, auto ph) __attribute__((always_inline)) {
    constexpr int k = spe_at(decltype(i)::value, decltype(seg)::value);
    if constexpr (k >= 0) spe_operand<decltype(ph)::value, k / 2, k % 2>(pe_mine, s_pe, pe_op[k], pe_v, lane);
  };
  using NoSigma = std::false_type;
  using Sigma = std::true_type;
  // one trunk layer (SKIP: layer 4 reads [h3, enc_x], 10 chunk-steps per group; SG: layer 7 starts the
  // density head).  Layers 1-3 and 5-6 run as loops of the plain body, layers 4 and 7 on their own:
  // one body with the skip and sigma variants behind runtime branches spilled (the register
  // allocator then has to serve every variant's live ranges at the loop's back edge).
  auto layer = [&](int L, auto skip_tag, auto sg_tag) __attribute__((always_inline)) {
    constexpr bool SKIP = decltype(skip_tag)::value;
    constexpr bool SG = decltype(sg_tag)::value;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      inv_cur[st] = cst[kS16InvW + L] / s_cur[st];
      if constexpr (SKIP) s_pe[st] = s_cur[st];
    }
    const float* bias_l = bias + L * kHidden;
    const int c0 = s16_chunk0(1) + (L - 1) * 16 + (L > kSkipLayer ? 4 : 0);
    if constexpr (SKIP) {
      // layer 4 reads [h3, enc_x]: its PE operands (k-steps 8, 9) are split just before they are read
      sgroup<0, 10, 0, 3, kSSkipPrev>(stream, c0, lds, lds_dma, voff, off, a, acc, op4,
                                      [&](auto i, auto seg, auto ph) __attribute__((always_inline)) {
                                        side_prev(i, seg, ph, NoSigma{});
                                        side_pe(i, seg, ph);
                                      });
    } else {
      sgroup<0, 8, 0, 3, kSPrev>(stream, c0, lds, lds_dma, voff, off, a, acc, act_operand,
                                 [&](auto i, auto seg, auto ph) __attribute__((always_inline)) {
                                   side_prev(i, seg, ph, NoSigma{});
                                 });
    }
    // the inputs of layer L are known: the scale of layer L+1's inputs from the bound on y_L
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const float ms = smax4(m[st]);
      float bound = cst[kS16R + L] * (SKIP ? fmaxf(ms, m_pe[st]) : ms) + cst[kS16B + L];
      if (L + 1 == kSkipLayer) bound = fmaxf(bound, m_pe[st]);    // layer 4 splits the PE at the same scale
      s_nxt[st] = pow2_scale(bound);
      m[st] = 0.0f;
    }
    if constexpr (SKIP) {
      sgroup<1, 10, 2, 3, kSSkipCur>(stream, c0 + 10, lds, lds_dma, voff, off, a, acc, op4,
                                     [&](auto i, auto seg, auto ph) __attribute__((always_inline)) {
                                       side_cur(i, seg, ph, bias_l, NoSigma{});
                                       side_pe(i, seg, ph);
                                     });
    } else {
      sgroup<1, 8, 0, 3, kSCur>(stream, c0 + 8, lds, lds_dma, voff, off, a, acc, act_operand,
                                [&](auto i, auto seg, auto ph) __attribute__((always_inline)) {
                                  side_cur(i, seg, ph, bias_l, sg_tag);
                                });
    }
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      inv_prev[st] = inv_cur[st];
      s_cur[st] = s_nxt[st];
    }
    bias_prev = bias_l;
  };
#pragma unroll 1
  for (int L = 1; L < kSkipLayer; ++L) layer(L, NoSigma{}, NoSigma{});
  layer(kSkipLayer, Sigma{}, NoSigma{});
#pragma unroll 1
  for (int L = kSkipLayer + 1; L < 7; ++L) layer(L, NoSigma{}, NoSigma{});
  layer(7, NoSigma{}, Sigma{});

  // ---- colour layer: h7 -> 128 (one group of 8 chunks); its side converts y_7 tiles 4-7 and
  // finishes the density head.  When N is a multiple of 32 the wave's samples lie on one ray: its
  // 1 KiB of ray features is DMA'd into LDS meanwhile (the stream's last vmcnt(0) covers it).
  const bool one_ray = (N & 31) == 0;
  float* feat_mine = lds + kSLdsFeat + wave * kRayFeat;
  if (one_ray) {
    const char* src = reinterpret_cast<const char*>(feat + (imin64(s0, M - 1) / N) * kRayFeat);
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
#pragma unroll
  for (int st = 0; st < 2; ++st) inv_cur[st] = cst[kS16InvW + 8] / s_cur[st];
  sgroup<0, 8, 0, 0, kSPrev>(stream, s16_chunk0(8), lds, lds_dma, voff, off, a, acc, act_operand,
                             [&](auto i, auto seg, auto ph) __attribute__((always_inline)) {
                               side_prev(i, seg, ph, Sigma{});
                             });

  // density head: sigma = ReLU(density_head(ReLU(h7))) (models.py:137-138), f32
  float sig[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) sig[st] = fmaxf(ssum4(part[st]) + ws[kHidden], 0.0f);
  // colour branch: h_dir = ReLU(W_dh ReLU(h7) + [b_dir + W_dd PE(d)]) + appearance (models.py:141-156)
  const float* wr = lds + kSLdsRgb;
  float pr[2][3] = {{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}};
  auto colour_head = [&](const float* fr, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int T = 0; T < 4; ++T)
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int n0 = 32 * T + 8 * r + nlane;
        const f32x4 fd = *reinterpret_cast<const f32x4*>(fr + n0);
        const f32x4 ap = *reinterpret_cast<const f32x4*>(fr + kDirHidden + n0);
        f32x4 hd;
#pragma unroll
        for (int e = 0; e < 4; ++e) hd[e] = fmaxf(fmaf(acc[T][r][st][e], inv_cur[st], fd[e]), 0.0f) + ap[e];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(wr + c * kDirHidden + n0);
#pragma unroll
          for (int e = 0; e < 4; ++e) pr[st][c] = fmaf(w[e], hd[e], pr[st][c]);
        }
      }
  };
  if (one_ray) {
    wait_vmcnt<0>();
    colour_head(feat_mine, 0);
    colour_head(feat_mine, 1);
  } else {
    colour_head(feat + (int64_t)((int)sample_of(0) / N) * kRayFeat, 0);
    colour_head(feat + (int64_t)((int)sample_of(1) / N) * kRayFeat, 1);
  }
  float out[2][3];
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = ssum4(pr[st][c]) + wr[3 * kDirHidden + c];
      out[st][c] = 1.0f / (1.0f + expf_rn(-v));                        // sigmoid (models.py:159-160)
    }
  // lane group st writes sample tile st
  if (g < 2) {
    const int st = g;
    if (s0 + 16 * st + li < M) {
      const int sm = (int)(s0 + 16 * st + li);
      const int64_t o_s = out_slot ? (int64_t)(sm / N) * out_T + out_slot[sm] : (int64_t)sm;
      sigma[o_s] = st ? sig[1] : sig[0];
#pragma unroll
      for (int c = 0; c < 3; ++c) rgb[3 * o_s + c] = st ? out[1][c] : out[0][c];
    }
  }
}

int launch_mlp16s(const float* packed, const float* o, const float* d, const float* z, int64_t R, int N,
                  const float* feat, float* rgb, float* sigma, const int* out_slot, int out_T, hipStream_t s) {
  const int64_t M = R * (int64_t)N;
  if (M == 0) return NERF_OK;
  constexpr int per_block = 32 * kW16Waves;
  const int64_t blocks = (M + per_block - 1) / per_block;
  hipLaunchKernelGGL(mlp16s_kernel, dim3((unsigned)blocks), dim3(64 * kW16Waves), 0, s, packed, o, d, z, M, N, feat,
                     rgb, sigma, out_slot, out_T);
  return check_launch("mlp16s_kernel");
}

}  // namespace nerf
