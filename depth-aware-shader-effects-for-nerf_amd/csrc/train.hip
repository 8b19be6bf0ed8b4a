// Training path (BASELINE config 5): backward of the render path and the
// optimizer step, all hand-written for gfx950.
//
// Reference: src/train.py:13-207 — volume_render (perturb=True, coarse only: render.py:83-86
// ignores n_importance), MSE against the target rgb (:87), loss.backward(), Adam (:90-92).
//
//   composite_backward_kernel   d loss / d(sigma, rgb) per sample from d loss / d rgb_map (one
//                               wave per ray, reverse double-precision scan)
//   mlp_backward_kernel         the data-gradient chain of NeRF.forward on fp32 MFMA, one wave per
//                               32 samples, mirroring mlp_kernel with transposed weights: writes
//                               every layer's d loss / d pre-activation (layout.h kGrad*)
//   wgrad_kernel + reduce       dW[n][k] = sum_m dpre[m][n] x[m][k] (+ the bias column) over the
//                               batch, chunked over samples with a deterministic reduction
//   app_grad_kernel             per-ray appearance-embedding gradient
//   adam_kernel                 torch.optim.Adam's update, element for element
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <utility>

#include "common.h"
#include "stream16.h"

namespace nerf {

static_assert(kSaveRow == NERF_SAVE_ROW && kGradRow == NERF_GRAD_ROW, "nerfmi_train.h rows out of sync");

// ---------------------------------------------------------------------------- composite bwd
// render.py:56-80 differentiated.  With g = d loss / d rgb_map (3), per sample s of a ray:
//   drgb_s = w_s g;  dw_s = g . rgb_s;  T_s = prod_{j<s} f_j, f_j = 1 - a_j + 1e-10
//   d a_s = dw_s T_s - (1/f_s) sum_{t>s} dw_t w_t;   d sigma_s = d a_s * dist_s * exp(-sigma_s dist_s)
// The training loss is mean((rgb_map - target)^2) over B x 3 (train.py:87): g = 2 (rgb_map - target)/(3B),
// sq_err[r] = sum_c (rgb_map - target)^2 for the loss value.  Given an arbitrary upstream gradient
// instead (autograd: grad_map (B,3) for rgb_map, grad_depth (B) for depth_map, each nullable = 0),
// g = grad_map[r] and the depth term of depth = S / (A + 1e-10), S = sum w z, A = sum w (:80) adds
//   dw_s += gd (z_s - S / (A + 1e-10)) / (A + 1e-10)
// with S and A re-accumulated (double) over the same float weights in the forward pass.
__global__ void __launch_bounds__(256)
composite_backward_kernel(const float* __restrict__ rgb, const float* __restrict__ sigma, const float* __restrict__ zv,
                          const float* __restrict__ rgb_map, const float* __restrict__ target,
                          const float* __restrict__ grad_map, const float* __restrict__ grad_depth, int64_t B, int N,
                          float scale, float* __restrict__ dsigma, float* __restrict__ drgb,
                          float* __restrict__ sq_err) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const int64_t base = r * N;
  float g[3], se = 0.0f;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (target) {
      const float e = rgb_map[3 * r + c] - target[3 * r + c];
      g[c] = scale * e;
      se += e * e;
    } else {
      g[c] = grad_map ? grad_map[3 * r + c] : 0.0f;
    }
  }
  const float gd = grad_depth ? grad_depth[r] : 0.0f;
  if (lane == 0 && sq_err) sq_err[r] = se;
  if (N == 1) {                       // the reference's per-sample tensors are empty (render.py:56-58)
    if (lane == 0) {
      dsigma[base] = 0.0f;
      drgb[3 * base] = drgb[3 * base + 1] = drgb[3 * base + 2] = 0.0f;
    }
    return;
  }
  // pass 1 (forward order): transmittance prefix, carried across 64-sample chunks (and, with a
  // depth gradient, S and A)
  // pass 2 (reverse order): suffix sums of dw*w; done chunk by chunk from the end, recomputing
  // each chunk's T from the stored chunk-start prefixes.
  const int nchunk = (N + 63) / 64;
  __shared__ double carry_lds[4][64]; // T at each chunk start (N <= 4096)
  double* carry_chunk = carry_lds[threadIdx.x >> 6];
  double carry = 1.0, wz = 0.0, ws = 0.0;
  for (int c = 0; c < nchunk; ++c) {
    const int s = c * 64 + lane;
    double f = 1.0;
    float alpha = 0.0f, z = 0.0f;
    if (s < N) {
      z = zv[base + s];
      const float dist = (s + 1 < N) ? zv[base + s + 1] - z : 1e-3f;
      alpha = 1.0f - expf_rn(-sigma[base + s] * dist);
      f = (double)((1.0f - alpha) + 1e-10f);
    }
    double incl = f;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double up = __shfl_up(incl, off);
      if (lane >= off) incl *= up;
    }
    if (gd != 0.0f) {
      double excl = __shfl_up(incl, 1);
      if (lane == 0) excl = 1.0;
      const float w = alpha * (float)(carry * excl);
      wz += (double)w * (double)z;
      ws += (double)w;
    }
    if (lane == 0) carry_chunk[c] = carry;
    carry *= __shfl(incl, 63);
  }
  double dinv = 0.0, dmean = 0.0;    // 1 / (A + 1e-10), S / (A + 1e-10)
  if (gd != 0.0f) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      wz += __shfl_xor(wz, off);
      ws += __shfl_xor(ws, off);
    }
    const double den = (double)((float)ws + 1e-10f);
    dinv = 1.0 / den;
    dmean = wz * dinv;
  }
  __builtin_amdgcn_wave_barrier();
  double suffix = 0.0;                // sum_{t > current chunk} dw_t w_t
  for (int c = nchunk - 1; c >= 0; --c) {
    const int s = c * 64 + lane;
    const bool valid = s < N;
    float alpha = 0.0f, dist = 0.0f, e = 1.0f, fs = 1.0f, sg = 0.0f, z = 0.0f;
    double f = 1.0;
    if (valid) {
      z = zv[base + s];
      dist = (s + 1 < N) ? zv[base + s + 1] - z : 1e-3f;
      sg = sigma[base + s];
      e = expf_rn(-sg * dist);
      alpha = 1.0f - e;
      fs = (1.0f - alpha) + 1e-10f;
      f = (double)fs;
    }
    double incl = f;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double up = __shfl_up(incl, off);
      if (lane >= off) incl *= up;
    }
    double excl = __shfl_up(incl, 1);
    if (lane == 0) excl = 1.0;
    const float T = (float)(carry_chunk[c] * excl);
    const float w = alpha * T;
    float dw = 0.0f;
    if (valid) {
      const int64_t e3 = 3 * (base + s);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        dw += g[k] * rgb[e3 + k];
        drgb[e3 + k] = w * g[k];
      }
      if (gd != 0.0f) dw += (float)((double)gd * ((double)z - dmean) * dinv);
    }
    // exclusive suffix sum of dw*w inside the chunk, plus the chunks after it
    double v = valid ? (double)dw * (double)w : 0.0;
    double incl_rev = v;                                   // inclusive suffix within the chunk
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double dn = __shfl_down(incl_rev, off);
      if (lane + off < 64) incl_rev += dn;
    }
    const double excl_rev = incl_rev - v + suffix;
    if (valid) {
      const float da = (float)((double)dw * (double)T - excl_rev / (double)fs);
      dsigma[base + s] = da * dist * e;
    }
    suffix += __shfl(incl_rev, 0);
  }
}

int launch_composite_backward(const float* rgb, const float* sigma, const float* z, const float* rgb_map,
                              const float* target, const float* grad_map, const float* grad_depth, int64_t B, int N,
                              float scale, float* dsigma, float* drgb, float* sq_err, hipStream_t s) {
  if (B == 0) return NERF_OK;
  hipLaunchKernelGGL(composite_backward_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, rgb, sigma, z,
                     rgb_map, target, grad_map, grad_depth, B, N, scale, dsigma, drgb, sq_err);
  return check_launch("composite_backward_kernel");
}

// ------------------------------------------------------------------------ transposed weights
// Fragment layout (layout.h) of W_l^T for trunk layers 1..7 (act part of layer 4) and of the
// h-part of dir_linear: matrix mt = 0..6 is W_{mt+1}^T (256 x 256), mt = 7 is W_dh^T (256 x 128).
// Rows are the forward layer's INPUT neurons (natural order), columns its OUTPUT neurons in the
// accumulator k order, so the backward chain feeds d pre-activations to the MFMA as they sit
// in registers, exactly like the forward.
NERF_HD constexpr int tmat_ksteps(int mt) { return mt == 7 ? kDirHidden / 2 : kActSteps; }
NERF_HD constexpr size_t tmat_offset(int mt) { return (size_t)mt * 8 * kActSteps * 64; }
constexpr size_t kPackedT32Floats = tmat_offset(7) + (size_t)8 * (kDirHidden / 2) * 64;   // 491520
// Split-f16 part (mlp_backward16_kernel), after the f32 part: W^T s_w of the same 8 matrices as f16
// hi/lo A fragments of v_mfma_f32_32x32x16_f16.  Matrix mt holds 2 tile groups x KS16 k-steps x
// 4 tiles x {hi, lo} pieces, each 64 lanes x 8 halves (4 words); the kernel streams them in that
// order.  Lane l of the piece for (tile tt, k-step ks) holds W^T[32 tt + (l & 31)][n_j], the
// k index n_j = 32 (ks >> 1) + 16 (ks & 1) + 8 (j >> 2) + 4 (l >> 5) + (j & 3) being the
// accumulator order in which the previous backward layer leaves its outputs (act_feature).
// s_w = 2^(14 - e) with max |W| < 2^e per matrix (layout.h s16_exponent), and its inverse, follow.
// The matrices lie in the order the data-gradient chain consumes them (dir_linear's h-part, then
// trunk layers 7 .. 1), so the f16 part is one contiguous stream of 16 KiB chunks (stream16.h):
// chunk c of the stream is at kPackedT32Floats + c * kChunkFloats.
NERF_HD constexpr int t16_ksteps(int mt) { return mt == 7 ? kDirHidden / 16 : kHidden / 16; }
NERF_HD constexpr size_t t16_offset(int mt) {
  return kPackedT32Floats + (mt == 7 ? 0 : (size_t)8 * kChunkFloats + (size_t)(6 - mt) * 16 * kChunkFloats);
}
constexpr int kBwChunks = 8 + 7 * 16;                                         // chunks of the stream
constexpr size_t kOffT16Consts = kPackedT32Floats + (size_t)kBwChunks * kChunkFloats;
// constants: s_w[8], 1/s_w[8], then the data-gradient bound constants C[8] (matrix mt's largest
// row L1 norm of W^T, x 1.0001: |W^T g| <= C max|g| rigorously) and max |density_head.weight|
constexpr int kT16S = 0, kT16InvS = 8, kT16C = 16, kT16WsigMax = 24, kT16Consts = 32;
constexpr size_t kPackedTFloats = kOffT16Consts + kT16Consts;                 // 983072
NERF_HD inline void store_t16_consts(float* consts, int mt, float mx) {
  const int e = s16_exponent(mx);
  consts[kT16S + mt] = ldexpf(1.0f, 14 - e);
  consts[kT16InvS + mt] = ldexpf(1.0f, e - 14);
}
static_assert(t16_offset(0) + 16 * kChunkFloats == kOffT16Consts && t16_offset(6) == t16_offset(7) + 8 * kChunkFloats,
              "the transposed stream is contiguous in consumption order");

NERF_HD inline float packT_value(const float* const* P, size_t e) {
  int mt = (int)(e / (8 * kActSteps * 64));
  if (mt > 7) mt = 7;
  const size_t rel = e - tmat_offset(mt);
  const int j = (int)(rel & 3);
  const int lane = (int)((rel >> 2) & 63);
  const size_t blk = rel >> 8;
  const int ksq = tmat_ksteps(mt) / 4;
  const int nt = (int)(blk / ksq), kq = (int)(blk % ksq);
  const int o = act_feature(4 * kq + j, lane >> 5);       // forward output neuron
  const int i = nt * 32 + (lane & 31);                   // forward input neuron
  if (mt == 7) return P[P_DIR_W][(size_t)o * (kHidden + kDirEnc) + i];
  const int layer = mt + 1;
  const int K = layer == kSkipLayer ? kHidden + kPosEnc : kHidden;
  return P[2 * layer][(size_t)o * K + i];
}

// W^T[i][o] of matrix mt (forward input neuron i, output neuron o)
NERF_HD inline float tmat_weight(const float* const* P, int mt, int i, int o) {
  if (mt == 7) return P[P_DIR_W][(size_t)o * (kHidden + kDirEnc) + i];
  const int layer = mt + 1;
  const int K = layer == kSkipLayer ? kHidden + kPosEnc : kHidden;
  return P[2 * layer][(size_t)o * K + i];
}

// max |W^T| of matrix mt over rows i (one thread per row)
NERF_HD inline float tmat_row_max(const float* const* P, int mt, int i) {
  const int outs = mt == 7 ? kDirHidden : kHidden;
  float m = 0.0f;
  for (int o = 0; o < outs; ++o) m = fmaxf(m, fabsf(tmat_weight(P, mt, i, o)));
  return m;
}



// word w (two halves) of the split-f16 part, w relative to t16_offset(0)
NERF_HD inline uint32_t packT16_word(const float* const* P, const float* consts, size_t w) {
  const size_t c = w / kChunkFloats;                    // chunk of the stream
  const int mt = c < 8 ? 7 : 6 - (int)((c - 8) / 16);
  const size_t rel = w - (t16_offset(mt) - kPackedT32Floats);
  const int KS = t16_ksteps(mt);
  const int jj = (int)(rel & 3), lane = (int)((rel >> 2) & 63);
  const size_t piece = rel >> 8;
  const int part = (int)(piece & 1), i = (int)((piece >> 1) & 3);
  const int step = (int)(piece >> 3), g = step / KS, ks = step % KS;
  const int row = 32 * (4 * g + i) + (lane & 31);
  uint32_t word = 0;
  for (int k = 0; k < 2; ++k) {
    const int j = 2 * jj + k;
    const int o = 32 * (ks >> 1) + 16 * (ks & 1) + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3);
    const float v = tmat_weight(P, mt, row, o) * consts[mt];
    const _Float16 hi = (_Float16)v;
    const _Float16 out = part == 0 ? hi : (_Float16)(v - (float)hi);
    uint16_t bits;
    memcpy(&bits, &out, 2);
    word |= (uint32_t)bits << (16 * k);
  }
  return word;
}

struct ParamPtrsT { const float* p[P_COUNT]; };

// (the last block also zeroes the split stream's constant slots, which statsT16_kernel's atomics fill)
__global__ void __launch_bounds__(256) packT_kernel(ParamPtrsT P, float* __restrict__ packed) {
  if (blockIdx.x == gridDim.x - 1) {
    if (threadIdx.x < kT16Consts) packed[kOffT16Consts + threadIdx.x] = 0.0f;
    return;
  }
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < kPackedT32Floats) packed[e] = packT_value(P.p, e);
}

// Statistics of the split scales (statsT16_kernel below): max |W^T| of matrix mt (= max |W| over its
// columns i < kHidden), 8 rows of W^T per block (thread = row i, coalesced over i), combined by
// atomicMax on the float bits (exact in any order) into consts[mt] (zeroed first); the last block
// turns the maxima into s_w and 1/s_w.
// Row L1 norm of W^T (a forward input neuron's weights over the outputs): four partial sums over
// the output quarters, each in order, added in order (the host's tmat_row_l1 is the same
// expression, so device and host constants are bit-identical); the matrix's maximum by atomicMax on
// the float bits (exact in any order).  One block per (matrix, 64 rows): thread = (row, quarter).
// One more block takes max |density_head.weight|.
NERF_HD inline float tmat_row_l1_part(const float* const* P, int mt, int i, int q) {
  const int outs = mt == 7 ? kDirHidden : kHidden, per = outs / 4;
  float l1 = 0.0f;
  for (int o = q * per; o < (q + 1) * per; ++o) l1 += fabsf(tmat_weight(P, mt, i, o));
  return l1;
}
NERF_HD inline float tmat_row_l1(const float* const* P, int mt, int i) {
  return ((tmat_row_l1_part(P, mt, i, 0) + tmat_row_l1_part(P, mt, i, 1)) + tmat_row_l1_part(P, mt, i, 2)) +
         tmat_row_l1_part(P, mt, i, 3);
}

// The three statistics passes in one launch (formerly scaleT16 / boundT16 / finalize kernels): the
// block counter (an unused constant slot, zeroed by packT_kernel, reset after) elects the last block
// to finish, which turns the maxima into the constants.  Blocks 0..255: max |W^T| (matrix b / 32,
// outputs 8 (b % 32) ..); 256..287: row L1 norms (matrix (b - 256) / 4); 288: max |density weight|.
constexpr int kT16Counter = kT16Consts - 1;
static_assert(kT16Counter > kT16WsigMax, "the counter slot is unused by the constants");
__global__ void __launch_bounds__(256) statsT16_kernel(ParamPtrsT P, float* __restrict__ packed) {
  __shared__ float part[4][64];
  __shared__ unsigned last;
  unsigned* c = reinterpret_cast<unsigned*>(packed + kOffT16Consts);
  const int b = blockIdx.x;
  if (b < 256) {
    const int mt = b / 32, i = threadIdx.x;
    const int outs = mt == 7 ? kDirHidden : kHidden;
    const int o0 = (b % 32) * 8;
    float m = 0.0f;
    for (int o = o0; o < o0 + 8 && o < outs; ++o) m = fmaxf(m, fabsf(tmat_weight(P.p, mt, i, o)));
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if ((threadIdx.x & 63) == 0) {
      atomicMax(c + mt, __float_as_uint(m));
      __threadfence();
    }
  } else if (b == 256 + 32) {
    float v = fabsf(P.p[P_SIGMA_W][threadIdx.x]);
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    if ((threadIdx.x & 63) == 0) {
      atomicMax(c + kT16WsigMax, __float_as_uint(v));
      __threadfence();
    }
  } else {
    const int bb = b - 256, mt = bb >> 2, r = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int i = (bb & 3) * 64 + r;
    part[q][r] = tmat_row_l1_part(P.p, mt, i, q);
    __syncthreads();
    if (q == 0) {
      float v = ((part[0][r] + part[1][r]) + part[2][r]) + part[3][r];
      for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
      if (r == 0) {
        atomicMax(c + kT16C + mt, __float_as_uint(v));
        __threadfence();
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(c + kT16Counter, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!last) return;   // (uniform)
  __threadfence();
  if (threadIdx.x < 8) {
    const int mt = threadIdx.x;
    const float mx = __uint_as_float(__hip_atomic_load(c + mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const float l1 = __uint_as_float(__hip_atomic_load(c + kT16C + mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    store_t16_consts(packed + kOffT16Consts, mt, mx);
    packed[kOffT16Consts + kT16C + mt] = l1 * 1.0001f;   // rounding margin on the float sums: a bound
  }
  if (threadIdx.x == 0) __hip_atomic_store(c + kT16Counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(256) packT16_kernel(ParamPtrsT P, float* __restrict__ packed) {
  const size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < kOffT16Consts - kPackedT32Floats)
    reinterpret_cast<uint32_t*>(packed)[kPackedT32Floats + w] = packT16_word(P.p, packed + kOffT16Consts, w);
}

int launch_packT(const float* const* params, float* packedT, hipStream_t s) {
  ParamPtrsT P;
  for (int i = 0; i < P_COUNT; ++i) P.p[i] = params[i];
  hipLaunchKernelGGL(packT_kernel, dim3((unsigned)((kPackedT32Floats + 255) / 256 + 1)), dim3(256), 0, s, P, packedT);
  if (int rc = check_launch("packT_kernel")) return rc;
  hipLaunchKernelGGL(statsT16_kernel, dim3(256 + 33), dim3(256), 0, s, P, packedT);
  if (int rc = check_launch("statsT16_kernel")) return rc;
  const size_t words = kOffT16Consts - kPackedT32Floats;
  hipLaunchKernelGGL(packT16_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, P, packedT);
  return check_launch("packT16_kernel");
}

void packT_host(const float* const* params, float* packedT) {
  for (size_t e = 0; e < kPackedT32Floats; ++e) packedT[e] = packT_value(params, e);
  float* consts = packedT + kOffT16Consts;
  for (int k = 0; k < kT16Consts; ++k) consts[k] = 0.0f;
  for (int mt = 0; mt < 8; ++mt) {
    float mx = 0.0f, l1 = 0.0f;
    for (int i = 0; i < kHidden; ++i) {
      mx = fmaxf(mx, tmat_row_max(params, mt, i));
      l1 = fmaxf(l1, tmat_row_l1(params, mt, i));
    }
    store_t16_consts(consts, mt, mx);
    consts[kT16C + mt] = l1 * 1.0001f;
  }
  for (int i = 0; i < kHidden; ++i) consts[kT16WsigMax] = fmaxf(consts[kT16WsigMax], fabsf(params[P_SIGMA_W][i]));
  uint32_t* words = reinterpret_cast<uint32_t*>(packedT);
  for (size_t w = 0; w < kOffT16Consts - kPackedT32Floats; ++w)
    words[kPackedT32Floats + w] = packT16_word(params, consts, w);
}

// ------------------------------------------------------------------------------ MLP backward
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x16 mfma32t(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <typename F, int... Is>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// out (8 tiles, 256 forward-input neurons) = W^T . in (KS k-steps of forward-output neurons in
// accumulator order), from a transposed fragment matrix.  Four tiles interleaved (independent
// MFMAs); weights streamed through a DEPTH-block register ring.
template <int KS>
__device__ __forceinline__ void dgrad(const float* __restrict__ wmat, const f32x16 (&in)[8], f32x16 (&out)[8],
                                      int lane) {
  constexpr int KSQ = KS / 4;
  constexpr int DEPTH = 8;
  constexpr int G = 8 * KSQ;
  const f32x4* __restrict__ wf = reinterpret_cast<const f32x4*>(wmat) + lane;
  auto blk = [](int g) { return ((g / (4 * KSQ)) * 4 + g % 4) * KSQ + (g / 4) % KSQ; };
  f32x4 ring[DEPTH];
#pragma unroll
  for (int p = 0; p < DEPTH; ++p) ring[p] = wf[blk(p) * 64];
  sfor<G / 4>([&](auto sc) __attribute__((always_inline)) {
    constexpr int st = decltype(sc)::value;
    constexpr int grp = st / KSQ, kq = st % KSQ;
    if constexpr (kq == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) out[4 * grp + i] = f32x16{};
    }
    sfor<4>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      constexpr int ks = 4 * kq + j;
      const float b = in[ks >> 4][ks & 15];
      sfor<4>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        out[4 * grp + i] = mfma32t(ring[(4 * st + i) % DEPTH][j], b, out[4 * grp + i]);
      });
    });
    sfor<4>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      constexpr int g = 4 * st + i;
      if constexpr (g + DEPTH < G) ring[g % DEPTH] = wf[blk(g + DEPTH) * 64];
    });
    __builtin_amdgcn_sched_barrier(0);
  });
}

// A wave's 32 gradient rows as a buffer resource sized to the rows that exist, so the stores of
// tail lanes fall outside it and are dropped: no branches around stores, which would otherwise
// split the loads and stores of the ReLU backward into one memory round trip per 16 bytes.
struct GradRows {
  __amdgpu_buffer_rsrc_t res;
  uint32_t loff;   // this lane's byte offset: row (lane & 31), lane half h
};

// (tile-major rows, layout.h: the wave's block of 32 samples; a lane's 4 features of a group at
// ((lane & 31) 8 + 4h) floats; a lane past M, or a wave past M, stores nothing)
__device__ __forceinline__ GradRows grad_rows(float* grad, int64_t s0, int64_t M, int lane) {
  const bool any = s0 < M;
  GradRows g;
  g.res = __builtin_amdgcn_make_buffer_rsrc(grad + (any ? s0 : 0) * kGradRow, (short)0, any ? 32 * kGradRow * 4 : 0,
                                            0x00020000);
  g.loff = s0 + (lane & 31) < M ? ((uint32_t)(lane & 31) * 8 + 4 * (uint32_t)(lane >> 5)) * 4 : 0x40000000u;
  return g;
}

// Sample s's place in its tile-major block: element f of the row at tile_row(...) + tile_col(f) + f % 8.
template <typename T>
__device__ __forceinline__ T* tile_row(T* base, int64_t s, int R) {
  return base + (s / 32) * 32 * (int64_t)R + (s % 32) * 8;
}

// 16 bytes at feature off (+ 4 h) of this lane's gradient row (off a multiple of 8)
__device__ __forceinline__ void grad_store4(const GradRows& g, int off, f32x4 v) {
  store16_rows<0>(v, g.res, g.loff + 4u * (uint32_t)tile_col(off));
}

// d pre-activation = d activation * [activation > 0] (ReLU backward; the saved activation is
// ReLU(pre), positive exactly where pre is), in place, and stored to the gradient row.
__device__ __forceinline__ void relu_back_store(f32x16 (&x)[8], int ntiles, const float* __restrict__ srow,
                                                int save_off, const GradRows& gr, int grad_off, int h) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    if (t >= ntiles) break;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(srow + tile_col(save_off + t * 32 + 8 * q) + 4 * h);
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = a[e] > 0.0f ? x[t][4 * q + e] : 0.0f;
        x[t][4 * q + e] = d;
        v[e] = d;
      }
      grad_store4(gr, grad_off + t * 32 + 8 * q, v);
    }
  }
}

__global__ void __launch_bounds__(256, 1)
mlp_backward_kernel(const float* __restrict__ packed, const float* __restrict__ packedT,
                    const float* __restrict__ save, const float* __restrict__ sigma, const float* __restrict__ rgb,
                    const float* __restrict__ dsigma, const float* __restrict__ drgb, int64_t M,
                    float* __restrict__ grad) {
  const int lane = threadIdx.x & 63;
  const int64_t s0 = ((int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 32;   // wave-uniform
  if (s0 >= M) return;
  const int h = lane >> 5;
  const int64_t s = imin64(s0 + (lane & 31), M - 1);
  const bool valid = s0 + (lane & 31) < M;
  const float* srow = tile_row(save, s, kSaveRow);
  float* grow = tile_row(grad, s, kGradRow);
  const GradRows gr = grad_rows(grad, s0, M, lane);

  // rgb head: rgb = sigmoid(v) -> dv = drgb * rgb (1 - rgb) (models.py:159-160)
  float dv[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float y = rgb[3 * s + c];
    dv[c] = drgb[3 * s + c] * (y * (1.0f - y));
  }
  // density head: sigma = ReLU(v_s) -> d v_s = dsigma * [sigma > 0]
  const float dsp = sigma[s] > 0.0f ? dsigma[s] : 0.0f;
  if (valid && h == 0) {
    grow[tile_col(kGradSigma)] = dsp;
    grow[tile_col(kMetaGradF) + kMetaGradF % 8] = 0.0f;   // no block exponent (layout.h)
#pragma unroll
    for (int c = 0; c < 3; ++c) grow[tile_col(kGradRgb) + c] = dv[c];
  }
  f32x16 A[8], B[8];
  // d hd = W_rgb^T dv (128, accumulator layout in A[0..3])
  const float* wr = packed + kOffRgbW;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = t * 32 + 8 * q + 4 * h + e;
        const float d = fmaf(dv[2], wr[2 * kDirHidden + n], fmaf(dv[1], wr[kDirHidden + n], dv[0] * wr[n]));
        A[t][4 * q + e] = d;
        v[e] = d;
      }
      grad_store4(gr, kGradHd + t * 32 + 8 * q, v);
    }
  // hd = ReLU(dir pre) + appearance: d dir_pre = d hd * [r_dir > 0]
  relu_back_store(A, 4, srow, kSaveRDir, gr, kGradDir, h);
  // d h7 = W_dh^T d dir_pre + w_sigma * d v_s
  dgrad<kDirHidden / 2>(packedT + tmat_offset(7), A, B, lane);
  const float* wsg = packed + kOffSigmaW;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(wsg + t * 32 + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) B[t][4 * q + e] = fmaf(dsp, w[e], B[t][4 * q + e]);
    }
  // trunk, top down: d pre_l = d h_l [h_l > 0]; d h_{l-1} = W_l^T d pre_l
#pragma unroll 1
  for (int p = 0; p < 3; ++p) {
    const int l1 = 7 - 2 * p, l2 = 6 - 2 * p;
    relu_back_store(B, 8, srow, save_h(l1), gr, l1 * kHidden, h);
    dgrad<kActSteps>(packedT + tmat_offset(l1 - 1), B, A, lane);
    relu_back_store(A, 8, srow, save_h(l2), gr, l2 * kHidden, h);
    dgrad<kActSteps>(packedT + tmat_offset(l2 - 1), A, B, lane);
  }
  relu_back_store(B, 8, srow, save_h(1), gr, 1 * kHidden, h);
  dgrad<kActSteps>(packedT + tmat_offset(0), B, A, lane);
  relu_back_store(A, 8, srow, save_h(0), gr, 0, h);
}

// ---------------------------------------------------------------- MLP backward, split f16
// The same chain on v_mfma_f32_32x32x16_f16 (nerf_arith F16X3), the arithmetic of mlp16_kernel:
// out = W^T g as hi(W s_w) hi(g s_g) + hi(W s_w) lo(g s_g) + lo(W s_w) hi(g s_g) with f32
// accumulation, unscaled by the exact inverses.  x s = hi + lo + O(2^-24 |x s|) for both operands
// and the dropped lo lo term is O(2^-22) of the products, so the result has fp32-level error.
// s_w is per matrix (pack time, packedT's split part); s_g is per sample, from the exact max |g|
// over the sample's gradient row (both lane halves): the whole row exists before the layer starts,
// so no bound is needed.  s_g = 2^(140 - E), E the biased exponent of the max (>= 14, so s_g stays
// a normal float): |g s_g| < 2^14.  Each 16-deep k-step is 3 x 32 MFMA cycles against 8 x 64 for
// v_mfma_f32_32x32x2_f32.  Weights stream per wave from L2 through a 3-step register ring (one
// step = 4 tiles x {hi, lo} = 8 KiB for 12 MFMAs).
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma16t(u32x4 a, h16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h16x8, a), b, c, 0, 0, 0);
}

// Split tiles 0..NT-1 of X (k-steps 2t + s: accumulator elements 8s..8s+7) at the sample's scale,
// negative for odd samples (lane & 1; see mlp_backward16_bound_kernel); returns 1 / s_g.
template <int NT>
__device__ __forceinline__ float split_rows(const f32x16 (&X)[8], h16x8 (&bh)[16], h16x8 (&bl)[16]) {
  float m = 0.0f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 16; ++g) m = fmaxf(m, fabsf(X[t][g]));
  m = fmaxf(m, __shfl_xor(m, 32));
  int E = (int)((__float_as_uint(m) >> 23) & 0xffu);
  E = E < 14 ? 14 : E;
  const float sgn = (threadIdx.x & 1) ? -1.0f : 1.0f;
  const float sc = sgn * __uint_as_float((uint32_t)(267 - E) << 23);
  typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < 8; j += 2) {   // a pair: hi by one v_cvt_pk_f16_f32, lo by split_lo_pair
        const float v0 = X[t][8 * q + j] * sc, v1 = X[t][8 * q + j + 1] * sc;
        const h16x2 hi2 = {(_Float16)v0, (_Float16)v1};
        const h16x2 lo2 = __builtin_bit_cast(h16x2, split_lo_pair(__builtin_bit_cast(uint32_t, hi2), v0, v1));
        bh[2 * t + q][j] = hi2[0];
        bh[2 * t + q][j + 1] = hi2[1];
        bl[2 * t + q][j] = lo2[0];
        bl[2 * t + q][j + 1] = lo2[1];
      }
  return sgn * __uint_as_float((uint32_t)(E - 13) << 23);
}

// out (8 tiles) = (W^T g) from the split operands of KS k-steps; inv_w = 1/s_w, inv_g = 1/s_g.
// Meanwhile the output's ReLU mask is fetched: the 128 saved activations this lane needs next
// (act, 32 chunks of 4 at act + 32 t + 8 q) are loaded a few per step and folded into 128 bits
// (chunk c = 4 t + q, element e -> bit 4 c + e), so the ReLU backward waits for no load.
__device__ __forceinline__ void fold_mask(uint32_t (&mask)[4], int c, f32x4 a) {
#pragma unroll
  for (int e = 0; e < 4; ++e) mask[c / 8] |= (a[e] > 0.0f ? 1u : 0u) << (4 * (c % 8) + e);
}

// (Without mask rows: nerf_mlp_backward called with masks = NULL.  The training path runs
// mlp_backward16_bound_kernel below.)
template <int KS>
__device__ __forceinline__ void dgrad16(const uint32_t* __restrict__ wmat, const h16x8 (&bh)[16],
                                        const h16x8 (&bl)[16], f32x16 (&out)[8], float inv_w, float inv_g,
                                        const float* __restrict__ act, uint32_t (&mask)[4], int lane) {
  constexpr int STEPS = 2 * KS, PIECES = 8 * STEPS, DEPTH = 24;
  constexpr int CPS = 32 / STEPS, LAG = 3, RS = (LAG + 1) * CPS;   // mask chunks per step, load->fold lag
  const u32x4* __restrict__ wf = reinterpret_cast<const u32x4*>(wmat) + lane;
  u32x4 ring[DEPTH];
  f32x4 pf[RS];
#pragma unroll
  for (int i = 0; i < 4; ++i) mask[i] = 0u;
#pragma unroll
  for (int p = 0; p < DEPTH; ++p) ring[p] = wf[p * 64];
  sfor<STEPS>([&](auto sc) __attribute__((always_inline)) {
    constexpr int st = decltype(sc)::value;
    constexpr int g = st / KS, ks = st % KS;
    if constexpr (st >= LAG) {
#pragma unroll
      for (int u = 0; u < CPS; ++u) fold_mask(mask, (st - LAG) * CPS + u, pf[((st - LAG) * CPS + u) % RS]);
    }
#pragma unroll
    for (int u = 0; u < CPS; ++u) {
      const int c = st * CPS + u;
      pf[c % RS] = *reinterpret_cast<const f32x4*>(act + 256 * c);   // tile-major: feature group c
    }
    if constexpr (ks == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) out[4 * g + i] = f32x16{};
    }
    // small products first: lo(W) hi(g), hi(W) lo(g), then hi(W) hi(g); tiles interleaved
    sfor<4>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      out[4 * g + i] = mfma16t(ring[(8 * st + 2 * i + 1) % DEPTH], bh[ks], out[4 * g + i]);
    });
    sfor<4>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      out[4 * g + i] = mfma16t(ring[(8 * st + 2 * i) % DEPTH], bl[ks], out[4 * g + i]);
    });
    sfor<4>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      out[4 * g + i] = mfma16t(ring[(8 * st + 2 * i) % DEPTH], bh[ks], out[4 * g + i]);
    });
    sfor<8>([&](auto qc) __attribute__((always_inline)) {
      constexpr int p = 8 * st + decltype(qc)::value;
      if constexpr (p + DEPTH < PIECES) ring[p % DEPTH] = wf[(p + DEPTH) * 64];
    });
    if constexpr (ks == KS - 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) out[4 * g + i] = (out[4 * g + i] * inv_w) * inv_g;
    }
    __builtin_amdgcn_sched_barrier(0);
  });
#pragma unroll
  for (int c = (STEPS - LAG) * CPS; c < 32; ++c) fold_mask(mask, c, pf[c % RS]);
}

// relu_back_store with the mask from dgrad16 (tiles 0..NT-1)
template <int NT = 8>
__device__ __forceinline__ void relu_mask_store(f32x16 (&x)[8], const uint32_t (&mask)[4], const GradRows& gr,
                                                int grad_off) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * t + q;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = (mask[c / 8] >> (4 * (c % 8) + e)) & 1u ? x[t][4 * q + e] : 0.0f;
        x[t][4 * q + e] = d;
        v[e] = d;
      }
      grad_store4(gr, grad_off + t * 32 + 8 * q, v);
    }
}

// Data gradient under f16x3 without mask rows (nerf_mlp_backward with masks = NULL): ReLU masks
// folded from the saved f32 activations, W^T fragments loaded per wave.
__global__ void __launch_bounds__(256, 1)
mlp_backward16_kernel(const float* __restrict__ packed, const float* __restrict__ packedT,
                      const float* __restrict__ save, const float* __restrict__ sigma, const float* __restrict__ rgb,
                      const float* __restrict__ dsigma, const float* __restrict__ drgb, int64_t M,
                      float* __restrict__ grad) {
  const int lane = threadIdx.x & 63;
  const int64_t s0 = ((int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 32;   // wave-uniform
  if (s0 >= M) return;
  const int h = lane >> 5;
  const int64_t s = imin64(s0 + (lane & 31), M - 1);
  const bool valid = s0 + (lane & 31) < M;
  const float* srow = tile_row(save, s, kSaveRow);
  float* grow = tile_row(grad, s, kGradRow);
  const GradRows gr = grad_rows(grad, s0, M, lane);
  const uint32_t* t16 = reinterpret_cast<const uint32_t*>(packedT);
  const float* invw = packedT + kOffT16Consts + 8;

  // heads, as mlp_backward_kernel
  float dv[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float y = rgb[3 * s + c];
    dv[c] = drgb[3 * s + c] * (y * (1.0f - y));
  }
  const float dsp = sigma[s] > 0.0f ? dsigma[s] : 0.0f;
  if (valid && h == 0) {
    grow[tile_col(kGradSigma)] = dsp;
    grow[tile_col(kMetaGradF) + kMetaGradF % 8] = 0.0f;   // no block exponent (layout.h)
#pragma unroll
    for (int c = 0; c < 3; ++c) grow[tile_col(kGradRgb) + c] = dv[c];
  }
  f32x16 X[8];
  h16x8 bh[16], bl[16];
  const float* wr = packed + kOffRgbW;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = t * 32 + 8 * q + 4 * h + e;
        const float d = fmaf(dv[2], wr[2 * kDirHidden + n], fmaf(dv[1], wr[kDirHidden + n], dv[0] * wr[n]));
        X[t][4 * q + e] = d;
        v[e] = d;
      }
      grad_store4(gr, kGradHd + t * 32 + 8 * q, v);
    }
  uint32_t mask[4];
  relu_back_store(X, 4, srow, kSaveRDir, gr, kGradDir, h);
  float inv_g = split_rows<4>(X, bh, bl);
  dgrad16<kDirHidden / 16>(t16 + t16_offset(7), bh, bl, X, invw[7], inv_g, srow + tile_col(save_h(7)) + 4 * h, mask, lane);
  const float* wsg = packed + kOffSigmaW;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = *reinterpret_cast<const f32x4*>(wsg + t * 32 + 8 * q + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) X[t][4 * q + e] = fmaf(dsp, w[e], X[t][4 * q + e]);
    }
#pragma unroll 1
  for (int l = 7; l >= 1; --l) {
    relu_mask_store(X, mask, gr, l * kHidden);
    inv_g = split_rows<8>(X, bh, bl);
    dgrad16<kHidden / 16>(t16 + t16_offset(l - 1), bh, bl, X, invw[l - 1], inv_g, srow + tile_col(save_h(l - 1)) + 4 * h, mask,
                          lane);
  }
  relu_mask_store(X, mask, gr, 0);
}

// ---- data gradient with split scales from a bound (f16x3, mask rows: the training path) ---------
// A split scale taken from the exact maximum of the layer's whole gradient row (round 2's kernel,
// in git history) leaves no output convertible before the last MFMA of the layer: the epilogue
// (mask, row store, maximum, split) sits exposed between layers (PMC: MFMA busy 25 %, 47 % of wave
// cycles in dependency waits).  Here the scale of d pre_{l-1} = mask . (W_l^T d pre_l)
// comes from the bound |W_l^T g| <= C_l max|g|, C_l the largest row L1 norm of W_l^T (pack-time,
// packedT kT16C), with max|g| the exact maximum of this layer's input, tracked while that input was
// being converted.  So the schedule is mlp16_kernel's (stream16.h): a layer's 8 output tiles run as
// two groups of 4 over all 16 k-steps; group A's side work converts the previous layer's tiles 4-7
// into operands 8..15, group B's converts this layer's tiles 0-3 into operands 0..7, each a quarter
// tile per half-step in the MFMA shadow.  A quarter: unscale, (layer 7: + dsigma w_sigma), ReLU mask
// from the forward's mask row, one 16-byte store of the gradient row, running max, split.  A loose
// bound only lowers the split's absolute error floor (2^-25 of the scaled unit: for a bound 2^k
// above the row's maximum, 2^(k-39) of that maximum), far below fp32 rounding.
// The head (rgb sigmoid, density ReLU, W_rgb^T, r_dir mask) and the dir layer's input split run
// first on the VALU; the dir layer's inputs sit in operands 8..15 (the dir layer has 8 k-steps), so
// its group B converts dh_7 tiles 0-3 straight into operands 0..7 for layer 7.
constexpr int kBoLdsMask = 4 * kChunkFloats;                          // after the 4-slot ring
constexpr int kBoLdsWsig = kBoLdsMask + 4 * 32 * kMaskRow;            // density-head weights (256)
constexpr int kBoLdsConsts = kBoLdsWsig + kHidden;                    // packedT's 32 constants
constexpr int kBoLdsFloats = kBoLdsConsts + kT16Consts;               // 99.6 KiB

struct GradAt {                      // where a layer's d pre-activations go, and its mask
  __amdgpu_buffer_rsrc_t rows;       // the wave's gradient rows (tail rows outside: stores dropped)
  uint32_t loff;                     // this lane's byte offset in the tile-major block: ((lane & 31) 8 + 4h) 4
  int slice;                         // the layer's first float in the row, uniform
  const uint32_t* mrow;              // this lane's mask words in LDS (sample row + 4h words)
  int mlay;                          // the layer's words in the row: 8 * layer, uniform
};
struct BwQuarter {
  uint32_t mw;                       // the quarter's mask word
  f32x4 w;                           // (layer 7) density-head weights
};

template <int T0, int QG, bool SIGMA>
__device__ __forceinline__ void bw_load4(const GradAt& g, const float* wsig, int h, BwQuarter& qv) {
  constexpr int T = T0 + QG / 4, q = QG % 4;
  qv.mw = g.mrow[g.mlay + T / 2];
  if constexpr (SIGMA) qv.w = *reinterpret_cast<const f32x4*>(wsig + 32 * T + 8 * q + 4 * h);
}

// Quarter QG of a 4-tile group = registers 4q..4q+3 of output tile T0 + QG/4 -> elements 4(q&1)..+3
// of operand in[OP0 + QG/2] (the forward's convert4 with the backward's epilogue).
template <int T0, int OP0, int QG, bool SIGMA, bool SPLIT>
__device__ __forceinline__ void bw_convert4(const f32x16 (&acc)[8], float inv, float dsp, const BwQuarter& qv,
                                            float s, Operand (&in)[16], float& m, const GradAt& g) {
  constexpr int T = T0 + QG / 4, q = QG % 4;
  constexpr int SH = 16 * (T % 2) + 4 * q;
  f32x4 dv;
  float xs[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float x = acc[T][4 * q + e] * inv;
    if constexpr (SIGMA) x = fmaf(dsp, qv.w[e], x);
    const float d = (qv.mw >> (SH + e)) & 1u ? x : 0.0f;
    dv[e] = d;
    m = fmaxf(m, fabsf(d));          // (layer 0, SPLIT = false: its block exponent record)
    if constexpr (SPLIT) xs[e] = d * s;
  }
  store16_rows<kRowStoreAux, true>(dv, g.rows,
                                   g.loff + 4u * (uint32_t)tile_col(g.slice) + 4u * (uint32_t)tile_col(32 * T + 8 * q));
  if constexpr (SPLIT) {   // hi pairs by v_cvt_pk_f16_f32, lo pairs by split_lo_pair
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
}

template <int PH, int T0, int OP0, int QG, bool SIGMA, bool SPLIT>
__device__ __forceinline__ void bw_quarter(const f32x16 (&acc)[8], float inv, float dsp, const float* wsig, int h,
                                           float s, Operand (&in)[16], float& m, BwQuarter& qv, const GradAt& g) {
  if constexpr (PH == 0) bw_load4<T0, QG, SIGMA>(g, wsig, h, qv);
  else bw_convert4<T0, OP0, QG, SIGMA, SPLIT>(acc, inv, dsp, qv, s, in, m, g);
}

__global__ void __launch_bounds__(64 * kW16Waves, 1)
mlp_backward16_bound_kernel(const float* __restrict__ packed, const float* __restrict__ packedT,
                            const uint32_t* __restrict__ masks, const float* __restrict__ sigma,
                            const float* __restrict__ rgb, const float* __restrict__ dsigma,
                            const float* __restrict__ drgb, int64_t M, float* __restrict__ grad, int store_dhd) {
  __shared__ __attribute__((aligned(16))) float lds[kBoLdsFloats];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t s0 = ((int64_t)blockIdx.x * kW16Waves + wave) * 32;
  // every wave runs to the end (the weight stream has barriers); tail lanes repeat sample M-1 and
  // store nothing
  const bool valid = s0 + (lane & 31) < M;
  const int64_t s = imin64(s0 + (lane & 31), M - 1);
  GradAt ga;                          // the wave's tile-major block (layout.h)
  ga.rows = __builtin_amdgcn_make_buffer_rsrc(grad + (s0 < M ? s0 : 0) * kGradRow, (short)0,
                                              s0 < M ? 32 * kGradRow * 4 : 0, 0x00020000);
  ga.loff = valid ? ((uint32_t)(lane & 31) * 8 + 4 * h) * 4 : 0x40000000u;
  // the wave's 32 mask rows (8,704 contiguous bytes) into LDS; constants and w_sigma
  uint32_t* mwave = reinterpret_cast<uint32_t*>(lds + kBoLdsMask) + wave * 32 * kMaskRow;
  for (int i = lane; i < 32 * kMaskRow / 4; i += 64) {
    const int row = i / (kMaskRow / 4), c = i % (kMaskRow / 4);
    reinterpret_cast<u32x4*>(mwave)[i] = reinterpret_cast<const u32x4*>(masks + imin64(s0 + row, M - 1) * kMaskRow)[c];
  }
  if (threadIdx.x < kHidden / 4)
    reinterpret_cast<f32x4*>(lds + kBoLdsWsig)[threadIdx.x] = reinterpret_cast<const f32x4*>(packed + kOffSigmaW)[threadIdx.x];
  if (threadIdx.x < kT16Consts) lds[kBoLdsConsts + threadIdx.x] = packedT[kOffT16Consts + threadIdx.x];
  ga.mrow = mwave + (lane & 31) * kMaskRow + 4 * h;
  ga.mlay = 0;
  ga.slice = 0;

  // heads (models.py:137-160 differentiated): rgb = sigmoid(v) -> dv = drgb rgb (1 - rgb); density
  // sigma = ReLU(v_s) -> d v_s = dsigma [sigma > 0]
  float dv[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float y = rgb[3 * s + c];
    dv[c] = drgb[3 * s + c] * (y * (1.0f - y));
  }
  const float dsp = sigma[s] > 0.0f ? dsigma[s] : 0.0f;
  const float* wr = packed + kOffRgbW;
  float dhd[4][16];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = t * 32 + 8 * q + 4 * h + e;
        dhd[t][4 * q + e] = fmaf(dv[2], wr[2 * kDirHidden + n], fmaf(dv[1], wr[kDirHidden + n], dv[0] * wr[n]));
      }
  __syncthreads();                    // mask rows, w_sigma and constants in LDS
  const float* cst = lds + kBoLdsConsts;
  const float* wsig = lds + kBoLdsWsig;
  float* grow = tile_row(grad, s, kGradRow);
  if (valid && h == 0) {
    grow[tile_col(kGradSigma)] = dsp;
#pragma unroll
    for (int c = 0; c < 3; ++c) grow[tile_col(kGradRgb) + c] = dv[c];
  }
  // d hd rows; d pre_dir = d hd [r_dir > 0] (hd = ReLU(dir pre) + appearance): rows, max, split at
  // the exact maximum into operands 8..15 (the dir layer's 8 k-steps)
  Operand in[16];
  float m_dir = 0.0f;
  {
    const uint32_t* md = mwave + (lane & 31) * kMaskRow + (kMaskRDirByte + 8 * h) / 4;
    const uint32_t mk[2] = {md[0], md[1]};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 a, b;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = dhd[t][4 * q + e];
          b[e] = (mk[t / 2] >> (16 * (t % 2) + 4 * q + e)) & 1u ? a[e] : 0.0f;
          dhd[t][4 * q + e] = b[e];
          m_dir = fmaxf(m_dir, fabsf(b[e]));
        }
        if (store_dhd)   // (uniform; the training step's fused per-ray sums read none, param_grads)
          store16_rows<0>(a, ga.rows, ga.loff + 4u * (uint32_t)tile_col(kGradHd + 32 * t + 8 * q));
        store16_rows<0>(b, ga.rows, ga.loff + 4u * (uint32_t)tile_col(kGradDir + 32 * t + 8 * q));
      }
  }
  m_dir = sample_max(m_dir);
  // block exponent records (layout.h): lane j < 8 gathers entry j; [dpre_dir | dsigma_pre] is entry 7
  float bexp = 0.0f;
  {
    const float rec = block_exp_record(wave_max_nn(fmaxf(m_dir, fabsf(dsp))));
    bexp = (lane & 31) == 7 ? rec : bexp;
  }
  // Every split scale carries the sample's sign sgn (odd samples negative).  The MFMA unit's f32
  // accumulation of f16 products is not correctly rounded and its error leans negative (-0.12 ulp
  // on average, profiles/r04/mfma_f16_accumulation_rounding.log); a gradient row of an odd sample is
  // computed negated, so its rounding error comes back with the opposite sign, and the per-column
  // errors cancel in the sums over samples that make the weight and bias gradients instead of adding
  // up.  (Each row's own error is unchanged; the sign is exact: the scales stay powers of two.)
  const float sgn = (lane & 1) ? -1.0f : 1.0f;
  const float s_dir = sgn * pow2_scale(m_dir);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) split_into(dhd[t][4 * q + e] * s_dir, in[8 + 2 * t + q / 2], 4 * (q & 1) + e);
  // d pre_7's scale: |W_dh^T g + dsigma w_sigma| <= C_dir max|g| + |dsigma| max|w_sigma|
  float s_cur = sgn * pow2_scale(cst[kT16C + 7] * m_dir + fabsf(dsp) * cst[kT16WsigMax]);
  float inv_prev = cst[kT16InvS + 7] / s_dir;

  // the weight stream: W^T fragments of dir_linear's h-part, then trunk layers 7 .. 1
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  const float* stream = packedT + kPackedT32Floats;
  const uint32_t lds_dma = (uint32_t)(uintptr_t)(lptr_t)lds + 1024u * wave;
  const uint32_t voff = 16u * lane + 1024u * wave;
  chunk_dma<0>(stream, 0, lds_dma, voff);
  chunk_dma<1>(stream, 1, lds_dma, voff);
  chunk_dma<2>(stream, 2, lds_dma, voff);
  wait_vmcnt<8>();
  __builtin_amdgcn_s_barrier();
  h16x8 a0[4][2], a1[4][2];
  read_kstep<0>(lds, a0, lane);
  f32x16 acc[8];
  float m = 0.0f;
  BwQuarter qv[2];
  using Yes = std::true_type;
  using No = std::false_type;

  // ---- dir layer: d h_7 = W_dh^T d pre_dir (8 k-steps, operands 8..15), 4 chunk-steps per group;
  // group B converts group A's tiles 0-3 (+ dsigma w_sigma, mask_7) into operands 0..7, two
  // quarters per half-step
  auto dir_operand = [&](auto i, auto kk) -> const Operand& { return in[8 + kstep_of(i, kk)]; };
  run_group<0, 4, 0, 3, kSideNone, true>(stream, 0, lds, lds_dma, voff, a0, a1, acc, lane, dir_operand, NoSide{});
  GradAt g_cur = ga, g_prev = ga;
  g_cur.slice = 7 * kHidden;
  g_cur.mlay = (kMaskLayerBytes / 4) * 7;
  run_group<1, 4, 0, 3, kSideHalf, true>(stream, 4, lds, lds_dma, voff, a0, a1, acc, lane, dir_operand,
                                         [&](auto i, auto kk, auto ph) __attribute__((always_inline)) {
                                           constexpr int hs = kstep_of(i, kk), P = decltype(ph)::value;
                                           bw_quarter<P, 0, 0, 2 * hs, true, true>(acc, inv_prev, dsp, wsig, h, s_cur,
                                                                                     in, m, qv[0], g_cur);
                                           bw_quarter<P, 0, 0, 2 * hs + 1, true, true>(acc, inv_prev, dsp, wsig, h,
                                                                                         s_cur, in, m, qv[1], g_cur);
                                         });

  // ---- trunk layers l = 7 .. 1: d h_{l-1} = W_l^T d pre_l.  On entry operands 0..7 hold d pre_l
  // tiles 0-3 split at s_cur, d h_l tiles 4-7 wait in acc[4..7] (unscaled by inv_prev), m holds the
  // max of d pre_l tiles 0-3.  Side-work schedule: mlp16_kernel's (kSidePrev / kSideCur).
  auto act_operand = [&](auto i, auto kk) -> const Operand& { return in[kstep_of(i, kk)]; };
  // group A's side: d pre_l tiles 4-7 (SG: layer 7 adds dsigma w_sigma)
  auto side_prev = [&](auto i, auto kk, auto ph, auto sg_tag) __attribute__((always_inline)) {
    constexpr int hs = kstep_of(i, kk), P = decltype(ph)::value;
    constexpr bool sg = decltype(sg_tag)::value;
    if constexpr (hs == 0) {
      bw_quarter<P, 4, 8, 0, sg, true>(acc, inv_prev, dsp, wsig, h, s_cur, in, m, qv[0], g_prev);
      bw_quarter<P, 4, 8, 1, sg, true>(acc, inv_prev, dsp, wsig, h, s_cur, in, m, qv[1], g_prev);
    } else if constexpr (hs <= 14) {
      bw_quarter<P, 4, 8, hs + 1, sg, true>(acc, inv_prev, dsp, wsig, h, s_cur, in, m, qv[0], g_prev);
    }
  };
  float s_nxt = 0.0f, inv_cur = 0.0f;
  // group B's side: d pre_{l-1} tiles 0-3 (SP: split for the next layer; layer 0 has no consumer)
  auto side_cur = [&](auto i, auto kk, auto ph, auto sp_tag) __attribute__((always_inline)) {
    constexpr int hs = kstep_of(i, kk), P = decltype(ph)::value;
    constexpr bool sp = decltype(sp_tag)::value;
    if constexpr (hs >= 1 && hs <= 14) {
      bw_quarter<P, 0, 0, hs - 1, false, sp>(acc, inv_cur, 0.0f, wsig, h, s_nxt, in, m, qv[0], g_cur);
    } else if constexpr (hs == 15) {
      bw_quarter<P, 0, 0, 14, false, sp>(acc, inv_cur, 0.0f, wsig, h, s_nxt, in, m, qv[0], g_cur);
      bw_quarter<P, 0, 0, 15, false, sp>(acc, inv_cur, 0.0f, wsig, h, s_nxt, in, m, qv[1], g_cur);
    }
  };
  auto layer = [&](int l, auto sg_tag, auto last_tag) __attribute__((always_inline)) {
    constexpr bool last = decltype(last_tag)::value;
    const int c0 = 8 + (7 - l) * 16;
    g_prev.slice = l * kHidden;
    g_prev.mlay = (kMaskLayerBytes / 4) * l;
    g_cur.slice = (l - 1) * kHidden;
    g_cur.mlay = (kMaskLayerBytes / 4) * (l - 1);
    inv_cur = cst[kT16InvS + l - 1] / s_cur;
    run_group<0, 8, 0, 3, kSidePrev, true>(stream, c0, lds, lds_dma, voff, a0, a1, acc, lane, act_operand,
                                           [&](auto i, auto kk, auto ph) __attribute__((always_inline)) {
                                             side_prev(i, kk, ph, sg_tag);
                                           });
    // the inputs of this layer are complete: the scale of d pre_{l-1} from the bound
    m = sample_max(m);
    {   // m = the sample's max |d pre_l|: entry l - 1 (uniform over the wave)
      const float rec = block_exp_record(wave_max_nn(m));
      bexp = (lane & 31) == l - 1 ? rec : bexp;
    }
    s_nxt = sgn * pow2_scale(cst[kT16C + l - 1] * m);
    m = 0.0f;
    if constexpr (last) {
      run_group<1, 8, 0, 0, kSideCur, true>(stream, c0 + 8, lds, lds_dma, voff, a0, a1, acc, lane, act_operand,
                                            [&](auto i, auto kk, auto ph) __attribute__((always_inline)) {
                                              side_cur(i, kk, ph, No{});
                                            });
    } else {
      run_group<1, 8, 0, 3, kSideCur, true>(stream, c0 + 8, lds, lds_dma, voff, a0, a1, acc, lane, act_operand,
                                            [&](auto i, auto kk, auto ph) __attribute__((always_inline)) {
                                              side_cur(i, kk, ph, Yes{});
                                            });
    }
    inv_prev = inv_cur;
    s_cur = s_nxt;
  };
  layer(7, Yes{}, No{});
#pragma unroll 1
  for (int l = 6; l >= 2; --l) layer(l, No{}, No{});
  layer(1, No{}, Yes{});
  // d pre_0 tiles 4-7: exposed (no MFMA left to hide behind)
  g_prev.slice = 0;
  g_prev.mlay = 0;
  static_for<16>([&](auto qc) __attribute__((always_inline)) {
    constexpr int QG = decltype(qc)::value;
    bw_quarter<0, 4, 8, QG, false, false>(acc, inv_prev, 0.0f, wsig, h, 0.0f, in, m, qv[0], g_prev);
    bw_quarter<1, 4, 8, QG, false, false>(acc, inv_prev, 0.0f, wsig, h, 0.0f, in, m, qv[0], g_prev);
  });
  {   // m = the sample's max |d pre_0| (tiles 0-3 from layer 1's group B, 4-7 above): entry 8, read by
      // the split-f16 layer-0 / skip-PE pair (wgrad_pair16_kernel)
    const float rec = block_exp_record(wave_max_nn(sample_max(m)));
    bexp = (lane & 31) == 8 ? rec : bexp;
  }
  // the records: sample j's feature kMetaGradF (lane half 1 writes a 0 four pad floats on; tail lanes'
  // offsets lie outside the buffer range)
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(h == 0 && (lane & 31) < 9 ? bexp : 0.0f), ga.rows,
                                        (int)ga.loff + 4 * (int)(tile_col(kMetaGradF) + kMetaGradF % 8), 0, 0);
}

// store_dhd = false (nerf_train_backward on the fused path of param_grads): the mask-row kernel leaves
// the d hd columns of the gradient rows unwritten (nothing reads them there).
int launch_mlp_backward(const float* packed, const float* packedT, const float* save, const uint32_t* masks,
                        const float* sigma, const float* rgb, const float* dsigma, const float* drgb, int64_t M,
                        float* grad, hipStream_t s, bool store_dhd = true) {
  if (M == 0) return NERF_OK;
  // tile-major gradient rows: the last block's rows past M are zeros (layout.h); its tail lanes store nothing
  if (M % 32 && hipMemsetAsync(grad + (M / 32) * 32 * kGradRow, 0, (size_t)32 * kGradRow * 4, s) != hipSuccess)
    return set_error(NERF_ERR_HIP, "mlp backward: hipMemsetAsync failed");
  if (g_mlp_arith == NERF_ARITH_F16X3) {
    if (masks)
      hipLaunchKernelGGL(mlp_backward16_bound_kernel, dim3((unsigned)((M + 127) / 128)), dim3(256), 0, s, packed,
                         packedT, masks, sigma, rgb, dsigma, drgb, M, grad, (int)store_dhd);
    else
      hipLaunchKernelGGL(mlp_backward16_kernel, dim3((unsigned)((M + 127) / 128)), dim3(256), 0, s, packed,
                         packedT, save, sigma, rgb, dsigma, drgb, M, grad);
    return check_launch("mlp_backward16_kernel");
  }
  hipLaunchKernelGGL(mlp_backward_kernel, dim3((unsigned)((M + 127) / 128)), dim3(256), 0, s, packed, packedT, save,
                     sigma, rgb, dsigma, drgb, M, grad);
  return check_launch("mlp_backward_kernel");
}

// ---------------------------------------------------------------------------------- wgrad
// partial[c][n*KP + k'] = sum over samples m of chunk c of a[m][n] * x'[m][k'], k' < KP = K + 1,
// where x'[m][k] = x[xrow(m)][k] for k < K and x'[m][K] = 1 (the bias column).  xrow(m) = m / x_div
// (x_div = 1: a per-sample input; = N: a per-ray input; 0: one broadcast row).  Each chunk's
// partial occupies wgrad_stride(N, K) floats (N*KP rounded up to 4, for 16-byte reduce loads, + 4).
constexpr int kWChunk = 2048;   // samples per chunk
// Chunk length of a (N, K) weight gradient outside the split-f16 GEMMs: short enough that a 2^18-sample
// step puts a block in every resident slot.  The 256x64-tile launches (K <= 64, N > 64: layer 0
// and the appearance projection) hold one block per CU and have one tile: 1024-sample chunks give
// 256 blocks instead of 128.  The 128x128-tile launches hold two blocks per CU; those with fewer
// than 3 tiles (the sigma and rgb heads) take 1024 / 512-sample chunks.
// (N = 160: dir_linear's 128 rows + the density head's, the tile-major training path only)
static inline bool wgrad_whole_tile(int N, int K) { return (N == 256 || N == 160) && K == 256; }
// Whole-tile chunks of 2,048 samples (128 per 262K-sample step, half the CUs): on split-f16 the
// launches are bound by HBM, not MFMA, and halving the chunk partials (~0.5 GB per step written and
// read back) paid +1.7 % on the training step against 1,024-sample chunks (same-box A/B,
// profiles/r05/ab_head3_pe_clen2k.log; under bf16x6 the 2,048-sample chunks had been 3.5 % slower).
// (Round 6, same box: 4,096-sample whole-tile chunks -11 % on the step, 64 chunks leave CUs idle; the
// layer-0 / skip-PE pair on 2,048-sample chunks instead of 1,024 +1.1 %, its partials halved:
// profiles/r06/ab_train_chunks.log.)
constexpr int kWholeClen = kWChunk, kWholeMinChunks = 128;       // whole-tile chunk length, minimum chunk count
constexpr int kPairClen = kWChunk, kPairMinChunks = 128;          // the layer-0 / skip-PE pair's
static inline int wgrad_chunk_len_big(int N, int K) {
  if (wgrad_whole_tile(N, K)) return kWholeClen;   // one block per chunk, 256 per step
  if (K <= 64 && N == 2 * kHidden) return kPairClen;   // (the layer-0 / skip-PE pair)
  if (K <= 64 && N > 64) return kWChunk / 2;       // (wgrad_bf_k64_kernel: 512-sample chunks ran the GEMM
                                                    // 3 % faster but doubled the reduction)
  const int tiles = ((N + 127) / 128) * ((K + 127) / 128);
  return tiles == 1 ? kWChunk / 4 : tiles == 2 ? kWChunk / 2 : kWChunk;
}
// Short GEMMs (the per-ray ones over B rows) halve the chunk down to one 16-sample stage until
// there are >= 256 chunks: 4,096 rays in 1,024-row chunks ran 8 blocks, 80-100 us per launch.
static inline int wgrad_chunk_len(int N, int K, int64_t M) {
  int c = wgrad_chunk_len_big(N, K);
  const int min_chunks = wgrad_whole_tile(N, K) ? kWholeMinChunks : (K <= 64 && N == 2 * kHidden) ? kPairMinChunks : 256;
  while (c > 16 && (M + c - 1) / c < min_chunks) c /= 2;
  return c;
}

// (+ 4 trailing floats: the split-f16 kernel's chunk exponent, wgrad_h16w_kernel)
NERF_HD inline int64_t wgrad_stride(int N, int K) { return ((((int64_t)N * (K + 1)) + 3) & ~(int64_t)3) + 4; }

// Fallback (unaligned operands): one wave per 32 (n) x 64 (k') tile of one chunk, operands
// loaded straight from global memory (A = a^T fragment: n = l&31, sample = l>>5; B = x'
// fragment: sample = l>>5, k = l&31).
__global__ void __launch_bounds__(256)
wgrad_kernel(const float* __restrict__ a, int64_t lda, int N, const float* __restrict__ x, int64_t ldx, int K,
             int64_t x_div, int64_t M, float* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int KP = K + 1;
  const int ntn = (N + 31) / 32, ntk = (KP + 63) / 64;
  const int tile = blockIdx.x * 4 + wave;
  if (tile >= ntn * ntk) return;
  const int n0 = (tile / ntk) * 32, k0 = (tile % ntk) * 64;
  const int64_t m0 = (int64_t)blockIdx.y * kWChunk;
  const int64_t m1 = m0 + kWChunk < M ? m0 + kWChunk : M;
  const int n = n0 + (lane & 31);
  const int ka = k0 + (lane & 31), kb = ka + 32;
  const int hm = lane >> 5;
  f32x16 acc0 = f32x16{}, acc1 = f32x16{};
  double bsum = 0.0;                  // the bias column, in double (one rounding per chunk)
  // uniform trip count for the whole wave (MFMA is a wave-wide instruction); a sample past the
  // chunk end contributes a zero a-operand
  const int pairs = (int)((m1 - m0 + 1) / 2);
  const int64_t mlast = m1 - 1;
  for (int p = 0; p < pairs; ++p) {
    const int64_t m = m0 + 2 * p + hm;
    const int64_t mc = m < mlast ? m : mlast;
    const float av = (n < N && m <= mlast) ? a[mc * lda + n] : 0.0f;
    bsum += (double)av;
    const int64_t xr = x_div == 0 ? 0 : (x_div == 1 ? mc : mc / x_div);
    const float x0 = ka < K ? x[xr * ldx + ka] : (ka == K ? 1.0f : 0.0f);
    const float x1 = kb < K ? x[xr * ldx + kb] : (kb == K ? 1.0f : 0.0f);
    acc0 = mfma32t(av, x0, acc0);
    acc1 = mfma32t(av, x1, acc1);
  }
  float* out = partial + (size_t)blockIdx.y * wgrad_stride(N, K);
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int row = n0 + (g & 3) + 8 * (g >> 2) + 4 * hm;
    if (row < N) {
      if (ka < KP) out[(size_t)row * KP + ka] = acc0[g];
      if (kb < KP) out[(size_t)row * KP + kb] = acc1[g];
    }
  }
  // the bias column again from the double sum (the MFMA's f32 value above is overwritten; stores of
  // one wave land in program order)
  bsum += __shfl_xor(bsum, 32);
  if (K >= k0 && K < k0 + 64 && hm == 0 && n < N) out[(size_t)n * KP + K] = (float)bsum;
}

// The main weight-gradient kernel.  A workgroup computes a (64 WN) x (64 WK) output tile of one
// 2048-sample chunk (WN * WK = 4 waves, each owning 64 x 64 = 2 x 2 accumulator tiles of
// v_mfma_f32_32x32x2_f32), streaming the chunk's a and x rows through LDS 16 samples at a time,
// double-buffered: the next stage's 16-byte global loads are in flight while the current
// stage's MFMAs run, one barrier per stage.  Per k-step (two samples) a wave reads 4 operand
// values from LDS for 4 MFMAs; a wave whose n or k range lies past N or K skips its MFMAs.  The
// bias column (sum over samples of a[m][n]) is accumulated from the staged a values by the
// k-tile-0 workgroups on the VALU.  Workgroups sharing a chunk are launched 8 apart so they run
// on the same XCD (blockIdx -> XCD is round-robin) and the chunk's rows come from HBM once per L2.
// Tile shapes: WN=2, WK=2 (128 x 128) for the 256-wide layers; WN=4, WK=1 (256 x 64) when K <= 64.
// Preconditions (host-checked): a, x 16-byte aligned, lda % 4 == 0, ldx % 4 == 0.
constexpr int kWS = 16;        // samples per LDS stage

__device__ __forceinline__ f32x4 load4_masked(const float* __restrict__ p, int valid) {
  if (valid >= 4) return *reinterpret_cast<const f32x4*>(p);
  f32x4 v;
  v[0] = valid > 0 ? p[0] : 0.0f;
  v[1] = valid > 1 ? p[1] : 0.0f;
  v[2] = valid > 2 ? p[2] : 0.0f;
  v[3] = 0.0f;
  return v;
}

// BLK: a in the tile-major row layout (layout.h), and x too when xblk (then x_div == 1); lda / ldx their
// row lengths.
template <int WN, int WK, bool BLK>
__global__ void __launch_bounds__(256, 2)
wgrad_lds_kernel(const float* __restrict__ a, int64_t lda, int N, const float* __restrict__ x, int64_t ldx, int K,
                 int64_t x_div, int xblk, int64_t M, int ntk, int tiles, int chunks, float* __restrict__ partial) {
  static_assert(WN * WK == 4, "four waves");
  constexpr int BN = 64 * WN, BK = 64 * WK;
  constexpr int APAD = BN + 32, XPAD = BK + 32;    // row s+1 lands 32 banks away from row s
  constexpr int AC4 = BN / 4, XC4 = BK / 4;        // float4 columns per staged row
  __shared__ float As[2][kWS][APAD];
  __shared__ float Xs[2][kWS][XPAD];
  __shared__ double bsum[256 / AC4][BN];
  const int b = blockIdx.x;
  const int grp = b / (8 * tiles), rem = b % (8 * tiles);
  const int chunk = grp * 8 + (rem & 7);
  const int tile = rem >> 3;
  if (chunk >= chunks) return;                     // uniform over the block, before any barrier
  const int n0 = (tile / ntk) * BN, k0 = (tile % ntk) * BK;
  const bool do_bias = (tile % ntk) == 0;
  const int64_t m0 = (int64_t)chunk * kWChunk;
  const int64_t m1 = m0 + kWChunk < M ? m0 + kWChunk : M;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wn = w % WN, wk = w / WN;
  // loader: thread tid moves float4 column tid % C4 of rows tid / C4 + (256 / C4) p
  const int a_c = (tid % AC4) * 4, a_r = tid / AC4;
  const int x_c = (tid % XC4) * 4, x_r = tid / XC4;
  constexpr int AROWS = 256 / AC4, XROWS = 256 / XC4;   // rows per pass
  const int a_valid = N - (n0 + a_c), x_valid = K - (k0 + x_c);
  f32x4 ra[WN], rx[WK];
  double bacc[4] = {0.0, 0.0, 0.0, 0.0};      // bias column in double: one rounding per chunk
  const f32x4 zero4 = {0.0f, 0.0f, 0.0f, 0.0f};
  auto load = [&](int64_t mb) __attribute__((always_inline)) {
    sfor<WN>([&](auto pc) __attribute__((always_inline)) {
      constexpr int p = decltype(pc)::value;
      const int64_t m = mb + a_r + AROWS * p;
      const float* ap = BLK ? a + tile_off(m, n0 + a_c, (int)lda) : a + m * lda + n0 + a_c;
      ra[p] = (m < m1 && a_valid > 0) ? load4_masked(ap, a_valid) : zero4;
    });
    sfor<WK>([&](auto pc) __attribute__((always_inline)) {
      constexpr int p = decltype(pc)::value;
      const int64_t m = mb + x_r + XROWS * p;
      const int64_t xr = x_div == 0 ? 0 : (x_div == 1 ? m : m / x_div);
      const float* xp = (BLK && xblk) ? x + tile_off(m, k0 + x_c, (int)ldx) : x + xr * ldx + k0 + x_c;
      rx[p] = (m < m1 && x_valid > 0) ? load4_masked(xp, x_valid) : zero4;
    });
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
    sfor<WN>([&](auto pc) __attribute__((always_inline)) {
      constexpr int p = decltype(pc)::value;
      *reinterpret_cast<f32x4*>(&As[buf][a_r + AROWS * p][a_c]) = ra[p];
      if (do_bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bacc[e] += (double)ra[p][e];
      }
    });
    sfor<WK>([&](auto pc) __attribute__((always_inline)) {
      constexpr int p = decltype(pc)::value;
      *reinterpret_cast<f32x4*>(&Xs[buf][x_r + XROWS * p][x_c]) = rx[p];
    });
  };
  const bool n_act0 = n0 + 64 * wn < N, n_act1 = n0 + 64 * wn + 32 < N;
  const bool k_act0 = k0 + 64 * wk < K, k_act1 = k0 + 64 * wk + 32 < K;
  f32x16 acc00 = f32x16{}, acc01 = f32x16{}, acc10 = f32x16{}, acc11 = f32x16{};
  const int nstages = (int)((m1 - m0 + kWS - 1) / kWS);
  load(m0);
  store(0);
  __syncthreads();
  const int h = lane >> 5, c = lane & 31;
  for (int st = 0; st < nstages; ++st) {
    const int buf = st & 1;
    if (st + 1 < nstages) load(m0 + (int64_t)kWS * (st + 1));
    if (n_act0 && k_act0) {
#pragma unroll
      for (int ks = 0; ks < kWS / 2; ++ks) {
        const float* ar = &As[buf][2 * ks + h][64 * wn + c];
        const float* xr = &Xs[buf][2 * ks + h][64 * wk + c];
        const float a0 = ar[0], a1 = ar[32], x0 = xr[0], x1 = xr[32];
        acc00 = mfma32t(a0, x0, acc00);
        if (k_act1) acc01 = mfma32t(a0, x1, acc01);
        if (n_act1) acc10 = mfma32t(a1, x0, acc10);
        if (n_act1 && k_act1) acc11 = mfma32t(a1, x1, acc11);
      }
    }
    if (st + 1 < nstages) store(buf ^ 1);
    __syncthreads();
  }
  const int KP = K + 1;
  float* out = partial + (size_t)chunk * wgrad_stride(N, K);
  auto emit = [&](const f32x16& acc, int i, int j) __attribute__((always_inline)) {
    const int kk = k0 + 64 * wk + 32 * j + c;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int nn = n0 + 64 * wn + 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;
      if (nn < N && kk < K) out[(size_t)nn * KP + kk] = acc[g];
    }
  };
  emit(acc00, 0, 0);
  emit(acc01, 0, 1);
  emit(acc10, 1, 0);
  emit(acc11, 1, 1);
  if (do_bias) {
    // every staged a row passed through store() exactly once (the prologue stores stage 0)
#pragma unroll
    for (int e = 0; e < 4; ++e) bsum[a_r][a_c + e] = bacc[e];
    __syncthreads();
    if (tid < BN && n0 + tid < N) {
      double sum = 0.0;
#pragma unroll
      for (int r = 0; r < AROWS; ++r) sum += bsum[r][tid];
      out[(size_t)(n0 + tid) * KP + K] = (float)sum;
    }
  }
}

// The bf16x6 weight-gradient kernel of the split MLP arithmetic (nerf_arith F16X3; the GEMMs the
// split-f16 kernels below do not take: in training the per-ray GEMMs over gradient sums, otherwise
// nerf_wgrad's other shapes): the same
// partial sums as wgrad_lds_kernel, on v_mfma_f32_32x32x16_bf16.  Every operand value is split into
// three bf16 parts, x = b0 + b1 + b2 + O(2^-27 x) (each part the RNE bf16 of the f32 remainder, the
// remainders exact), and a k-step accumulates the six products of order >= 2^-16,
//   b0c2 + b1c1 + b2c0 + b0c1 + b1c0 + b0c0   (small terms first; dropped ones O(2^-24)),
// so the result has fp32-level error, at 6 x 32 MFMA cycles per 16 samples against 8 x 64 for
// v_mfma_f32_32x32x2_f32.  bf16 has f32's exponent range: no scaling (gradient rows reach 1e-9).
// A workgroup computes a (64 WN) x (64 WK) tile of one 2048-sample chunk; 16-sample stages are
// split by the loader (a thread owns 8 samples of one column: 8 coalesced dword loads, three
// 16-byte LDS writes) into [part][column][sample] rows of 24 bf16 (48-byte stride: the MFMA
// operand reads, 16 bytes per lane from 16 consecutive rows, are bank-conflict free), double
// buffered with the next stage's loads in flight during the MFMAs.  The bias column sums the
// loader's f32 values.  Workgroups sharing a chunk are launched 8 apart (same XCD).
constexpr int kBfStage = 16;   // samples per stage = one MFMA k-step
constexpr int kBfRow = 24;     // bf16 per LDS row (16 samples + pad)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// XD1 (x_div == 1, one x row per sample: every trunk/head layer): the loader's per-sample offsets
// are stage-invariant VGPRs and only the buffer descriptors move per stage (no VALU address work;
// the generic x path divides and carries per sample, ~130 VALU per stage).
// BLK: a (and x when XD1) tile-major (layout.h): a stage of 16 samples lies in one 32-sample block,
// the stage's resource is based at its first sample's place in that block, a sample j of a slot at
// +32 j bytes; past the chunk end only the sentinel stage (an empty resource) and the zero padding
// of the last block are read.
template <int WN, int WK, bool XD1, bool BLK>
__global__ void __launch_bounds__(256, WN == 4 ? 1 : 2)   // 256 x 64 tiles: 94 KB of LDS, one block per CU
wgrad_bf_kernel(const float* __restrict__ a, int64_t lda, int N, const float* __restrict__ x, int64_t ldx, int K,
                int64_t x_div, int64_t M, int ntk, int tiles, int chunks, int clen, float* __restrict__ partial) {
  static_assert(WN * WK == 4, "four waves");
  constexpr int BN = 64 * WN, BK = 64 * WK;
  constexpr int SA = 2 * BN / 256 > 0 ? 2 * BN / 256 : 1;    // loader slots per thread (column, octet)
  constexpr int SX = 2 * BK / 256 > 0 ? 2 * BK / 256 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][3][BN][kBfRow];
  __shared__ __attribute__((aligned(16))) __bf16 Xs[2][3][BK][kBfRow];
  __shared__ double bsum[2][BN];
  const int b = blockIdx.x;
  const int grp = b / (8 * tiles), rem = b % (8 * tiles);
  const int chunk = grp * 8 + (rem & 7);
  const int tile = rem >> 3;
  if (chunk >= chunks) return;                     // uniform over the block, before any barrier
  const int n0 = (tile / ntk) * BN, k0 = (tile % ntk) * BK;
  const bool do_bias = (tile % ntk) == 0;
  const int64_t m0 = (int64_t)chunk * clen;
  const int64_t m1 = m0 + clen < M ? m0 + clen : M;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wn = w % WN, wk = w / WN;
  float ra[2][SA][8], rx[2][SX][8];   // two stages in flight: stage k's values in set k % 2
  double bacc[SA];                   // bias column in double: one rounding per chunk
#pragma unroll
  for (int q = 0; q < SA; ++q) bacc[q] = 0.0;
  // Operands through buffer loads (an out-of-range offset reads 0, so no branches in the loader).
  // a: one resource per stage, based at the stage's first row, sized to the chunk's remaining rows;
  // a slot's sample j sits at byte aoff + j*lda4 (past the resource for samples >= m1), and a
  // column >= N gets an offset >= 2^31 (> any resource size: host-checked lda < 2^18).
  // x: based at the chunk's first x row; sample m reads row xrow(m) - xrow(m0) = (r0 + rel) / xd
  // (rel = m - m0, r0 = m0 % xd; xd = 1 per sample, N per ray, "infinite" for one broadcast row),
  // stepped over a slot's 8 samples by a carry instead of a division.
  const uint32_t lda4 = (uint32_t)lda * 4u, ldx4 = (uint32_t)ldx * 4u;
  constexpr uint32_t kOut = 0x80000000u;
  uint32_t aoff[SA], xcol[SX];
#pragma unroll
  for (int q = 0; q < SA; ++q) {
    const int slot = tid + 256 * q, col = slot % BN, oct = slot / BN;
    const int nc = n0 + col;
    aoff[q] = (slot < 2 * BN && nc < N)
                  ? (BLK ? 4u * (uint32_t)(tile_col(nc) + nc % 8 + 64 * oct) : (uint32_t)(8 * oct) * lda4 + 4u * (uint32_t)nc)
                  : kOut;
  }
#pragma unroll
  for (int q = 0; q < SX; ++q) {
    const int slot = tid + 256 * q, col = slot % BK;
    xcol[q] = (slot < 2 * BK && k0 + col < K) ? 4u * (uint32_t)(k0 + col) : kOut;
  }
  uint32_t avo[SA][8], xvo[SX][8];   // XD1: sample j of a slot at a stage-invariant offset
#pragma unroll
  for (int q = 0; q < SA; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) avo[q][j] = aoff[q] == kOut ? kOut : aoff[q] + (uint32_t)j * (BLK ? 32u : lda4);
  if constexpr (XD1) {
#pragma unroll
    for (int q = 0; q < SX; ++q) {
      const int oct = (tid + 256 * q) / BK;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        xvo[q][j] = xcol[q] == kOut ? kOut
                    : BLK ? 4u * (uint32_t)(tile_col(xcol[q] / 4) + (xcol[q] / 4) % 8 + 8 * (8 * oct + j))
                          : (uint32_t)(8 * oct + j) * ldx4 + xcol[q];
    }
  }
  const uint32_t xd = x_div == 0 ? 0xFFFFFFFFu : (uint32_t)x_div;
  const int64_t xr0 = x_div == 0 ? 0 : m0 / x_div;
  const uint32_t r0 = x_div == 0 ? 0u : (uint32_t)(m0 - xr0 * x_div);
  const uint32_t xrows = x_div == 0 ? 1u : (uint32_t)((m1 - 1) / x_div - xr0 + 1);
  const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x + xr0 * ldx), (short)0, (int)(xrows * ldx4), 0x00020000);
  const uint32_t mrel_end = (uint32_t)(m1 - m0);
  // stage `stage` (< nstages) into register set SET; past the last stage it loads nothing
  auto load = [&](auto set_c, int stage) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    const uint32_t rel0 = (uint32_t)(kBfStage * stage);
    const int64_t ms = m0 + rel0;             // BLK: the stage's place in its block; empty past the chunk
    const bool live = rel0 < mrel_end;
    const __amdgpu_buffer_rsrc_t ares = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(BLK ? a + (ms / 32) * 32 * lda + (ms % 32) * 8 : a + ms * lda), (short)0,
        BLK ? (live ? (int)(32 * lda4 - (ms % 32) * 32) : 0) : (int)((mrel_end - rel0) * lda4), 0x00020000);
#pragma unroll
    for (int q = 0; q < SA; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        ra[SET][q][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ares, (int)avo[q][j], 0, kRowLoadAux));
    if constexpr (XD1) {
      const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(BLK ? x + (ms / 32) * 32 * ldx + (ms % 32) * 8 : x + ms * ldx), (short)0,
          BLK ? (live ? (int)(32 * ldx4 - (ms % 32) * 32) : 0) : (int)((mrel_end - rel0) * ldx4), 0x00020000);
#pragma unroll
      for (int q = 0; q < SX; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          rx[SET][q][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xs, (int)xvo[q][j], 0, kRowLoadAux));
      return;
    }
#pragma unroll
    for (int q = 0; q < SX; ++q) {
      const int slot = tid + 256 * q, oct = slot / BK;
      const uint32_t rel = rel0 + 8u * (uint32_t)oct;
      uint32_t row = (r0 + rel) / xd, r = (r0 + rel) - row * xd;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = rel + j < mrel_end && xcol[q] != kOut;
        const uint32_t off = ok ? row * ldx4 + xcol[q] : kOut;
        rx[SET][q][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xres, (int)off, 0, kRowLoadAux));
        if (++r == xd) {
          r = 0;
          ++row;
        }
      }
    }
  };
  auto split_store = [&](float (&v)[8], __bf16 (*dst)[kBfRow], int col, int oct, int plane_stride) {
    bf16x8 p0, p1, p2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const __bf16 h0 = (__bf16)v[j];
      const float r1 = v[j] - (float)h0;
      const __bf16 h1 = (__bf16)r1;
      const float r2 = r1 - (float)h1;
      p0[j] = h0;
      p1[j] = h1;
      p2[j] = (__bf16)r2;
    }
    *reinterpret_cast<bf16x8*>(&dst[col][8 * oct]) = p0;
    *reinterpret_cast<bf16x8*>(&dst[col + plane_stride][8 * oct]) = p1;
    *reinterpret_cast<bf16x8*>(&dst[col + 2 * plane_stride][8 * oct]) = p2;
  };
  auto store = [&](auto set_c, int buf) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
#pragma unroll
    for (int q = 0; q < SA; ++q) {
      const int slot = tid + 256 * q, col = slot % BN, oct = slot / BN;
      if (slot < 2 * BN) {
        if (do_bias) {
#pragma unroll
          for (int j = 0; j < 8; ++j) bacc[q] += (double)ra[SET][q][j];
        }
        split_store(ra[SET][q], &As[buf][0][0], col, oct, BN);
      }
    }
#pragma unroll
    for (int q = 0; q < SX; ++q) {
      const int slot = tid + 256 * q, col = slot % BK, oct = slot / BK;
      if (slot < 2 * BK) split_store(rx[SET][q], &Xs[buf][0][0], col, oct, BK);
    }
  };
  const bool n_act0 = n0 + 64 * wn < N, n_act1 = n0 + 64 * wn + 32 < N;
  const bool k_act0 = k0 + 64 * wk < K, k_act1 = k0 + 64 * wk + 32 < K;
  f32x16 acc[2][2] = {{f32x16{}, f32x16{}}, {f32x16{}, f32x16{}}};
  const int nstages = (int)((m1 - m0 + kBfStage - 1) / kBfStage);
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  // Loads run two stages ahead of the MFMAs: iteration st issues stage st+2's loads, splits stage
  // st+1's values (loaded a whole iteration earlier) into the other LDS buffer, and runs stage st's
  // MFMAs.  (One stage ahead, the split waited on loads issued only one MFMA stage before.)
  load(S0{}, 0);
  if (nstages > 1) load(S1{}, 1);
  store(S0{}, 0);
  __syncthreads();
  const int h = lane >> 5, c = lane & 31;
  auto iteration = [&](auto set_c, int st) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;            // st % 2
    using Other = std::integral_constant<int, 1 - SET>;
    const int buf = SET;
    if (st + 2 < nstages) load(set_c, st + 2);
    if (n_act0 && k_act0) {
      bf16x8 fa[2][3], fx[2][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          fa[i][p] = *reinterpret_cast<const bf16x8*>(&As[buf][p][64 * wn + 32 * i + c][8 * h]);
          fx[i][p] = *reinterpret_cast<const bf16x8*>(&Xs[buf][p][64 * wk + 32 * i + c][8 * h]);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if ((i == 1 && !n_act1) || (j == 1 && !k_act1)) continue;
          f32x16 t = acc[i][j];
          t = mfma_bf16(fa[i][0], fx[j][2], t);
          t = mfma_bf16(fa[i][1], fx[j][1], t);
          t = mfma_bf16(fa[i][2], fx[j][0], t);
          t = mfma_bf16(fa[i][0], fx[j][1], t);
          t = mfma_bf16(fa[i][1], fx[j][0], t);
          acc[i][j] = mfma_bf16(fa[i][0], fx[j][0], t);
        }
    }
    if (st + 1 < nstages) store(Other{}, buf ^ 1);
    __syncthreads();
  };
  for (int st = 0; st < nstages; st += 2) {
    iteration(S0{}, st);
    if (st + 1 < nstages) iteration(S1{}, st + 1);
  }
  const int KP = K + 1;
  float* out = partial + (size_t)chunk * wgrad_stride(N, K);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kk = k0 + 64 * wk + 32 * j + c;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int nn = n0 + 64 * wn + 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;
        if (nn < N && kk < K) out[(size_t)nn * KP + kk] = acc[i][j][g];
      }
    }
  if (do_bias) {
    // every staged a value passed through store() exactly once (the prologue stores stage 0)
#pragma unroll
    for (int q = 0; q < SA; ++q) {
      const int slot = tid + 256 * q, col = slot % BN, oct = slot / BN;
      if (slot < 2 * BN) bsum[oct][col] = bacc[q];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < N) out[(size_t)(n0 + tid) * KP + K] = (float)(bsum[0][tid] + bsum[1][tid]);
  }
}

// The whole-tile (256 x 256) weight gradients: the trunk layers' d pre_l over h_{l-1}, the skip
// layer's h3 block and dir/density over h7.
constexpr int kWT = 256;
__device__ __forceinline__ void split3_bf16(const float (&v)[8], bf16x8& p0, bf16x8& p1, bf16x8& p2) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h0 = (__bf16)v[j];
    const float r1 = v[j] - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    const float r2 = r1 - (float)h1;
    p0[j] = h0;
    p1[j] = h1;
    p2[j] = (__bf16)r2;
  }
}
// ------------------------------------------------- split-f16 ("f16x3") weight gradient, 256 columns
// The whole-tile GEMM (a chunk's 256 x 256 weight gradient in one workgroup) on
// v_mfma_f32_32x32x16_f16 with three products per fp32 product instead of bf16x6's six: every operand value is split as v s = hi + lo (f16 each, lo =
// f16(v s - hi), the residual exact in f32) and a k-step accumulates lo(a)hi(x) + hi(a)lo(x) +
// hi(a)hi(x) (small terms first; the dropped lo lo term and the split residual are O(2^-22) of the
// product), half the MFMAs and two thirds of the split VALU of bf16x6.  f16 lacks f32's exponent
// range, so each operand carries one power-of-two scale per chunk, s = 2^(14 - e) with e the
// exponent of the chunk's largest |value| (every v s < 2^14: no f16 overflow).  The MFMAs accumulate
// in place (AGPRs) at those scales and the partial is unscaled once at the store (exact: powers of
// two).  A value far below its chunk's maximum keeps an absolute error <= 2^-25 / s = 2^-39 of that
// maximum, far below an fp32 sum's rounding of the terms near it.
// The chunk maxima come from the producers: the f16x3 forward and data-gradient kernels record each
// 32-sample block's exponent per operand slice (layout.h, block exponents); the kernel takes the
// largest over its chunk's blocks.  Without records (rows from another writer) it first reads the
// chunk once to find them (workgroup-uniform branch before the GEMM).
constexpr int kH16EMin = -100;        // scale floor exponent (an all-zero or tiny chunk)
struct H16Meta {                      // where the block exponents of a and x are (nullable: absent)
  const float* a = nullptr;           // record of block 0; block b at + b * a_stride
  int64_t a_stride = 0;
  const float* x = nullptr;
  int64_t x_stride = 0;
  int a_cols = 256;                   // a columns whose values count (the partial's kept rows)
};

// v s = hi + lo for 8 values at scale s (hi by v_cvt_pk_f16_f32, lo by split_lo_pair)
__device__ __forceinline__ void split2_f16(const float (&v)[8], float s, h16x8& hi, h16x8& lo) {
  typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float x0 = v[2 * p] * s, x1 = v[2 * p + 1] * s;
    const h16x2 hi2 = {(_Float16)x0, (_Float16)x1};
    const h16x2 lo2 = __builtin_bit_cast(h16x2, split_lo_pair(__builtin_bit_cast(uint32_t, hi2), x0, x1));
    hi[2 * p] = hi2[0];
    hi[2 * p + 1] = hi2[1];
    lo[2 * p] = lo2[0];
    lo[2 * p + 1] = lo2[1];
  }
}

// The chunk's exponents (Ea, Ex; wave-uniform, the same in every wave of the workgroup) for the
// split-f16 whole-tile GEMMs: from the block records (lanes 0..31: one block each), else by a pass
// over the chunk's whole 32-sample blocks (the records' span: a chunk shorter than a block gets the
// exponents the records would give it; a: column tid of the staged rows, counting meta.a_cols of
// them; x: the wave's fragment columns).  wmax: 8 floats of LDS.
template <bool BLK>
__device__ __forceinline__ void h16_chunk_exps(const float* __restrict__ a, int64_t lda, const float* __restrict__ x,
                                               int64_t ldx, int64_t M, int64_t m0, int64_t m1, const H16Meta& meta,
                                               float (&wmax)[4][2], int& Ea, int& Ex) {
  const int tid = threadIdx.x, lane = tid & 63, wk = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int64_t b0 = m0 / 32, nb = (m1 - 1) / 32 - b0 + 1;   // blocks of the chunk (<= 64)
  float ra_rec = 0.0f, rx_rec = 0.0f, bad = 0.0f;            // 1000 + e of the lane's blocks; 1: a record absent
  if (meta.a && meta.x) {
    for (int64_t b = lane; b < nb; b += 64) {
      const float va = meta.a[(b0 + b) * meta.a_stride], vx = meta.x[(b0 + b) * meta.x_stride];
      bad = (block_exp_valid(va) && block_exp_valid(vx)) ? bad : 1.0f;
      ra_rec = fmaxf(ra_rec, -va);
      rx_rec = fmaxf(rx_rec, -vx);
    }
  }
  const bool have = meta.a && meta.x && wave_max_nn(bad) == 0.0f;   // uniform (every wave alike)
  if (have) {
    Ea = (int)wave_max_nn(ra_rec) - kBlockExpBias;
    Ex = (int)wave_max_nn(rx_rec) - kBlockExpBias;
  } else {
    const uint32_t lda4 = (uint32_t)lda * 4u, ldx4 = (uint32_t)ldx * 4u;
    const uint32_t avo = BLK ? 4u * (uint32_t)(tile_col(tid) + tid % 8) : 4u * (uint32_t)tid;
    const uint32_t as4 = BLK ? 32u : lda4, xs4 = BLK ? 32u : ldx4;
    uint32_t xvo[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int xc = 64 * wk + 32 * t + c;
      xvo[t] = BLK ? 4u * (uint32_t)(tile_col(xc) + xc % 8 + 64 * h) : (uint32_t)(8 * h) * ldx4 + 4u * (uint32_t)xc;
    }
    float ma = 0.0f, mx = 0.0f;
    const int64_t f0 = b0 * 32, f1 = (b0 + nb) * 32 < M ? (b0 + nb) * 32 : M;
    for (int64_t ms = f0; ms < f1; ms += kBfStage) {
      const uint32_t left = (uint32_t)(f1 - ms);
      const __amdgpu_buffer_rsrc_t ares = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(BLK ? a + (ms / 32) * 32 * lda + (ms % 32) * 8 : a + ms * lda), (short)0,
          BLK ? (int)(32 * lda4 - (ms % 32) * 32) : (int)((left < kBfStage ? left : kBfStage) * lda4), 0x00020000);
      const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(BLK ? x + (ms / 32) * 32 * ldx + (ms % 32) * 8 : x + ms * ldx), (short)0,
          BLK ? (int)(32 * ldx4 - (ms % 32) * 32) : (int)((left < kBfStage ? left : kBfStage) * ldx4), 0x00020000);
#pragma unroll
      for (int j = 0; j < 16; ++j)
        ma = fmaxf(ma, fabsf(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ares, (int)avo, (int)(j * as4), 0))));
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          mx = fmaxf(mx, fabsf(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xres, (int)xvo[t], (int)(j * xs4), 0))));
    }
    ma = wave_max_nn(tid < meta.a_cols ? ma : 0.0f);
    mx = wave_max_nn(mx);
    wmax[wk][0] = ma;                // (every lane the same value)
    wmax[wk][1] = mx;
    __syncthreads();
    ma = fmaxf(fmaxf(wmax[0][0], wmax[1][0]), fmaxf(wmax[2][0], wmax[3][0]));
    mx = fmaxf(fmaxf(wmax[0][1], wmax[1][1]), fmaxf(wmax[2][1], wmax[3][1]));
    Ea = (int)(-block_exp_record(ma)) - kBlockExpBias;
    Ex = (int)(-block_exp_record(mx)) - kBlockExpBias;
  }
  Ea = __builtin_amdgcn_readfirstlane(Ea < kH16EMin ? kH16EMin : Ea);
  Ex = __builtin_amdgcn_readfirstlane(Ex < kH16EMin ? kH16EMin : Ex);
}

typedef _Float16 H16Stage[2][2][kWT][kBfRow];   // [buffer][hi, lo][column][sample]
template <bool BLK, int NRT>
__device__ __forceinline__ void h16w_chunk(const float* __restrict__ a, int64_t lda, const float* __restrict__ x,
                                           int64_t ldx, int64_t M, int clen, const H16Meta& meta,
                                           float* __restrict__ partial, int chunk, H16Stage& As, float (&wmax)[4][2]) {
  const int64_t m0 = (int64_t)chunk * clen;
  const int64_t m1 = m0 + clen < M ? m0 + clen : M;
  const int tid = threadIdx.x, lane = tid & 63, wk = tid >> 6;   // wave wk: columns 64 wk ..
  const int h = lane >> 5, c = lane & 31;
  const uint32_t lda4 = (uint32_t)lda * 4u, ldx4 = (uint32_t)ldx * 4u;
  // (NRT < 8: the columns past the kept rows are not read: an offset beyond any buffer range)
  const uint32_t avo = tid >= 32 * NRT ? 0x80000000u : BLK ? 4u * (uint32_t)(tile_col(tid) + tid % 8) : 4u * (uint32_t)tid;
  const uint32_t as4 = BLK ? 32u : lda4, xs4 = BLK ? 32u : ldx4;
  uint32_t xvo[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int xc = 64 * wk + 32 * t + c;
    xvo[t] = BLK ? 4u * (uint32_t)(tile_col(xc) + xc % 8 + 64 * h) : (uint32_t)(8 * h) * ldx4 + 4u * (uint32_t)xc;
  }
  const uint32_t mrel_end = (uint32_t)(m1 - m0);
  float ra[4][16], rx[4][2][8];
  double bacc = 0.0;
  auto load = [&](auto set_c, int stage) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    const uint32_t rel0 = (uint32_t)(kBfStage * stage) < mrel_end ? (uint32_t)(kBfStage * stage) : mrel_end;
    const int64_t ms = m0 + rel0;
    const bool live = rel0 < mrel_end;
    const __amdgpu_buffer_rsrc_t ares = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(BLK ? a + (ms / 32) * 32 * lda + (ms % 32) * 8 : a + ms * lda), (short)0,
        BLK ? (live ? (int)(32 * lda4 - (ms % 32) * 32) : 0) : (int)((mrel_end - rel0) * lda4), 0x00020000);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(BLK ? x + (ms / 32) * 32 * ldx + (ms % 32) * 8 : x + ms * ldx), (short)0,
        BLK ? (live ? (int)(32 * ldx4 - (ms % 32) * 32) : 0) : (int)((mrel_end - rel0) * ldx4), 0x00020000);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      ra[SET][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ares, (int)avo, (int)(j * as4), kRowLoadAux));
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        rx[SET][t][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xres, (int)xvo[t], (int)(j * xs4), kRowLoadAux));
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;

  // ---- the chunk's exponents (records, else a pass over the chunk)
  int Ea, Ex;
  h16_chunk_exps<BLK>(a, lda, x, ldx, M, m0, m1, meta, wmax, Ea, Ex);
  const float sa = ldexpf(1.0f, 14 - Ea), sx = ldexpf(1.0f, 14 - Ex);

  h16x8 fx[2][2][2];                   // split x fragments of stages st (fx[st & 1]) and st+1: [t][hi, lo]
  auto split_x = [&](auto set_c, auto fb_c) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value, FB = decltype(fb_c)::value;
#pragma unroll
    for (int t = 0; t < 2; ++t) split2_f16(rx[SET][t], sx, fx[FB][t][0], fx[FB][t][1]);
  };
  auto split_a = [&](auto set_c, int buf) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
#pragma unroll
    for (int j = 0; j < 16; ++j) bacc += (double)ra[SET][j];
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = ra[SET][8 * o + j];
      h16x8 hi, lo;
      split2_f16(v, sa, hi, lo);
      *reinterpret_cast<h16x8*>(&As[buf][0][tid][8 * o]) = hi;
      *reinterpret_cast<h16x8*>(&As[buf][1][tid][8 * o]) = lo;
    }
  };
  f32x16 acc[NRT][2];
#pragma unroll
  for (int i = 0; i < NRT; ++i) acc[i][0] = acc[i][1] = f32x16{};
  const int nstages = (int)((mrel_end + 4 * kBfStage - 1) / (4 * kBfStage)) * 4;
  load(C0{}, 0);
  load(C1{}, 1);
  load(C2{}, 2);
  split_x(C0{}, C0{});
  split_a(C0{}, 0);
  __syncthreads();
  // iteration st (set st % 4, buffers st % 2): stage st+3's loads; stage st's MFMAs with stage st+1's
  // splits in their shadow; barrier
  auto iteration = [&](auto set_c, int st) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value, FB = SET & 1;
    using Nxt = std::integral_constant<int, (SET + 1) & 3>;
    using Ld = std::integral_constant<int, (SET + 3) & 3>;
    using FBn = std::integral_constant<int, FB ^ 1>;
    load(Ld{}, st + 3);
    __builtin_amdgcn_sched_barrier(0);
    h16x8 fa[2][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) fa[0][p] = *reinterpret_cast<const h16x8*>(&As[FB][p][c][8 * h]);
#pragma unroll
    for (int i = 0; i < NRT; ++i) {
      if (i + 1 < NRT) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
          fa[(i + 1) & 1][p] = *reinterpret_cast<const h16x8*>(&As[FB][p][32 * (i + 1) + c][8 * h]);
      }
      const h16x8 (&f)[2] = fa[i & 1];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16 t = acc[i][j];
        t = mfma16(f[1], fx[FB][j][0], t);
        t = mfma16(f[0], fx[FB][j][1], t);
        acc[i][j] = mfma16(f[0], fx[FB][j][0], t);
      }
    }
    split_x(Nxt{}, FBn{});
    split_a(Nxt{}, FB ^ 1);
    // schedule: per row tile 2 fragment reads (the next tile's), then its 6 MFMAs each followed by
    // VALU of the next stage's splits; the split's LDS writes last
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);         // tile 0's reads
#pragma unroll
    for (int i = 0; i < NRT; ++i) {
      if (i + 1 < NRT) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS reads (tile i+1)
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, NRT >= 8 ? 2 : 3, 0);     // VALU
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x200, 4, 0);         // DS writes
    __syncthreads();
  };
  for (int st = 0; st < nstages; st += 4) {
    iteration(C0{}, st);
    iteration(C1{}, st + 1);
    iteration(C2{}, st + 2);
    iteration(std::integral_constant<int, 3>{}, st + 3);
  }
  // the partial at the chunk's scales; its exponent eo (true = stored 2^eo) in the partial's trailing
  // slot, applied by the reduction (a VALU unscale here would pull the accumulators out of the AGPRs)
  constexpr int KP = kWT + 1;
  const int64_t stride = wgrad_stride(32 * NRT, kWT);
  float* out = partial + (size_t)chunk * stride;
#pragma unroll
  for (int i = 0; i < NRT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kk = 64 * wk + 32 * j + c;
#pragma unroll
      for (int g = 0; g < 16; ++g) out[(size_t)(32 * i + (g & 3) + 8 * (g >> 2) + 4 * h) * KP + kk] = acc[i][j][g];
    }
  if (tid < 32 * NRT) out[(size_t)tid * KP + kWT] = (float)bacc;   // (the bias column: unscaled)
  if (tid == 0) reinterpret_cast<int*>(out)[stride - 4] = Ea + Ex - 28;   // acc = sum (a 2^(14-Ea)) (x 2^(14-Ex))
}

template <bool BLK, int NRT = 8>
__global__ void __launch_bounds__(256, 1)
wgrad_h16w_kernel(const float* __restrict__ a, int64_t lda, const float* __restrict__ x, int64_t ldx, int64_t M,
                  int clen, H16Meta meta, float* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) H16Stage As;
  __shared__ float wmax[4][2];
  h16w_chunk<BLK, NRT>(a, lda, x, ldx, M, clen, meta, partial, blockIdx.x, As, wmax);
}

// The same 256 x 256 GEMM (tile-major rows) with two workgroups per CU: each workgroup computes half
// the output rows (a columns 128 half .. +127: 4 row tiles x 2 column tiles per wave, 128 accumulators)
// so the two workgroups' waves (two per SIMD) fill each other's load, split and barrier waits, which a
// lone workgroup per CU runs in lock-step ("What bounds the phase now").  Both halves read
// all of x: block b runs chunk (b / 16) 8 + b % 8, half (b / 8) % 2, so the halves of a chunk sit on
// one XCD (b and b + 8) and the second read of x hits its L2.  NS raw-load sets: loads run NS - 1
// stages ahead; the x split runs just before its stage's MFMAs (one fragment set, not two).
// nrows < 256 (the dir/density launch: 160): a columns from nrows on are not read (zeros) and
// output rows from nrows on are not stored; the partial has nrows rows (wgrad_stride(nrows, 256)).
// The bias column: each a column has two threads (samples 0-7 and 8-15 of every stage), each summing
// in double; their sums are added once at the end (wgrad_h16w_kernel: one thread, all 16).
// SUMS (the dir/density launch, rays of N % 32 == 0 samples): the threads of a columns 0..127
// (d pre_dir) also write each stage's sum of their 8 raw values (in double, rounded once) to
// sums[(m / 8) * 128 + column], m the first of the 8 samples: the per-ray inputs' GEMMs (dir_linear's
// PE_4(d) columns) then run over M / 8 rows of these sums instead of re-reading the gradient rows
// (ray_sums_kernel's 256 columns per sample).
template <int NS, bool SUMS = false>
__global__ void __launch_bounds__(256, 2)
wgrad_h16h_kernel(const float* __restrict__ a, int64_t lda, const float* __restrict__ x, int64_t ldx, int64_t M,
                  int clen, int chunks, int nrows, H16Meta meta, float* __restrict__ partial,
                  float* __restrict__ sums = nullptr) {
  __shared__ __attribute__((aligned(16))) _Float16 As[2][2][128][kBfRow];   // [buffer][hi, lo][column][sample]
  __shared__ float wmax[4][2];
  __shared__ double bsum[128];
  const int b = blockIdx.x;
  const int chunk = (b >> 4) * 8 + (b & 7), half = (b >> 3) & 1;
  if (chunk >= chunks) return;
  const int64_t m0 = (int64_t)chunk * clen;
  const int64_t m1 = m0 + clen < M ? m0 + clen : M;
  const int tid = threadIdx.x, lane = tid & 63, wk = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const uint32_t lda4 = (uint32_t)lda * 4u, ldx4 = (uint32_t)ldx * 4u;
  const int ac = 128 * half + (tid & 127), as0 = 8 * (tid >> 7);   // the thread's a column, its first sample
  // a columns past the kept rows' whole feature groups (meta.a_cols; the dir/density launch: 129 of 160
  // -> 136) are not read: their rows are dropped, and an offset beyond the resource reads 0
  const int acols = (meta.a_cols + 7) / 8 * 8 < nrows ? (meta.a_cols + 7) / 8 * 8 : nrows;
  const uint32_t avo = ac < acols ? 4u * (uint32_t)(tile_col(ac) + ac % 8) + 32u * (uint32_t)as0 : 0x80000000u;
  uint32_t xvo[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int xc = 64 * wk + 32 * t + c;
    xvo[t] = 4u * (uint32_t)(tile_col(xc) + xc % 8 + 64 * h);
  }
  const uint32_t mrel_end = (uint32_t)(m1 - m0);
  float ra[NS][8], rx[NS][2][8];
  double bacc = 0.0;
  auto load = [&](auto set_c, int stage) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    const uint32_t rel0 = (uint32_t)(kBfStage * stage) < mrel_end ? (uint32_t)(kBfStage * stage) : mrel_end;
    const int64_t ms = m0 + rel0;
    const bool live = rel0 < mrel_end;
    const __amdgpu_buffer_rsrc_t ares = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a + (ms / 32) * 32 * lda + (ms % 32) * 8), (short)0,
        live ? (int)(32 * lda4 - (ms % 32) * 32) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(x + (ms / 32) * 32 * ldx + (ms % 32) * 8), (short)0,
        live ? (int)(32 * ldx4 - (ms % 32) * 32) : 0, 0x00020000);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      ra[SET][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ares, (int)avo, j * 32, kRowLoadAux));
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        rx[SET][t][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xres, (int)xvo[t], j * 32, kRowLoadAux));
  };
  int Ea, Ex;
  h16_chunk_exps<true>(a, lda, x, ldx, M, m0, m1, meta, wmax, Ea, Ex);
  const float sa = ldexpf(1.0f, 14 - Ea), sx = ldexpf(1.0f, 14 - Ex);
  __amdgpu_buffer_rsrc_t sres;   // SUMS: this chunk's rows of 8-sample sums (half 0 only)
  if constexpr (SUMS)
    sres = __builtin_amdgcn_make_buffer_rsrc(sums + (m0 / 8) * kDirHidden, (short)0,
                                             half == 0 ? (int)(mrel_end / 8 * kDirHidden * 4) : 0, 0x00020000);
  auto split_a = [&](auto set_c, int buf, int stage) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    double ps = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) ps += (double)ra[SET][j];
    bacc += ps;
    // float (m0 + 16 stage + as0) / 8 * 128 + (tid & 127) = (m0 / 8 + 2 stage) 128 + tid; past the
    // chunk (and in the half-1 workgroups) the store falls outside the resource and is dropped
    if constexpr (SUMS)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)ps), sres, 4 * tid, 2 * kDirHidden * 4 * stage,
                                            kRowStoreAux);
    h16x8 hi, lo;
    split2_f16(ra[SET], sa, hi, lo);
    *reinterpret_cast<h16x8*>(&As[buf][0][tid & 127][as0]) = hi;
    *reinterpret_cast<h16x8*>(&As[buf][1][tid & 127][as0]) = lo;
  };
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x16{};
  constexpr int U = NS % 2 ? 2 * NS : NS;
  const int nstages = (int)((mrel_end + U * kBfStage - 1) / (U * kBfStage)) * U;   // (extra stages add zeros)
  load(std::integral_constant<int, 0>{}, 0);
  if constexpr (NS > 2) load(std::integral_constant<int, (NS > 2 ? 1 : 0)>{}, 1);
  if constexpr (NS > 3) load(std::integral_constant<int, (NS > 3 ? 2 : 0)>{}, 2);
  split_a(std::integral_constant<int, 0>{}, 0, 0);
  __syncthreads();
  // iteration st (IT = st mod U: set IT % NS, buffer IT % 2): stage st+NS-1's loads; stage st's x
  // split and MFMAs, stage st+1's a split in their shadow; barrier
  auto iteration = [&](auto it_c, int st) __attribute__((always_inline)) {
    constexpr int IT = decltype(it_c)::value, SET = IT % NS, FB = IT & 1;
    using Nxt = std::integral_constant<int, (IT + 1) % NS>;
    using Ld = std::integral_constant<int, (IT + NS - 1) % NS>;
    load(Ld{}, st + NS - 1);
    __builtin_amdgcn_sched_barrier(0);
    h16x8 fx[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) split2_f16(rx[SET][t], sx, fx[t][0], fx[t][1]);
    h16x8 fa[2][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) fa[0][p] = *reinterpret_cast<const h16x8*>(&As[FB][p][c][8 * h]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i + 1 < 4) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
          fa[(i + 1) & 1][p] = *reinterpret_cast<const h16x8*>(&As[FB][p][32 * (i + 1) + c][8 * h]);
      }
      const h16x8 (&f)[2] = fa[i & 1];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16 t = acc[i][j];
        t = mfma16(f[1], fx[j][0], t);
        t = mfma16(f[0], fx[j][1], t);
        acc[i][j] = mfma16(f[0], fx[j][0], t);
      }
    }
    split_a(Nxt{}, FB ^ 1, st + 1);
    __builtin_amdgcn_sched_group_barrier(0x002, 40, 0);        // the x split
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);         // tile 0's reads
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i + 1 < 4) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
    __syncthreads();
  };
#define NERF_H_IT(I) \
  if constexpr (I < U) iteration(std::integral_constant<int, (I < U ? I : 0)>{}, st + I);
  for (int st = 0; st < nstages; st += U) {
    NERF_H_IT(0) NERF_H_IT(1) NERF_H_IT(2) NERF_H_IT(3) NERF_H_IT(4) NERF_H_IT(5)
  }
#undef NERF_H_IT
  static_assert(NS >= 2 && NS <= 3, "1..2 stages of loads in flight");
  constexpr int KP = kWT + 1;
  const int64_t stride = wgrad_stride(nrows, kWT);
  float* out = partial + (size_t)chunk * stride;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (128 * half + 32 * i < nrows) {   // (uniform: whole row tiles past the kept rows are dropped)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int kk = 64 * wk + 32 * j + c;
#pragma unroll
        for (int g = 0; g < 16; ++g)
          out[(size_t)(128 * half + 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h) * KP + kk] = acc[i][j][g];
      }
    }
  }
  if (tid >= 128) bsum[tid - 128] = bacc;   // samples 8..15 of each stage
  __syncthreads();
  if (tid < 128 && ac < nrows) out[(size_t)ac * KP + kWT] = (float)(bacc + bsum[tid]);
  if (tid == 0 && half == 0) reinterpret_cast<int*>(out)[stride - 4] = Ea + Ex - 28;
}

// 256 x (K <= 64) weight gradients with one x row per sample (layer 0 and the skip layer's PE
// columns): 8 waves, wave w owns output rows 32w .. 32w+31 (one MFMA row tile, two column tiles).
// Each wave loads its own a columns straight in A-fragment order (lane (c, h): column 32w + c,
// samples 8h .. 8h+7) and splits them in registers; x (64 columns, shared by all waves) is split
// once per workgroup into LDS (each thread: one column, two samples).  Little LDS and few
// registers, so two workgroups share a CU and keep more loads in flight (1 KiB of a + 252 B of x
// per sample).  Loads run two stages ahead, unconditionally.  75 us per 262K-sample launch against
// 105 us on 256 x 64 tiles of wgrad_bf_kernel (scripts/wgrad_libs_trace.sh, K=63).
// (The split arithmetic's layer-0 / skip-PE pair runs wgrad_pair16_kernel below: this kernel serves
// nerf_wgrad's 256 x (K <= 64) GEMMs under f16x3.)
template <bool BLK>   // BLK: a and x tile-major (layout.h; see wgrad_bf_kernel)
__global__ void __launch_bounds__(512)
wgrad_bf_k64_kernel(const float* __restrict__ a, int64_t lda, const float* __restrict__ x, int64_t ldx, int K,
                    int64_t M, int clen, float* __restrict__ partial) {
  constexpr int NW = 8;
  constexpr int XS = 16 / NW;        // x samples per thread and stage
  __shared__ __attribute__((aligned(16))) __bf16 Xs[2][3][64][kBfRow];
  const int chunk = blockIdx.x;
  const int64_t m0 = (int64_t)chunk * clen;
  const int64_t m1 = m0 + clen < M ? m0 + clen : M;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, c = lane & 31;
  const uint32_t lda4 = (uint32_t)lda * 4u, ldx4 = (uint32_t)ldx * 4u;
  const int ac = 32 * (w & 7) + c;
  const uint32_t avo = BLK ? 4u * (uint32_t)(tile_col(ac) + ac % 8 + 64 * h) : (uint32_t)(8 * h) * lda4 + 4u * (uint32_t)ac;
  const uint32_t as4 = BLK ? 32u : lda4, xs4 = BLK ? 32u : ldx4;   // byte step from sample j to j + 1
  // x loader: column tid % 64 (past K: an offset beyond any resource, reads 0), samples XS p .. + XS-1
  const int xc = tid & 63, xp = tid >> 6;
  const uint32_t xvo = xc < K ? (BLK ? 4u * (uint32_t)(tile_col(xc) + xc % 8 + 8 * XS * xp)
                                     : (uint32_t)(XS * xp) * ldx4 + 4u * (uint32_t)xc)
                              : 0x80000000u;
  const uint32_t mrel_end = (uint32_t)(m1 - m0);
  float ra[2][8], rx[2][XS];
  double bacc = 0.0;                 // bias column in double: one rounding per chunk
  auto load = [&](auto set_c, int stage) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    const uint32_t rel0 = (uint32_t)(kBfStage * stage) < mrel_end ? (uint32_t)(kBfStage * stage) : mrel_end;
    const int64_t ms = m0 + rel0;
    const bool live = rel0 < mrel_end;
    const __amdgpu_buffer_rsrc_t ares = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(BLK ? a + (ms / 32) * 32 * lda + (ms % 32) * 8 : a + ms * lda), (short)0,
        BLK ? (live ? (int)(32 * lda4 - (ms % 32) * 32) : 0) : (int)((mrel_end - rel0) * lda4), 0x00020000);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(BLK ? x + (ms / 32) * 32 * ldx + (ms % 32) * 8 : x + ms * ldx), (short)0,
        BLK ? (live ? (int)(32 * ldx4 - (ms % 32) * 32) : 0) : (int)((mrel_end - rel0) * ldx4), 0x00020000);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      ra[SET][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ares, (int)avo, (int)(j * as4), kRowLoadAux));
#pragma unroll
    for (int j = 0; j < XS; ++j)
      rx[SET][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xres, (int)xvo, (int)(j * xs4), kRowLoadAux));
  };
  auto store_x = [&](auto set_c, int buf) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    __bf16 p[3][XS];
#pragma unroll
    for (int j = 0; j < XS; ++j) {
      const float v = rx[SET][j];
      const __bf16 h0 = (__bf16)v;
      const float r1 = v - (float)h0;
      const __bf16 h1 = (__bf16)r1;
      p[0][j] = h0;
      p[1][j] = h1;
      p[2][j] = (__bf16)(r1 - (float)h1);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if constexpr (XS == 2) {
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<bf16x2*>(&Xs[buf][q][xc][2 * xp]) = bf16x2{p[q][0], p[q][1]};
      } else {
        Xs[buf][q][xc][xp] = p[q][0];
      }
    }
  };
  f32x16 acc[2] = {f32x16{}, f32x16{}};
  const int nstages = (int)((m1 - m0 + 2 * kBfStage - 1) / (2 * kBfStage)) * 2;   // even; the extra reads zeros
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  load(S0{}, 0);
  load(S1{}, 1);
  store_x(S0{}, 0);
  __syncthreads();
  // iteration st: split stage st's a (set st % 2) into fragments, reuse the set for stage st+2,
  // stage st's MFMAs (x from LDS buffer st % 2), stage st+1's x into the other buffer
  auto iteration = [&](auto set_c, int st) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    using Other = std::integral_constant<int, 1 - SET>;
    const int buf = SET;
    bf16x8 fa[3];
#pragma unroll
    for (int j = 0; j < 8; ++j) bacc += (double)ra[SET][j];
    split3_bf16(ra[SET], fa[0], fa[1], fa[2]);
    load(set_c, st + 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x8 fx[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) fx[q] = *reinterpret_cast<const bf16x8*>(&Xs[buf][q][32 * t + c][8 * h]);
      f32x16 v = acc[t];
      v = mfma_bf16(fa[0], fx[2], v);
      v = mfma_bf16(fa[1], fx[1], v);
      v = mfma_bf16(fa[2], fx[0], v);
      v = mfma_bf16(fa[0], fx[1], v);
      v = mfma_bf16(fa[1], fx[0], v);
      acc[t] = mfma_bf16(fa[0], fx[0], v);
    }
    store_x(Other{}, buf ^ 1);   // (after the last stage: zeros into the idle buffer)
    __syncthreads();
  };
  for (int st = 0; st < nstages; st += 2) {
    iteration(S0{}, st);
    iteration(S1{}, st + 1);
  }
  const int KP = K + 1;
  float* out = partial + (size_t)chunk * wgrad_stride(32 * NW, K);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kk = 32 * t + c;
    if (kk < K) {
#pragma unroll
      for (int g = 0; g < 16; ++g) out[(size_t)(32 * w + (g & 3) + 8 * (g >> 2) + 4 * h) * KP + kk] = acc[t][g];
    }
  }
  // bias column: this lane summed column 32w + c over its 8 samples of every stage
  bacc += __shfl_xor(bacc, 32);
  if (h == 0) out[(size_t)(32 * w + c) * KP + K] = (float)bacc;
}

// Layer 0's weight gradient (d pre_0 over enc_x) and the skip layer's PE columns (d pre_4 over enc_x)
// of the split arithmetic as one 512 x 63 GEMM on split-f16 MFMA (wgrad_bf_k64_kernel<true, 16>'s
// shape with wgrad_h16h_kernel's arithmetic: three f16 products per fp32 product instead of bf16x6's
// six, two f16 parts to split instead of three bf16 parts).  16 waves per chunk (kPairClen): wave w
// owns output rows 32w .. 32w+31 (waves 0-7 of d pre_0, 8-15 of d pre_4; one MFMA row tile, two
// column tiles), loads its a columns straight in A-fragment order and splits them in registers; x =
// enc_x (63 columns + the pad slot, which is never read) is split once per workgroup into LDS, one
// sample of one column per thread and stage.  enc_x is read once for both gradients.
// Scales: one power of two per chunk and operand, s = 2^(14 - e) (h16_chunk_exps), from the producers'
// block exponent records (layout.h: d pre_0 = gradient entry 8, d pre_4 = entry 3, enc_x = save entry
// 8), else from a pass over the chunk (workgroup-uniform branch).  The two halves' a scales differ, so
// each wave unscales its 32 accumulators itself (exact: powers of two) and the partial is plain fp32
// (wgrad_reduce_kernel, scaled = 0).  The bias column sums the raw a values in double.
// 274 us per step beside the other stream against 298 us for the bf16x6 kernel it replaced; a variant
// without LDS or barriers (every wave loading and splitting all 64 enc_x columns itself) took 372 us:
// the 16 waves' dword gathers of x cost more than the per-stage barrier (profiles/r06/
// kernel_stats_train_a.csv, kernel_stats_train_b.csv).
constexpr int kPairWaves = 16;
__global__ void __launch_bounds__(64 * kPairWaves)
wgrad_pair16_kernel(const float* __restrict__ grad, const float* __restrict__ save, int64_t M, int clen,
                    float* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) _Float16 Xs[2][2][64][kBfRow];   // [buffer][hi, lo][column][sample]
  __shared__ float wmax[kPairWaves][2];
  const int chunk = blockIdx.x;
  const int64_t m0 = (int64_t)chunk * clen;
  const int64_t m1 = m0 + clen < M ? m0 + clen : M;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, c = lane & 31, half = w >> 3;
  const float* a = grad + tile_col(half ? kSkipLayer * kHidden : 0);     // (wave-uniform)
  const float* x = save + tile_col(kSaveEncX);
  constexpr uint32_t lda4 = kGradRow * 4u, ldx4 = kSaveRow * 4u;
  const int ac = 32 * (w & 7) + c;
  const uint32_t avo = 4u * (uint32_t)(tile_col(ac) + ac % 8 + 64 * h);   // sample j of the stage at + 32 j bytes
  const int xc = tid & 63, xp = tid >> 6;                                 // x: column xc, sample xp of a stage
  const uint32_t xvo = xc < kPosEnc ? 4u * (uint32_t)(tile_col(xc) + xc % 8 + 8 * xp) : 0x80000000u;
  const uint32_t mrel_end = (uint32_t)(m1 - m0);

  // ---- the chunk's exponents: records (every wave reads all three, so the branch is uniform)
  const int64_t b0 = m0 / 32, nb = (m1 - 1) / 32 - b0 + 1;
  const float* rec0 = grad + tile_col(kMetaGradF) + kMetaGradF % 8 + 8 * 8;   // entry 8: d pre_0
  const float* rec4 = grad + tile_col(kMetaGradF) + kMetaGradF % 8 + 8 * 3;   // entry 3: d pre_4
  const float* recx = save + tile_col(kMetaSaveF) + kMetaSaveF % 8 + 8 * 8;   // entry 8: enc_x
  float r0 = 0.0f, r4 = 0.0f, rx_ = 0.0f, bad = 0.0f;
  for (int64_t b = lane; b < nb; b += 64) {
    const float v0 = rec0[(b0 + b) * 32 * kGradRow], v4 = rec4[(b0 + b) * 32 * kGradRow];
    const float vx = recx[(b0 + b) * 32 * kSaveRow];
    bad = (block_exp_valid(v0) && block_exp_valid(v4) && block_exp_valid(vx)) ? bad : 1.0f;
    r0 = fmaxf(r0, -v0);
    r4 = fmaxf(r4, -v4);
    rx_ = fmaxf(rx_, -vx);
  }
  int Ea, Ex;
  if (wave_max_nn(bad) == 0.0f) {
    Ea = (int)wave_max_nn(half ? r4 : r0) - kBlockExpBias;
    Ex = (int)wave_max_nn(rx_) - kBlockExpBias;
  } else {   // absent: the chunk's whole 32-sample blocks read once (the records' span)
    float ma = 0.0f, mx = 0.0f;
    const int64_t f0 = b0 * 32, f1 = (b0 + nb) * 32 < M ? (b0 + nb) * 32 : M;
    for (int64_t ms = f0; ms < f1; ms += kBfStage) {
      const __amdgpu_buffer_rsrc_t ares = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(a + (ms / 32) * 32 * kGradRow + (ms % 32) * 8), (short)0, (int)(32 * lda4 - (ms % 32) * 32),
          0x00020000);
      const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(x + (ms / 32) * 32 * kSaveRow + (ms % 32) * 8), (short)0, (int)(32 * ldx4 - (ms % 32) * 32),
          0x00020000);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        ma = fmaxf(ma, fabsf(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ares, (int)avo, j * 32, 0))));
      mx = fmaxf(mx, fabsf(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xres, (int)xvo, 0, 0))));
    }
    ma = wave_max_nn(ma);
    mx = wave_max_nn(mx);
    if (lane == 0) {
      wmax[w][0] = ma;
      wmax[w][1] = mx;
    }
    __syncthreads();
    ma = 0.0f;
    mx = 0.0f;
    for (int v = 0; v < kPairWaves; ++v) {
      if ((v >> 3) == half) ma = fmaxf(ma, wmax[v][0]);
      mx = fmaxf(mx, wmax[v][1]);
    }
    Ea = (int)(-block_exp_record(ma)) - kBlockExpBias;
    Ex = (int)(-block_exp_record(mx)) - kBlockExpBias;
  }
  Ea = __builtin_amdgcn_readfirstlane(Ea < kH16EMin ? kH16EMin : Ea);
  Ex = __builtin_amdgcn_readfirstlane(Ex < kH16EMin ? kH16EMin : Ex);
  const float sa = ldexpf(1.0f, 14 - Ea), sx = ldexpf(1.0f, 14 - Ex);

  float ra[2][8], rx[2];
  double bacc = 0.0;                 // bias column (this lane's column, its 8 samples of every stage)
  auto load = [&](auto set_c, int stage) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    const uint32_t rel0 = (uint32_t)(kBfStage * stage) < mrel_end ? (uint32_t)(kBfStage * stage) : mrel_end;
    const int64_t ms = m0 + rel0;
    const bool live = rel0 < mrel_end;   // past the chunk: an empty resource, the loads read zeros
    const __amdgpu_buffer_rsrc_t ares = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a + (ms / 32) * 32 * kGradRow + (ms % 32) * 8), (short)0,
        live ? (int)(32 * lda4 - (ms % 32) * 32) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t xres = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(x + (ms / 32) * 32 * kSaveRow + (ms % 32) * 8), (short)0,
        live ? (int)(32 * ldx4 - (ms % 32) * 32) : 0, 0x00020000);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      ra[SET][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ares, (int)avo, j * 32, kRowLoadAux));
    rx[SET] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xres, (int)xvo, 0, kRowLoadAux));
  };
  auto store_x = [&](auto set_c, int buf) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    const float v = rx[SET] * sx;
    const _Float16 hi = (_Float16)v;
    Xs[buf][0][xc][xp] = hi;
    Xs[buf][1][xc][xp] = split_lo(v, hi);
  };
  f32x16 acc[2] = {f32x16{}, f32x16{}};
  const int nstages = (int)((m1 - m0 + 2 * kBfStage - 1) / (2 * kBfStage)) * 2;   // even; the extra reads zeros
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  load(S0{}, 0);
  load(S1{}, 1);
  store_x(S0{}, 0);
  __syncthreads();
  // iteration st: split stage st's a (set st % 2) in registers, reuse the set for stage st+2's loads,
  // stage st's MFMAs (x from LDS buffer st % 2), stage st+1's x into the other buffer
  auto iteration = [&](auto set_c, int st) __attribute__((always_inline)) {
    constexpr int SET = decltype(set_c)::value;
    using Other = std::integral_constant<int, 1 - SET>;
    const int buf = SET;
#pragma unroll
    for (int j = 0; j < 8; ++j) bacc += (double)ra[SET][j];
    h16x8 fh, fl;
    split2_f16(ra[SET], sa, fh, fl);
    load(set_c, st + 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const h16x8 xh = *reinterpret_cast<const h16x8*>(&Xs[buf][0][32 * t + c][8 * h]);
      const h16x8 xl = *reinterpret_cast<const h16x8*>(&Xs[buf][1][32 * t + c][8 * h]);
      f32x16 v = mfma16(fl, xh, acc[t]);   // small products first
      v = mfma16(fh, xl, v);
      acc[t] = mfma16(fh, xh, v);
    }
    store_x(Other{}, buf ^ 1);   // (after the last stage: zeros into the idle buffer)
    __syncthreads();
  };
  for (int st = 0; st < nstages; st += 2) {
    iteration(S0{}, st);
    iteration(S1{}, st + 1);
  }
  // acc = sum (a 2^(14-Ea)) (x 2^(14-Ex)): unscaled here by two exact power-of-two factors (each
  // normal for any exponent the clamps allow)
  const int e = Ea + Ex - 28;
  const float u0 = ldexpf(1.0f, e / 2), u1 = ldexpf(1.0f, e - e / 2);
  constexpr int KP = kPosEnc + 1;
  float* out = partial + (size_t)chunk * wgrad_stride(2 * kHidden, kPosEnc);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kk = 32 * t + c;
    if (kk < kPosEnc) {
#pragma unroll
      for (int g = 0; g < 16; ++g) out[(size_t)(32 * w + (g & 3) + 8 * (g >> 2) + 4 * h) * KP + kk] = (acc[t][g] * u0) * u1;
    }
  }
  bacc += __shfl_xor(bacc, 32);
  if (h == 0) out[(size_t)(32 * w + c) * KP + kPosEnc] = (float)bacc;
}

// The rgb head's weight gradient (rgb_linear: 3 rows over hd, K = 128) on tile-major rows: a
// streaming kernel, not a GEMM tile (an MFMA tile would keep 3 of its 128 rows).  A workgroup owns a
// chunk of 16 blocks (512 samples); wave w the feature groups 4w..4w+3 of hd.  Per block and group
// a lane reads one float4 (the group's 32 samples x 8 features are 1 KiB contiguous: lane l holds
// sample l/2, features 8g + 4(l&1)..+3) and the sample's d rgb_pre (3 floats), and accumulates the
// 3 x 4 products in double; at the chunk's end the 32 lanes of each parity are summed (shuffles,
// double) into the chunk's partial (N = 3, K = 128 layout of wgrad_reduce_kernel; the bias column
// from wave 0).  Reads hd once at full lines: ~134 MB per 262K-sample step.
// SUMS (rays of N % 32 == 0 samples under the split arithmetic, the fused per-ray sums): the launch
// also writes what the appearance projection's and dir_linear's per-ray GEMMs need from the head,
// since it holds every block's d rgb_pre anyway (models.py:154-160: d hd = W_rgb^T d rgb_pre is linear
// in the sample, so a block's sum of d hd needs only its 3 column sums): per 32-sample block b (all on
// one ray) S_hd[b] = W_rgb^T (the block's d rgb_pre sums, in double, rounded once), and for a ray's
// first block E[ray] = the ray's PE_4(d) (its first sample's save row).  Wave (b - b0) % 4 takes
// block b.  (Until round 6 a separate block_head_sums_kernel read the d rgb_pre rows again.)
constexpr int kHeadChunkBlocks = 16;   // (512 chunks per 262K-sample step: two workgroups per CU)
template <bool SUMS = false>
__global__ void __launch_bounds__(256)
wgrad_head3_kernel(const float* __restrict__ a, const float* __restrict__ x, int64_t M, float* __restrict__ partial,
                   const float* __restrict__ save = nullptr, const float* __restrict__ packed = nullptr, int N = 0,
                   float* __restrict__ S_hd = nullptr, float* __restrict__ E = nullptr) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float wr[3][2];   // SUMS: rgb_linear.weight columns lane, lane + 64
  if constexpr (SUMS) {
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int q = 0; q < 2; ++q) wr[c][q] = packed[kOffRgbW + c * kDirHidden + 64 * q + lane];
  }
  const int64_t nblk = (M + 31) / 32;
  const int64_t b0 = (int64_t)blockIdx.x * kHeadChunkBlocks;
  const int64_t b1 = b0 + kHeadChunkBlocks < nblk ? b0 + kHeadChunkBlocks : nblk;
  const int j = lane >> 1, par = lane & 1;
  double acc[4][3][4] = {};
  double bacc[3] = {0.0, 0.0, 0.0};
  // the block's rows: gradient rows at d rgb_pre's group, save rows at hd's first group; the next
  // block's loads are issued before this block's products
  auto load = [&](int64_t b, f32x4& dv, f32x4 (&v)[4]) __attribute__((always_inline)) {
    const float* ab = a + b * 32 * kGradRow;
    const float* xb = x + b * 32 * kSaveRow;
    dv = *reinterpret_cast<const f32x4*>(ab + 8 * j);
#pragma unroll
    for (int g = 0; g < 4; ++g) v[g] = *reinterpret_cast<const f32x4*>(xb + (4 * w + g) * 256 + 4 * lane);
  };
  f32x4 dv_n, v_n[4];
  if (b0 < b1) load(b0, dv_n, v_n);
  for (int64_t b = b0; b < b1; ++b) {
    const f32x4 dv = dv_n;
    f32x4 v[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) v[g] = v_n[g];
    if (b + 1 < b1) load(b + 1, dv_n, v_n);
    if constexpr (SUMS) {
      if ((int)((b - b0) & 3) == w) {   // (wave-uniform)
        double ds[3];   // lane (j, par) holds sample j's d rgb_pre: xor 2 .. 32 sums one parity's 32 lanes
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          ds[c] = (double)dv[c];
#pragma unroll
          for (int m = 2; m < 64; m <<= 1) ds[c] += __shfl_xor(ds[c], m);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q)
          S_hd[b * kDirHidden + 64 * q + lane] =
              (float)(ds[0] * (double)wr[0][q] + ds[1] * (double)wr[1][q] + ds[2] * (double)wr[2][q]);
        if ((b * 32) % N == 0 && lane < 32) E[(b * 32 / N) * 32 + lane] = save[tile_off(b * 32, kSaveEncD + lane, kSaveRow)];
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double d = (double)dv[c];
      bacc[c] += par == 0 ? d : 0.0;
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[g][c][e] = fma(d, (double)v[g][e], acc[g][c][e]);
    }
  }
  // sum the 32 lanes of each parity (xor 2 .. 32 keeps the parity), in a fixed order
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int m = 2; m < 64; m <<= 1) acc[g][c][e] += __shfl_xor(acc[g][c][e], m);
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int m = 2; m < 64; m <<= 1) bacc[c] += __shfl_xor(bacc[c], m);
  constexpr int KP = kDirHidden + 1;
  float* out = partial + (size_t)blockIdx.x * wgrad_stride(3, kDirHidden);
  if (lane < 2) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) out[c * KP + 8 * (4 * w + g) + 4 * lane + e] = (float)acc[g][c][e];
    if (w == 0 && lane == 0) {
#pragma unroll
      for (int c = 0; c < 3; ++c) out[c * KP + kDirHidden] = (float)bacc[c];
    }
  }
}

// x_blk: x tile-major (BLK and x_div == 1); under BLK a row-major x with x_div == 1 (the appearance
// rows of one-sample "rays") takes the generic x loader, which reads row-major rows.
template <int WN, int WK, bool BLK>
static int launch_wgrad_bf(const float* a, int64_t lda, int N, const float* x, int64_t ldx, int K, int64_t x_div,
                           bool x_blk, int64_t M, int chunks, int clen, float* ws, hipStream_t s) {
  const int ntn = (N + 64 * WN - 1) / (64 * WN), ntk = (K + 64 * WK - 1) / (64 * WK);
  const int tiles = ntn * ntk;
  const int blocks = ((chunks + 7) / 8) * 8 * tiles;
  if (x_div == 1 && (!BLK || x_blk))
    hipLaunchKernelGGL((wgrad_bf_kernel<WN, WK, true, BLK>), dim3((unsigned)blocks), dim3(256), 0, s, a, lda, N, x,
                       ldx, K, x_div, M, ntk, tiles, chunks, clen, ws);
  else
    hipLaunchKernelGGL((wgrad_bf_kernel<WN, WK, false, BLK>), dim3((unsigned)blocks), dim3(256), 0, s, a, lda, N, x,
                       ldx, K, x_div, M, ntk, tiles, chunks, clen, ws);
  return check_launch("wgrad_bf_kernel");
}

struct WgradSplit {                  // rows n0 <= n < n_end of a weight gradient belong to a second parameter
  int n0 = 0;
  float* out_w = nullptr;            // its weight gradient, ld ldo, the first k columns
  int ldo = 0, k = 0;
  float* out_b = nullptr;            // its bias gradient (the bias column), nullable
  int n_end = 1 << 30;               // rows from n_end on are dropped (padding rows of a whole-tile launch)
};

// out_w[n][k] (ld K) and out_b[n] (nullable) = (accumulate ? out : 0) + sum over chunks, in chunk
// order; with a WgradSplit, rows n >= split.n0 go to split.out_w[n - n0][k < split.k] and
// split.out_b[n - n0] instead.  A workgroup owns 64 float4 columns of the partial layout; its
// kRedParts waves each sum a contiguous 1/kRedParts of the chunks (fixed order, eight loads in flight
// per lane), then the parts are added in order: deterministic.  The reductions run beside the other
// stream's GEMMs: eight waves per workgroup made the step 2-3 % slower than four (same-box A/B,
// profiles/r03_ab_train_reduce_parts.log).
constexpr int kRedParts = 4;
__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ partial, int chunks, int N, int K,
                                                  float* __restrict__ out_w, int ldo, float* __restrict__ out_b,
                                                  int accumulate, const WgradSplit& split, int scaled) {
  // the chunk partials are added in double and rounded once: a gradient entry is a sum over up to
  // 2^18 samples with heavy cancellation (random-sign upstream gradients), and an fp32 running sum of
  // its 256 chunk partials cost up to ~10x the fp32 CPU autograd's error on the bias columns
  // (tests/test_gpu_accuracy.py::test_gradients_vs_float64, scripts/diag_grad_masks.py)
  typedef double f64x4 __attribute__((ext_vector_type(4)));
  __shared__ f64x4 part[kRedParts][64];
  const int KP = K + 1;
  const int64_t stride = wgrad_stride(N, K);
  const int64_t col4 = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  const int per = (chunks + kRedParts - 1) / kRedParts;
  const int c0 = q * per < chunks ? q * per : chunks, c1 = c0 + per < chunks ? c0 + per : chunks;
  f64x4 acc = {0.0, 0.0, 0.0, 0.0};
  auto add = [&](const f32x4& v) __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] += (double)v[e];
  };
  if (col4 * 4 < stride && !scaled) {
    const f32x4* p = reinterpret_cast<const f32x4*>(partial) + col4;
    const int64_t s4 = stride / 4;
    int c = c0;
    for (; c + 8 <= c1; c += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(c + u) * s4];
#pragma unroll
      for (int u = 0; u < 8; ++u) add(v[u]);
    }
    for (; c < c1; ++c) add(p[c * s4]);
  } else if (col4 * 4 < stride) {
    // split-f16 partials: chunk c's values times 2^(its exponent), the bias column as stored (exact in
    // double: powers of two)
    const f32x4* p = reinterpret_cast<const f32x4*>(partial) + col4;
    const int* ex = reinterpret_cast<const int*>(partial) + stride - 4;
    const int64_t s4 = stride / 4;
    bool bias[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = (col4 * 4 + e) % (K + 1) == K;
    auto add_scaled = [&](const f32x4& v, int x) __attribute__((always_inline)) {
      const double sc = ldexp(1.0, x);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += bias[e] ? (double)v[e] : (double)v[e] * sc;
    };
    int c = c0;
    for (; c + 8 <= c1; c += 8) {
      f32x4 v[8];
      int x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = p[(c + u) * s4];
        x[u] = ex[(c + u) * stride];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) add_scaled(v[u], x[u]);
    }
    for (; c < c1; ++c) add_scaled(p[c * s4], ex[c * stride]);
  }
  part[q][threadIdx.x & 63] = acc;
  __syncthreads();
  if (q != 0 || col4 * 4 >= stride) return;
  f64x4 sum64 = part[0][threadIdx.x];
#pragma unroll
  for (int r = 1; r < kRedParts; ++r) sum64 += part[r][threadIdx.x];
  f32x4 sum;
#pragma unroll
  for (int e = 0; e < 4; ++e) sum[e] = (float)sum64[e];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t idx = col4 * 4 + e;
    if (idx >= (int64_t)N * KP) break;
    const int n = (int)(idx / KP), k = (int)(idx % KP);
    float* dst;
    if (split.out_w && n >= split.n0) {   // rows from n0 on belong to a second output (WgradSplit)
      if (n >= split.n_end) continue;
      const int n2 = n - split.n0;
      dst = k < split.k ? split.out_w + (size_t)n2 * split.ldo + k : (k == K && split.out_b ? split.out_b + n2 : nullptr);
    } else {
      dst = k < K ? out_w + (size_t)n * ldo + k : (out_b ? out_b + n : nullptr);
    }
    if (dst) *dst = accumulate ? *dst + sum[e] : sum[e];
  }
}
__global__ void __launch_bounds__(64 * kRedParts)
wgrad_reduce_kernel(const float* __restrict__ partial, int chunks, int N, int K, float* __restrict__ out_w, int ldo,
                    float* __restrict__ out_b, int accumulate, WgradSplit split, int scaled) {
  wgrad_reduce_body(partial, chunks, N, K, out_w, ldo, out_b, accumulate, split, scaled);
}

size_t wgrad_workspace_floats(int64_t M, int N, int K) {
  const int clen = wgrad_chunk_len(N, K, M);   // >= the chunk count of every path of launch_wgrad
  const int64_t chunks = (M + clen - 1) / clen;
  return (size_t)chunks * wgrad_stride(N, K);
}

template <int WN, int WK, bool BLK>
static int launch_wgrad_lds(const float* a, int64_t lda, int N, const float* x, int64_t ldx, int K, int64_t x_div,
                            bool x_blk, int64_t M, int chunks, float* ws, hipStream_t s) {
  const int ntn = (N + 64 * WN - 1) / (64 * WN), ntk = (K + 64 * WK - 1) / (64 * WK);
  const int tiles = ntn * ntk;
  const int blocks = ((chunks + 7) / 8) * 8 * tiles;
  hipLaunchKernelGGL((wgrad_lds_kernel<WN, WK, BLK>), dim3((unsigned)blocks), dim3(256), 0, s, a, lda, N, x, ldx, K,
                     x_div, (int)(BLK && x_blk && x_div == 1), M, ntk, tiles, chunks, ws);
  return check_launch("wgrad_lds_kernel");
}

// sums (nullable): S_hd and E of the fused per-ray sums (rays of N % 32 == 0 samples), save / packed
// the rows and weights they come from
struct HeadSums { const float* save; const float* packed; int N; float* S_hd; float* E; };
static int launch_wgrad_head3(const float* a, const float* x, int64_t M, float* out_w, float* out_b, float* ws,
                              size_t ws_floats, hipStream_t s, const HeadSums* sums = nullptr) {
  if (M == 0) return NERF_OK;
  const int chunks = (int)(((M + 31) / 32 + kHeadChunkBlocks - 1) / kHeadChunkBlocks);
  if ((size_t)chunks * wgrad_stride(3, kDirHidden) > ws_floats) return set_error(NERF_ERR_WORKSPACE, "wgrad_head3: workspace");
  if (sums)
    hipLaunchKernelGGL(wgrad_head3_kernel<true>, dim3((unsigned)chunks), dim3(256), 0, s, a, x, M, ws, sums->save,
                       sums->packed, sums->N, sums->S_hd, sums->E);
  else
    hipLaunchKernelGGL(wgrad_head3_kernel<false>, dim3((unsigned)chunks), dim3(256), 0, s, a, x, M, ws);
  if (int rc = check_launch("wgrad_head3_kernel")) return rc;
  const int64_t cols4 = wgrad_stride(3, kDirHidden) / 4;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((cols4 + 63) / 64)), dim3(64 * kRedParts), 0, s, ws, chunks, 3,
                     kDirHidden, out_w, kDirHidden, out_b, 0, WgradSplit{}, 0);
  return check_launch("wgrad_reduce_kernel");
}

// Layer 0's weight gradient (d pre_0 over enc_x) and the skip layer's PE columns (d pre_4 over
// enc_x) as one 512 x 63 split-f16 GEMM over the tile-major rows (wgrad_pair16_kernel): enc_x is read
// once; rows 0..255 go to layer 0's weight + bias, rows 256.. to the skip weight's PE columns.
static int launch_wgrad_pe_pair(const float* save, const float* grad, int64_t M, float* w0, float* b0, float* w4,
                                float* ws, size_t ws_floats, hipStream_t s) {
  if (M == 0) return NERF_OK;
  const int clen = wgrad_chunk_len(2 * kHidden, kPosEnc, M);
  const int chunks = (int)((M + clen - 1) / clen);
  if ((size_t)chunks * wgrad_stride(2 * kHidden, kPosEnc) > ws_floats)
    return set_error(NERF_ERR_WORKSPACE, "wgrad pe pair: workspace");
  hipLaunchKernelGGL(wgrad_pair16_kernel, dim3((unsigned)chunks), dim3(64 * kPairWaves), 0, s, grad, save, M, clen, ws);
  if (int rc = check_launch("wgrad_pair16_kernel")) return rc;
  const WgradSplit skip{kHidden, w4 + kHidden, kHidden + kPosEnc, kPosEnc, nullptr};
  const int64_t cols4 = wgrad_stride(2 * kHidden, kPosEnc) / 4;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((cols4 + 63) / 64)), dim3(64 * kRedParts), 0, s, ws, chunks,
                     2 * kHidden, kPosEnc, w0, kPosEnc, b0, 0, skip, 0);
  return check_launch("wgrad_reduce_kernel");
}

// tiled: a (and x when x_div == 1 and x_tiled) are tile-major rows (layout.h) of row length lda / ldx,
// each pointer at its slice's tile_col; the training path (param_grads).  Otherwise row-major.  The
// appearance projection's x (the embedding rows, one per ray) is row-major: x_tiled = false.
// meta: the block exponents of a and x (layout.h) for the split-f16 whole-tile kernel (nullable).
int launch_wgrad(const float* a, int64_t lda, int N, const float* x, int64_t ldx, int K, int64_t x_div, int64_t M,
                 float* out_w, int ldo, float* out_b, int accumulate, float* ws, hipStream_t s,
                 const WgradSplit* split = nullptr, bool tiled = false, bool x_tiled = true,
                 const H16Meta* meta = nullptr, float* sums = nullptr) {
  const H16Meta hm = meta ? *meta : H16Meta{};
  if (M == 0) return NERF_OK;
  const int KP = K + 1;
  int chunks = (int)((M + kWChunk - 1) / kWChunk);
  const bool aligned = ((uintptr_t)a % 16 == 0) && ((uintptr_t)x % 16 == 0) && lda % 4 == 0 && ldx % 4 == 0;
  if (tiled && !(aligned && lda % 8 == 0 && (x_div != 1 || ldx % 8 == 0)))
    return set_error(NERF_ERR_BAD_ARG, "wgrad: tile-major operands must be aligned with row lengths % 8 == 0");
  const bool x_blk = tiled && x_tiled && x_div == 1;   // x tile-major
  int rc;
  bool sums_done = false;                               // (sums: written by the h16h launch only)
  bool scaled = false;                                  // partials of wgrad_h16w_kernel (chunk exponents)
  // the split arithmetic (buffer offsets of a chunk's rows must stay below 2^31): the whole-tile
  // GEMMs on split-f16 MFMA, the rest on bf16x6
  if (g_mlp_arith == NERF_ARITH_F16X3 && K >= 1 && lda < (1 << 18) && ldx < (1 << 18)) {
    const int clen = wgrad_chunk_len(N, K, M);
    chunks = (int)((M + clen - 1) / clen);
    if (wgrad_whole_tile(N, K) && x_div == 1 && tiled && x_blk) {
      // tile-major rows (the training path): two workgroups per CU, half the rows each; the
      // dir_linear + density launch (N = 160) keeps 160 of 256 rows
      if (sums)   // (the dir/density launch also writes d pre_dir's 8-sample sums, wgrad_h16h_kernel)
        hipLaunchKernelGGL((wgrad_h16h_kernel<3, true>), dim3((unsigned)((chunks + 7) / 8 * 16)), dim3(256), 0, s, a, lda,
                           x, ldx, M, clen, chunks, N, hm, ws, sums);
      else
        hipLaunchKernelGGL(wgrad_h16h_kernel<3>, dim3((unsigned)((chunks + 7) / 8 * 16)), dim3(256), 0, s, a, lda, x, ldx,
                           M, clen, chunks, N, hm, ws, nullptr);
      rc = check_launch("wgrad_h16h_kernel");
      scaled = true;
      sums_done = true;
    } else if (N == kWT && wgrad_whole_tile(N, K) && x_div == 1 && !tiled) {   // nerf_wgrad's row-major operands
      hipLaunchKernelGGL(wgrad_h16w_kernel<false>, dim3((unsigned)chunks), dim3(256), 0, s, a, lda, x, ldx, M, clen, hm, ws);
      rc = check_launch("wgrad_h16w_kernel");
      scaled = true;
    } else if (N == kWT && K <= 64 && x_div == 1 && (!tiled || x_blk)) {
      if (tiled)
        hipLaunchKernelGGL(wgrad_bf_k64_kernel<true>, dim3((unsigned)chunks), dim3(512), 0, s, a, lda, x, ldx, K, M,
                           clen, ws);
      else
        hipLaunchKernelGGL(wgrad_bf_k64_kernel<false>, dim3((unsigned)chunks), dim3(512), 0, s, a, lda, x, ldx, K, M,
                           clen, ws);
      rc = check_launch("wgrad_bf_k64_kernel");
    } else if (K <= 64 && N > 64) {
      rc = tiled ? launch_wgrad_bf<4, 1, true>(a, lda, N, x, ldx, K, x_div, x_blk, M, chunks, clen, ws, s)
                 : launch_wgrad_bf<4, 1, false>(a, lda, N, x, ldx, K, x_div, x_blk, M, chunks, clen, ws, s);
    } else {
      rc = tiled ? launch_wgrad_bf<2, 2, true>(a, lda, N, x, ldx, K, x_div, x_blk, M, chunks, clen, ws, s)
                 : launch_wgrad_bf<2, 2, false>(a, lda, N, x, ldx, K, x_div, x_blk, M, chunks, clen, ws, s);
    }
  } else if (aligned && K >= 1 && K <= 64 && N > 64) {
    rc = tiled ? launch_wgrad_lds<4, 1, true>(a, lda, N, x, ldx, K, x_div, x_blk, M, chunks, ws, s)
               : launch_wgrad_lds<4, 1, false>(a, lda, N, x, ldx, K, x_div, x_blk, M, chunks, ws, s);
  } else if (aligned && K >= 1) {
    rc = tiled ? launch_wgrad_lds<2, 2, true>(a, lda, N, x, ldx, K, x_div, x_blk, M, chunks, ws, s)
               : launch_wgrad_lds<2, 2, false>(a, lda, N, x, ldx, K, x_div, x_blk, M, chunks, ws, s);
  } else {
    const int tiles = ((N + 31) / 32) * ((KP + 63) / 64);
    hipLaunchKernelGGL(wgrad_kernel, dim3((unsigned)((tiles + 3) / 4), (unsigned)chunks), dim3(256), 0, s, a, lda, N,
                       x, ldx, K, x_div, M, ws);
    rc = check_launch("wgrad_kernel");
  }
  if (rc) return rc;
  if (sums && !sums_done) return set_error(NERF_ERR_BAD_ARG, "wgrad: 8-sample sums need the split-f16 whole-tile launch");
  const int64_t cols4 = wgrad_stride(N, K) / 4;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((cols4 + 63) / 64)), dim3(64 * kRedParts), 0, s, ws, chunks, N, K,
                     out_w, ldo, out_b, accumulate, split ? *split : WgradSplit{}, (int)scaled);
  return check_launch("wgrad_reduce_kernel");
}

// ------------------------------------------------------------------- appearance gradient
// d app_row(r) = appearance_projection.weight^T . S_r, S_r = sum over the samples that used row r of
// d hd (models.py:154-156: hd += W_app app + b_app).  Row r's samples are src rows
// [r*group, (r+1)*group) with stride ld: per-ray rows pass the gradient rows (group = N); a single
// broadcast row passes the already-reduced bias gradient of appearance_projection (group = 1).
__global__ void __launch_bounds__(128)
app_grad_kernel(const float* __restrict__ src, int64_t ld, int group, int tiled, const float* __restrict__ packed,
                float* __restrict__ dapp) {
  __shared__ float sum[kDirHidden];
  const int64_t r = blockIdx.x;
  const int n = threadIdx.x;
  double acc = 0.0;
  for (int s = 0; s < group; ++s) {
    const int64_t m = r * group + s;     // tiled: gradient rows (layout.h), src at the slice's tile_col
    acc += (double)src[tiled ? tile_off(m, n, (int)ld) : m * ld + n];
  }
  sum[n] = (float)acc;
  __syncthreads();
  if (n < kAppDim) {
    const float* W = packed + kOffAppW;      // (128 x 32) row-major
    float v = 0.0f;
    for (int j = 0; j < kDirHidden; ++j) v = fmaf(W[j * kAppDim + n], sum[j], v);
    dapp[r * kAppDim + n] = v;
  }
}

int launch_app_grad(const float* src, int64_t ld, int64_t rows, int group, const float* packed, float* dapp,
                    hipStream_t s, bool tiled) {
  if (rows == 0) return NERF_OK;
  hipLaunchKernelGGL(app_grad_kernel, dim3((unsigned)rows), dim3(128), 0, s, src, ld, group, (int)tiled, packed, dapp);
  return check_launch("app_grad_kernel");
}

// ---------------------------------------------------------------- per-ray gradient sums
// Inputs that are constant along a ray (PE_4(d) of dir_linear's last 27 columns, the appearance
// row) make their weight gradient a GEMM over rays: sum_m g[m][n] x[ray(m)][k] = sum_r S[r][n] x[r][k]
// with S[r] = sum over the ray's samples of g (distributivity; the sums in double).  Ray r's block:
// S[r] = [sum d pre_dir (128) | sum d hd (128)] from the tile-major gradient rows, and E[r] = the
// ray's PE_4(d) (its first sample's save row, kSaveEncD: 27 values + zeros) as a row-major row.
__global__ void __launch_bounds__(256)
ray_sums_kernel(const float* __restrict__ grad, const float* __restrict__ save, int N, float* __restrict__ S,
                float* __restrict__ E) {
  const int64_t r = blockIdx.x;
  const int t = threadIdx.x;
  const int col = t < kDirHidden ? kGradDir + t : kGradHd + (t - kDirHidden);
  const int64_t m0 = r * N;
  double acc = 0.0;
#pragma unroll 8
  for (int j = 0; j < N; ++j) acc += (double)grad[tile_off(m0 + j, col, kGradRow)];
  S[r * 256 + t] = (float)acc;
  if (t < 32) E[r * 32 + t] = save[tile_off(m0, kSaveEncD + t, kSaveRow)];
}

// The ray-sum buffers for any N >= kRaySumMinN (B = M / N <= M / kRaySumMinN rays): region A holds
// S (B x 256, ray_sums_kernel) or the fused path's 8-sample sums of d pre_dir ((M / 8) x 128), region
// B the fused path's S_hd ((M / 32) x 128), region C E (B x 32).
constexpr int kRaySumMinN = kEncDPerRayMinN;   // (enc_d per ray from there on, layout.h)
// The fused per-ray sums (the split arithmetic's dir/density launch writes d pre_dir's 8-sample sums,
// the rgb head's launch, wgrad_head3_kernel<true>, the rest): 32-sample blocks on one ray.  Then
// nothing reads d hd's columns.
static bool fused_ray_sums(int N) { return g_mlp_arith == NERF_ARITH_F16X3 && N >= kRaySumMinN && N % 32 == 0; }
static size_t ray_sum_a_floats(int64_t M) { return (size_t)(M / 8 + 1) * kDirHidden; }   // >= (M / 32 + 1) 256
static size_t ray_sum_b_floats(int64_t M) { return (size_t)(M / 32 + 1) * kDirHidden; }
static size_t ray_sum_floats(int64_t M) { return ray_sum_a_floats(M) + ray_sum_b_floats(M) + (size_t)(M / 32 + 1) * 32 + 64; }

// ------------------------------------------------------------------------------------ Adam
// torch.optim.Adam (amsgrad=False, maximize=False, weight_decay=0) element for element:
//   m = lerp(m, g, 1-beta1);  v = v*beta2 + (1-beta2) g^2
//   p = p - step_size * m / (sqrt(v)/bc2_sqrt + eps),  step_size = lr / bc1
__global__ void __launch_bounds__(256)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
            int64_t n, float w1, float beta2, float one_m_beta2, float bc2_sqrt, float eps, float neg_step) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i];
  const float mi = m[i];
  // lerp as ATen's vectorised CPU kernel evaluates it (fused multiply-add), addcmul left to right
  const float m_new = w1 < 0.5f ? fmaf(w1, gi - mi, mi) : fmaf(w1 - 1.0f, gi - mi, gi);
  const float v_new = v[i] * beta2 + (one_m_beta2 * gi) * gi;
  m[i] = m_new;
  v[i] = v_new;
  const float denom = sqrtf(v_new) / bc2_sqrt + eps;
  p[i] = p[i] + neg_step * (m_new / denom);
}

int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1, double beta2,
                double eps, int64_t step, hipStream_t s) {
  if (n == 0) return NERF_OK;
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, g, m, v, n,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)sqrt(bc2), (float)eps,
                     (float)(-(lr / bc1)));
  return check_launch("adam_kernel");
}

}  // namespace nerf

namespace nerf {
// loss = sum(sq_err) / (3B) (F.mse_loss, reduction='mean', train.py:87), summed in double
__global__ void __launch_bounds__(256) loss_kernel(const float* __restrict__ sq_err, int64_t B, float* __restrict__ loss) {
  __shared__ double part[256];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < B; i += 256) acc += (double)sq_err[i];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = (float)(part[0] / (3.0 * (double)B));
}

// Training workspace carve (each region 256-B aligned), M = B*N samples:
//   dirs (B,3) | z (B,N) | feat (B,256) | encd (B,32) | rgb (M,3) | sigma (M) | maps (B,4)
//   | dsigma (M) | drgb (M,3) | sq_err (B) | save (M,kSaveRow) | masks (M,kMaskRow) | grad (M,kGradRow)
//   | wgrad partials
enum { T_DIRS, T_Z, T_FEAT, T_ENCD, T_RGB, T_SIG, T_MAPS, T_DSIG, T_DRGB, T_SQE, T_SAVE, T_MASK, T_GRAD, T_WG,
       T_COUNT };

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// the largest wgrad partial buffer over the parameter list of param_grads (one stream's)
static size_t wgrad_stream_floats(int64_t M) {
  const int Ks[] = {kPosEnc, kHidden, kHidden + kPosEnc, kHidden + kDirEnc, kAppDim, kDirHidden};
  size_t m = 0;
  for (int K : Ks) {
    const size_t f = wgrad_workspace_floats(M, kHidden, K);
    if (f > m) m = f;
  }
  return m;
}
// param_grads' workspace: two streams' partial buffers + the ray-sum buffers
static size_t max_wgrad_floats(int64_t M) {
  return 2 * ((wgrad_stream_floats(M) + 63) & ~(size_t)63) + ray_sum_floats(M) + 64;
}

// Which MLP arithmetic the last nerf_train_forward on a workspace ran under (the f32 forward writes no
// mask rows): nerf_train_backward picks the mask source from it, not from the setting in force at
// backward time.  A small host-side table keyed by workspace address.
static std::mutex g_ws_mu;
static std::unordered_map<const void*, int> g_ws_arith;
static void remember_forward_arith(const void* ws, int arith) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  if (g_ws_arith.size() > 4096) g_ws_arith.clear();
  g_ws_arith[ws] = arith;
}
static int forward_arith(const void* ws) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  const auto it = g_ws_arith.find(ws);
  return it == g_ws_arith.end() ? -1 : it->second;
}

static size_t train_carve(int64_t B, int N, size_t* off) {
  const size_t b = (size_t)B, M = b * (size_t)N, MT = (size_t)tile_rows((int64_t)M);   // tile-major rows (layout.h)
  const size_t sizes[T_COUNT] = {b * 3, b * N, b * kRayFeat, b * 32, M * 3, M, b * 4, M, M * 3, b,
                                 MT * kSaveRow, M * kMaskRow, MT * kGradRow, max_wgrad_floats((int64_t)M)};
  size_t at = 0;
  for (int i = 0; i < T_COUNT; ++i) {
    off[i] = at;
    at += align256(sizes[i] * 4);
  }
  return at;
}
}  // namespace nerf

using namespace nerf;

#define TREQUIRE(cond, ...)                                        \
  do {                                                             \
    if (!(cond)) return set_error(NERF_ERR_BAD_ARG, __VA_ARGS__);  \
  } while (0)

extern "C" {

size_t nerf_packed_transposed_floats(void) { return kPackedTFloats; }

int nerf_pack_weights_transposed(const float* const* params, float* packedT, nerf_stream_t stream) {
  TREQUIRE(params && packedT, "nerf_pack_weights_transposed: null pointer");
  for (int i = 0; i < P_COUNT; ++i) TREQUIRE(params[i], "nerf_pack_weights_transposed: parameter %d is null", i);
  return launch_packT(params, packedT, (hipStream_t)stream);
}

int nerf_pack_weights_transposed_host(const float* const* params, float* packedT) {
  TREQUIRE(params && packedT, "nerf_pack_weights_transposed_host: null pointer");
  for (int i = 0; i < P_COUNT; ++i) TREQUIRE(params[i], "nerf_pack_weights_transposed_host: parameter %d is null", i);
  packT_host(params, packedT);
  return NERF_OK;
}

int nerf_ray_features_train(const float* packed, const float* dirs, int64_t R, const float* app, int64_t app_rows,
                            float* feat, float* enc_d, nerf_stream_t stream) {
  TREQUIRE(R >= 0, "nerf_ray_features_train: R=%lld", (long long)R);
  TREQUIRE(app_rows == 0 || app_rows == 1 || app_rows == R, "nerf_ray_features_train: app_rows=%lld with R=%lld",
           (long long)app_rows, (long long)R);
  TREQUIRE(R == 0 || (packed && dirs && feat && enc_d && (app_rows == 0 || app)),
           "nerf_ray_features_train: null pointer");
  return launch_ray_features(packed, dirs, R, app, app_rows, feat, (hipStream_t)stream, enc_d);
}

int nerf_mlp_forward_train(const float* packed, const float* origins, const float* dirs, const float* z_vals,
                           int64_t R, int N, const float* ray_feat, const float* enc_d, float* rgb, float* sigma,
                           float* save, uint32_t* masks, nerf_stream_t stream) {
  TREQUIRE(R >= 0 && N >= 1, "nerf_mlp_forward_train: R=%lld N=%d", (long long)R, N);
  TREQUIRE(R == 0 || (packed && origins && dirs && z_vals && ray_feat && enc_d && rgb && sigma && save),
           "nerf_mlp_forward_train: null pointer");
  TREQUIRE(R == 0 || masks || g_mlp_arith != NERF_ARITH_F16X3, "nerf_mlp_forward_train: masks required under f16x3");
  return launch_mlp(packed, origins, dirs, z_vals, R, N, ray_feat, rgb, sigma, nullptr, 0, (hipStream_t)stream, save,
                    enc_d, masks);
}

int nerf_composite_backward(const float* rgb, const float* sigma, const float* z_vals, const float* rgb_map,
                            const float* target, int64_t B, int N, float scale, float* dsigma, float* drgb,
                            float* sq_err, nerf_stream_t stream) {
  TREQUIRE(B >= 0, "nerf_composite_backward: B=%lld", (long long)B);
  if (N < 1 || N > 4096) return set_error(NERF_ERR_UNSUPPORTED, "nerf_composite_backward: N=%d (1..4096)", N);
  TREQUIRE(B == 0 || (rgb && sigma && z_vals && rgb_map && target && dsigma && drgb && sq_err),
           "nerf_composite_backward: null pointer");
  return launch_composite_backward(rgb, sigma, z_vals, rgb_map, target, nullptr, nullptr, B, N, scale, dsigma, drgb,
                                   sq_err, (hipStream_t)stream);
}

int nerf_composite_backward_grad(const float* rgb, const float* sigma, const float* z_vals, const float* grad_rgb_map,
                                 const float* grad_depth_map, int64_t B, int N, float* dsigma, float* drgb,
                                 nerf_stream_t stream) {
  TREQUIRE(B >= 0, "nerf_composite_backward_grad: B=%lld", (long long)B);
  if (N < 1 || N > 4096) return set_error(NERF_ERR_UNSUPPORTED, "nerf_composite_backward_grad: N=%d (1..4096)", N);
  TREQUIRE(B == 0 || (rgb && sigma && z_vals && dsigma && drgb), "nerf_composite_backward_grad: null pointer");
  return launch_composite_backward(rgb, sigma, z_vals, nullptr, nullptr, grad_rgb_map, grad_depth_map, B, N, 0.0f,
                                   dsigma, drgb, nullptr, (hipStream_t)stream);
}

int nerf_mlp_backward(const float* packed, const float* packedT, const float* save, const uint32_t* masks,
                      const float* sigma, const float* rgb, const float* dsigma, const float* drgb, int64_t M,
                      float* grad, nerf_stream_t stream) {
  TREQUIRE(M >= 0, "nerf_mlp_backward: M=%lld", (long long)M);
  TREQUIRE(M == 0 || (packed && packedT && save && sigma && rgb && dsigma && drgb && grad),
           "nerf_mlp_backward: null pointer");
  return launch_mlp_backward(packed, packedT, save, masks, sigma, rgb, dsigma, drgb, M, grad, (hipStream_t)stream);
}

size_t nerf_wgrad_workspace_bytes(int64_t M, int N, int K) {
  if (M < 0 || N < 1 || K < 0) return 0;
  return wgrad_workspace_floats(M, N, K) * 4;
}

int nerf_wgrad(const float* a, int64_t lda, int N, const float* x, int64_t ldx, int K, int64_t x_div, int64_t M,
               float* out_w, float* out_b, int accumulate, void* workspace, size_t ws_bytes, nerf_stream_t stream) {
  TREQUIRE(M >= 0 && M < ((int64_t)1 << 31) && N >= 1 && K >= 0 && x_div >= 0, "nerf_wgrad: M=%lld N=%d K=%d",
           (long long)M, N, K);
  TREQUIRE(lda >= N && (K == 0 || ldx >= K), "nerf_wgrad: lda=%lld ldx=%lld", (long long)lda, (long long)ldx);
  TREQUIRE(M == 0 || (a && (K == 0 || x) && (K == 0 || out_w) && workspace), "nerf_wgrad: null pointer");
  if (ws_bytes < wgrad_workspace_floats(M, N, K) * 4)
    return set_error(NERF_ERR_WORKSPACE, "nerf_wgrad: workspace %zu < %zu bytes", ws_bytes,
                     wgrad_workspace_floats(M, N, K) * 4);
  return launch_wgrad(a, lda, N, x, ldx, K, x_div, M, out_w, K, out_b, accumulate, (float*)workspace,
                      (hipStream_t)stream);
}

// Every parameter gradient of NeRF (+ the appearance rows) from the saved activations and the
// per-sample gradient rows; param_grads follows nerf_pack_weights' 24-pointer order.
//
// Two streams.  The GEMMs are independent (each reads its slices of the save and gradient rows and
// writes its own parameters), so they run on the caller's stream and on a second library stream,
// each with its own partial buffer: one launch's tail, the small reductions and the memory-bound
// ray sums overlap the other stream's GEMMs.  Every output is still written by one GEMM and one
// fixed-order reduction (deterministic).  The second stream forks from the caller's after
// everything queued there (the gradient rows) and the caller's stream waits for it at the end.
struct PgStreams {
  hipStream_t s2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
static int pg_streams(PgStreams** out) {
  static thread_local PgStreams per_dev[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return set_error(NERF_ERR_HIP, "param_grads: hipGetDevice");
  PgStreams& p = per_dev[dev];
  if (!p.s2) {
    if (hipStreamCreateWithFlags(&p.s2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&p.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&p.join, hipEventDisableTiming) != hipSuccess)
      return set_error(NERF_ERR_HIP, "param_grads: stream/event creation failed");
  }
  *out = &p;
  return NERF_OK;
}

// Where the block exponents of gradient entry ja and save entry jx live (layout.h)
static H16Meta block_exps(const float* save, const float* grad, int ja, int jx) {
  H16Meta m;
  if (ja < 0 || jx < 0) return m;
  m.a = grad + tile_col(kMetaGradF) + 8 * ja + kMetaGradF % 8;
  m.a_stride = 32 * (int64_t)kGradRow;
  m.x = save + tile_col(kMetaSaveF) + 8 * jx + kMetaSaveF % 8;
  m.x_stride = 32 * (int64_t)kSaveRow;
  return m;
}

// The jobs, on streams sa / sb with partial buffers wa / wb (wfl floats each) and the ray-sum
// buffers at `rays` (N >= kRaySumMinN).
static int param_grads_jobs(const float* save, const float* grad, int64_t M, int N, const float* app, int64_t app_rows,
                            const float* packed, float* const* g, float* dapp, float* wa, float* wb, size_t wfl,
                            float* rays, hipStream_t sa, hipStream_t sb) {
  // Job: columns [k0, k0 + K) of parameter p's weight gradient (row length ldo) from x; the bias
  // gradient with the first column block only.  The skip layer's [h3 | enc_x] runs as a 256 x 256
  // block (the whole-tile kernel) plus the 63 PE columns, instead of one 256 x 319 GEMM on 128 x 128
  // tiles (416 -> ~300 us per step).
  // save and grad are tile-major rows (layout.h): a slice starting at feature c is the same layout at
  // float offset tile_col(c).  Stream B: the K <= 64 GEMMs, layers 6-7 and the heads below.
  // ja / jx: the block-exponent entries of a and x (layout.h; -1: none)
  struct Job { int a; int n; int x; int K; int p; int k0; int ldo; bool bias; bool b; int ja; int jx; };
  constexpr int kSkipK = kHidden + kPosEnc;
  const Job jobs[] = {
      {0, kHidden, kSaveEncX, kPosEnc, 0, 0, kPosEnc, true, true, -1, -1},
      {1 * kHidden, kHidden, save_h(0), kHidden, 2, 0, kHidden, true, false, 0, 0},
      {2 * kHidden, kHidden, save_h(1), kHidden, 4, 0, kHidden, true, false, 1, 1},
      {3 * kHidden, kHidden, save_h(2), kHidden, 6, 0, kHidden, true, false, 2, 2},
      {4 * kHidden, kHidden, save_h(3), kHidden, 8, 0, kSkipK, true, false, 3, 3},                  // h3 ..
      {4 * kHidden, kHidden, save_h(3) + kHidden, kPosEnc, 8, kHidden, kSkipK, false, true, -1, -1},  // .. | enc_x
      {5 * kHidden, kHidden, save_h(4), kHidden, 10, 0, kHidden, true, false, 4, 4},
      {6 * kHidden, kHidden, save_h(5), kHidden, 12, 0, kHidden, true, true, 5, 5},
      {7 * kHidden, kHidden, save_h(6), kHidden, 14, 0, kHidden, true, true, 6, 6},
      {kGradRgb, 3, kSaveHd, kDirHidden, P_RGB_W, 0, kDirHidden, true, false, -1, -1},
  };
  static_assert(kSaveEncX == save_h(3) + kHidden, "the skip layer's input [h3 | enc_x] is contiguous in the save row");
  int rc;
  // layer 0 and the skip layer's PE columns (both over enc_x): one launch of the split arithmetic's
  // pair kernel; under f32 two K = 63 jobs on the f32 GEMM like every other weight gradient
  const bool pe_pair = g_mlp_arith == NERF_ARITH_F16X3;
  if (pe_pair && (rc = launch_wgrad_pe_pair(save, grad, M, g[0], g[1], g[8], wb, wfl, sb))) return rc;
  // fused per-ray sums (the split arithmetic's dir/density launch writes d pre_dir's 8-sample sums,
  // the rgb head's launch d hd's block sums; blocks of 32 samples lie on one ray): below, on stream B
  const bool fused = rays && fused_ray_sums(N);
  for (const Job& j : jobs) {
    if (pe_pair && j.K == kPosEnc) continue;            // (in the pair above)
    if (fused && j.a == kGradRgb) continue;             // (with the per-ray sums below)
    if (wgrad_workspace_floats(M, j.n, j.K) > wfl) return set_error(NERF_ERR_WORKSPACE, "param_grads: workspace");
    if (j.a == kGradRgb) {   // the rgb head: the streaming kernel (3 rows)
      if ((rc = launch_wgrad_head3(grad + tile_col(kGradRgb), save + tile_col(kSaveHd), M, g[j.p], g[j.p + 1],
                                   j.b ? wb : wa, wfl, j.b ? sb : sa)))
        return rc;
      continue;
    }
    const H16Meta hm = block_exps(save, grad, j.ja, j.jx);
    if ((rc = launch_wgrad(grad + tile_col(j.a), kGradRow, j.n, save + tile_col(j.x), kSaveRow, j.K, 1, M, g[j.p] + j.k0,
                           j.ldo, j.bias ? g[j.p + 1] : nullptr, 0, j.b ? wb : wa, j.b ? sb : sa, nullptr, true, true,
                           j.ja >= 0 ? &hm : nullptr)))
      return rc;
  }
  static_assert(kGradSigma == kGradDir + kDirHidden, "the density head's gradient follows dir_linear's");
  if (rays) {
    // Rays of N >= 32 samples.  dir_linear's h7 columns and the density head (1 row over h7) run as
    // one 160 x 256 GEMM on the whole-tile kernel (5 row tiles) over a = the gradient columns from
    // d pre_dir on ([d pre_dir | d sigma | pad | d hd...]) and x = h7: rows 0..127 are dir_linear's
    // gradient (+ its bias column), row 128 the density head's, rows 129.. are dropped (h7 is read once).
    // dir_linear's PE_4(d) columns and the appearance projection take per-ray inputs: GEMMs over
    // per-ray (or per-block) gradient sums, which replace two M-row GEMMs: under the split arithmetic
    // with N % 32 == 0 the dir/density launch itself writes d pre_dir's 8-sample sums and the rgb
    // head's launch d hd's block sums from d rgb_pre; otherwise ray_sums_kernel reads the
    // 256 gradient columns of every sample.
    const int64_t B = M / N;
    float* S = rays;                                       // B x 256 (fused: S8, (M / 8) x 128)
    float* S_hd = S + ray_sum_a_floats(M);                 // fused: (M / 32) x 128
    float* E = S_hd + ray_sum_b_floats(M);                 // B x 32
    constexpr int kDirRows = 160;
    if (wgrad_workspace_floats(M, kDirRows, kWT) > wfl) return set_error(NERF_ERR_WORKSPACE, "param_grads: workspace");
    const WgradSplit heads{kDirHidden, g[P_SIGMA_W], kHidden, kHidden, g[P_SIGMA_B], kDirHidden + 1};
    H16Meta hm = block_exps(save, grad, 7, 7);
    hm.a_cols = kDirHidden + 1;                            // d pre_dir, d sigma (rows 129.. are dropped)
    if ((rc = launch_wgrad(grad + tile_col(kGradDir), kGradRow, kDirRows, save + tile_col(save_h(7)), kSaveRow, kHidden, 1,
                           M, g[P_DIR_W], kHidden + kDirEnc, g[P_DIR_B], 0, wb, sb, &heads, true, true, &hm,
                           fused ? S : nullptr)))
      return rc;
    if (fused) {
      const HeadSums hs{save, packed, N, S_hd, E};   // (rgb_linear's weight gradient + S_hd, E)
      if ((rc = launch_wgrad_head3(grad + tile_col(kGradRgb), save + tile_col(kSaveHd), M, g[P_RGB_W], g[P_RGB_B], wb, wfl,
                                   sb, &hs)))
        return rc;
      // dir_linear's PE_4(d) columns over the M / 8 rows of 8-sample sums (row m: samples 8m .. 8m+7,
      // ray 8m / N)
      if ((rc = launch_wgrad(S, kDirHidden, kDirHidden, E, 32, kDirEnc, N / 8, M / 8, g[P_DIR_W] + kHidden,
                             kHidden + kDirEnc, nullptr, 0, wb, sb)))
        return rc;
      if (app_rows == 0) return NERF_OK;     // no appearance: the projection is unused (models.py:146)
      if ((rc = launch_wgrad(S_hd, kDirHidden, kDirHidden, app, kAppDim, kAppDim, app_rows == 1 ? 0 : N / 32, M / 32,
                             g[P_APP_W], kAppDim, g[P_APP_B], 0, wb, sb)))
        return rc;
      if (!dapp) return NERF_OK;
      if (app_rows == 1) return launch_app_grad(g[P_APP_B], 1, 1, 1, packed, dapp, sb, false);
      return launch_app_grad(S_hd, kDirHidden, app_rows, N / 32, packed, dapp, sb, false);
    }
    hipLaunchKernelGGL(ray_sums_kernel, dim3((unsigned)B), dim3(256), 0, sb, grad, save, N, S, E);
    if ((rc = check_launch("ray_sums_kernel"))) return rc;
    if ((rc = launch_wgrad(S, 256, kDirHidden, E, 32, kDirEnc, 1, B, g[P_DIR_W] + kHidden, kHidden + kDirEnc, nullptr,
                           0, wb, sb)))
      return rc;
    if (app_rows == 0) return NERF_OK;     // no appearance: the projection is unused (models.py:146)
    if ((rc = launch_wgrad(S + kDirHidden, 256, kDirHidden, app, kAppDim, kAppDim, app_rows == 1 ? 0 : 1, B,
                           g[P_APP_W], kAppDim, g[P_APP_B], 0, wb, sb)))
      return rc;
    if (!dapp) return NERF_OK;
    if (app_rows == 1) return launch_app_grad(g[P_APP_B], 1, 1, 1, packed, dapp, sb, false);
    return launch_app_grad(S + kDirHidden, 256, app_rows, 1, packed, dapp, sb, false);
  }
  // dir_linear (128 rows over [h7 | enc_d]) and the density head (1 row over h7) in one GEMM: the
  // gradient row holds [d pre_dir | d sigma], so rows 0..127 are dir_linear's gradient and row 128
  // (its first 256 columns and the bias column) the density head's: h7 is read once
  if (wgrad_workspace_floats(M, kDirHidden + 1, kHidden + kDirEnc) > wfl)
    return set_error(NERF_ERR_WORKSPACE, "param_grads: workspace");
  const WgradSplit heads{kDirHidden, g[P_SIGMA_W], kHidden, kHidden, g[P_SIGMA_B]};
  if ((rc = launch_wgrad(grad + tile_col(kGradDir), kGradRow, kDirHidden + 1, save + tile_col(save_h(7)), kSaveRow,
                         kHidden + kDirEnc, 1, M, g[P_DIR_W], kHidden + kDirEnc, g[P_DIR_B], 0, wb, sb, &heads, true)))
    return rc;
  if (app_rows == 0) {   // no appearance: the projection is unused (models.py:146)
    return NERF_OK;
  }
  // appearance_projection: x = the ray's embedding row (broadcast when app_rows == 1; row-major)
  const int64_t xdiv = app_rows == 1 ? 0 : N;
  if ((rc = launch_wgrad(grad + tile_col(kGradHd), kGradRow, kDirHidden, app, kAppDim, kAppDim, xdiv, M, g[P_APP_W],
                         kAppDim, g[P_APP_B], 0, wb, sb, nullptr, true, /*x_tiled=*/false)))
    return rc;
  if (!dapp) return NERF_OK;
  if (app_rows == 1) return launch_app_grad(g[P_APP_B], 1, 1, 1, packed, dapp, sb, false);
  return launch_app_grad(grad + tile_col(kGradHd), kGradRow, app_rows, N, packed, dapp, sb, true);
}

static int param_grads(const float* save, const float* grad, int64_t M, int N, const float* app, int64_t app_rows,
                       const float* packed, float* const* g, float* dapp, float* ws, size_t ws_floats,
                       hipStream_t s) {
  const bool ray_path = N >= kRaySumMinN;
  const size_t rf = ray_path ? ray_sum_floats(M) : 0;
  if (ws_floats < rf + 64) return set_error(NERF_ERR_WORKSPACE, "param_grads: workspace");
  const size_t avail = (ws_floats - rf) & ~(size_t)63;   // partial buffers; the ray sums after them, aligned
  float* rays = ray_path ? ws + avail : nullptr;
  const size_t w1 = (wgrad_stream_floats(M) + 63) & ~(size_t)63;
  const bool two = avail >= 2 * w1;
  if (!two) return param_grads_jobs(save, grad, M, N, app, app_rows, packed, g, dapp, ws, ws, avail, rays, s, s);
  PgStreams* ps;
  int rc;
  if ((rc = pg_streams(&ps))) return rc;
  if (hipEventRecord(ps->fork, s) != hipSuccess || hipStreamWaitEvent(ps->s2, ps->fork, 0) != hipSuccess)
    return set_error(NERF_ERR_HIP, "param_grads: stream fork failed");
  rc = param_grads_jobs(save, grad, M, N, app, app_rows, packed, g, dapp, ws, ws + w1, w1, rays, s, ps->s2);
  // join even after a failed launch, so the caller's stream never runs ahead of queued work
  if (hipEventRecord(ps->join, ps->s2) != hipSuccess || hipStreamWaitEvent(s, ps->join, 0) != hipSuccess)
    return rc ? rc : set_error(NERF_ERR_HIP, "param_grads: stream join failed");
  return rc;
}

int nerf_param_grads(const float* save, const float* grad, int64_t M, int N, const float* app, int64_t app_rows,
                     const float* packed, float* const* param_grads_out, float* dapp, void* workspace,
                     size_t ws_bytes, nerf_stream_t stream) {
  TREQUIRE(M >= 0 && M < ((int64_t)1 << 31) && N >= 1 && M % N == 0, "nerf_param_grads: M=%lld N=%d",
           (long long)M, N);
  TREQUIRE(app_rows == 0 || app_rows == 1 || app_rows * N == M, "nerf_param_grads: app_rows=%lld", (long long)app_rows);
  TREQUIRE(param_grads_out && packed && workspace && (M == 0 || (save && grad)) && (app_rows == 0 || app),
           "nerf_param_grads: null pointer");
  for (int i = 0; i < P_COUNT; ++i) TREQUIRE(param_grads_out[i], "nerf_param_grads: gradient %d is null", i);
  if (M == 0) return NERF_OK;
  return param_grads(save, grad, M, N, app, app_rows, packed, param_grads_out, dapp, (float*)workspace, ws_bytes / 4,
                     (hipStream_t)stream);
}

size_t nerf_param_grads_workspace_bytes(int64_t M) { return M < 0 ? 0 : max_wgrad_floats(M) * 4; }

int nerf_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr, double beta1,
              double beta2, double eps, int64_t step, nerf_stream_t stream) {
  TREQUIRE(n >= 0 && step >= 1, "nerf_adam: n=%lld step=%lld", (long long)n, (long long)step);
  TREQUIRE(n == 0 || (param && grad && exp_avg && exp_avg_sq), "nerf_adam: null pointer");
  return launch_adam(param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, step, (hipStream_t)stream);
}

size_t nerf_train_workspace_bytes(int64_t B, int N) {
  if (B < 0 || N < 1) return 0;
  size_t off[T_COUNT];
  return train_carve(B, N, off);
}

int nerf_train_forward(const float* packed, const float* rays_o, const float* rays_d, int64_t B, double near,
                       double far, int N, const float* t_vals, int perturb, const float* t_rand, uint64_t seed,
                       const float* app, int64_t app_rows, float* rgb_map, float* depth_map, float* weights_out,
                       float* z_out, void* workspace, size_t ws_bytes, nerf_stream_t stream) {
  TREQUIRE(B >= 0, "nerf_train_forward: B=%lld", (long long)B);
  if (N < 1 || N > 4096) return set_error(NERF_ERR_UNSUPPORTED, "nerf_train_forward: N=%d (1..4096)", N);
  TREQUIRE(app_rows == 0 || app_rows == 1 || app_rows == B, "nerf_train_forward: app_rows=%lld with B=%lld",
           (long long)app_rows, (long long)B);
  if (B == 0) return NERF_OK;
  TREQUIRE((int64_t)B * N < ((int64_t)1 << 31), "nerf_train_forward: B*N=%lld too large", (long long)B * N);
  TREQUIRE(packed && rays_o && rays_d && t_vals && rgb_map && depth_map && workspace && (app_rows == 0 || app),
           "nerf_train_forward: null pointer");
  size_t off[T_COUNT];
  const size_t need = train_carve(B, N, off);
  if (ws_bytes < need) return set_error(NERF_ERR_WORKSPACE, "nerf_train_forward: workspace %zu < %zu bytes", ws_bytes, need);
  char* ws = (char*)workspace;
  auto R = [&](int i) { return (float*)(ws + off[i]); };
  hipStream_t s = (hipStream_t)stream;
  int rc;
  // the directions normalised (render.py:19) by the ray-feature kernel, which writes them to T_DIRS
  if ((rc = launch_ray_features(packed, rays_d, B, app, app_rows, R(T_FEAT), s, R(T_ENCD), R(T_DIRS)))) return rc;
  if ((rc = launch_stratified(rays_o, R(T_DIRS), B, (float)near, (float)(far - near), N, t_vals, perturb, t_rand,
                              seed, R(T_Z), nullptr, s)))
    return rc;                                                                                          // :22
  if ((rc = launch_mlp(packed, rays_o, R(T_DIRS), R(T_Z), B, N, R(T_FEAT), R(T_RGB), R(T_SIG), nullptr, 0, s,
                       R(T_SAVE), R(T_ENCD), (uint32_t*)R(T_MASK))))
    return rc;                                                                                          // :49
  remember_forward_arith(workspace, g_mlp_arith);
  if ((rc = launch_composite(R(T_RGB), R(T_SIG), R(T_Z), B, N, rgb_map, depth_map, weights_out, s))) return rc;  // :56-80
  if (z_out && hipMemcpyAsync(z_out, R(T_Z), (size_t)B * N * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return set_error(NERF_ERR_HIP, "nerf_train_forward: z copy failed");
  return NERF_OK;
}

int nerf_train_backward(const float* packed, const float* packedT, const float* rgb_map, const float* target,
                        int64_t B, int N, const float* app, int64_t app_rows, float* const* param_grads_out,
                        float* dapp, float* loss, void* workspace, size_t ws_bytes, nerf_stream_t stream) {
  TREQUIRE(B >= 0 && N >= 1 && N <= 4096, "nerf_train_backward: B=%lld N=%d", (long long)B, N);
  TREQUIRE(app_rows == 0 || app_rows == 1 || app_rows == B, "nerf_train_backward: app_rows=%lld", (long long)app_rows);
  TREQUIRE(packed && packedT && param_grads_out && loss && workspace && (B == 0 || (rgb_map && target)) &&
               (app_rows == 0 || app),
           "nerf_train_backward: null pointer");
  for (int i = 0; i < P_COUNT; ++i) TREQUIRE(param_grads_out[i], "nerf_train_backward: gradient %d is null", i);
  if (B == 0) return NERF_OK;
  size_t off[T_COUNT];
  const size_t need = train_carve(B, N, off);
  if (ws_bytes < need) return set_error(NERF_ERR_WORKSPACE, "nerf_train_backward: workspace %zu < %zu bytes", ws_bytes, need);
  char* ws = (char*)workspace;
  auto R = [&](int i) { return (float*)(ws + off[i]); };
  hipStream_t s = (hipStream_t)stream;
  // the mask rows exist only when this workspace's forward ran under f16x3; the backward's kernels
  // follow the arithmetic in force now (an f16x3 backward after an f32 forward reads the ReLU masks
  // from the saved activations instead)
  const int fwd_arith = forward_arith(workspace);
  if (fwd_arith < 0)
    return set_error(NERF_ERR_BAD_ARG, "nerf_train_backward: no nerf_train_forward wrote this workspace");
  const uint32_t* masks = fwd_arith == NERF_ARITH_F16X3 ? (const uint32_t*)R(T_MASK) : nullptr;
  const int64_t M = B * N;
  int rc;
  const float scale = (float)(2.0 / (3.0 * (double)B));                                              // train.py:87
  if ((rc = launch_composite_backward(R(T_RGB), R(T_SIG), R(T_Z), rgb_map, target, nullptr, nullptr, B, N, scale,
                                      R(T_DSIG),
                                      R(T_DRGB), R(T_SQE), s)))
    return rc;
  hipLaunchKernelGGL(loss_kernel, dim3(1), dim3(256), 0, s, R(T_SQE), B, loss);
  if ((rc = check_launch("loss_kernel"))) return rc;
  if ((rc = launch_mlp_backward(packed, packedT, R(T_SAVE), masks, R(T_SIG), R(T_RGB), R(T_DSIG), R(T_DRGB), M,
                                R(T_GRAD), s, /*store_dhd=*/!fused_ray_sums(N))))
    return rc;
  const size_t wg_floats = (need - off[T_WG]) / 4;
  return param_grads(R(T_SAVE), R(T_GRAD), M, N, app, app_rows, packed, param_grads_out, dapp, R(T_WG), wg_floats, s);
}

}  // extern "C"
