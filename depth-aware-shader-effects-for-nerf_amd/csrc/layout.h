// Packed-weight layout of the fused MLP (shared by the device pack kernel, the host
// packer and the MLP kernel).  DESIGN.md §"Weight layout" explains it; in short:
//
// The MLP runs every dense layer as out^T = W . in^T on v_mfma_f32_32x32x2_f32 with
// A = W (32 output neurons x 2 inputs per instruction) and B = the activations
// (2 inputs x 32 samples).  The 32x32 accumulator of one layer holds, in lane l and
// register g, sample (l & 31) and neuron (g&3) + 8(g>>2) + 4(l>>5) of a 32-neuron
// tile.  The next layer consumes that register directly as its B operand (k-step
// "register g of tile t"), so the k order of every weight matrix is permuted to
// match, here, once, at pack time.  Positional-encoding inputs use a fixed k order
// too (pe_feature below).
//
// A fragment block is one (n-tile, 4 consecutive k-steps) pair: 64 lanes x 4 floats,
// lane l holding W[nt*32 + (l&31)][col(ks, l>>5)] for ks = 4*kq .. 4*kq+3, so one
// wave reads a block with one coalesced 16-byte-per-lane load.
#pragma once
#include <stdint.h>
#include <stddef.h>

#if defined(__HIPCC__)
#define NERF_HD __host__ __device__
#else
#define NERF_HD
#endif

namespace nerf {

constexpr int kHidden = 256;
constexpr int kPosLevels = 10;
constexpr int kDirLevels = 4;
constexpr int kPosEnc = 3 * (1 + 2 * kPosLevels);  // 63
constexpr int kDirEnc = 3 * (1 + 2 * kDirLevels);  // 27
constexpr int kAppDim = 32;
constexpr int kDirHidden = kHidden / 2;             // 128
constexpr int kSkipLayer = 4;
constexpr int kPeSteps = 32;                        // PE padded 63 -> 64 inputs = 32 k-steps
constexpr int kActSteps = kHidden / 2;              // 256 inputs = 128 k-steps
constexpr int kRayFeat = 2 * kDirHidden;            // per-ray [dir part | appearance part]

// Matrices held as fragments: 0 = layer 0 (PE input), 1..7 = the 256 activation inputs of
// trunk layers 1..7, 8 = the h-part of dir_linear, 9 = the PE part of the skip layer
// (layer 4 input is cat[h, enc_x], models.py:130-131).
constexpr int kNumFragMats = 10;
constexpr int kSkipPeMat = 9;
NERF_HD constexpr bool frag_is_pe(int m) { return m == 0 || m == kSkipPeMat; }
NERF_HD constexpr int frag_ntiles(int m) { return m == 8 ? 4 : 8; }
NERF_HD constexpr int frag_act_steps(int m) { return frag_is_pe(m) ? 0 : kActSteps; }
NERF_HD constexpr int frag_pe_steps(int m) { return frag_is_pe(m) ? kPeSteps : 0; }
NERF_HD constexpr int frag_ksteps(int m) { return frag_act_steps(m) + frag_pe_steps(m); }
NERF_HD constexpr size_t frag_floats(int m) { return (size_t)frag_ntiles(m) * frag_ksteps(m) * 64; }
NERF_HD constexpr size_t frag_offset(int m) {
  size_t off = 0;
  for (int i = 0; i < m; ++i) off += frag_floats(i);
  return off;
}
constexpr size_t kFragFloats = frag_offset(kNumFragMats);   // 524288 floats = 2 MiB

// Raw vectors after the fragments (each rounded up to 4 floats for 16-B loads).
constexpr size_t kOffBias = kFragFloats;                        // 8 x 256 trunk biases
constexpr size_t kOffSigmaW = kOffBias + 8 * kHidden;           // density_head.weight (256)
constexpr size_t kOffSigmaB = kOffSigmaW + kHidden;             // density_head.bias (1, padded 4)
constexpr size_t kOffDirB = kOffSigmaB + 4;                     // dir_linear.bias (128)
constexpr size_t kOffDirWd = kOffDirB + kDirHidden;             // dir_linear.weight[:,256:283] (128 x 27)
constexpr size_t kOffAppW = kOffDirWd + kDirHidden * kDirEnc;   // appearance_projection.weight (128 x 32)
constexpr size_t kOffAppB = kOffAppW + kDirHidden * kAppDim;    // appearance_projection.bias (128)
constexpr size_t kOffRgbW = kOffAppB + kDirHidden;              // rgb_linear.weight (3 x 128)
constexpr size_t kOffRgbB = kOffRgbW + 3 * kDirHidden;          // rgb_linear.bias (3, padded 4)
constexpr size_t kF32Floats = kOffRgbB + 4;                     // end of the exact-f32 path's data

// ---- split-f16 ("f16x3") fragments: the same 10 matrices as f16 hi/lo pairs --------------------
// The f16x3 MLP runs every dense layer on v_mfma_f32_32x32x16_f16 as three products
// hi(W)hi(a) + hi(W)lo(a) + lo(W)hi(a), where x*s = hi + lo + O(2^-24 x*s) with hi = f16(x*s)
// and lo = f16(x*s - hi), s a power of two (per layer for W, per sample for a) that keeps every
// value under 2^15.  The dropped lo*lo term is O(2^-24): fp32-level accuracy at 3 x 32 MFMA
// cycles per 16-deep k-step against 8 x 64 for the exact f32 instruction.
//
// A k-step is 16 inputs; lane l supplies 8 of them, k = 8(l>>5) + j (j = 0..7), for row or
// column l&31.  Activation k-step ks = 2t + s reads registers 8s..8s+7 of the previous layer's
// accumulator tile t as they stand, so element j of lane half h is input feature
// 32t + 16s + 8(j>>2) + 4h + (j&3).  PE k-step q reads PE slot p = 8q + j (pe_feature).
//
// Nine "layers" stream their weights in the order the kernel consumes them: trunk layers 0..7
// (layer 4 = its activation part, matrix 4, then its PE part, matrix 9) and the colour layer
// (dir_linear's h part, matrix 8).  A trunk layer's 8 output tiles run as two groups of 4
// (tiles 0-3, then 4-7), each over all of the layer's k-steps; the colour layer is one group.
// The stream is a sequence of 16 KiB CHUNKS, each 2 k-steps x 4 tiles x {hi, lo} "pieces" of
// 64 lanes x 8 halves (1 KiB): piece (kk*4 + ti)*2 + part of chunk i of group g of layer L holds
// k-step 2i + kk of tile 4g + ti.
constexpr int kS16Layers = 9;                                    // 0..7 trunk, 8 = colour
NERF_HD constexpr int s16_layer_ks(int L) { return L == 0 ? 4 : (L == kSkipLayer ? 20 : 16); }
NERF_HD constexpr int s16_layer_groups(int L) { return L == 8 ? 1 : 2; }
NERF_HD constexpr int s16_layer_chunks(int L) { return s16_layer_groups(L) * s16_layer_ks(L) / 2; }
NERF_HD constexpr int s16_chunk0(int L) {                        // first chunk of layer L
  int c = 0;
  for (int i = 0; i < L; ++i) c += s16_layer_chunks(i);
  return c;
}
constexpr int kS16Chunks = s16_chunk0(kS16Layers);               // 128
constexpr int kChunkFloats = 4096;                               // 16 KiB
static_assert(kS16Chunks * kChunkFloats == (int)kFragFloats, "the stream holds exactly the 10 matrices");
constexpr size_t kOff16 = (kF32Floats + 255) / 256 * 256;       // 1 KiB aligned
// Per-layer constants after the stream: s_w, 1/s_w (9 each); R = max row L1 norm of W over all of
// the layer's inputs, B = max |bias| (8 trunk layers each); bound |y| <= R max|a| + B.
constexpr size_t kOffScale16 = kOff16 + kFragFloats;
constexpr int kS16Sw = 0, kS16InvW = 9, kS16R = 18, kS16B = 26, kS16Consts = 48;
constexpr size_t kPackedFloats = kOffScale16 + kS16Consts;

// Matrix and its k-step for k-step ks of layer L.
NERF_HD inline int s16_matrix(int L, int ks) { return L == 8 ? 8 : (L == kSkipLayer && ks >= 16 ? kSkipPeMat : L); }
NERF_HD inline int s16_matrix_ks(int L, int ks) { return L == kSkipLayer && ks >= 16 ? ks - 16 : ks; }

// Index of a state_dict tensor in the 24-pointer parameter list of nerf_pack_weights.
enum Param {
  P_PTS_W0 = 0,  // pts_linears.i.weight = 2i, .bias = 2i+1
  P_SIGMA_W = 16, P_SIGMA_B, P_DIR_W, P_DIR_B, P_APP_W, P_APP_B, P_RGB_W, P_RGB_B, P_COUNT
};

// Positional-encoding input of PE k-step p for lane half h (reference feature order,
// models.py:36-44: [x, sin(x), cos(x), sin(2x), cos(2x), ...] in blocks of 3).
// Steps 0..29: frequency i = p/3, component c = p%3; half 0 carries sin, half 1 cos.
// Step 30: x0 | x1.  Step 31: x2 | padding (-1).
NERF_HD inline int pe_feature(int p, int h) {
  if (p < 3 * kPosLevels) {
    const int i = p / 3, c = p % 3;
    return 3 + 6 * i + (h ? 3 : 0) + c;
  }
  if (p == 30) return h ? 1 : 0;
  return h ? -1 : 2;
}

// Input column of the activation k-step ks (0..127) for lane half h: register g of
// accumulator tile t of the previous layer holds neuron 32t + (g&3) + 8(g>>2) + 4h.
NERF_HD inline int act_feature(int ks, int h) {
  const int t = ks >> 4, g = ks & 15;
  return 32 * t + (g & 3) + 8 * (g >> 2) + 4 * h;
}

// Source of packed fragment element (matrix m, n-tile nt, k-step ks, lane l):
// returns the column of W (row nt*32 + (l&31)) or -1 for zero padding.
NERF_HD inline int frag_source_col(int m, int ks, int lane) {
  const int h = lane >> 5;
  const int act = frag_act_steps(m);
  if (ks < act) return act_feature(ks, h);
  const int f = pe_feature(ks - act, h);
  if (f < 0) return -1;
  return (m == kSkipPeMat ? kHidden : 0) + f;   // skip layer input is cat[h, enc_x] (models.py:131)
}

// Input feature of element j of k-step ks (lane half h) of f16 matrix m, or -1 for padding.
NERF_HD inline int s16_source_col(int m, int ks, int h, int j) {
  if (!frag_is_pe(m)) {
    const int t = ks >> 1, s = ks & 1;
    return 32 * t + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
  }
  const int f = pe_feature(8 * ks + j, h);
  if (f < 0) return -1;
  return (m == kSkipPeMat ? kHidden : 0) + f;
}

// Power-of-two scale that maps |x| <= m to |x*s| < 2^14 (so f16 rounding stays under 2^15).
NERF_HD inline int s16_exponent(float m) {
  int e = 0;
  float v = m;
  if (!(v > 0.0f)) return 0;
  while (v >= 1.0f && e < 200) { v *= 0.5f; ++e; }
  while (v < 0.5f && e > -200) { v *= 2.0f; --e; }
  return e;   // m = v * 2^e, v in [0.5, 1): m < 2^e
}

}  // namespace nerf

namespace nerf {
// Training: per-sample activation row saved by the forward pass (nerf_mlp_forward_train),
// laid out so every weight-gradient input is one contiguous slice:
//   [h0 | h1 | h2 | h3 | enc_x(64) | h4 | h5 | h6 | h7 | enc_d(32) | r_dir(128) | hd(128)]
// h_l = ReLU(layer l) (256 each), enc_x = PE_10(x) (63 + a zero), enc_d = PE_4(d) (27 + 5 zeros),
// r_dir = ReLU(dir_linear(...)), hd = r_dir + appearance feature (the rgb head's input).
// Layer 4's input [h3, enc_x] and the colour branch's [h7, enc_d] are contiguous
// (models.py:131, :141).
constexpr int kSaveEncX = 4 * kHidden;                       // 1024
NERF_HD constexpr int save_h(int l) { return l < 4 ? l * kHidden : kSaveEncX + 64 + (l - 4) * kHidden; }
constexpr int kSaveEncD = 1088 + 4 * kHidden;                // 2112
// enc_d is constant along a ray: rays of N >= kEncDPerRayMinN samples carry it in their first
// sample's row only (the weight gradients read it per ray there, train.hip param_grads); shorter rays
// in every row (the dir GEMM reads [h7 | enc_d] per sample)
constexpr int kEncDPerRayMinN = 32;
constexpr int kSaveRDir = kSaveEncD + 32;                    // 2144
constexpr int kSaveHd = kSaveRDir + kDirHidden;              // 2272
constexpr int kSaveRow = kSaveHd + kDirHidden;               // 2400 floats per sample
// Training ReLU masks (written by the f16x3 forward, read by the split-f16 backward), one row of
// 272 bytes per sample in their own buffer: for trunk layer l, 32 bytes = lane half h's 16-byte
// slot at 32 l + 16 h (tile T's 16 bits at byte 2T, bit 4q + e = neuron 32T + 8q + 4h + e), then
// r_dir's 8 bytes per lane half at 256 + 8h.  The backward reads one slot per layer instead of the
// layer's 1 KiB of f32 activations.  (Kept out of the save rows: a 2,496-float row stride cost the
// training forward 9 %, same-box A/B.)
constexpr int kMaskLayerBytes = 32;
constexpr int kMaskRDirByte = 8 * kMaskLayerBytes;           // 256
constexpr int kMaskRowBytes = kMaskRDirByte + 16;            // 272
constexpr int kMaskRow = kMaskRowBytes / 4;                  // 68 words per sample

// Per-sample gradient row written by the backward pass (nerf_mlp_backward):
//   [dpre_0 .. dpre_7 (256 each) | dpre_dir (128) | dsigma_pre + pad | dhd (128) | drgb_pre (3) + pad]
// dpre_l = d loss / d (pre-activation of trunk layer l), dhd = d loss / d hd.  Every slice starts
// on an 8-float boundary (a whole group of the tile-major layout below).  dsigma_pre follows
// dpre_dir: both heads read h7, so their weight gradients run as one 129-row GEMM over
// [h7 | enc_d] (param_grads), which reads h7 once.
constexpr int kGradDir = 8 * kHidden;                        // 2048
constexpr int kGradSigma = kGradDir + kDirHidden;            // 2176
constexpr int kGradHd = kGradSigma + 8;                      // 2184
constexpr int kGradRgb = kGradHd + kDirHidden;               // 2312
constexpr int kGradRow = kGradRgb + 8;                       // 2320

// Tile-major rows.  The save rows and the gradient rows are stored per block of 32 samples (one
// wave's), feature groups of 8 outermost: element f of sample m's row (row length R, a multiple
// of 8) is float
//     (m / 32) * 32 R  +  (f / 8) * 256  +  (m % 32) * 8  +  f % 8.
// A kernel's quarter-tile store (4 features of each of a wave's 32 samples, both lane halves) is
// then one contiguous KiB instead of 32 separate 32-byte pieces of 32 rows: the row-major
// pieces cost the training forward and the data gradient ~0.3 ms each per 262K-sample launch
// (same-box A/B, profiles/r03_ab_train_store_variants.log).  Buffers hold tile_rows(M) rows: the
// last block is whole; its rows past M are zero (the writers clear that block first), so the
// weight-gradient GEMMs read whole blocks and the padding adds nothing.  A slice starting at
// feature c (c % 8 == 0) is the same layout at float offset tile_col(c).
NERF_HD constexpr int64_t tile_rows(int64_t M) { return (M + 31) / 32 * 32; }
NERF_HD constexpr int64_t tile_col(int c) { return (int64_t)(c / 8) * 256; }
NERF_HD constexpr int64_t tile_off(int64_t m, int f, int R) {
  return (m / 32) * 32 * (int64_t)R + (int64_t)(f / 8) * 256 + (m % 32) * 8 + f % 8;
}
// Block exponents (the split arithmetic's weight gradients, train.hip wgrad_h16h_kernel and
// wgrad_pair16_kernel).  The f16x3 forward and data-gradient kernels record, for each 32-sample block
// and each weight-gradient operand, the exponent e of the block's largest |value| (max < 2^e; an
// all-zero block e = kBlockExpZero), as the integer-valued float -(kBlockExpBias + e), in row padding:
//   save rows: entry j (j < 8: h_j; j = 8: enc_x) in enc_x's pad slot (feature kSaveEncX + 63) of
//   sample j;
//   gradient rows: entry j (j < 7: dpre_{j+1}; j = 7: [dpre_dir | dsigma_pre]; j = 8: dpre_0) in the
//   first pad float after dsigma_pre (feature kGradSigma + 1) of sample j.
// Every other writer leaves those slots 0 (the f32 forward's zero pad, the other backward kernels),
// which reads as "absent": the GEMM then finds the chunk's maximum itself.
constexpr int kMetaSaveF = kSaveEncX + 63;
constexpr int kMetaGradF = kGradSigma + 1;
constexpr int kBlockExpBias = 1000;
constexpr int kBlockExpZero = -126;
NERF_HD constexpr bool block_exp_valid(float v) { return v <= -500.0f; }

static_assert(kSaveRow % 8 == 0 && kGradRow % 8 == 0 && kSaveEncX % 8 == 0 && kSaveEncD % 8 == 0 &&
                  kSaveRDir % 8 == 0 && kSaveHd % 8 == 0 && kGradSigma % 8 == 0 && kGradHd % 8 == 0 &&
                  kGradRgb % 8 == 0,
              "every slice of the tile-major rows starts on a feature group");

// Float offset, inside matrix m's fragment array, of element j of lane `lane` in the
// fragment block (n-tile nt, k-step quad kq): ks = 4*kq + j.
NERF_HD inline size_t frag_elem(int m, int nt, int kq, int lane, int j) {
  return frag_offset(m) + ((size_t)(nt * (frag_ksteps(m) / 4) + kq) * 64 + lane) * 4 + j;
}
}  // namespace nerf
