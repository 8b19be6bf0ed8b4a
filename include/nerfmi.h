/*
 * nerfmi.h — C ABI of libnerfmi.so, the MI355X (gfx950) NeRF render path.
 *
 * The reference (ByeongKyuPark/Depth-Aware-Shader-Effects-for-NeRF) has no
 * native FFI: its hot path is the Python surface of src/ray_utils.py,
 * src/models.py and src/render.py.  Each entry point below replaces one of
 * those functions; the cited file:line is the reference interface it stands in
 * for.  INTEGRATION.md shows the ctypes binding a maintainer would add on the
 * reference side.
 *
 * Conventions
 *  - Every array argument is a DEVICE pointer, contiguous, fp32 unless noted;
 *    the caller allocates every input, output and workspace.  The library
 *    never allocates or frees device memory.
 *  - Ray-major layouts: rays (B,3); per-sample arrays (B,N) or (B,N,3), sample
 *    s of ray r at index r*N + s.
 *  - Every call is asynchronous and ordered on `stream` (a hipStream_t, NULL =
 *    the default stream).  No call synchronises the device.
 *  - Every call returns NERF_OK (0) or an error code; the message of the last
 *    failure on the calling thread is nerf_last_error().  No C++ exception
 *    crosses the ABI.
 */
#ifndef NERFMI_H
#define NERFMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* nerf_stream_t; /* == hipStream_t */

enum nerf_status {
  NERF_OK = 0,
  NERF_ERR_BAD_ARG = 1,     /* null pointer, negative size, out-of-range count */
  NERF_ERR_HIP = 2,         /* a HIP runtime call or kernel launch failed      */
  NERF_ERR_UNSUPPORTED = 3, /* shape outside what the kernels are built for    */
  NERF_ERR_WORKSPACE = 4    /* workspace smaller than nerf_render_workspace_bytes */
};

/* Message of the last failed call on this thread ("" if none). */
const char* nerf_last_error(void);
/* ABI version (bumped on any signature or layout change; 7: ReLU mask rows in the training forward
 * and backward, include/nerfmi_train.h; 8: nerf_frame_fog; 9: nerf_render_rays' ray0 (in-kernel
 * draws keyed by the global ray index), nerf_train_forward's weights/z outputs,
 * nerf_composite_backward_grad; 10: tile-major save / gradient rows, NERF_TILE_ROWS, and the
 * two-stream nerf_param_grads with its larger workspace; 11: nerf_render_chunk_rays (calls past
 * the launch-size limit run in ray chunks), block exponent records in the save / gradient rows'
 * padding, the split-f16 weight gradient). */
int nerf_abi_version(void);

/* ------------------------------------------------------------------ R1 rays
 * get_rays (src/ray_utils.py:4-50).  Rays of image rows [row0, row0+nrows) of
 * an H x W pinhole camera; c2w is a HOST array of 12 floats, the 3x4 row-major
 * top of the camera-to-world matrix.  rays_o (nullable: the reference returns a
 * 0-stride view there) and rays_d are (nrows*W, 3), row-major pixel order. */
int nerf_get_rays(int H, int W, float focal, const float* c2w_host, int row0, int nrows,
                  float* rays_o, float* rays_d, nerf_stream_t stream);

/* F.normalize(rays_d, dim=-1), eps 1e-12 (src/render.py:19). */
int nerf_normalize_dirs(const float* rays_d, int64_t B, float* out, nerf_stream_t stream);

/* PositionalEncoding.__call__ (src/models.py:14-47): x (M,dims) -> out
 * (M, dims*(2*levels + include_input)) = [x, sin(2^0 x), cos(2^0 x), ...]. */
int nerf_positional_encoding(const float* x, int64_t M, int dims, int levels, int include_input,
                             float* out, nerf_stream_t stream);

/* The in-kernel uniform generator (splitmix64 finaliser of seed + golden*(i+1), top 24 bits):
 * out[i] = u(seed, first + i).  Stratified jitter of sample s of ray r uses u(seed, r*N + s);
 * inside nerf_render_rays, whose rays are global rays ray0 .. ray0+B-1, the jitter of sample s of
 * ray r uses u(seed, (ray0 + r)*N + s) and the inverse-CDF draw j u(seed ^ 0x5DEECE66D,
 * (ray0 + r)*Nf + j): a frame rendered as ray shards (each with its own ray0) draws exactly the
 * uniforms of the same frame rendered in one call.  The per-stage entry points take the key of
 * their first ray, seed + 0x9E3779B97F4A7C15 * first (mod 2^64), the same stream shifted. */
int nerf_rng_uniforms(uint64_t seed, int64_t first, int64_t n, float* out, nerf_stream_t stream);

/* Per-launch timing of the fused MLP (bench.py's roofline): after nerf_profile_mlp_begin(cap),
 * each MLP launch inside nerf_render_rays / nerf_mlp_forward (up to cap) is bracketed by HIP
 * events on its own stream; nerf_profile_mlp_end synchronises them and writes each launch's
 * milliseconds and sample count (min(recorded, capacity) entries; *count = launches recorded)
 * and stops recording.  Process-wide; for one host thread. */
int nerf_profile_mlp_begin(int capacity);
int nerf_profile_mlp_end(float* ms, int64_t* samples, int capacity, int* count);

/* ------------------------------------------------------------ R2 stratified
 * sample_stratified (src/ray_utils.py:52-88).  t_vals = torch.linspace(0,1,N)
 * (N floats, device).  perturb: t_rand (B,N) uniforms when non-null, else an
 * in-kernel counter hash keyed by `seed`.  pts (B,N,3) is nullable. */
int nerf_sample_stratified(const float* rays_o, const float* rays_d, int64_t B, double near,
                           double far, int N, const float* t_vals, int perturb,
                           const float* t_rand, uint64_t seed, float* z_vals, float* pts,
                           nerf_stream_t stream);

/* ------------------------------------------------------- R3 inverse-CDF, H1
 * sample_importance (src/ray_utils.py:90-149) with the H1 clamp of the z
 * gather index to N-1.  weights (B,N) are the squeezed
 * coarse weights; u_lin = torch.linspace(0,1,Nf+1)[:-1] (Nf floats); u_rand
 * (B,Nf) nullable (counter hash keyed by seed).  z_all (B,N+Nf) sorted; pts_all
 * (B,N+Nf,3) nullable.  N <= 256, Nf <= 1024. */
int nerf_sample_importance(const float* rays_o, const float* rays_d, const float* z_vals,
                           const float* weights, int64_t B, int N, int Nf, const float* u_lin,
                           const float* u_rand, uint64_t seed, float* z_all, float* pts_all,
                           nerf_stream_t stream);

/* The same resample fused with the coarse-evaluation reuse of the hierarchical pass:
 * besides z_all it scatters the coarse (rgb_c (B,N,3), sigma_c (B,N)) into their merged
 * slots of rgb_all (B,N+Nf,3) / sigma_all (B,N+Nf), and emits the fine samples z_fine (B,Nf)
 * with their merged slots fine_slot (B,Nf), for nerf_mlp_forward(..., out_slot=fine_slot). */
int nerf_sample_importance_merge(const float* z_vals, const float* weights, const float* rgb_c,
                                 const float* sigma_c, int64_t B, int N, int Nf,
                                 const float* u_lin, const float* u_rand, uint64_t seed,
                                 float* z_all, float* rgb_all, float* sigma_all, float* z_fine,
                                 int32_t* fine_slot, nerf_stream_t stream);

/* -------------------------------------------------------- R5 packed weights
 * NeRF parameters (src/models.py:58-103) in the MFMA fragment layout of the
 * fused MLP.  params: 24 device pointers in state_dict order
 *   pts_linears.{0..7}.{weight,bias}, density_head.{weight,bias},
 *   dir_linear.{weight,bias}, appearance_projection.{weight,bias},
 *   rgb_linear.{weight,bias}
 * with the shapes of NeRF(Config()) (hidden 256, 8 layers, skip [4], PE 10/4,
 * appearance 32).  `packed` holds nerf_packed_weights_floats() floats. */
size_t nerf_packed_weights_floats(void);
int nerf_pack_weights(const float* const* params, float* packed, nerf_stream_t stream);
/* Same layout built on the host from host pointers (tests, offline packing). */
int nerf_pack_weights_host(const float* const* params, float* packed);

/* ---------------------------------------------------- per-ray MLP features
 * The direction and appearance parts of the colour branch, hoisted out of the
 * per-sample MLP (src/models.py:141-156): for each of R rays,
 *   feat[r][0:128]   = dir_linear.bias + dir_linear.weight[:,256:283] . PE_4(dirs[r])
 *   feat[r][128:256] = appearance_projection(app row)   (zeros when app_rows == 0)
 * app_rows: 0 = no appearance, 1 = one (32,) row broadcast, R = one row per ray. */
int nerf_ray_features(const float* packed, const float* dirs, int64_t R, const float* app,
                      int64_t app_rows, float* feat, nerf_stream_t stream);

/* ------------------------------------------------------ MLP arithmetic
 * The MLP's dense layers run on one of two MFMA arithmetics (process-wide,
 * default NERF_ARITH_F16X3); both give fp32-level results:
 *   NERF_ARITH_F32   v_mfma_f32_32x32x2_f32: exact f32 products, 157 TFLOP/s peak.
 *   NERF_ARITH_F16X3 v_mfma_f32_32x32x16_f16 on a hi/lo f16 split of
 *                    power-of-two-scaled operands, three products per k-step
 *                    (hi.hi + hi.lo + lo.hi): split residual and dropped term
 *                    O(2^-24), f32 accumulation; 5.3x the f32 MFMA rate.
 * nerf_set_mlp_arith returns the previous setting (or -1 for an unknown one). */
enum nerf_arith { NERF_ARITH_F32 = 0, NERF_ARITH_F16X3 = 1 };
int nerf_set_mlp_arith(int arith);
int nerf_get_mlp_arith(void);

/* ----------------------------------------------- R4+R6 fused PE -> NeRF MLP
 * NeRF.forward (src/models.py:105-162) for M = R*N samples on MFMA
 * (nerf_set_mlp_arith).
 * With z_vals non-null sample s of ray r sits at pts = origins[r] + dirs[r]*z[r*N+s]
 * (src/ray_utils.py:86); with z_vals null the (R,3) `origins` ARE the points
 * (N must be 1).  ray_feat: (R,256) from nerf_ray_features.  Outputs rgb (M,3),
 * sigma (M) (== (M,1)); with out_slot (R,N) non-null, sample s of ray r is written at
 * row r*out_T + out_slot[r*N+s] instead (the scatter of the hierarchical fine pass). */
int nerf_mlp_forward(const float* packed, const float* origins, const float* dirs,
                     const float* z_vals, int64_t R, int N, const float* ray_feat, float* rgb,
                     float* sigma, const int32_t* out_slot, int out_T, nerf_stream_t stream);

/* ------------------------------------------------------------- R7 composite
 * Alpha compositing of volume_render (src/render.py:56-80): dists padded with
 * 1e-3, alpha = 1-exp(-sigma*dist), T = exclusive cumprod(1-alpha+1e-10),
 * w = alpha*T, rgb_map = sum w*c, depth = sum w*z / (sum w + 1e-10).
 * rgb (B,N,3), sigma (B,N), z (B,N) -> rgb_map (B,3), depth (B), weights (B,N)
 * nullable.  N <= 4096. */
int nerf_composite(const float* rgb, const float* sigma, const float* z_vals, int64_t B, int N,
                   float* rgb_map, float* depth_map, float* weights, nerf_stream_t stream);

/* ------------------------------------------------------------ the whole path
 * volume_render (src/render.py:5-97): normalise dirs, stratified sampling,
 * ray features, fused MLP, composite; with Nf > 0 the H1 hierarchical pass
 * (resample, fused MLP over the Nf new samples with the N coarse evaluations reused —
 * bit-identical to evaluating all N+Nf merged samples — composite over N+Nf).  Nf == 0 is
 * the reference's compat mode (its n_importance is ignored, render.py:83-86).
 * Outputs: rgb_map (B,3), depth_map (B) of the final pass; weights_out
 * (B,N+Nf or N) and z_out (same) nullable; coarse_rgb/coarse_depth nullable
 * (only written when Nf > 0).  ray0: global index of the first ray (keys the in-kernel draws,
 * nerf_rng_uniforms; 0 for a whole batch).  The workspace must hold
 * nerf_render_workspace_bytes(B, N, Nf) bytes. */
size_t nerf_render_workspace_bytes(int64_t B, int N, int Nf);
/* Rays per launch chunk: one launch spans at most 2^30 samples (the grid limit of the sample-
 * parallel kernels), so nerf_render_rays (and nerf_mlp_forward, with Nf = 0) run a call of more
 * than nerf_render_chunk_rays(N, Nf) rays as consecutive chunks of that many rays, bit-identical
 * to one launch (the draws are keyed by the global ray index); nerf_render_workspace_bytes covers
 * one chunk.  0 when N and Nf are both < 1. */
int64_t nerf_render_chunk_rays(int N, int Nf);
int nerf_render_rays(const float* packed, const float* rays_o, const float* rays_d, int64_t B,
                     double near, double far, int N, int Nf, const float* t_vals,
                     const float* u_lin, int perturb, const float* t_rand, const float* u_rand,
                     uint64_t seed, int64_t ray0, const float* app, int64_t app_rows, float* rgb_map,
                     float* depth_map, float* weights_out, float* z_out, float* coarse_rgb,
                     float* coarse_depth, void* workspace, size_t ws_bytes,
                     nerf_stream_t stream);

/* ------------------------------------------------- depth-aware post effects
 * The depth-reading effects of the reference's PostProcessor (src/post_processor.py) on the
 * frame run.py renders.  image / out: uint8 (H,W,3) RGB; depth: fp32 (H,W)
 * or the first channel of (H,W,C) with depth_stride = C, nullable (each effect's no-depth
 * branch).  workspace: nerf_effect_workspace_bytes(H, W) device bytes.
 *   nerf_depth_normalize   run.py:248: (d - min) / (max - min + 1e-6) over n values.
 *   nerf_effect_fog        Fog (post_processor.py:451-493): white fog, fog_start < 1.
 *   nerf_frame_fog         the CLI's `--shader Fog` frame from the render outputs in one pass after
 *                          the depth reduction: rgb fp32 (H,W,3) -> uint8 by truncation (run.py:233),
 *                          depth fp32 (H,W) normalised (run.py:248), then Fog; equal, bit for bit,
 *                          to nerf_depth_normalize + nerf_effect_fog on the truncated image.
 *                          workspace >= 256 bytes.
 *   nerf_effect_toon       Toon Shader (post_processor.py:64-117): colours quantised to `levels`
 *                          (> 0; any real value, used as float32 like the reference's numpy scalar),
 *                          depth edges (bilateral 9/75/75, Sobel, threshold 0.05, 3x3 dilation) or,
 *                          without depth, colour edges (gray Laplacian, threshold 0.1) darkened by
 *                          edge_strength.  The cv2 steps are OpenCV 4's algorithms restated. */
size_t nerf_effect_workspace_bytes(int H, int W);
int nerf_depth_normalize(const float* depth, int64_t n, float* out, void* workspace, size_t ws_bytes,
                         nerf_stream_t stream);
int nerf_effect_fog(const uint8_t* image, const float* depth, int64_t depth_stride, int H, int W,
                    double fog_start, uint8_t* out, void* workspace, size_t ws_bytes,
                    nerf_stream_t stream);
int nerf_frame_fog(const float* rgb, const float* depth, int H, int W, double fog_start, uint8_t* out,
                   void* workspace, size_t ws_bytes, nerf_stream_t stream);
int nerf_effect_toon(const uint8_t* image, const float* depth, int64_t depth_stride, int H, int W,
                     double levels, double edge_strength, uint8_t* out, void* workspace,
                     size_t ws_bytes, nerf_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* NERFMI_H */
