/*
 * nerfmi_train.h — training entry points of libnerfmi.so (gfx950).
 *
 * They replace the autograd backward and optimizer step of the reference's training loop,
 * src/train.py:13-207: volume_render(perturb=True) → F.mse_loss(rgb, target) (:87) →
 * loss.backward() (:90) → torch.optim.Adam.step() (:91).  Conventions are those of
 * nerfmi.h (device pointers, caller-owned memory, stream-ordered, status codes).
 *
 * Two levels:
 *  - whole step: nerf_train_forward + nerf_train_backward share one workspace
 *    (nerf_train_workspace_bytes) that carries the saved activations between them;
 *  - stages (for tests and other hosts): forward with saves, composite backward, MLP
 *    backward, parameter gradients, generic weight-gradient GEMM, Adam.
 *
 * `params` / `param_grads` arrays are the 24 state_dict tensors in nerf_pack_weights order:
 * pts_linears.{0..7}.{weight,bias}, density_head, dir_linear, appearance_projection,
 * rgb_linear (.weight, .bias each).
 */
#ifndef NERFMI_TRAIN_H
#define NERFMI_TRAIN_H

#include "nerfmi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Per-sample rows the forward saves / the backward writes (floats). */
#define NERF_SAVE_ROW 2400 /* [h0..h3 | enc_x(64) | h4..h7 | enc_d(32) | r_dir(128) | hd(128)] */
#define NERF_GRAD_ROW 2320 /* [dpre_0..7 (256 each) | dpre_dir(128) | dsigma+pad(8) | dhd(128) | drgb(3)+pad(8)] */
/* Both are stored tile-major: per block of 32 samples, feature groups of 8 outermost.  Element f
 * of sample m's row (row length R) is float (m/32)*32*R + (f/8)*256 + (m%32)*8 + f%8, and a buffer
 * of M samples holds NERF_TILE_ROWS(M) rows (the last block whole; its rows past M are zero). */
#define NERF_TILE_ROWS(M) ((((M) + 31) / 32) * 32)
/* Block exponents (ABI 11, f16x3 only): sample j of each 32-sample block carries, in enc_x's pad
 * slot (save feature 1087) the exponent record of h_j (j < 8) or enc_x (j = 8), and in the float after
 * dsigma (gradient feature 2177) that of dpre_{j+1} (j < 7), [dpre_dir | dsigma] (j = 7) or dpre_0
 * (j = 8): -(1000 + e)
 * with e = frexp's exponent of the block's largest |value| (-126 for an all-zero block); 0 = absent.
 * nerf_param_grads' split-f16 weight gradient scales each chunk from them (csrc/layout.h). */
/* ReLU masks the f16x3 training forward writes for the backward (uint32 words per sample):
 * trunk layers 0..7 (256 bits each) and r_dir (128 bits), 272 bytes (csrc/layout.h kMaskRow). */
#define NERF_MASK_ROW 68

/* ---------------------------------------------------------------- whole step
 * Forward of train.py:77-84 (coarse volume_render, n_importance ignored as in
 * render.py:83-86) keeping every activation the backward needs in `workspace`.
 * Arguments as nerf_render_rays with Nf = 0 and ray0 = 0; weights_out (B,N) and z_out (B,N)
 * are nullable (volume_render's extras).  B*N < 2^31. */
size_t nerf_train_workspace_bytes(int64_t B, int N);
int nerf_train_forward(const float* packed, const float* rays_o, const float* rays_d, int64_t B,
                       double near, double far, int N, const float* t_vals, int perturb,
                       const float* t_rand, uint64_t seed, const float* app, int64_t app_rows,
                       float* rgb_map, float* depth_map, float* weights_out, float* z_out,
                       void* workspace, size_t ws_bytes, nerf_stream_t stream);
/* loss = mse(rgb_map, target) (train.py:87) into *loss (device float) and its gradient
 * with respect to every parameter (written, not accumulated) and, when dapp is non-null,
 * to the appearance rows (app_rows x 32).  packedT from nerf_pack_weights_transposed.  The
 * workspace must hold a nerf_train_forward's saves; the mask source follows the arithmetic that
 * forward ran under (NERF_ERR_BAD_ARG if no forward wrote it). */
int nerf_train_backward(const float* packed, const float* packedT, const float* rgb_map,
                        const float* target, int64_t B, int N, const float* app, int64_t app_rows,
                        float* const* param_grads, float* dapp, float* loss, void* workspace,
                        size_t ws_bytes, nerf_stream_t stream);

/* -------------------------------------------------------------------- stages */
/* W^T of trunk layers 1..7 and of dir_linear's h-part in MFMA fragment layout. */
size_t nerf_packed_transposed_floats(void);
int nerf_pack_weights_transposed(const float* const* params, float* packedT, nerf_stream_t stream);
int nerf_pack_weights_transposed_host(const float* const* params, float* packedT);

/* nerf_ray_features plus enc_d (R,32): PE_4(d) (models.py:122), zero-padded. */
int nerf_ray_features_train(const float* packed, const float* dirs, int64_t R, const float* app,
                            int64_t app_rows, float* feat, float* enc_d, nerf_stream_t stream);
/* nerf_mlp_forward (no scatter) that also writes save (NERF_TILE_ROWS(R*N), NERF_SAVE_ROW,
 * tile-major, padding rows zeroed; enc_d, constant along a ray, only in each ray's first row when
 * N >= 32) and, under the f16x3
 * arithmetic, masks (R*N, NERF_MASK_ROW) (required there; ignored under f32, may be null). */
int nerf_mlp_forward_train(const float* packed, const float* origins, const float* dirs,
                           const float* z_vals, int64_t R, int N, const float* ray_feat,
                           const float* enc_d, float* rgb, float* sigma, float* save,
                           uint32_t* masks, nerf_stream_t stream);
/* d/d(sigma, rgb) of the composite (render.py:66-78) given g = scale*(rgb_map - target);
 * sq_err (B) = per-ray sum of squared errors. */
int nerf_composite_backward(const float* rgb, const float* sigma, const float* z_vals,
                            const float* rgb_map, const float* target, int64_t B, int N,
                            float scale, float* dsigma, float* drgb, float* sq_err,
                            nerf_stream_t stream);
/* The same for an arbitrary upstream gradient (autograd of volume_render, src/render.py:56-80):
 * grad_rgb_map (B,3) = d loss / d rgb_map, grad_depth_map (B) = d loss / d depth_map, each
 * nullable (= 0); dsigma (B,N), drgb (B,N,3) out. */
int nerf_composite_backward_grad(const float* rgb, const float* sigma, const float* z_vals,
                                 const float* grad_rgb_map, const float* grad_depth_map, int64_t B,
                                 int N, float* dsigma, float* drgb, nerf_stream_t stream);
/* Data gradients of NeRF.forward (models.py:105-162) on MFMA: grad (NERF_TILE_ROWS(M),
 * NERF_GRAD_ROW, tile-major; save as the forward wrote it).  Under
 * f16x3 the ReLU masks come from `masks` when non-null (an f16x3 forward's), else from the saved
 * activations; the f32 backward always reads the activations. */
int nerf_mlp_backward(const float* packed, const float* packedT, const float* save,
                      const uint32_t* masks, const float* sigma, const float* rgb,
                      const float* dsigma, const float* drgb, int64_t M, float* grad,
                      nerf_stream_t stream);
/* Every parameter gradient (+ appearance rows) from the tile-major save and grad rows. */
size_t nerf_param_grads_workspace_bytes(int64_t M);
int nerf_param_grads(const float* save, const float* grad, int64_t M, int N, const float* app,
                     int64_t app_rows, const float* packed, float* const* param_grads, float* dapp,
                     void* workspace, size_t ws_bytes, nerf_stream_t stream);
/* Plain row-major operands: out_w[n][k] = sum_m a[m*lda+n] x[(m/x_div)*ldx+k] (x_div 0: row 0), out_b[n] = sum_m a[m*lda+n]
 * (nullable); accumulate adds to the outputs instead of overwriting. */
size_t nerf_wgrad_workspace_bytes(int64_t M, int N, int K);
int nerf_wgrad(const float* a, int64_t lda, int N, const float* x, int64_t ldx, int K, int64_t x_div,
               int64_t M, float* out_w, float* out_b, int accumulate, void* workspace,
               size_t ws_bytes, nerf_stream_t stream);
/* torch.optim.Adam step (amsgrad off, no weight decay), `step` counted from 1. */
int nerf_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
              double lr, double beta1, double beta2, double eps, int64_t step, nerf_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* NERFMI_TRAIN_H */
