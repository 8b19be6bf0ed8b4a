"""Training loop of the reference (src/train.py:13-207) on the nerfmi HIP kernels.

One iteration (train.py:77-92) is: volume_render(perturb=True) over a batch of rays of one image
→ F.mse_loss against the pixels → loss.backward() → Adam.step().  Here that is four C-ABI
calls (include/nerfmi_train.h) and one RCCL all-reduce:

  nerf_train_forward    normalise, stratified samples, fused PE→MLP forward on MFMA saving every
                        activation, composite (csrc/train.hip, csrc/mlp.hip)
  nerf_train_backward   loss, composite backward (reverse scan), MLP data-gradient chain on MFMA
                        with transposed weight fragments, every weight gradient as an MFMA
                        reduction over the batch, appearance-row gradient
  all_reduce            data parallel: the flat gradient buffer averaged over ranks (one RCCL
                        collective of 2.4 MB + the appearance table)
  nerf_adam             torch.optim.Adam's update on the flat parameter buffer (one launch)

Parameters, gradients and Adam moments live in flat device buffers; the NeRF module's parameters
are views into the parameter buffer, so the model, its state_dict and checkpoints always see the
trained values.  The reference's quirks are kept: the first 5 iterations
use min(64, batch_size) rays (train.py:26,56-57), StepLR steps only when i % step_size == 0
(train.py:95-96), n_importance is ignored by the coarse-only volume_render (render.py:83-86),
and one image's rays form each batch (dataset.py:249-277).
"""
import ctypes
import math
import os
import time

import numpy as np
import torch

from . import _lib
from .models import NeRF, STATE_KEYS, state_tensors
from .ray_utils import linspace_table

_APP_DIM = 32


class Trainer:
    """Flat-buffer NeRF (+ appearance table) trainer: one object per rank.

    ``group``: a torch.distributed process group for data parallelism (gradients averaged over
    it before the optimizer step, as DDP would); None trains on this process alone."""

    def __init__(self, config, model=None, appearance_embeddings=None, n_images=None, group=None,
                 lr=None, betas=(0.9, 0.999), eps=1e-8, near=None, far=None):
        self.config = config
        # the sampling interval: the dataset's near/far (train.py:79 passes dataset.near/far), the
        # config's when no dataset is given
        self.near = float(config.near if near is None else near)
        self.far = float(config.far if far is None else far)
        self.dev = _lib.device()
        self.lib = _lib.load()
        self.group = group
        model = model if model is not None else NeRF(config)
        self.model = model.to(self.dev)
        named = dict(self.model.named_parameters())
        # 24 parameter slots in STATE_KEYS order; a use_appearance=False model has no
        # appearance_projection (models.py:99-103): its slots stay zero and are not parameters
        self.present = [k in named for k in STATE_KEYS]
        tensors = state_tensors(named, self.dev)
        self.shapes = [tuple(t.shape) for t in tensors]
        self.sizes = [t.numel() for t in tensors]
        if config.use_appearance:
            if appearance_embeddings is None:
                appearance_embeddings = torch.randn(n_images or 100, config.appearance_dim)
            self.n_images = appearance_embeddings.shape[0]
            self.sizes.append(appearance_embeddings.numel())
            self.shapes.append(tuple(appearance_embeddings.shape))
        else:
            self.n_images = 0
        self.offsets = np.concatenate([[0], np.cumsum(self.sizes)]).tolist()
        total = self.offsets[-1]
        self.flat = torch.empty(total, device=self.dev)
        self.grad = torch.zeros(total, device=self.dev)
        self.exp_avg = torch.zeros(total, device=self.dev)
        self.exp_avg_sq = torch.zeros(total, device=self.dev)
        with torch.no_grad():
            for i, t in enumerate(tensors):
                self.view(self.flat, i).copy_(t.detach())
            if self.n_images:
                self.view(self.flat, len(tensors)).copy_(appearance_embeddings.detach())
            # the module's parameters become views of the flat buffer
            for i, k in enumerate(STATE_KEYS):
                if not self.present[i]:
                    continue
                mod_name, pname = k.rsplit(".", 1)
                mod = self.model.get_submodule(mod_name)
                setattr(mod, pname, torch.nn.Parameter(self.view(self.flat, i), requires_grad=False))
        self.appearance_embeddings = self.view(self.flat, len(tensors)) if self.n_images else None
        if isinstance(appearance_embeddings, torch.nn.Parameter):
            # the caller's table (dataset.appearance_embeddings, an nn.Parameter as dataset.py:81-83)
            # becomes a view of the flat buffer, so every optimizer step updates it in place as
            # the reference's Adam does (train.py:36-39)
            appearance_embeddings.data = self.appearance_embeddings
        # Adam's parameter numbering (model.parameters() order, then the appearance table)
        self.param_slots = [i for i in range(24) if self.present[i]] + ([24] if self.n_images else [])
        self.rank = 0
        if group is not None:
            import torch.distributed as dist
            self.rank = dist.get_rank(group)
        # every rank starts from rank 0's weights and table, as DDP's constructor does
        broadcast_state([self.flat], group)
        self.param_ptrs = (ctypes.c_void_p * 24)(*[self.view(self.flat, i).data_ptr() for i in range(24)])
        self.grad_ptrs = (ctypes.c_void_p * 24)(*[self.view(self.grad, i).data_ptr() for i in range(24)])
        self.app_grad = self.view(self.grad, 24) if self.n_images else None
        self.packed = torch.empty(self.lib.nerf_packed_weights_floats(), device=self.dev)
        self.packedT = torch.empty(self.lib.nerf_packed_transposed_floats(), device=self.dev)
        self.dapp = torch.empty(1, _APP_DIM, device=self.dev)
        self.loss_buf = torch.empty(1, device=self.dev)
        self.lr = config.learning_rate if lr is None else lr
        self.initial_lr = self.lr
        self.betas, self.eps = betas, eps
        self.steps = 0
        self._ws = None
        self._tvals = {}
        self._side = None          # side stream for the transposed packing (forward_backward)

    def view(self, buf, i):
        return buf[self.offsets[i]: self.offsets[i + 1]].view(self.shapes[i])

    def _workspace(self, B, N):
        need = self.lib.nerf_train_workspace_bytes(B, N)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.dev)
        return self._ws

    # ------------------------------------------------------------------------------ one step
    def forward_backward(self, rays_o, rays_d, target, app_idx=None, *, t_rand=None, seed=None, _marks=None):
        """Loss (device scalar) and gradients in self.grad for one batch (train.py:77-90).
        rays (B,3) and target (B,3) on the device; app_idx: the batch's image (appearance row).
        t_rand (B,N) = the torch.rand draw of ray_utils.py:80; else the in-kernel RNG on `seed`."""
        lib, s, P = self.lib, _lib.stream(), _lib.ptr
        N = self.config.num_samples
        o = rays_o.reshape(-1, 3).to(self.dev, torch.float32).contiguous()
        d = rays_d.reshape(-1, 3).to(self.dev, torch.float32).contiguous()
        tgt = target.reshape(-1, 3).to(self.dev, torch.float32).contiguous()
        B = o.shape[0]
        if t_rand is not None:
            t_rand = t_rand.to(self.dev, torch.float32).contiguous()
            assert t_rand.shape == (B, N)
        if seed is None:
            seed = step_seed(self.steps + 1, self.rank)
        _lib.check(lib.nerf_pack_weights(self.param_ptrs, P(self.packed), s), "nerf_pack_weights")
        # The transposed weights are read only by the backward: they are packed on a side stream while
        # the forward runs (forked after everything queued so far, so after the previous step's
        # backward read them; joined before this step's backward).
        main = torch.cuda.current_stream(self.dev)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.dev)
            self._fork, self._join = torch.cuda.Event(), torch.cuda.Event()
        self._fork.record(main)
        self._side.wait_event(self._fork)
        _lib.check(lib.nerf_pack_weights_transposed(self.param_ptrs, P(self.packedT), self._side.cuda_stream),
                   "nerf_pack_weights_transposed")
        if self.app_grad is not None:    # the table's gradient is one row this step: zeroed beside the forward
            with torch.cuda.stream(self._side):
                self.app_grad.zero_()
        self._join.record(self._side)
        if N not in self._tvals:
            self._tvals[N] = linspace_table(N, self.dev)
        ws = self._workspace(B, N)
        rgb_map = torch.empty(B, 3, device=self.dev)
        depth = torch.empty(B, device=self.dev)
        if self.n_images and app_idx is not None:
            app, rows = self.appearance_embeddings[int(app_idx)].reshape(1, _APP_DIM), 1
        else:
            app, rows = None, 0
        _lib.check(lib.nerf_train_forward(P(self.packed), P(o), P(d), B, self.near, self.far, N,
                                          P(self._tvals[N]), 1, P(t_rand), int(seed), P(app), rows, P(rgb_map),
                                          P(depth), None, None, P(ws), ws.numel(), s),
                   "nerf_train_forward")
        if _marks is not None:
            _marks[1].record(torch.cuda.current_stream())
        # d app of the batch's image goes straight into its row of the table's gradient
        dapp = self.app_grad[int(app_idx)] if rows else None
        main.wait_event(self._join)
        _lib.check(lib.nerf_train_backward(P(self.packed), P(self.packedT), P(rgb_map), P(tgt), B, N, P(app), rows,
                                           self.grad_ptrs, P(dapp), P(self.loss_buf), P(ws), ws.numel(), s),
                   "nerf_train_backward")
        if rows == 0:   # appearance_projection unused: its gradient is zero, as torch leaves it (None → no update)
            self.view(self.grad, 20).zero_()
            self.view(self.grad, 21).zero_()
        return self.loss_buf[0], rgb_map

    def profile_step(self, rays_o, rays_d, target, app_idx=None, seed=12345):
        """Event-timed phases of one training step through the stage entry points (no parameter
        update): {phase: ms} for the forward MLP, the MLP data-gradient chain, the weight
        gradients and the whole forward+backward."""
        lib, s, P = self.lib, _lib.stream(), _lib.ptr
        cur = torch.cuda.current_stream()
        N = self.config.num_samples
        o = rays_o.reshape(-1, 3).to(self.dev, torch.float32).contiguous()
        d = rays_d.reshape(-1, 3).to(self.dev, torch.float32).contiguous()
        tgt = target.reshape(-1, 3).to(self.dev, torch.float32).contiguous()
        B = o.shape[0]
        M = B * N
        dev = self.dev
        dn, z = torch.empty(B, 3, device=dev), torch.empty(B, N, device=dev)
        feat, encd = torch.empty(B, 256, device=dev), torch.empty(B, 32, device=dev)
        rgb, sigma = torch.empty(M, 3, device=dev), torch.empty(M, device=dev)
        MT = _lib.tile_rows(M)                                       # tile-major save/grad rows
        save, grad = torch.empty(MT, _lib.SAVE_ROW, device=dev), torch.empty(MT, _lib.GRAD_ROW, device=dev)
        masks = torch.empty(M, _lib.MASK_ROW, dtype=torch.int32, device=dev)
        rgb_map, depth = torch.empty(B, 3, device=dev), torch.empty(B, device=dev)
        dsig, drgb, sq = torch.empty(M, device=dev), torch.empty(M, 3, device=dev), torch.empty(B, device=dev)
        grads = [torch.empty_like(self.view(self.grad, i)) for i in range(24)]
        gptr = (ctypes.c_void_p * 24)(*[g.data_ptr() for g in grads])
        wsz = self.lib.nerf_param_grads_workspace_bytes(M)
        ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
        app, rows = (self.appearance_embeddings[int(app_idx)].reshape(1, _APP_DIM), 1) \
            if (self.n_images and app_idx is not None) else (None, 0)
        if N not in self._tvals:
            self._tvals[N] = linspace_table(N, dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
        ck = _lib.check
        ev[0].record(cur)
        ck(lib.nerf_pack_weights(self.param_ptrs, P(self.packed), s), "pack")
        ck(lib.nerf_pack_weights_transposed(self.param_ptrs, P(self.packedT), s), "packT")
        ev[1].record(cur)
        ck(lib.nerf_normalize_dirs(P(d), B, P(dn), s), "normalize")
        ck(lib.nerf_sample_stratified(P(o), P(dn), B, self.near, self.far, N,
                                      P(self._tvals[N]), 1, None, seed, P(z), None, s), "stratified")
        ck(lib.nerf_ray_features_train(P(self.packed), P(dn), B, P(app), rows, P(feat), P(encd), s), "features")
        ev[2].record(cur)
        ck(lib.nerf_mlp_forward_train(P(self.packed), P(o), P(dn), P(z), B, N, P(feat), P(encd), P(rgb), P(sigma),
                                      P(save), P(masks), s), "mlp_forward_train")
        ev[3].record(cur)
        ck(lib.nerf_composite(P(rgb), P(sigma), P(z), B, N, P(rgb_map), P(depth), None, s), "composite")
        ck(lib.nerf_composite_backward(P(rgb), P(sigma), P(z), P(rgb_map), P(tgt), B, N, 2.0 / (3 * B), P(dsig),
                                       P(drgb), P(sq), s), "composite_backward")
        ev[4].record(cur)
        mk = masks if _lib.get_mlp_arith() == "f16x3" else None    # the f16x3 forward wrote them
        ck(lib.nerf_mlp_backward(P(self.packed), P(self.packedT), P(save), P(mk), P(sigma), P(rgb), P(dsig), P(drgb),
                                 M, P(grad), s), "mlp_backward")
        ev[5].record(cur)
        ck(lib.nerf_param_grads(P(save), P(grad), M, N, P(app), rows, P(self.packed), gptr, P(self.dapp), P(ws),
                                wsz, s), "param_grads")
        ev[6].record(cur)
        torch.cuda.synchronize()
        return {"pack_ms": ev[0].elapsed_time(ev[1]), "rays_ms": ev[1].elapsed_time(ev[2]),
                "mlp_forward_ms": ev[2].elapsed_time(ev[3]), "composite_fwd_bwd_ms": ev[3].elapsed_time(ev[4]),
                "mlp_backward_ms": ev[4].elapsed_time(ev[5]), "param_grads_ms": ev[5].elapsed_time(ev[6]),
                "total_ms": ev[0].elapsed_time(ev[6])}

    def all_reduce(self):
        """Average the gradients over the data-parallel group (one RCCL all-reduce)."""
        average_gradients(self.grad, self.group)

    def optimizer_step(self):
        """torch.optim.Adam.step() on every parameter (train.py:91), one launch."""
        self.steps += 1
        _lib.check(self.lib.nerf_adam(_lib.ptr(self.flat), _lib.ptr(self.grad), _lib.ptr(self.exp_avg),
                                      _lib.ptr(self.exp_avg_sq), self.flat.numel(), float(self.lr),
                                      float(self.betas[0]), float(self.betas[1]), float(self.eps), self.steps,
                                      _lib.stream()), "nerf_adam")
        self.model._packed = None          # the module's cached inference packing is stale now

    def step(self, rays_o, rays_d, target, app_idx=None, *, t_rand=None, seed=None):
        loss, rgb = self.forward_backward(rays_o, rays_d, target, app_idx, t_rand=t_rand, seed=seed)
        self.all_reduce()
        self.optimizer_step()
        return loss

    # ---------------------------------------------------------------------- checkpoints
    def optimizer_state_dict(self):
        """torch.optim.Adam.state_dict() layout (train.py:116,178): per-parameter step/exp_avg/exp_avg_sq,
        parameters numbered model.parameters() order then the appearance table."""
        n = len(self.param_slots)
        state = {}
        if self.steps:
            for i, slot in enumerate(self.param_slots):
                state[i] = {"step": torch.tensor(float(self.steps)),
                            "exp_avg": self.view(self.exp_avg, slot).detach().cpu().clone(),
                            "exp_avg_sq": self.view(self.exp_avg_sq, slot).detach().cpu().clone()}
        group = {"lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": 0, "amsgrad": False,
                 "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
                 "decoupled_weight_decay": False, "initial_lr": self.initial_lr, "params": list(range(n))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, sd):
        st = sd["state"]
        if len(sd["param_groups"][0]["params"]) != len(self.param_slots):
            raise ValueError(f"optimizer state has {len(sd['param_groups'][0]['params'])} parameters, "
                             f"this trainer {len(self.param_slots)}")
        for i, e in st.items():
            slot = self.param_slots[int(i)]
            self.view(self.exp_avg, slot).copy_(e["exp_avg"])
            self.view(self.exp_avg_sq, slot).copy_(e["exp_avg_sq"])
            self.steps = int(float(e["step"]))
        self.lr = sd["param_groups"][0]["lr"]
        broadcast_state([self.exp_avg, self.exp_avg_sq], self.group)

    def checkpoint(self, loss, psnr, iteration):
        """The dict train.py:114-125 saves."""
        ck = {"model_state_dict": {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()},
              "optimizer_state_dict": self.optimizer_state_dict(), "loss": loss, "psnr": psnr,
              "iteration": iteration}
        if self.n_images:
            ck["appearance_embeddings"] = self.appearance_embeddings.detach().cpu().clone()
        return ck


def step_seed(key, rank):
    """Key of a step's in-kernel jitter stream: distinct per step and per data-parallel rank (the
    reference draws torch.rand per call, ray_utils.py:80; ranks must not share draws)."""
    return (int(key) & ((1 << 40) - 1)) | (int(rank) << 40)


def broadcast_state(tensors, group):
    """Rank 0's copy of each tensor on every rank of `group` (a no-op alone)."""
    if group is None:
        return
    import torch.distributed as dist
    src = dist.get_global_rank(group, 0)
    for t in tensors:
        dist.broadcast(t, src=src, group=group)


def average_gradients(flat_grad, group):
    """Data-parallel gradient sync: one all-reduce of the whole flat gradient buffer (2.4 MB of
    NeRF weights + the appearance table), then / world — the mean-loss gradient of the union of
    the ranks' batches.  One large collective suits xGMI's per-link ring bandwidth better than
    per-tensor buckets."""
    if group is None:
        return
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dist.all_reduce(flat_grad, group=group)     # (world 1 included: the collective runs whenever a group exists)
    if world > 1:
        flat_grad.div_(world)


def train_nerf(config, dataset, save_dir="checkpoints", group=None, num_iterations=None, log_every=10,
               checkpoint_every=1000, seed=None, plots=True, return_metrics=False):
    """src/train.py:13-207 on nerfmi: returns the trained model, as the reference does
    (train.py:207; run.py:347 assigns it).  ``return_metrics=True`` returns (model, losses, psnrs)
    instead; the per-iteration losses and PSNRs are also left on ``train_nerf.losses`` /
    ``train_nerf.psnrs``.  The dataset's appearance table (an nn.Parameter, dataset.py:81-83) is
    trained in place (train.py:36-39).  Every ``checkpoint_every`` iterations rank 0 writes
    checkpoint_{i:06d}.pt and the validation render render_{i:06d}.png of train.py:127-173.
    Under data parallelism every rank draws its own batch (its own image, its own jitter
    stream) and the gradients are averaged; rank 0 writes."""
    import torch.distributed as dist
    rank = dist.get_rank(group) if group is not None else 0
    if rank == 0:
        os.makedirs(save_dir, exist_ok=True)
    initial_batch_size = min(64, config.batch_size)                    # train.py:26
    trainer = Trainer(config, appearance_embeddings=getattr(dataset, "appearance_embeddings", None),
                      n_images=len(dataset), group=group, near=getattr(dataset, "near", None),
                      far=getattr(dataset, "far", None))
    iters = config.num_iterations if num_iterations is None else num_iterations
    losses, psnrs = [], []
    train_nerf.losses, train_nerf.psnrs = losses, psnrs
    start = time.time()
    loss_v = psnr_v = float("nan")
    for i in range(1, iters + 1):
        batch = dataset.get_rays(batch_size=initial_batch_size) if i <= 5 else dataset.get_rays()
        app_idx = batch["appearance_idx"] if config.use_appearance else None
        loss = trainer.step(batch["rays_o"], batch["rays_d"], batch["rgb"], app_idx,
                            seed=None if seed is None else step_seed(seed * 1_000_003 + i, trainer.rank))
        if i % config.scheduler_step_size == 0:                          # StepLR, train.py:95-96
            trainer.lr *= config.scheduler_gamma
        loss_v = float(loss)
        psnr_v = -10.0 * math.log10(loss_v) if loss_v > 0 else float("inf")
        losses.append(loss_v)
        psnrs.append(psnr_v)
        if rank == 0 and log_every and i % log_every == 0:
            print(f"iter {i}: Loss: {loss_v:.5f}, PSNR: {psnr_v:.2f}")
        if rank == 0 and checkpoint_every and i % checkpoint_every == 0:
            torch.save(trainer.checkpoint(loss_v, psnr_v, i), os.path.join(save_dir, f"checkpoint_{i:06d}.pt"))
            if plots:
                validation_render(trainer.model, dataset, config, i, save_dir)
    if rank == 0:
        torch.save(trainer.checkpoint(loss_v, psnr_v, iters), os.path.join(save_dir, "checkpoint_final.pt"))
        if plots:
            _plot_curves(losses, psnrs, os.path.join(save_dir, "training_curves.png"))
        print(f"Training completed in {time.time() - start:.2f}s")
    if return_metrics:
        return trainer.model, losses, psnrs
    return trainer.model


@torch.no_grad()
def validation_render(model, dataset, config, iteration, save_dir):
    """The sample render of train.py:127-173: the first 1000 rays of the last image, coarse
    volume_render with perturb=False, RGB and viridis depth side by side in
    render_{iteration:06d}.png.  Returns (rgb (1000,3), depth (1000,1))."""
    from .render import volume_render
    val = dataset.get_rays(idx=len(dataset) - 1)
    o, d = val["rays_o"][:1000], val["rays_d"][:1000]
    app = None
    if config.use_appearance:
        app = dataset.appearance_embeddings[val["appearance_idx"]]
    rgb, depth, _ = volume_render(model, o, d, near=dataset.near, far=dataset.far, n_samples=config.num_samples,
                                  n_importance=config.num_importance, appearance_embedding=app, perturb=False)
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    rgb_viz = rgb.reshape(-1, 3).cpu().numpy()
    n = int(np.sqrt(rgb_viz.shape[0]))
    plt.figure(figsize=(10, 5))
    plt.subplot(1, 2, 1)
    plt.imshow(np.clip(rgb_viz[:n * n].reshape(n, n, 3), 0, 1))
    plt.title(f"RGB - Iteration {iteration}")
    plt.axis("off")
    plt.subplot(1, 2, 2)
    plt.imshow(depth.reshape(-1).cpu().numpy()[:n * n].reshape(n, n), cmap="viridis")
    plt.title(f"Depth - Iteration {iteration}")
    plt.colorbar()
    plt.axis("off")
    plt.savefig(os.path.join(save_dir, f"render_{iteration:06d}.png"))
    plt.close()
    return rgb, depth


def _plot_curves(losses, psnrs, path):
    """training_curves.png of train.py:189-204."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.figure(figsize=(10, 5))
    plt.subplot(1, 2, 1)
    plt.plot(losses)
    plt.title("Training Loss")
    plt.xlabel("Iteration")
    plt.ylabel("Loss")
    plt.subplot(1, 2, 2)
    plt.plot(psnrs)
    plt.title("Training PSNR")
    plt.xlabel("Iteration")
    plt.ylabel("PSNR (dB)")
    plt.savefig(path)
    plt.close()
