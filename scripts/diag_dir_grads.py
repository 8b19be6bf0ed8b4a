"""Diagnostic (GPU): where the head gradients' error comes from.  The training step of
tests/test_gpu_train.py::test_trainer_matches_oracle_over_steps (step 0: chair circle frame 0, 512
rays x 64 samples, seed 21), staged through the C ABI: the composite backward's per-sample d rgb and
d sigma, the data-gradient rows d pre_dir (= d hd x mask) and d pre_7, and the bias sums over
samples, each against float64 autograd on the GPU's own ReLU branches, beside the fp32 CPU autograd
against float64 on its branches.  Prints rel-L2 and the mean signed error (a bias shows there)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from oracle import nerf_oracle as O  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def bias(a, b):
    """mean signed error relative to the rms of the reference"""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float((a - b).mean() / max(np.sqrt((b ** 2).mean()), 1e-300))


def oracle_parts(st, table, img, o, d, target, t_rand, dtype, masks=None, record=None):
    """fp32/float64 autograd of one step, keeping d rgb, d sigma (per sample), d pre_dir, d pre_7 and
    the parameter gradients."""
    sd = {k: v.detach().to(dtype).clone().requires_grad_(True) for k, v in st.items()}
    keep = {}

    def relu(pre, i):
        if record is not None:
            record.append(pre.detach() > 0)
        if i in (7, 9):
            pre.retain_grad()
            keep[i] = pre
        return torch.relu(pre) if masks is None else pre * masks[i].to(dtype)
    oo, dd = o.to(dtype), O.normalize(d.to(dtype))
    z, pts = O.sample_stratified(oo, dd, 2.0, 6.0, 64, t_rand.to(dtype))
    app = table[img].to(dtype)
    with torch.enable_grad():
        b, n = z.shape
        d_exp = dd.unsqueeze(1).expand(-1, n, -1).reshape(-1, 3)
        rgb, sigma = O.nerf_forward(sd, pts.reshape(-1, 3), d_exp, app.expand(b * n, -1), relu=relu)
        rgb.retain_grad()
        sigma.retain_grad()
        rgb_map, _, _ = O.composite(rgb.reshape(b, n, 3), sigma.reshape(b, n, 1), z)
        loss = torch.nn.functional.mse_loss(rgb_map, target.to(dtype))
        loss.backward()
    out = {"rgb": rgb.detach().double().numpy(), "sigma": sigma.detach().double().numpy().ravel(),
           "rgb_map": rgb_map.detach().double().numpy(),
           "drgb": rgb.grad.double().numpy(), "dsigma": sigma.grad.double().numpy().ravel(),
           "dpre_dir": keep[9].grad.double().numpy(), "dpre_7": keep[7].grad.double().numpy()}
    out.update({k: v.grad.double().numpy() for k, v in sd.items()})
    return out


def main():
    import nerfmi
    from nerfmi import _lib as L
    from nerfmi import cameras, get_rays
    from nerfmi.ray_utils import linspace_table
    from test_gpu_train import _trainer
    from conftest import REPO as _  # noqa: F401
    for arith in ("f16x3", "f32"):
        L.set_mlp_arith(arith)
        ref_state = O.random_state(0)
        tr, table = _trainer(ref_state, n_images=4)
        g = torch.Generator().manual_seed(21)
        c2w = cameras.frame_c2w("chair", "circle", 0, 120).float()
        o_all, d_all = get_rays(800, 800, cameras.synthetic_focal(800), c2w.to(tr.dev))
        sel = torch.randperm(800 * 800, generator=g)[:512]
        o, d = o_all.reshape(-1, 3)[sel.to(tr.dev)], d_all.reshape(-1, 3)[sel.to(tr.dev)]
        target = torch.rand(512, 3, generator=g)
        t_rand = torch.rand(512, 64, generator=g)
        img = 0
        tr.forward_backward(o, d, target.to(tr.dev), img, t_rand=t_rand)
        torch.cuda.synchronize()
        grads = {n: tr.view(tr.grad, i).detach().cpu().double().numpy()
                 for i, n in enumerate(list(O.STATE_KEYS) + ["appearance_embeddings"])}
        # staged: the same kernels, keeping the intermediate rows
        lib, P, s, dev = L.load(), L.ptr, L.stream(), tr.dev
        B, N = 512, 64
        M = B * N
        dn, z = torch.empty(B, 3, device=dev), torch.empty(B, N, device=dev)
        feat, encd = torch.empty(B, 256, device=dev), torch.empty(B, 32, device=dev)
        rgb, sigma = torch.empty(M, 3, device=dev), torch.empty(M, device=dev)
        save = torch.empty(L.tile_rows(M), L.SAVE_ROW, device=dev)
        grad = torch.zeros(L.tile_rows(M), L.GRAD_ROW, device=dev)
        masks = torch.empty(M, L.MASK_ROW, dtype=torch.int32, device=dev)
        rgb_map, depth = torch.empty(B, 3, device=dev), torch.empty(B, device=dev)
        dsig, drgb, sq = torch.empty(M, device=dev), torch.empty(M, 3, device=dev), torch.empty(B, device=dev)
        app = tr.appearance_embeddings[img].reshape(1, 32)
        oo, dd = o.contiguous(), d.contiguous()
        L.check(lib.nerf_normalize_dirs(P(dd), B, P(dn), s), "n")
        L.check(lib.nerf_sample_stratified(P(oo), P(dn), B, 2.0, 6.0, N, P(linspace_table(N, dev)), 1,
                                           P(t_rand.to(dev).contiguous()), 0, P(z), None, s), "s")
        L.check(lib.nerf_ray_features_train(P(tr.packed), P(dn), B, P(app), 1, P(feat), P(encd), s), "f")
        L.check(lib.nerf_mlp_forward_train(P(tr.packed), P(oo), P(dn), P(z), B, N, P(feat), P(encd), P(rgb), P(sigma),
                                           P(save), P(masks), s), "fw")
        L.check(lib.nerf_composite(P(rgb), P(sigma), P(z), B, N, P(rgb_map), P(depth), None, s), "c")
        L.check(lib.nerf_composite_backward(P(rgb), P(sigma), P(z), P(rgb_map), P(target.to(dev).contiguous()), B, N,
                                            2.0 / (3 * B), P(dsig), P(drgb), P(sq), s), "cb")
        L.check(lib.nerf_mlp_backward(P(tr.packed), P(tr.packedT), P(save), P(masks) if arith == "f16x3" else None,
                                      P(sigma), P(rgb), P(dsig), P(drgb), M, P(grad), s), "bw")
        torch.cuda.synchronize()
        rows, grows = L.untile(save.cpu(), M), L.untile(grad.cpu(), M).double().numpy()
        offs = [0, 256, 512, 768, 1088, 1344, 1600, 1856]
        m_gpu = [rows[:, a:a + 256] > 0 for a in offs] + [(sigma.cpu() > 0).reshape(M, 1), rows[:, 2144:2272] > 0]
        st = {k: v.clone() for k, v in ref_state.items()}
        m_cpu = []
        c32 = oracle_parts(st, table, img, o.cpu(), d.cpu(), target, t_rand, torch.float32, record=m_cpu)
        c64 = oracle_parts(st, table.double(), img, o.cpu(), d.cpu(), target, t_rand, torch.float64, masks=m_cpu)
        g64 = oracle_parts(st, table.double(), img, o.cpu(), d.cpu(), target, t_rand, torch.float64, masks=m_gpu)
        gpu = {"rgb": rgb.cpu().double().numpy(), "sigma": sigma.cpu().double().numpy(),
               "rgb_map": rgb_map.cpu().double().numpy(),
               "drgb": drgb.cpu().double().numpy(), "dsigma": dsig.cpu().double().numpy(),
               "dpre_dir": grows[:, 2048:2176], "dpre_7": grows[:, 1792:2048]}
        print(f"== {arith}: rel-L2 / mean signed error vs float64 (own branches): gpu | cpu fp32")
        for k in ("rgb", "sigma", "rgb_map", "drgb", "dsigma", "dpre_dir", "dpre_7"):
            print(f"  {k:10s} {rel(gpu[k], g64[k]):.3g} {bias(gpu[k], g64[k]):+.3g} | "
                  f"{rel(c32[k], c64[k]):.3g} {bias(c32[k], c64[k]):+.3g}")
        if os.environ.get("DIAG_SAVE"):
            np.savez(os.path.join(os.environ["DIAG_SAVE"], f"composite_inputs_{arith}.npz"), rgb=gpu["rgb"].astype(np.float32),
                     sigma=gpu["sigma"].astype(np.float32), z=z.cpu().numpy(), rgb_map=gpu["rgb_map"].astype(np.float32),
                     target=target.numpy(), drgb=gpu["drgb"].astype(np.float32))
        # the composite alone: float64 render + mse backward from the GPU's own rgb / sigma / z
        rgb_t = torch.from_numpy(gpu["rgb"]).reshape(B, N, 3).requires_grad_(True)
        with torch.enable_grad():
            rm, _, _ = O.composite(rgb_t, torch.from_numpy(gpu["sigma"]).reshape(B, N, 1), z.cpu().double())
            torch.nn.functional.mse_loss(rm, target.double()).backward()
        dr64 = rgb_t.grad.reshape(-1, 3).numpy()
        # the reference's own fp32 composite (O.composite in float32, torch CPU) on the same GPU inputs
        rgb_32 = torch.from_numpy(gpu["rgb"]).float().reshape(B, N, 3).requires_grad_(True)
        with torch.enable_grad():
            rm32, _, _ = O.composite(rgb_32, torch.from_numpy(gpu["sigma"]).float().reshape(B, N, 1), z.cpu())
            torch.nn.functional.mse_loss(rm32, target).backward()
        print(f"  cpu fp32 composite on the gpu's inputs: rgb_map {rel(rm32.detach().numpy(), rm.detach().numpy()):.3g} "
              f"{bias(rm32.detach().numpy(), rm.detach().numpy()):+.3g}  drgb "
              f"{rel(rgb_32.grad.reshape(-1, 3).numpy(), dr64):.3g} {bias(rgb_32.grad.reshape(-1, 3).numpy(), dr64):+.3g}")
        print(f"  composite only: rgb_map {rel(gpu['rgb_map'], rm.detach().numpy()):.3g} "
              f"{bias(gpu['rgb_map'], rm.detach().numpy()):+.3g}  drgb {rel(gpu['drgb'], dr64):.3g} {bias(gpu['drgb'], dr64):+.3g}")
        for k in ("dpre_dir", "dpre_7"):
            sg, s64, sc, s64c = (x.sum(0) for x in (gpu[k], g64[k], c32[k], c64[k]))
            print(f"  sum_m {k:6s} {rel(sg, s64):.3g} | {rel(sc, s64c):.3g}")
        for k in ("dir_linear.bias", "dir_linear.weight", "density_head.bias", "pts_linears.7.bias"):
            print(f"  grad {k:18s} {rel(grads[k], g64[k]):.3g} | {rel(c32[k], c64[k]):.3g}")


if __name__ == "__main__":
    main()
