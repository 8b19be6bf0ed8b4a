"""Diagnostic (GPU): the F7 / multi-step training parity checks against a float64 trajectory.

F7 (one reference training step): per sampled gradient tensor, the distribution (max, p99.9, median)
of |GPU - float64| and of |reference - float64| (F7 is the reference's own fp32 CPU step), relative to
the tensor's largest float64 entry.  Then the parameters after the step and after 3 oracle steps
(test_trainer_matches_oracle_over_steps' batches): how many entries of each tensor the GPU and the fp32
CPU oracle leave more than 2e-6 from the float64 trajectory.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def stats(e):
    return e.max(), np.quantile(e, 0.999), np.median(e)


def main():
    from conftest import GOLDEN, seeded_uniform
    from oracle import nerf_oracle as O
    from test_gpu_train import _trainer
    from nerfmi import _lib, cameras, get_rays
    f7 = dict(np.load(os.path.join(GOLDEN, "f7_train_step.npz")))
    meta = json.load(open(os.path.join(GOLDEN, "golden.json")))["F7"]
    ref = O.random_state(0)
    t_rand = seeded_uniform(meta["seed_t_rand"], (256, 64), meta["t_rand_sha256"])
    o, d, tgt = (torch.from_numpy(f7[k]) for k in ("o", "d", "target"))
    for arith in ("f16x3", "f32"):
        _lib.set_mlp_arith(arith)
        tr, table = _trainer(ref)
        st64 = {k: v.double().clone() for k, v in ref.items()}
        tab64 = table.double().clone()
        _, _, g64, _ = O.train_step(st64, tab64, 0, o.double(), d.double(), tgt.double(), 2.0, 6.0, 64,
                                    t_rand.double())
        dev = tr.dev
        tr.forward_backward(o.to(dev), d.to(dev), tgt.to(dev), 0, t_rand=t_rand)
        grads = {n: tr.view(tr.grad, i).detach().cpu().clone() for i, n in enumerate(meta["names"])}
        tr.optimizer_step()
        torch.cuda.synchronize()
        for i, name in enumerate(meta["names"]):
            sel = torch.from_numpy(f7[f"idx/{name}"]) if f"idx/{name}" in f7 else None
            e64 = g64[name].reshape(-1)
            e64 = (e64[sel] if sel is not None else e64).numpy()
            g = grads[name].reshape(-1).double()
            g = (g[sel] if sel is not None else g).numpy()
            b = f7[f"grad/{name}"].astype(np.float64).reshape(-1)
            sc = np.abs(e64).max() + 1e-300
            sg, sr = stats(np.abs(g - e64) / sc), stats(np.abs(b - e64) / sc)
            p = tr.view(tr.flat, i).detach().cpu().reshape(-1).double()
            p = (p[sel] if sel is not None else p).numpy()
            q64 = (st64[name] if name in st64 else tab64).detach().reshape(-1)
            q64 = (q64[sel] if sel is not None else q64).numpy()
            pr = f7[f"param/{name}"].astype(np.float64).reshape(-1)
            print(f"F7 {arith} {name:28s} grad |gpu-f64| {sg[0]:.2e} {sg[1]:.2e} {sg[2]:.2e}  |ref-f64| {sr[0]:.2e} "
                  f"{sr[1]:.2e} {sr[2]:.2e} | params off f64: gpu {int((np.abs(p - q64) > 2e-6).sum())} "
                  f"ref {int((np.abs(pr - q64) > 2e-6).sum())} of {p.size}")
        # three steps (test_trainer_matches_oracle_over_steps)
        tr, table = _trainer(ref, n_images=4)
        st32, tab32 = {k: v.clone() for k, v in ref.items()}, table.clone()
        st64, tab64 = {k: v.double().clone() for k, v in ref.items()}, table.double().clone()
        opt32 = opt64 = None
        focal = cameras.synthetic_focal(800)
        g = torch.Generator().manual_seed(21)
        for step in range(3):
            c2w = cameras.frame_c2w("chair", "circle", 10 * step, 120).float()
            o_all, d_all = get_rays(800, 800, focal, c2w.to(tr.dev))
            sel = torch.randperm(800 * 800, generator=g)[:512]
            oo, dd = o_all.reshape(-1, 3)[sel.to(tr.dev)], d_all.reshape(-1, 3)[sel.to(tr.dev)]
            target = torch.rand(512, 3, generator=g)
            tr_ = torch.rand(512, 64, generator=g)
            img = step % 4
            _, _, _, opt32 = O.train_step(st32, tab32, img, oo.cpu(), dd.cpu(), target, 2.0, 6.0, 64, tr_, optimizer=opt32)
            _, _, _, opt64 = O.train_step(st64, tab64, img, oo.cpu().double(), dd.cpu().double(), target.double(), 2.0,
                                          6.0, 64, tr_.double(), optimizer=opt64)
            tr.forward_backward(oo, dd, target.to(tr.dev), img, t_rand=tr_)
            tr.optimizer_step()
        torch.cuda.synchronize()
        names = list(O.STATE_KEYS) + ["appearance_embeddings"]
        for i, n in enumerate(names):
            got = tr.view(tr.flat, i).detach().cpu().double().numpy().ravel()
            c32 = (tab32 if n == "appearance_embeddings" else st32[n]).detach().double().numpy().ravel()
            c64 = (tab64 if n == "appearance_embeddings" else st64[n]).detach().numpy().ravel()
            print(f"3-step {arith} {n:28s} params off f64 >2e-6: gpu {int((np.abs(got - c64) > 2e-6).sum())} "
                  f"cpu32 {int((np.abs(c32 - c64) > 2e-6).sum())}  gpu-vs-cpu32 {int((np.abs(got - c32) > 2e-6).sum())}"
                  f" of {got.size}; max |gpu-f64| {np.abs(got - c64).max():.2e} cpu {np.abs(c32 - c64).max():.2e}")


if __name__ == "__main__":
    main()
