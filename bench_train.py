"""Benchmark of the training step (BASELINE config 5).

    python bench_train.py [--gpus N] [--steps K] [--warmup W] [--batch 4096]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench_train.py --gpus N

`python bench_train.py --gpus N` starts its own N ranks (nerfmi/launch.py, as bench.py); --dry-run
rehearses the data-parallel plumbing (gloo process group, the flat-gradient all-reduce of
train.average_gradients, rank-0 broadcast, barrier + max-over-ranks timing) on the CPU.

One step = one iteration of the reference's train_nerf (src/train.py:77-92) per GPU on a
4096-ray batch of one image, 64 stratified samples per ray (perturb=True; n_importance is
ignored by the reference's volume_render, render.py:83-86): weight packing, forward with
activation saves, mse loss, backward (composite, MLP data gradients, weight gradients), the
data-parallel RCCL all-reduce of the flat gradient buffer, and the Adam update.  Batches come
from the teacher-rendered synthetic scene (nerfmi.dataset.SyntheticNeRFDataset at 800x800; no
dataset exists here) and are generated before the timed region (inputs resident in HBM).
Rank 0 prints one JSON line; value = rays trained per second over all ranks (weak scaling:
4096 rays per GPU per step).

roofline: per-sample algorithmic FLOP of the three MFMA kernels (forward 1,048,832; data
gradients 983,040; weight gradients 1,066,752 including bias columns — DESIGN.md §Training)
over their event-timed durations; for the weight-gradient phase, whose every operand row is
streamed once, the binding roofline is HBM when its algorithmic bytes (18,188 per sample) at
8 TB/s take longer than its MFMA work at peak: then bound "hbm" in GB/s, the MFMA figures under
"mfma".  The forward runs on the MLP arithmetic selected by --arith
(f16x3 default: split-f16 MFMA, peak 2516.8/3 = 838.9 TFLOP/s of fp32-equivalent work; f32:
157.3).  Under f16x3 the data gradients run on split-f16 MFMA too (838.9) and the weight
gradients on block-scaled split-f16 MFMA (three f16 products per fp32 product at per-chunk
power-of-two scales, 838.9); under f32 both run on fp32 MFMA (157.3).
cpu_baseline: the oracle's train_step (PyTorch-CPU autograd + torch.optim.Adam) on the measured
config's own batch (--batch, 4096 rays x 64 samples; at least 3 steps) on this host's cores.
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

MFMA_F32_PEAK_TFLOPS = 157.3
FLOP_FWD = 1_048_832
FLOP_DGRAD = 2 * (7 * 256 * 256 + 256 * 128)                                   # 983,040
FLOP_WGRAD = 2 * (64 * 256 + 6 * 257 * 256 + 320 * 256 + 257 + 284 * 128 + 33 * 128 + 129 * 3)
# the weight gradients' MFMA arithmetic under f16x3: the 256-column GEMMs (7 of the 8 big ones and
# dir/sigma) on split-f16 with per-chunk power-of-two scales (three f16 products per fp32 product:
# 2516.8/3 = 838.9 TFLOP/s; vendor f16 GEMM 1,323.5 / 3).
# HBM: bytes the weight-gradient phase must read once per sample (fp32 rows, layout.h): gradient rows
# d pre_0..7 (8 x 256), [d pre_dir | d sigma] (129), d rgb (3); saved rows enc_x (63), h_0..h_7
# (8 x 256), hd (128).  (d hd's 128 columns were read per sample until round 5; under f16x3 the per-ray
# sums now come from the dir/density launch and the block sums of d rgb, train.hip.)  Against 8 TB/s
# this is the phase's binding roofline under f16x3 (0.58 ms per 262,144 samples, against 0.33 ms of
# MFMA work at 838.9 TFLOP/s).
HBM_PEAK_GBS = 8000.0
WGRAD_ALG_BYTES = 4 * (8 * 256 + 129 + 3 + 63 + 8 * 256 + 128)   # 17,676
WGRAD_ARITH, WGRAD_PRODUCTS, WGRAD_VENDOR = "block-scaled f16x3", 3, 1323.5 / 3


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=10)   # (3: the timed steps still ramp up, ~2 % slow)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--arith", default="f16x3", choices=("f16x3", "f32"), help="forward MLP MFMA arithmetic")
    p.add_argument("--dry-run", action="store_true", help="CPU/gloo rehearsal of the N-rank plumbing (no GPU)")
    return p.parse_args()


def cpu_baseline(target_s, B=4096, min_steps=3):
    from oracle import nerf_oracle as O
    from nerfmi import cameras
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    state = O.random_state(0)
    torch.manual_seed(1)
    table = torch.randn(100, 32)
    o, d = O.get_rays(800, 800, cameras.synthetic_focal(800), cameras.frame_c2w("chair"))
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    g = torch.Generator().manual_seed(3)
    opt, n, t = None, 0, 0.0
    while (t < target_s or n < min_steps) and n < 50:
        sel = torch.randperm(o.shape[0], generator=g)[:B]
        t_rand = torch.rand(B, 64, generator=g)
        target = torch.rand(B, 3, generator=g)
        t0 = time.perf_counter()
        _, _, _, opt = O.train_step(state, table, 0, o[sel], d[sel], target, 2.0, 6.0, 64, t_rand, optimizer=opt)
        t += time.perf_counter() - t0
        n += 1
    return {"value": n * B / t, "unit": "rays/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} training steps of {B} rays (64 samples, fwd+bwd+Adam), oracle/nerf_oracle.py "
                      f"train_step on PyTorch-CPU fp32, {t:.1f} s"}


PMC_SUMMARY = (sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                          "r*_pmc_summary_train.json"))) or [""])[-1]   # the latest round's


def pmc_traffic():
    """HBM bytes per step of the weight-gradient phase (every wgrad GEMM and chunk reduction) and
    per data-gradient launch, from the committed PMC passes of `scripts/profile_pmc.sh <dir> train`
    (2 x FETCH_SIZE + WRITE_SIZE; scripts/summarize_pmc.py).  Steps in the profiled run = its
    data-gradient launches (one per step)."""
    try:
        k = json.load(open(PMC_SUMMARY))["kernels"]
        bw = next(v for n, v in k.items() if "mlp_backward16" in n)   # (the LDS-stream kernel since r02)
        wgrad = sum(v["hbm_bytes_per_dispatch"] * v["dispatches"] for n, v in k.items()
                    if "wgrad" in n or "ray_sums" in n or "app_grad" in n)   # param_grads
        return {"wgrad": wgrad / bw["dispatches"], "mlp_backward": bw["hbm_bytes_per_dispatch"]}
    except (OSError, KeyError, ValueError, ZeroDivisionError, StopIteration):
        return {}


def dry_run(args, world, rank):
    """Data-parallel plumbing of a training step on the CPU: every rank fills the flat gradient
    buffer (534,276 + 3,200 floats) with its own values, train.average_gradients all-reduces it, and
    the result must be the mean over ranks; rank 0's parameters are broadcast first."""
    from nerfmi.train import average_gradients, broadcast_state
    group = None
    if world > 1:
        dist.init_process_group("gloo")
        group = dist.group.WORLD
    n = 534_276 + 3_200
    flat = torch.full((n,), float(rank))
    broadcast_state([flat], group)
    ok = bool((flat == 0).all())
    grad = torch.empty(n)
    for _ in range(args.warmup):
        average_gradients(grad.fill_(rank + 1.0), group)
    if group is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        average_gradients(grad.fill_(rank + 1.0), group)
    if group is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ok = ok and bool(torch.allclose(grad, torch.full((n,), (world + 1) / 2.0)))
    got = [(rank, 1e3 * elapsed / args.steps)]
    if group is not None:
        got = [None] * world
        dist.all_gather_object(got, (rank, 1e3 * elapsed / args.steps))
    ranks, rank_ms = [g[0] for g in got], [g[1] for g in got]
    elapsed = max(rank_ms) * args.steps * 1e-3
    if rank == 0:
        print(json.dumps({"metric": "training steps/sec (dry run: gradient all-reduce only, gloo)",
                          "value": args.steps / elapsed, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
                          "higher_is_better": True, "scaling": "weak", "dry_run": True, "ranks": ranks,
                          "rank_ms": rank_ms, "allreduce_ok": ok, "config": {"parallelism": f"dp{world} (gloo all-reduce)"}}), flush=True)
    if group is not None:
        dist.destroy_process_group()


def measure(args, world, rank, group, ranks):
    """Time args.steps training steps on this rank (args: steps, warmup, batch, arith,
    no_cpu_baseline, cpu_seconds); every rank calls it, rank 0 gets the result dict (else None).
    bench.py calls it for its "train" leg in the same process as the render bench."""
    import nerfmi
    from nerfmi.dataset import SyntheticNeRFDataset
    from nerfmi.train import Trainer
    prev_arith = nerfmi.get_mlp_arith()
    nerfmi.set_mlp_arith(args.arith)
    cfg = nerfmi.Config()
    np.random.seed(100 + rank)                    # each rank draws its own images / pixels
    ds = SyntheticNeRFDataset(cfg, n_images=100)
    batches = [ds.get_rays(batch_size=args.batch) for _ in range(args.warmup + args.steps)]
    torch.manual_seed(0)
    tr = Trainer(cfg, appearance_embeddings=ds.appearance_embeddings, group=group)
    stream = torch.cuda.current_stream()

    # stage timing: events around each stage on the launch stream
    pending = []

    def step(b, timed):
        marks = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if timed else None
        if timed:
            marks[0].record(stream)
        tr.forward_backward(b["rays_o"], b["rays_d"], b["rgb"], b["appearance_idx"], seed=tr.steps + 1,
                            _marks=marks)
        if timed:
            marks[2].record(stream)
        tr.all_reduce()
        if timed:
            marks[3].record(stream)
        tr.optimizer_step()
        if timed:
            marks[4].record(stream)
            pending.append(marks)

    for i in range(args.warmup):
        step(batches[i], False)
    torch.cuda.synchronize()
    if group is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed steps carry no instrumentation (a stream event between kernels costs the GPU a few us);
    # the stage split comes from as many instrumented steps after them
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(batches[args.warmup + i], False)
    torch.cuda.synchronize()
    if group is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rank_ms = gather_rank_ms(1e3 * elapsed / args.steps, group)
    elapsed = max(rank_ms) * args.steps * 1e-3
    for i in range(args.steps):
        step(batches[args.warmup + i], True)
    torch.cuda.synchronize()
    stage = {"fwd": [], "bwd": [], "allreduce": [], "adam": []}
    for m in pending:
        stage["fwd"].append(m[0].elapsed_time(m[1]))
        stage["bwd"].append(m[1].elapsed_time(m[2]))
        stage["allreduce"].append(m[2].elapsed_time(m[3]))
        stage["adam"].append(m[3].elapsed_time(m[4]))
    stage_ms = {k: float(np.mean(v)) for k, v in stage.items()}
    # kernel-level timing of one extra (untimed) step: forward, data-gradient and weight-gradient phases
    kt = tr.profile_step(batches[-1]["rays_o"], batches[-1]["rays_d"], batches[-1]["rgb"],
                         batches[-1]["appearance_idx"])
    out = None
    if rank == 0:
        M = args.batch * cfg.num_samples
        rays = args.batch * args.steps * world
        kern = {"mlp_forward_train": (FLOP_FWD, kt["mlp_forward_ms"]), "mlp_backward": (FLOP_DGRAD, kt["mlp_backward_ms"]),
                "wgrad": (FLOP_WGRAD, kt["param_grads_ms"])}
        peaks = {"mlp_forward_train": MFMA_F32_PEAK_TFLOPS * (16 / 3 if args.arith == "f16x3" else 1),
                 "mlp_backward": MFMA_F32_PEAK_TFLOPS * (16 / 3 if args.arith == "f16x3" else 1),
                 "wgrad": MFMA_F32_PEAK_TFLOPS * (16 / WGRAD_PRODUCTS if args.arith == "f16x3" else 1)}
        vendor = ({"mlp_forward_train": 1323.5 / 3, "mlp_backward": 1323.5 / 3, "wgrad": WGRAD_VENDOR}
                  if args.arith == "f16x3" else None)
        dominant = max(kern, key=lambda k: kern[k][1])
        flop, ms = kern[dominant]
        ach = M * flop / (ms * 1e-3) / 1e12
        # the binding roofline of the dominant phase: MFMA time at peak against HBM time at peak (the
        # weight gradients stream every saved and gradient row once)
        hbm = None
        if dominant == "wgrad":
            t_mfma = M * flop / (peaks[dominant] * 1e12)
            t_hbm = M * WGRAD_ALG_BYTES / (HBM_PEAK_GBS * 1e9)
            if t_hbm > t_mfma:
                hbm = {"bound": "hbm", "achieved": M * WGRAD_ALG_BYTES / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": M * WGRAD_ALG_BYTES / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                       "alg_bytes_per_sample": WGRAD_ALG_BYTES, "roofline_ms": {"hbm": t_hbm * 1e3, "mfma": t_mfma * 1e3}}
        traffic = pmc_traffic() if args.arith == "f16x3" else {}
        out = {"metric": "training rays/sec, 4096-ray batches, 64 samples, fwd+bwd+Adam (BASELINE config 5)",
               "value": rays / elapsed, "unit": "rays/s", "n_gpus": world, "ranks": ranks,
               "rank_ms": rank_ms,
               "process_group": "nccl (RCCL)" if group is not None else None, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None,
               "dtype": f"fp32 (f16x3 split forward/data gradients, {WGRAD_ARITH} split weight gradients)"
                        if args.arith == "f16x3" else "fp32",
               "data": "synthetic: teacher-rendered 800x800 scene (SyntheticNeRFDataset, 100 poses), batches "
                       "pre-generated in HBM; student = torch.manual_seed(0); NeRF(Config())",
               "config": {"workload": "chair-style training loop, one image per batch", "rays_per_gpu_per_step":
                          args.batch, "n_samples": cfg.num_samples,
                          "parallelism": f"dp{world} (RCCL all-reduce)" if group is not None
                          else "dp1 (no process group, no collective)"},
               "mlp_arith_forward": args.arith,
               "roofline": {"bound": "mfma", "kernel": dominant, "achieved": ach, "peak": peaks[dominant],
                            "unit": "TFLOP/s", "frac": ach / peaks[dominant],
                            **(hbm or {}),
                            **({"mfma": {"achieved": ach, "peak": peaks[dominant], "unit": "TFLOP/s",
                                         "frac": ach / peaks[dominant]}} if hbm else {}),
                            "traffic": traffic.get(dominant), "traffic_unit": "bytes/phase (one step)",
                            "traffic_source": os.path.relpath(PMC_SUMMARY, os.path.dirname(os.path.abspath(__file__)))
                            if traffic.get(dominant) is not None else None,
                            "traffic_by_kernel": traffic,
                            "kernels_ms": {k: v[1] for k, v in kern.items()},
                            "kernels_tflops": {k: M * v[0] / (v[1] * 1e-3) / 1e12 for k, v in kern.items()},
                            "kernels_frac": {k: M * v[0] / (v[1] * 1e-3) / 1e12 / peaks[k] for k, v in kern.items()},
                            "kernels_peak": peaks,
                            # hipBLASLt's own sustained dense GEMM on this part (profiles/r02_gemm_f16_ceiling.log):
                            # f16 1,323.5 and bf16 1,377.1 TFLOP/s, divided by the split's product count
                            "kernels_frac_of_vendor_gemm": {k: M * v[0] / (v[1] * 1e-3) / 1e12 / vendor[k]
                                                            for k, v in kern.items()} if vendor else None},
               "stage_ms": stage_ms, "phase_ms": kt}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.batch)
    nerfmi.set_mlp_arith(prev_arith)
    del tr, ds, batches
    return out


def gather_rank_ms(ms, group):
    """Every rank's ms per step (rank order); [ms] without a process group."""
    if group is None:
        return [ms]
    t = torch.tensor([ms], dtype=torch.float64, device="cuda")
    got = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(got, t, group=group)
    return [float(g.item()) for g in got]


def main():
    args = parse()
    from nerfmi import launch
    rc = launch.world_or_launch(args.gpus, os.path.abspath(__file__), sys.argv[1:], check_devices=not args.dry_run)
    if rc is not None:
        sys.exit(rc)
    if args.dry_run:
        alone = not launch.under_launcher()
        return dry_run(args, 1 if alone else int(os.environ["WORLD_SIZE"]), 0 if alone else int(os.environ.get("RANK", "0")))
    # under a launcher (WORLD_SIZE set, 1 included) the RCCL group exists: broadcast, gradient
    # all-reduce, barriers and the max-over-ranks timing all run on the device
    world, rank, local, group = launch.init_ranks("nccl")
    if group is None:
        torch.cuda.set_device(local)
    ranks = launch.rank_list(group)
    out = measure(args, world, rank, group, ranks)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if group is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
