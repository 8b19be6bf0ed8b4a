"""Benchmark: rays/s of the hierarchical render path at 800x800, 64 coarse + 128 fine samples.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong] [--scene chair|hotdog]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`python bench.py --gpus N` (N > 1, WORLD_SIZE unset) starts the N ranks itself: it runs
torch.distributed.run as a child process before anything touches the GPU and exits with its status
(nerfmi/launch.py).  Under a launcher, --gpus must equal WORLD_SIZE (else exit 2).
--dry-run: the same launcher, process group (gloo, CPU), step plan, all-gather reassembly and
max-over-ranks timing with a CPU stand-in renderer and 64x64 frames, so the N-rank plumbing is
tested without a GPU (tests/test_bench_launch.py); its JSON line says "dry_run": true.

One step = get_rays -> render_rays (hierarchical H1: coarse 64, inverse-CDF 128, fine composite
over the 192 merged samples, the 64 coarse evaluations reused bit-identically so the fine MLP
evaluates 128) with in-kernel stratified / inverse-CDF RNG, on a random-init NeRF of the
reference architecture (torch.manual_seed(0); NeRF(Config())), through the shipped path: one
nerf_render_rays C call per rank per step (frames.render_path_frames).  The rays of the step's
frames (run.py circle path) are sharded contiguously over the N ranks and reassembled on every
rank with one RCCL all-gather of [r,g,b,depth] per ray (frames.py).
  --scaling weak (default): N frames per step, rank r renders frame r (640,000 rays per GPU).
  --scaling strong: one frame per step sharded over the N ranks (BASELINE config 4 with
                    --scene hotdog: one 800x800 frame ray-chunk sharded across the GPUs).
Rank 0 prints one JSON line.  value = rays of all ranks / max-over-ranks wall time.

roofline: the dominant kernel is the fused PE->MLP kernel.  Its algorithmic work is 1,048,832
FLOP per evaluated sample; each step launches it twice (B*64 and B*128
samples: 192 evaluations per ray).  achieved = algorithmic FLOP / kernel time, the time measured
live in the timed steps by HIP events the library records on the launch's own stream around each
MLP launch inside nerf_render_rays (nerf_profile_mlp_begin/_end; no change to what runs).
--arith selects the MLP arithmetic (include/nerfmi.h, nerf_arith), both fp32-accurate:
  f16x3 (default, mlp16s_kernel): every fp32 product is three f16 MFMA products of a hi/lo split;
        peak = the f16 dense MFMA peak / 3 = 2516.8 / 3 = 838.9 TFLOP/s of fp32-equivalent work
        (MI355X_MICROARCH.md: f16 = 16x the f32 MFMA rate); "mfma_busy" reports the issued f16
        MFMA FLOP (6144 v_mfma_f32_16x16x32_f16 per 32 samples, the FLOP of 3072 32x32x16) against
        2516.8 TFLOP/s;
  f32   (mlp_kernel): v_mfma_f32_32x32x2_f32, peak 157.3 TFLOP/s.
cpu_baseline: the oracle (PyTorch-CPU restatement, oracle/nerf_oracle.py) timed on a
bounded sample of the same workload on this host's cores (rank 0, N=1 only); the GPU renders
the same rays with the same uniforms and the line reports the PSNR of its rgb against the
oracle's (the metric's "PSNR vs reference").  The oracle evaluates all 256 MLP points per ray
(the reference's formulation) where the GPU evaluates 192 (coarse reuse, bit-identical).
The same line carries two more legs, measured in the same process after the headline steps:
  f32_exact (N = 1): --f32-steps frames of the headline workload on the exact-f32 MLP
        (mlp_kernel, v_mfma_f32_32x32x2_f32: the reference's arithmetic), roofline against 157.3;
  train (every rank, data parallel over the same group): bench_train.measure, BASELINE config 5 —
        --train-steps steps of 4,096 rays x 64 samples, fwd + bwd + RCCL all-reduce + Adam, with
        per-phase kernels_ms and the roofline of each MFMA phase.
rank_ms: every rank's ms per step (the max is ms_per_step), so an unbalanced N-GPU run shows it.
cpu_baseline.rays_outside_1e-4: rays whose rgb/depth leave the 1e-4 parity tolerance, GPU against
the fp32 oracle, and GPU and fp32 oracle each against the oracle evaluated in float64.
traffic: HBM bytes per MLP launch from the rocprofv3 PMC passes of scripts/profile_pmc.sh
(FETCH_SIZE doubled per MI355X_MICROARCH.md + WRITE_SIZE), read from the newest
profiles/r*_pmc_summary.json when present (PMC counters cannot be read inside this process).
"""
import argparse
import glob
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

H = W = 800
N_COARSE, N_FINE = 64, 128
FLOP_PER_SAMPLE = 1_048_832           # SURVEY.md §8d, DESIGN.md §Roofline
MFMA_F32_PEAK_TFLOPS = 157.3          # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense
MFMA_F16_PEAK_TFLOPS = 16 * MFMA_F32_PEAK_TFLOPS   # f16/bf16 dense MFMA = 16x the f32 rate
F16X3_ISSUED_FLOP_PER_SAMPLE = 6144 * 16 * 16 * 32 * 2 // 32   # mlp16s_kernel MFMAs per 32-sample wave
# Measured power-limited ceiling of the f16 MFMA stream the render kernel is built from:
# the trunk's MFMAs alone with their LDS fragment reads, no side work, every CU, random operands.  The
# render kernel runs v_mfma_f32_16x16x32_f16 since round 6: that stream holds 1.99 GHz = 1,574 f16
# TFLOP/s = 525 TFLOP/s of f16x3 work; the 32x32x16 stream of round 5's kernel (and of the training
# kernels) 1.44 GHz = 1,447 f16 TFLOP/s = 482 TFLOP/s.
F16X3_POWER_CEILING = {"value": 1574.0 / 3, "unit": "TFLOP/s", "shape": "v_mfma_f32_16x16x32_f16",
                       "source": "profiles/r02_mfma_shape_side.log (scripts/microbench/mfma_shape_side.hip, "
                                 "shape 16, NV=0)",
                       "shape_32x32x16": {"value": 1447.0 / 3, "unit": "TFLOP/s"}}
# The vendor library's sustained f16 GEMM on the same part (torch.matmul -> hipBLASLt, 8192^3, random
# operands, 3 s back to back): 1,323.5 TFLOP/s = 0.526 of the dense f16 peak.
VENDOR_F16_GEMM = {"f16_tflops": 1323.5, "frac_of_f16_peak": 1323.5 / MFMA_F16_PEAK_TFLOPS,
                   "source": "profiles/r02_gemm_f16_ceiling.log (scripts/microbench/gemm_f16_ceiling.py)"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scene", default="chair")
    p.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                   help="weak: one frame per rank per step; strong: one frame per step over all ranks")
    p.add_argument("--arith", default="f16x3", choices=("f16x3", "f32"), help="MLP MFMA arithmetic")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="target length of the CPU baseline sample")
    p.add_argument("--dry-run", action="store_true", help="CPU/gloo rehearsal of the N-rank plumbing (no GPU)")
    p.add_argument("--dry-size", type=int, default=64, help="frame side of the --dry-run frames")
    p.add_argument("--no-train", action="store_true", help="skip the training leg (BASELINE config 5)")
    p.add_argument("--train-steps", type=int, default=20)
    p.add_argument("--no-f32", action="store_true", help="skip the exact-f32 render leg")
    p.add_argument("--f32-steps", type=int, default=3)
    return p.parse_args()


def cpu_baseline(target_s, gpu_render=None, f64_rays=2048):
    """Oracle H1 render of a centre block of the same frame on the host cores; with gpu_render,
    the PSNR of the GPU's rgb on the same rays and uniforms against the oracle's, and the number of
    rays outside the 1e-4 parity tolerance: GPU against the fp32 oracle on every sampled ray, and on
    the first `f64_rays` of them both the GPU and the fp32 oracle against the oracle evaluated in
    float64 (the fine pass is ill-conditioned, so two fp32 evaluations disagree on a
    few rays; the float64 counts show the GPU is no further from the truth than the CPU)."""
    from oracle import nerf_oracle as O
    from nerfmi import cameras
    state = O.random_state(0)
    torch.manual_seed(1)
    app = torch.randn(100, 32)[0]
    o, d = O.get_rays(H, W, cameras.synthetic_focal(W), cameras.frame_c2w("chair"))
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    centre = (H // 2) * W + W // 2

    def run(n):
        sl = slice(centre - n // 2, centre - n // 2 + n)
        torch.manual_seed(2)
        t_rand = torch.rand(n, N_COARSE)
        u_rand = torch.rand(n, N_FINE)
        args = (o[sl].contiguous(), d[sl].contiguous())
        t0 = time.perf_counter()
        rgb, depth, _ = O.render_rays_h1(state, *args, 2.0, 6.0, N_COARSE, N_FINE, app, t_rand, u_rand)
        return time.perf_counter() - t0, args, t_rand, u_rand, rgb, depth

    n = 512
    dt = run(n)[0]
    n = int(min(65536, max(n, n * target_s / max(dt, 1e-3))))
    n = max(512, (n // 512) * 512)
    dt, rays, t_rand, u_rand, rgb_ref, depth_ref = run(n)
    out = {"value": n / dt, "unit": "rays/s", "cores": torch.get_num_threads(), "kind": "port",
           "sample": f"{n} contiguous rays at the centre of the 800x800 chair frame 0, hierarchical "
                     f"{N_COARSE}+{N_FINE} (H1), perturbed, oracle/nerf_oracle.py on PyTorch-CPU fp32, {dt:.1f} s"}
    psnr = None
    if gpu_render is not None:
        rgb, depth = (t.cpu() for t in gpu_render(*rays, app, t_rand, u_rand))
        mse = float(((rgb - rgb_ref) ** 2).mean())
        psnr = float("inf") if mse == 0 else -10.0 * math.log10(mse)
        got = torch.cat([rgb, depth.reshape(-1, 1)], 1).double()
        ref = torch.cat([rgb_ref, depth_ref.reshape(-1, 1)], 1).double()

        def outside(a, b):       # rays with any of r, g, b, depth outside |a-b| <= 1e-4|b| + 1e-6
            return int(((a - b).abs() > 1e-4 * b.abs() + 1e-6).any(1).sum())

        k = min(f64_rays, n)
        st64 = {key: v.double() for key, v in state.items()}
        t0 = time.perf_counter()
        r64, d64, _ = O.render_rays_h1(st64, rays[0][:k].double(), rays[1][:k].double(), 2.0, 6.0, N_COARSE,
                                       N_FINE, app.double(), t_rand[:k].double(), u_rand[:k].double())
        t64 = time.perf_counter() - t0
        ref64 = torch.cat([r64, d64.reshape(-1, 1)], 1)
        out["rays_outside_1e-4"] = {
            "gpu_vs_oracle_fp32": outside(got, ref), "of_rays": n,
            "gpu_vs_float64": outside(got[:k], ref64), "oracle_fp32_vs_float64": outside(ref[:k], ref64),
            "of_rays_float64": k,
            "max_rel_err_vs_float64": {"gpu": float(((got[:k] - ref64).abs() / (ref64.abs() + 1e-6)).max()),
                                       "oracle_fp32": float(((ref[:k] - ref64).abs() / (ref64.abs() + 1e-6)).max())},
            "criterion": "per ray, any of rgb/depth with |a-b| > 1e-4*|b| + 1e-6; float64 = the oracle's "
                         f"expressions in float64 on the same fp32 inputs and uniforms ({t64:.1f} s)"}
    return out, psnr


def pmc_traffic(arith):
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_summary{'_f16x3' if arith == 'f16x3' else ''}.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        js = json.load(f)
    return js.get("mlp_hbm_bytes_per_launch"), os.path.relpath(paths[-1], REPO)


def workload(scene, world, scaling):
    """Poses of one step: weak = one circle-path frame per rank (frame k on rank k), strong = one
    frame for all ranks.  frames.render_path_frames shards the poses' rays contiguously over the
    ranks either way (tests/test_frames_dist.py runs this plan through gloo)."""
    from nerfmi import cameras
    n = world if scaling == "weak" else 1
    return [cameras.frame_c2w(scene, "circle", frame=k % 120, num_frames=120) for k in range(n)]


def dry_run(args, world, rank):
    """The N-rank plumbing of a bench step on the CPU: gloo process group, bench.workload's poses,
    frames.render_frames_sharded's shard plan and all-gather, barrier + max-over-ranks timing; the
    renderer is a deterministic CPU stand-in (no GPU, no oracle)."""
    from nerfmi import cameras, frames
    if world > 1:
        dist.init_process_group("gloo")
    Hd = Wd = args.dry_size
    poses = workload(args.scene, world, args.scaling)
    focal = cameras.synthetic_focal(Wd)

    def ray_fn(frame, row0, nrows):
        c2w = torch.as_tensor(poses[frame], dtype=torch.float32)
        i, j = torch.meshgrid(torch.arange(row0, row0 + nrows, dtype=torch.float32),
                              torch.arange(Wd, dtype=torch.float32), indexing="ij")
        dirs = torch.stack([(j - Wd * .5) / focal, -(i - Hd * .5) / focal, -torch.ones_like(i)], -1)
        d = (dirs[..., None, :] * c2w[:3, :3]).sum(-1).reshape(-1, 3)
        return c2w[:3, 3].expand(d.shape), d

    def render_fn(o, d, offset):
        idx = torch.arange(offset, offset + o.shape[0], dtype=torch.float64)
        return torch.sigmoid(o + d).float(), (idx % 997).float()[:, None]

    for _ in range(args.warmup):
        frames.render_frames_sharded(ray_fn, render_fn, Hd, Wd, len(poses))
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rgb, depth = frames.render_frames_sharded(ray_fn, render_fn, Hd, Wd, len(poses))
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    start, end, _ = frames.shard_range(Hd * Wd * len(poses), world, rank)
    mine = {"rank": rank, "ms": 1e3 * elapsed / args.steps, "shard": [start, end]}
    got = [mine]
    if world > 1:
        got = [None] * world
        dist.all_gather_object(got, mine)
    ranks = [g["rank"] for g in got]
    rank_ms = [g["ms"] for g in got]
    elapsed = max(rank_ms) * args.steps * 1e-3
    shards = [g["shard"] for g in got]
    ok = bool(torch.equal(depth.reshape(-1), (torch.arange(depth.numel(), dtype=torch.float64) % 997).float()))
    if rank == 0:
        total = Hd * Wd * len(poses) * args.steps
        print(json.dumps({"metric": "rays/sec (dry run: CPU stand-in renderer, gloo)", "value": total / elapsed,
                          "unit": "rays/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
                          "scaling": args.scaling, "dry_run": True, "ranks": ranks, "rank_ms": rank_ms,
                          "shards": shards, "rows_per_rank": [(e - s_) / Wd for s_, e in shards],
                          "reassembly_ok": ok,
                          "config": {"workload": f"{args.scene} {Hd}x{Wd}, {len(poses)} frame(s) per step",
                                     "parallelism": f"ray-shard x{world} + all-gather (gloo)"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def time_render(step, first, steps, group):
    """steps timed calls of step(first + i) between barriers + synchronize; returns (this rank's
    seconds, the MLP launches [(ms, samples)] timed by libnerfmi's events on the MLP's stream)."""
    from nerfmi import _lib
    torch.cuda.synchronize()
    if group is not None:
        dist.barrier()
    cap = 4 * steps + 8
    torch.cuda.synchronize()
    _lib.profile_mlp_begin(cap)
    t0 = time.perf_counter()
    for i in range(steps):
        step(first + i)
    torch.cuda.synchronize()
    if group is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return elapsed, _lib.profile_mlp_end(cap)


def mlp_roofline(launches, arith):
    """(achieved TFLOP/s, peak, kernel, mfma_busy) of the MLP launches under `arith`."""
    mlp_ms = sum(ms for ms, _ in launches)
    mlp_samples = sum(n for _, n in launches)
    achieved = mlp_samples * FLOP_PER_SAMPLE / (mlp_ms * 1e-3) / 1e12 if mlp_ms else 0.0
    if arith == "f16x3":
        busy = mlp_samples * F16X3_ISSUED_FLOP_PER_SAMPLE / (mlp_ms * 1e-3) / 1e12 / MFMA_F16_PEAK_TFLOPS \
            if mlp_ms else 0.0
        return achieved, MFMA_F16_PEAK_TFLOPS / 3, "nerf::mlp16s_kernel", busy
    return achieved, MFMA_F32_PEAK_TFLOPS, "nerf::mlp_kernel", achieved / MFMA_F32_PEAK_TFLOPS


def main():
    args = parse()
    from nerfmi import launch
    rc = launch.world_or_launch(args.gpus, os.path.abspath(__file__), sys.argv[1:], check_devices=not args.dry_run)
    if rc is not None:
        sys.exit(rc)
    if args.dry_run:
        alone = not launch.under_launcher()
        return dry_run(args, 1 if alone else int(os.environ["WORLD_SIZE"]), 0 if alone else int(os.environ.get("RANK", "0")))
    # under a launcher (WORLD_SIZE set, 1 included) the RCCL group exists and every collective below runs
    world, rank, local, group = launch.init_ranks("nccl")
    ranks = launch.rank_list(group)
    import nerfmi
    from nerfmi import cameras, frames
    import bench_train
    nerfmi.set_mlp_arith(args.arith)

    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(0)
    model = nerfmi.NeRF(nerfmi.Config()).to(dev).eval()
    torch.manual_seed(1)
    app = torch.randn(100, 32)[0].to(dev)
    focal = cameras.synthetic_focal(W)
    poses = workload(args.scene, world, args.scaling)
    B = H * W

    @torch.no_grad()
    def step(i):
        rgb, depth = frames.render_path_frames(model, poses, H, W, focal, 2.0, 6.0, N_COARSE, N_FINE,
                                               appearance_embedding=app, perturb=True, hierarchical=True, seed=i)
        return rgb

    for i in range(args.warmup):
        step(i)
    elapsed, launches = time_render(step, args.warmup, args.steps, group)
    rank_ms = bench_train.gather_rank_ms(1e3 * elapsed / args.steps, group)
    elapsed = max(rank_ms) * args.steps * 1e-3           # max over ranks

    rays_per_rank = B * len(poses) // world
    per_kind = {}
    for ms, n in launches:
        per_kind.setdefault("coarse" if n == rays_per_rank * N_COARSE else "fine", []).append(ms)
    achieved, peak, kernel, busy = mlp_roofline(launches, args.arith)
    mlp_ms = sum(ms for ms, _ in launches)

    # --- exact-f32 leg (rank 0 alone, N = 1): the reference's arithmetic, v_mfma_f32_32x32x2_f32
    f32_exact = None
    if world == 1 and not args.no_f32 and args.arith != "f32":
        nerfmi.set_mlp_arith("f32")
        step(10_000)                                       # warmup under the f32 kernel
        e32, l32 = time_render(step, 10_001, args.f32_steps, None)
        nerfmi.set_mlp_arith(args.arith)
        a32, p32, k32, _ = mlp_roofline(l32, "f32")
        f32_exact = {"value": B * len(poses) * args.f32_steps / e32, "unit": "rays/s", "steps": args.f32_steps,
                     "warmup": 1, "ms_per_step": 1e3 * e32 / args.f32_steps, "dtype": "fp32", "mlp_arith": "f32",
                     "workload": "the headline workload above with the exact-f32 MLP (--arith f32)",
                     "roofline": {"bound": "mfma", "kernel": k32, "achieved": a32, "peak": p32, "unit": "TFLOP/s",
                                  "frac": a32 / p32, "launches": len(l32),
                                  "avg_launch_ms": sum(ms for ms, _ in l32) / max(len(l32), 1),
                                  "timing": "HIP events recorded by libnerfmi on the MLP's stream"}}

    # --- training leg (BASELINE config 5), every rank: data parallel over the same group
    train = None
    if not args.no_train:
        # (10 untimed steps: after 3 the step still runs ~2 % slow, profiles/r05/train_warmup.log)
        targs = argparse.Namespace(steps=args.train_steps, warmup=10, batch=4096, arith=args.arith,
                                   no_cpu_baseline=args.no_cpu_baseline, cpu_seconds=8.0)
        train = bench_train.measure(targs, world, rank, group, ranks)
        if train is not None:
            for k in ("metric", "higher_is_better", "vs_baseline", "data", "scaling", "ranks", "process_group"):
                train.pop(k, None)

    if rank == 0:
        total_rays = B * len(poses) * args.steps
        traffic, traffic_src = pmc_traffic(args.arith)
        ceiling = None
        if args.arith == "f16x3":
            ceiling = dict(F16X3_POWER_CEILING, frac=achieved / F16X3_POWER_CEILING["value"],
                           vendor_f16_gemm=dict(VENDOR_F16_GEMM, mlp16_issued_f16_tflops=busy * MFMA_F16_PEAK_TFLOPS))
            dtype = "fp32 (f16x3 split)"
        else:
            dtype = "fp32"
        per_gpu = "one frame per GPU" if args.scaling == "weak" else f"one frame sharded over {world} GPU(s)"
        line = {
            "metric": "rays/sec at 800x800, 64 coarse + 128 fine samples",
            "value": total_rays / elapsed,
            "unit": "rays/s",
            "n_gpus": world,
            "ranks": ranks,
            "rank_ms": rank_ms,
            "process_group": "nccl (RCCL)" if group is not None else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic: run.py circle-path poses, random-init NeRF "
                    "(torch.manual_seed(0); NeRF(Config())), no dataset/checkpoint in the environment",
            "config": {"workload": f"{args.scene} 800x800, {per_gpu} per step, hierarchical {N_COARSE} coarse + "
                                   f"{N_FINE} fine (H1; fine composite over 192 merged samples, coarse "
                                   f"evaluations reused), perturb=True, one nerf_render_rays call per rank",
                       "rays_per_step": B * len(poses), "rays_per_gpu_per_step": rays_per_rank,
                       "n_coarse": N_COARSE, "n_fine": N_FINE, "mlp_evals_per_ray": N_COARSE + N_FINE,
                       "parallelism": f"ray-shard x{world} + RCCL all-gather" if group is not None
                       else "ray-shard x1 (no process group, no collective)"},
            "mlp_arith": args.arith,
            "roofline": {"bound": "mfma", "kernel": kernel, "achieved": achieved,
                         "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak, "mfma_busy": busy,
                         "power_limited_ceiling": ceiling,
                         "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                         "launches": len(launches), "avg_launch_ms": mlp_ms / max(len(launches), 1),
                         "avg_launch_ms_by_pass": {k: sum(v) / len(v) for k, v in per_kind.items()},
                         "flop_per_sample": FLOP_PER_SAMPLE,
                         "timing": "HIP events recorded by libnerfmi on the MLP's stream inside the timed steps"},
            "cpu_baseline": None,
            "psnr_vs_reference_db": None,
            "f32_exact": f32_exact,
            "train": train,
        }
        if world == 1 and not args.no_cpu_baseline:
            @torch.no_grad()
            def gpu_render(o, d, a, t_rand, u_rand):
                rgb, depth, _ = nerfmi.render_rays(model, o.to(dev), d.to(dev), 2.0, 6.0, N_COARSE, N_FINE,
                                                   appearance_embedding=a.to(dev), perturb=True, hierarchical=True,
                                                   t_rand=t_rand, u_rand=u_rand)
                return rgb, depth
            line["cpu_baseline"], line["psnr_vs_reference_db"] = cpu_baseline(args.cpu_seconds, gpu_render)
        print(json.dumps(line), flush=True)
    if group is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
