"""Ray-chunk sharding of frames across ranks (frames.py) on CPU with gloo, world_size 1 and 2.

The HIP renderer is replaced by the oracle (a small frame) or by a function of the ray itself,
so what is tested is the sharding, the per-rank ray generation and the all-gather reassembly:
the assembled frames must equal the single-process ones bit for bit, in ray order."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nerf_oracle as O
from nerfmi import cameras, frames

H, W = 6, 10


def ray_fn_for(poses, focal):
    def ray_fn(frame, row0, nrows):
        o, d = O.get_rays(H, W, focal, poses[frame])
        return o[row0:row0 + nrows].reshape(-1, 3), d[row0:row0 + nrows].reshape(-1, 3)
    return ray_fn


def fake_render(o, d, offset):
    # depends on the ray and on its global index: a mis-ordered gather or a wrong offset shows
    idx = torch.arange(offset, offset + o.shape[0], dtype=torch.float32)
    return d * 0.5 + 0.5, (o.sum(-1) + idx)[:, None]


def poses():
    return [cameras.frame_c2w("chair", "circle", k, 120) for k in range(3)]


def test_shard_range_covers_everything():
    for n in (0, 1, 7, 640000, 640001):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, e, per = frames.shard_range(n, world, r)
                assert e - s <= per
                seen += list(range(s, e)) if n < 1000 else [s, e]
            if n < 1000:
                assert seen == list(range(n))


def test_shard_rays_slices_rows_exactly():
    ps = poses()
    ray_fn = ray_fn_for(ps, 7.5)
    full_o = torch.cat([ray_fn(f, 0, H)[0] for f in range(3)])
    full_d = torch.cat([ray_fn(f, 0, H)[1] for f in range(3)])
    for start, end in ((0, 180), (3, 57), (55, 125), (119, 121), (60, 60)):
        o, d = frames.shard_rays(ray_fn, H, W, 3, start, end)
        if end == start:
            assert o is None
            continue
        assert torch.equal(o, full_o[start:end]) and torch.equal(d, full_d[start:end])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ps = poses()
        rgb, depth = frames.render_frames_sharded(ray_fn_for(ps, 7.5), fake_render, H, W, len(ps))
        # a real (oracle) render of one frame, strong-scaled
        state = O.random_state(0)

        def oracle_render(o, d, offset):
            r, dep, _ = O.volume_render(state, o, d, 2.0, 6.0, 8, None)
            return r, dep
        rgb1, depth1 = frames.render_frames_sharded(ray_fn_for(ps[:1], 7.5), oracle_render, H, W, 1)
        if rank == 0:
            torch.save({"rgb": rgb, "depth": depth, "rgb1": rgb1, "depth1": depth1}, out)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_world2_reassembles_the_single_process_frames(tmp_path):
    ps = poses()
    ref_rgb, ref_depth = frames.render_frames_sharded(ray_fn_for(ps, 7.5), fake_render, H, W, len(ps))
    state = O.random_state(0)
    o, d = ray_fn_for(ps[:1], 7.5)(0, 0, H)
    r_ref, d_ref, _ = O.volume_render(state, o, d, 2.0, 6.0, 8, None)
    out = str(tmp_path / "rank0.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert torch.equal(got["rgb"], ref_rgb) and torch.equal(got["depth"], ref_depth)
    # the oracle's CPU GEMM blocks differently for 30- and 60-ray batches: equal to rounding
    assert torch.allclose(got["rgb1"].reshape(-1, 3), r_ref, rtol=1e-5, atol=1e-7)
    assert torch.allclose(got["depth1"].reshape(-1), d_ref[:, 0], rtol=1e-5, atol=1e-7)


def _worker_bench(rank, world, port, out):
    """bench.py's own step plan (bench.workload) through frames.render_frames_sharded, both
    scaling modes, at world 2 over gloo."""
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        for scaling in ("weak", "strong"):
            ps = bench.workload("hotdog", world, scaling)
            res[scaling] = frames.render_frames_sharded(ray_fn_for(ps, 7.5), fake_render, H, W, len(ps))
        if rank == 0:
            torch.save(res, out)
    finally:
        dist.destroy_process_group()


def test_bench_plans_world2(tmp_path):
    """Strong scaling (BASELINE config 4: one hotdog frame sharded over the ranks) and weak
    scaling (one frame per rank) reassemble exactly the single-process frames."""
    import bench
    assert len(bench.workload("hotdog", 2, "strong")) == 1 and len(bench.workload("hotdog", 2, "weak")) == 2
    out = str(tmp_path / "bench.pt")
    mp.spawn(_worker_bench, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    for scaling in ("weak", "strong"):
        ps = bench.workload("hotdog", 2, scaling)
        ref = frames.render_frames_sharded(ray_fn_for(ps, 7.5), fake_render, H, W, len(ps))
        assert torch.equal(got[scaling][0], ref[0]) and torch.equal(got[scaling][1], ref[1]), scaling
