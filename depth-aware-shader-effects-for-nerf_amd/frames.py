"""Frame rendering sharded by ray chunk over the GPUs of one node.

The reference renders a frame as a loop over independent ray chunks (run.py:209-231).
Here the rays of a batch of frames — frame-major, row-major inside a frame, exactly the
order run.py concatenates its chunks in (run.py:230-231) — are cut into one contiguous
shard per rank.  Each rank generates only its own rays (get_rays on the rows it needs),
renders them, and one all-gather (torch.distributed, backend "nccl" = RCCL over xGMI)
reassembles [r, g, b, depth] of every ray on every rank in ray order.  Rays are independent
and every ray costs the same, so there is no other exchange.

With one pose and N ranks this is strong scaling of one frame; with N poses and N ranks
each rank renders one whole frame (weak scaling, what bench.py measures).
The ray source and the renderer are injectable so the sharding and reassembly logic is
tested with gloo on CPU (tests/test_frames_dist.py) with no GPU.
"""
import torch
import torch.distributed as dist


def shard_range(n_rays, world, rank):
    """Contiguous [start, end) of rank `rank` and the padded shard length (all shards equal)."""
    per = -(-n_rays // world) if n_rays else 0
    start = min(rank * per, n_rays)
    return start, min(start + per, n_rays), per


def _world(group):
    """(world, rank, collective): collective is True whenever a process group exists, world 1
    included, so the all-gather runs on the device under any launcher (tests/test_gpu_rccl.py)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group), True
    return 1, 0, False


def shard_rays(ray_fn, H, W, n_frames, start, end):
    """(o, d) of global rays [start, end): frame f = ray // (H*W), generated per frame on the
    rows that hold the range and sliced to it.  ray_fn(frame, row0, nrows) -> (o, d), each
    (nrows*W, 3)."""
    P = H * W
    os_, ds_ = [], []
    r = start
    while r < end:
        f = r // P
        lo = r - f * P
        hi = min(end - f * P, P)
        row0, row1 = lo // W, -(-hi // W)
        o, d = ray_fn(f, row0, row1 - row0)
        os_.append(o[lo - row0 * W: hi - row0 * W])
        ds_.append(d[lo - row0 * W: hi - row0 * W])
        r = f * P + hi
    if not os_:
        return None, None
    return torch.cat(os_), torch.cat(ds_)


def _render_shard(ray_fn, render_fn, H, W, n_frames, start, end, buf):
    if end > start:
        o, d = shard_rays(ray_fn, H, W, n_frames, start, end)
        rgb, depth = render_fn(o, d, start)
        buf[: end - start, :3] = rgb.to(buf.device)
        buf[: end - start, 3:] = depth.reshape(-1, 1).to(buf.device)


@torch.no_grad()
def render_frames_sharded(ray_fn, render_fn, H, W, n_frames, group=None, device=None, virtual_shards=None):
    """Render n_frames HxW frames over the ranks of `group`.

    ray_fn(frame, row0, nrows) -> (rays_o, rays_d) for those rows (row-major, (nrows*W, 3));
    render_fn(rays_o, rays_d, ray_offset) -> (rgb (n,3), depth (n,1)); ray_offset is the global
    index of the first ray (it keys per-ray randomness, so the result does not depend on the
    world size).
    virtual_shards=G (one process only): render the G shards G ranks would render, one after the
    other, and reassemble them as the all-gather would (the 1-GPU "G virtual shards"
    check of the sharding and reassembly of a G-GPU run).
    Returns (rgb (n_frames,H,W,3), depth (n_frames,H,W)) on every rank.  Inference only (no autograd
    graph: the outputs are copied into the reassembly buffer, as the reference renders its frames
    under torch.no_grad(), run.py:217).
    """
    world, rank, collective = _world(group)
    total = n_frames * H * W
    if virtual_shards is not None:
        if world != 1:
            raise ValueError("render_frames_sharded: virtual_shards runs in one process (world size 1)")
        G = int(virtual_shards)
        per = shard_range(total, G, 0)[2]
        out = torch.zeros(G * per, 4, device=device)
        for r in range(G):
            start, end, _ = shard_range(total, G, r)
            _render_shard(ray_fn, render_fn, H, W, n_frames, start, end, out[r * per:(r + 1) * per])
    else:
        start, end, per = shard_range(total, world, rank)
        buf = torch.zeros(per, 4, device=device)
        _render_shard(ray_fn, render_fn, H, W, n_frames, start, end, buf)
        if collective:
            out = torch.empty(world * per, 4, device=buf.device)
            dist.all_gather_into_tensor(out, buf, group=group)
        else:
            out = buf
    frames = out[:total].reshape(n_frames, H, W, 4)
    return frames[..., :3], frames[..., 3]


@torch.no_grad()
def render_path_frames(model, poses, H, W, focal, near, far, n_samples, n_importance=0, appearance_embedding=None,
                       perturb=False, hierarchical=False, seed=0, group=None, timing=None, virtual_shards=None):
    """render_frames_sharded with nerfmi's HIP get_rays / render_rays (one list entry per frame:
    a (3,4)/(4,4) c2w, kept on the host: ray generation takes the pose by value, so no shard
    synchronises on a device-to-host copy).  The in-kernel draws are keyed by `seed` and the global
    ray index, so the frames are bit-identical for every world size.  timing: passed to
    render_rays (per-launch MLP events)."""
    from . import _lib
    from .ray_utils import rays_on_device
    from .render import render_rays
    dev = _lib.device()
    c2ws = [torch.as_tensor(p, dtype=torch.float32).detach().cpu() for p in poses]

    def ray_fn(frame, row0, nrows):
        return rays_on_device(H, W, focal, c2ws[frame], (row0, nrows), dev)

    def render_fn(o, d, offset):
        rgb, depth, _ = render_rays(model, o, d, near, far, n_samples, n_importance,
                                    appearance_embedding=appearance_embedding, perturb=perturb,
                                    hierarchical=hierarchical, seed=int(seed) & (2 ** 62 - 1), ray_offset=offset,
                                    timing=timing)
        return rgb, depth

    return render_frames_sharded(ray_fn, render_fn, H, W, len(c2ws), group=group, device=dev,
                                 virtual_shards=virtual_shards)
