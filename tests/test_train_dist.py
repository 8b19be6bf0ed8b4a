"""Data-parallel training sync (train.py average_gradients) on CPU with gloo, world_size 2.

Each rank computes the gradients of half the batch with the oracle's autograd (the HIP path needs
a GPU; what is tested here is the data-parallel arithmetic the product uses), flattens them the
way nerfmi.train.Trainer lays out its gradient buffer, and calls the product's
average_gradients.  The result must be the full-batch gradient of the single-process step: the
mean-loss gradient of the union of the ranks' batches."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import nerf_oracle as O
from nerfmi import cameras
from nerfmi.train import average_gradients


def batch():
    focal = cameras.synthetic_focal(800)
    c2w = cameras.frame_c2w("chair", "circle", 3, 120).float()
    o, d = O.get_rays(800, 800, focal, c2w)
    g = torch.Generator().manual_seed(5)
    sel = torch.randperm(800 * 800, generator=g)[:64]
    return (o.reshape(-1, 3)[sel], d.reshape(-1, 3)[sel], torch.rand(64, 3, generator=g),
            torch.rand(64, 16, generator=g))


def flat_grads(o, d, target, t_rand):
    state = O.random_state(0)
    torch.manual_seed(1)
    table = torch.randn(4, 32)
    _, _, grads, _ = O.train_step(state, table, 2, o, d, target, 2.0, 6.0, 16, t_rand)
    return torch.cat([grads[k].reshape(-1) for k in list(O.STATE_KEYS) + ["appearance_embeddings"]])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o, d, target, t_rand = batch()
        half = slice(32 * rank, 32 * (rank + 1))
        g = flat_grads(o[half], d[half], target[half], t_rand[half])
        average_gradients(g, dist.group.WORLD)
        if rank == 0:
            torch.save(g, out)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_world2_average_is_the_full_batch_gradient(tmp_path):
    o, d, target, t_rand = batch()
    full = flat_grads(o, d, target, t_rand)
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert got.shape == full.shape
    assert torch.allclose(got, full, rtol=1e-4, atol=1e-9)


def test_single_process_sync_is_identity():
    g = torch.arange(10.0)
    average_gradients(g, None)
    assert torch.equal(g, torch.arange(10.0))


def _worker_broadcast(rank, world, port, out):
    """Ranks built from different seeds (as ranks that load different checkpoints or reach the
    constructor with different RNG states would): after broadcast_state every rank holds rank 0's
    flat buffer, and one averaged-gradient Adam step keeps them identical."""
    from nerfmi.train import broadcast_state
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(100 + rank)
        flat = torch.randn(1000)
        broadcast_state([flat], dist.group.WORLD)
        p = torch.nn.Parameter(flat.clone())
        opt = torch.optim.Adam([p], lr=1e-3)
        g = torch.randn(1000)              # each rank's own (different) gradient
        average_gradients(g, dist.group.WORLD)
        p.grad = g
        opt.step()
        torch.save(p.detach(), f"{out}.{rank}")
    finally:
        dist.destroy_process_group()


def test_world2_ranks_start_from_rank0_and_stay_identical(tmp_path):
    out = str(tmp_path / "p")
    mp.spawn(_worker_broadcast, args=(2, _free_port(), out), nprocs=2, join=True)
    p0, p1 = torch.load(out + ".0", weights_only=True), torch.load(out + ".1", weights_only=True)
    assert torch.equal(p0, p1)
    torch.manual_seed(100)
    start = torch.randn(1000)
    assert not torch.equal(p0, start) and (p0 - start).abs().max() <= 1.01e-3


def test_step_seeds_differ_per_rank_and_step():
    from nerfmi.train import step_seed
    seeds = {step_seed(i, r) for i in range(1, 50) for r in range(8)}
    assert len(seeds) == 49 * 8
