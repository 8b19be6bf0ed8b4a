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
