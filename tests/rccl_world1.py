"""Child of tests/test_gpu_rccl.py, started by torch.distributed.run with one rank on the GPU: the
RCCL ("nccl") group exists at world size 1 and the device collectives of the render and training
paths run through it.  Prints one line "RCCL_CHECK {json}"."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import torch.distributed as dist
    from nerfmi import launch
    world, rank, local, group = launch.init_ranks("nccl")
    assert group is not None and dist.get_backend(group) == "nccl", dist.get_backend(group)
    import nerfmi
    from nerfmi import cameras, frames
    from nerfmi.dataset import SyntheticNeRFDataset
    from nerfmi.train import Trainer
    out = {"world": world, "rank": rank, "ranks": launch.rank_list(group)}
    # config 4's path (run.py:212-231 as frames.py shards it): the hotdog frame, 64 + 128 H1, perturbed,
    # with the all-gather over the RCCL group against the same frame reassembled without a collective
    torch.manual_seed(0)
    model = nerfmi.NeRF(nerfmi.Config()).cuda().eval()
    torch.manual_seed(1)
    app = torch.randn(100, 32)[0].cuda()
    pose = cameras.frame_c2w("hotdog")
    H = W = 96
    kw = dict(appearance_embedding=app, perturb=True, hierarchical=True, seed=7)
    focal = cameras.synthetic_focal(W)
    rgb_g, depth_g = frames.render_path_frames(model, [pose], H, W, focal, 2.0, 6.0, 64, 128, group=group, **kw)
    rgb_n, depth_n = frames.render_path_frames(model, [pose], H, W, focal, 2.0, 6.0, 64, 128, virtual_shards=1, **kw)
    out["frame_equal"] = bool(torch.equal(rgb_g, rgb_n) and torch.equal(depth_g, depth_n))
    out["frame_finite"] = bool(torch.isfinite(rgb_g).all() and torch.isfinite(depth_g).all())
    # config 5's exchange: Trainer.all_reduce over the RCCL group leaves world-1 gradients unchanged
    import numpy as np
    cfg = nerfmi.Config()
    np.random.seed(0)
    ds = SyntheticNeRFDataset(cfg, n_images=2, H=64, W=64)
    torch.manual_seed(0)
    tr = Trainer(cfg, appearance_embeddings=ds.appearance_embeddings, group=group)
    b = ds.get_rays(batch_size=1024)
    tr.forward_backward(b["rays_o"], b["rays_d"], b["rgb"], b["appearance_idx"], seed=1)
    before = tr.grad.detach().clone()
    tr.all_reduce()
    torch.cuda.synchronize()
    out["allreduce_equal"] = bool(torch.equal(before, tr.grad))
    out["grad_nonzero"] = bool(before.abs().sum() > 0)
    dist.destroy_process_group()
    print("RCCL_CHECK " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
