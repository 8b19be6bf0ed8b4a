"""Child of tests/test_gpu_train.py::test_weight_gradient_kernels_agree: one production-size training
step's gradients (4,096 rays x 64 samples) in this process, whose environment (set by the parent)
selects a weight-gradient variant of libnerfmi (NERFMI_WGRAD_HALF); saves them
for the parent."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def grads(out_path=None, arith=None):
    import nerfmi
    from nerfmi.train import Trainer
    if arith:
        nerfmi.set_mlp_arith(arith)
    torch.manual_seed(0)
    model = nerfmi.NeRF(nerfmi.Config())
    torch.manual_seed(1)
    table = torch.randn(4, 32)
    tr = Trainer(nerfmi.Config(), model=model, appearance_embeddings=table)
    g = torch.Generator().manual_seed(5)
    B = 4096
    o = torch.randn(B, 3, generator=g) * 0.2
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=-1)
    target = torch.rand(B, 3, generator=g)
    t_rand = torch.rand(B, 64, generator=g)
    tr.forward_backward(o.cuda(), d.cuda(), target.cuda(), 1, t_rand=t_rand)
    torch.cuda.synchronize()
    out = {str(i): tr.view(tr.grad, i).detach().cpu().clone() for i in range(25)}
    if out_path:
        torch.save(out, out_path)
    return out


if __name__ == "__main__":
    grads(sys.argv[1], sys.argv[2])
