"""Diagnostic (GPU): gradient error of NeRF.forward's training kernels against float64 on each ReLU branch.

For the adversarial weights of tests/test_gpu_accuracy.py (and seed-0 weights), under both MLP
arithmetics: per parameter tensor, the GPU's rel-L2 error against float64 autograd evaluated (a) on
float64's own branches, (b) on the GPU's branches (masks from the GPU forward's saved activations),
(c) on the CPU fp32's branches; the CPU fp32's error likewise; and the number of ReLU decisions per
layer where the GPU, the CPU fp32 and float64 disagree.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import nerfmi
    from nerfmi import _lib
    from oracle import nerf_oracle as O
    from test_gpu_accuracy import adversarial_state, gpu_relu_masks
    ref = O.random_state(0)
    torch.manual_seed(1)
    app = torch.randn(100, 32)[0]
    modes = os.environ.get("DIAG_MODES", "f16x3,f32,f16x3>f32").split(",")
    for which, st in (("seed0", ref), ("adversarial", adversarial_state(ref))):
        for mode in modes:     # "a>b": forward under a, backward under b
            arith, bw = (mode.split(">") + [None])[:2]
            _lib.set_mlp_arith(arith)
            model = nerfmi.NeRF(nerfmi.Config())
            model.load_state_dict(st)
            model = model.cuda()
            g = torch.Generator().manual_seed(13)
            M = 8192
            x = torch.rand(M, 3, generator=g) * 3 - 1.5
            d = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
            g_rgb, g_sig = torch.randn(M, 3, generator=g), torch.randn(M, 1, generator=g)
            rgb, sigma = model(x.cuda(), d.cuda(), app.cuda())
            if bw:
                _lib.set_mlp_arith(bw)
            ((rgb * g_rgb.cuda()).sum() + (sigma * g_sig.cuda()).sum()).backward()
            _lib.set_mlp_arith(arith)
            with torch.no_grad():
                m_gpu = gpu_relu_masks(model, x.cuda(), d.cuda(), app)

            def ref_grads(dtype, masks=None, record=None):
                sd = {k: v.detach().clone().to(dtype).requires_grad_(True) for k, v in st.items()}

                def relu(pre, i):
                    if record is not None:
                        record.append(pre.detach() > 0)
                    return torch.relu(pre) if masks is None else pre * masks[i].to(dtype)
                with torch.enable_grad():
                    r, s = O.nerf_forward(sd, x.to(dtype), d.to(dtype), app.to(dtype), relu=relu)
                    ((r * g_rgb.to(dtype)).sum() + (s * g_sig.to(dtype)).sum()).backward()
                return {k: v.grad.double() for k, v in sd.items()}

            m_cpu, m64 = [], []
            g32 = ref_grads(torch.float32, record=m_cpu)
            g64 = ref_grads(torch.float64, record=m64)
            g64_gpu, g64_cpu = ref_grads(torch.float64, masks=m_gpu), ref_grads(torch.float64, masks=m_cpu)

            def rel(a, b):
                return float((a - b).norm() / (b.norm() + 1e-300))
            print(f"== {which} {mode}: ReLU decisions GPU!=f64 per layer {[int((a != b).sum()) for a, b in zip(m_gpu, m64)]}"
                  f" CPU!=f64 {[int((a != b).sum()) for a, b in zip(m_cpu, m64)]}")
            for k, p in model.named_parameters():
                gg = p.grad.cpu().double()
                print(f"  {k:32s} gpu: own-f64 {rel(gg, g64[k]):.3g} gpu-branch {rel(gg, g64_gpu[k]):.3g} "
                      f"cpu-branch {rel(gg, g64_cpu[k]):.3g} | cpu32: own-f64 {rel(g32[k], g64[k]):.3g} "
                      f"cpu-branch {rel(g32[k], g64_cpu[k]):.3g}")


if __name__ == "__main__":
    main()
