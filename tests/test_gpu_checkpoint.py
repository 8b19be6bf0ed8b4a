"""Drop-in contract of the training entry points on the GPU:
train_nerf on a nerf_synthetic-style PNG scene returns the model (src/train.py:207), trains the
dataset's appearance table in place (train.py:36-39), writes the checkpoints and validation
renders of train.py:112-187; the checkpoint loads into torch.optim.Adam and renders through
run.py --checkpoint exactly as render_rays renders the trained weights; the use_appearance=False
model (models.py:99-103) against fixture F8."""
import os

import numpy as np
import pytest
import torch

import nerfmi
from oracle import nerf_oracle as O
from test_dataset import _config, write_synthetic_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def trained(tmp_path_factory):
    from nerfmi.dataset import NeRFDataset
    from nerfmi.train import train_nerf
    root = tmp_path_factory.mktemp("scene")
    write_synthetic_scene(root, n=4, H=24, W=24, seed=2)
    cfg = _config(root, batch_size=256)
    np.random.seed(0)
    torch.manual_seed(0)
    ds = NeRFDataset(cfg)
    table0 = ds.appearance_embeddings.detach().clone()
    save = str(root / "ckpt")
    model = train_nerf(cfg, ds, save_dir=save, num_iterations=4, checkpoint_every=2, seed=1, log_every=0)
    return dict(cfg=cfg, ds=ds, table0=table0, save=save, model=model)


def test_train_nerf_returns_model_and_writes_outputs(trained):
    from nerfmi.train import train_nerf
    model, save = trained["model"], trained["save"]
    assert isinstance(model, nerfmi.NeRF)                                          # train.py:207
    files = set(os.listdir(save))
    for f in ("checkpoint_000002.pt", "checkpoint_000004.pt", "render_000002.png", "render_000004.png",
              "checkpoint_final.pt", "training_curves.png"):
        assert f in files, (f, files)
    assert len(train_nerf.losses) == 4 and np.all(np.isfinite(train_nerf.losses))
    ck = torch.load(os.path.join(save, "checkpoint_final.pt"), map_location="cpu", weights_only=True)
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "loss", "psnr", "iteration",
                       "appearance_embeddings"}
    assert ck["iteration"] == 4 and ck["loss"] == train_nerf.losses[-1]
    for k, v in model.state_dict().items():
        assert torch.equal(ck["model_state_dict"][k], v.cpu()), k


def test_appearance_table_trained_in_place(trained):
    ds = trained["ds"]
    tab = ds.appearance_embeddings
    assert isinstance(tab, torch.nn.Parameter)
    assert not torch.equal(tab.detach().cpu(), trained["table0"])       # Adam moved it
    ck = torch.load(os.path.join(trained["save"], "checkpoint_final.pt"), map_location="cpu", weights_only=True)
    assert torch.equal(ck["appearance_embeddings"], tab.detach().cpu())


def test_checkpoint_loads_into_torch_adam(trained):
    """The optimizer_state_dict is torch.optim.Adam's own layout (train.py:116,178): a torch Adam
    over model.parameters() + [appearance table] loads it, and one more torch step from it
    matches one more nerfmi step on the same gradients."""
    cfg = trained["cfg"]
    ck = torch.load(os.path.join(trained["save"], "checkpoint_final.pt"), map_location="cpu", weights_only=True)
    m = nerfmi.NeRF(cfg)
    m.load_state_dict(ck["model_state_dict"])
    tab = torch.nn.Parameter(ck["appearance_embeddings"].clone())
    params = list(m.parameters()) + [tab]
    opt = torch.optim.Adam(params, lr=cfg.learning_rate)
    opt.load_state_dict(ck["optimizer_state_dict"])
    for p in params:
        st = opt.state[p]
        assert st["exp_avg"].shape == p.shape and float(st["step"]) == 4.0
    # continue both optimizers one step on the same synthetic gradients
    from nerfmi.train import Trainer
    tr = Trainer(cfg, model=nerfmi.NeRF(cfg), appearance_embeddings=torch.zeros_like(tab))
    with torch.no_grad():
        for i, k in enumerate(O.STATE_KEYS):
            tr.view(tr.flat, i).copy_(ck["model_state_dict"][k])
        tr.view(tr.flat, 24).copy_(tab)
    tr.load_optimizer_state_dict(ck["optimizer_state_dict"])
    g = torch.Generator().manual_seed(3)
    grads = [torch.randn(p.shape, generator=g) * 1e-3 for p in params]
    for p, gr in zip(params, grads):
        p.grad = gr.clone()
    opt.step()
    with torch.no_grad():
        for slot, gr in zip(tr.param_slots, grads):
            tr.view(tr.grad, slot).copy_(gr)
    tr.optimizer_step()
    torch.cuda.synchronize()
    for slot, p in zip(tr.param_slots, params):
        np.testing.assert_allclose(tr.view(tr.flat, slot).cpu().numpy(), p.detach().numpy(), rtol=1e-6, atol=1e-7)


def test_run_py_renders_the_checkpoint_like_render_rays(trained, tmp_path):
    """run.py --checkpoint (run.py:361-366) renders the trained weights exactly as render_rays
    does on the same rays: the raw depth bit for bit, the uint8 rgb identical."""
    from PIL import Image
    import run as cli
    from nerfmi import cameras, get_rays, render_rays
    ckpt = os.path.join(trained["save"], "checkpoint_final.pt")
    out = str(tmp_path / "out")
    assert cli.main(["--mode", "render", "--scene", "chair", "--checkpoint", ckpt, "--frames", "1", "--width", "40",
                     "--height", "24", "--quality", "preview", "--output_dir", out, "--raw_output",
                     "--save_depth"]) == 0
    ck = torch.load(ckpt, map_location="cpu", weights_only=True)
    m = nerfmi.NeRF(nerfmi.Config())
    m.load_state_dict(ck["model_state_dict"])
    m = m.cuda()
    c2w = torch.tensor(cameras.look_at_c2w(cameras.camera_position("circle", *[a[0] for a in cameras.path_angles(
        "circle", 1, "chair")]), *cameras.scene_center_up("chair")), dtype=torch.float32)
    focal = cameras.synthetic_focal(800) * (40 / 800)
    o, d = get_rays(24, 40, focal, c2w.cuda())
    with torch.no_grad():
        rgb, depth, _ = render_rays(m, o.reshape(-1, 3), d.reshape(-1, 3), 2.0, 6.0, 32, 0,
                                    appearance_embedding=ck["appearance_embeddings"][0].cuda(), perturb=False)
    dep = np.load(os.path.join(out, "raw", "depth_000.npy"))
    assert np.array_equal(dep, depth.reshape(24, 40).cpu().numpy())
    img = np.array(Image.open(os.path.join(out, "raw", "rgb_000.png")))
    assert np.array_equal(img, (rgb.reshape(24, 40, 3).cpu() * 255).numpy().astype(np.uint8))


def test_validation_render_matches_volume_render(trained, tmp_path):
    from nerfmi.render import volume_render
    from nerfmi.train import validation_render
    ds, cfg, model = trained["ds"], trained["cfg"], trained["model"]
    rgb, depth = validation_render(model, ds, cfg, 7, str(tmp_path))
    assert os.path.exists(tmp_path / "render_000007.png")
    val = ds.get_rays(idx=len(ds) - 1)
    args = (model, val["rays_o"][:1000], val["rays_d"][:1000], 2.0, 6.0, cfg.num_samples, 0)
    kw = dict(appearance_embedding=ds.appearance_embeddings[len(ds) - 1], perturb=False)
    with torch.no_grad():                              # (train.py:128-140 renders under no_grad)
        r2, d2, _ = volume_render(*args, **kw)
    assert rgb.shape == (576, 3)                       # the first 1000 rays of a 24x24 image: all 576
    assert torch.equal(rgb, r2) and torch.equal(depth, d2)
    # With gradients enabled the same call takes the differentiable path, whose forward is the
    # training kernel (32 x 32 MFMA tiles; the render kernel runs 16 x 16 x 32): the same
    # arithmetic with the products summed in another order inside the MFMA, so equal to fp32 rounding
    r3, d3, _ = volume_render(*args, **kw)
    assert torch.allclose(r3, r2, rtol=1e-5, atol=1e-6) and torch.allclose(d3, d2, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("arith", ["f16x3", "f32"])
def test_no_appearance_model_matches_f8(golden, noapp_state, arith):
    from nerfmi import _lib as L
    prev = L.set_mlp_arith(arith)
    try:
        f8 = golden("f8_no_appearance.npz")
        cfg = nerfmi.Config()
        cfg.use_appearance = False
        torch.manual_seed(0)
        m = nerfmi.NeRF(cfg).cuda().eval()
        app = torch.from_numpy(f8["app"]).cuda()
        with torch.no_grad():
            rgb, sigma = m(torch.from_numpy(f8["x"]).cuda(), torch.from_numpy(f8["d"]).cuda(), app)
        np.testing.assert_allclose(rgb.cpu().numpy(), f8["rgb"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(sigma.cpu().numpy(), f8["sigma"], rtol=1e-4, atol=1e-6)
        f1 = golden("f1_get_rays.npz")
        o, d = torch.from_numpy(f1["chair_o"][:512]).cuda(), torch.from_numpy(f1["chair_d"][:512]).cuda()
        with torch.no_grad():
            rgb, depth, _ = nerfmi.render_rays(m, o, d, 2.0, 6.0, 64, 0, appearance_embedding=app, perturb=False)
        np.testing.assert_allclose(rgb.cpu().numpy(), f8["render_rgb"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(depth.cpu().numpy(), f8["render_depth"], rtol=1e-4, atol=1e-6)
    finally:
        L.set_mlp_arith(prev)
