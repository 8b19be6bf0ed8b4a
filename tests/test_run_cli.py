"""run.py (the reference's render CLI, run.py:15-61,63-282) on the host side: flags, scene
metadata fallback, output files.  The GPU render itself is covered in test_gpu_parity.py."""
import os

import numpy as np
import pytest
import torch

import run as cli


def test_flags_match_the_reference():
    a = cli.parse_args(["--mode", "render", "--scene", "chair", "--frames", "3", "--quality", "preview",
                        "--camera_path", "spiral", "--height_range", "-0.2", "0.3", "--save_depth", "--raw_output"])
    assert (a.mode, a.scene, a.frames, a.quality, a.camera_path) == ("render", "chair", 3, "preview", "spiral")
    assert a.height_range == [-0.2, 0.3] and a.save_depth and a.raw_output
    d = cli.parse_args([])
    assert (d.mode, d.scene, d.width, d.height, d.frames, d.quality, d.fps) == ("train", "hotdog", 800, 800, 120,
                                                                               "high", 30)


def test_scene_info_without_dataset(tmp_path):
    import nerfmi
    cfg = nerfmi.Config()
    cfg.dataset_path = str(tmp_path)
    cfg.scene = "chair"
    s = cli.SceneInfo(cfg)
    assert (s.W, s.H, s.near, s.far) == (800, 800, 2.0, 6.0)
    assert abs(s.focal - 1111.1110311937682) < 1e-9
    assert s.appearance_embeddings.shape == (100, 32)


def test_scene_info_reads_transforms(tmp_path):
    import json
    from PIL import Image
    import nerfmi
    d = tmp_path / "lego" / "test"
    d.mkdir(parents=True)
    Image.fromarray(np.zeros((40, 60, 4), np.uint8)).save(d / "r_0.png")
    (tmp_path / "lego" / "transforms_test.json").write_text(
        json.dumps({"camera_angle_x": 0.5, "frames": [{"file_path": "./test/r_0"}] * 7}))
    cfg = nerfmi.Config()
    cfg.dataset_path = str(tmp_path)
    s = cli.SceneInfo(cfg)
    assert (s.W, s.H) == (60, 40) and abs(s.focal - 0.5 * 60 / np.tan(0.25)) < 1e-12
    assert s.appearance_embeddings.shape[0] == 7


def test_write_frame_outputs(tmp_path):
    from PIL import Image
    rgb = torch.rand(12, 16, 3)
    depth = torch.rand(12, 16) * 4 + 2
    cli.write_frame(str(tmp_path), 7, rgb, depth, save_depth=True, raw_output=True)
    img = np.array(Image.open(tmp_path / "rgb_007.png"))
    assert img.shape == (12, 16, 3) and np.array_equal(img, (rgb * 255).numpy().astype(np.uint8))
    assert np.array_equal(np.load(tmp_path / "raw" / "depth_007.npy"), depth.numpy())
    assert (tmp_path / "raw" / "rgb_007.png").exists() and (tmp_path / "depth_007.png").exists()


def test_out_of_scope_modes_say_so(capsys):
    assert cli.main(["--mode", "video"]) == 2
    assert "video" in capsys.readouterr().out


@pytest.mark.gpu
def test_unknown_shader_is_refused(capsys):
    assert cli.main(["--mode", "render", "--random_init", "0", "--shader", "Sepia"]) == 2
    assert "Sepia" in capsys.readouterr().out


@pytest.mark.gpu
def test_render_with_shader_applies_the_effect(tmp_path):
    """--shader Fog writes the GPU Fog of the plain frame, with run.py:248's depth normalisation."""
    from PIL import Image
    from nerfmi.post_processor import PostProcessor, normalize_depth
    base = ["--mode", "render", "--scene", "chair", "--random_init", "0", "--frames", "1", "--width", "40",
            "--height", "24", "--quality", "preview", "--save_depth"]
    plain, fog = str(tmp_path / "plain"), str(tmp_path / "fog")
    assert cli.main(base + ["--output_dir", plain]) == 0
    assert cli.main(base + ["--output_dir", fog, "--shader", "Fog"]) == 0
    img = np.array(Image.open(os.path.join(plain, "rgb_000.png")))
    depth = np.load(os.path.join(plain, "raw", "depth_000.npy"))
    pp = PostProcessor()
    pp.current_effect = "Fog"
    exp = pp.apply_effect(img, normalize_depth(depth))
    assert np.array_equal(np.array(Image.open(os.path.join(fog, "rgb_000.png"))), exp)


@pytest.mark.gpu
def test_train_mode_runs_the_training_loop(tmp_path, monkeypatch):
    """--mode train (run.py:326-347) on the synthetic scene: a few iterations, a final checkpoint in
    train_nerf's default directory 'checkpoints' (train.py:13; run.py:347 passes no save_dir)."""
    monkeypatch.chdir(tmp_path)
    assert cli.main(["--mode", "train", "--scene", "chair", "--iterations", "3", "--random_init", "0"]) == 0
    files = os.listdir(tmp_path / "checkpoints")
    assert any(f.endswith(".pt") for f in files), files


@pytest.mark.gpu
def test_render_mode_end_to_end(tmp_path):
    from PIL import Image
    out = str(tmp_path / "out")
    rc = cli.main(["--mode", "render", "--scene", "chair", "--random_init", "0", "--frames", "2", "--width", "48",
                   "--height", "32", "--quality", "preview", "--output_dir", out, "--save_depth"])
    assert rc == 0
    for i in range(2):
        assert np.array(Image.open(os.path.join(out, f"rgb_{i:03d}.png"))).shape == (32, 48, 3)
        dep = np.load(os.path.join(out, "raw", f"depth_{i:03d}.npy"))
        assert dep.shape == (32, 48) and np.isfinite(dep).all()
    # chunked rendering gives the same frames as whole-frame rendering (preview: no randomness)
    out2 = str(tmp_path / "out2")
    cli.main(["--mode", "render", "--scene", "chair", "--random_init", "0", "--frames", "2", "--width", "48",
              "--height", "32", "--quality", "preview", "--output_dir", out2, "--save_depth", "--chunk", "500"])
    for i in range(2):
        assert np.array_equal(np.load(os.path.join(out, "raw", f"depth_{i:03d}.npy")),
                              np.load(os.path.join(out2, "raw", f"depth_{i:03d}.npy")))
