"""Drop-in render CLI for the reference's run.py (render path only), on the nerfmi HIP renderer.

    python run.py --mode render --scene chair --checkpoint checkpoints_chair/checkpoint_final.pt
    python run.py --mode render --scene hotdog --random_init 0 --frames 4 --quality preview
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 run.py --mode render ...

Same flags, camera paths (circle / spiral / hemisphere / horizontal_only, run.py:118-147),
quality presets (run.py:88-100) and outputs as the reference's render mode (run.py:63-282):
rgb_{i:03d}.png (uint8 by truncation, run.py:233), a viridis depth_{i:03d}.png
(run.py:271-275), raw/rgb_*.png and raw/depth_*.npy with --raw_output / --save_depth.
Added flags: --random_init SEED renders a seeded random-init model when no checkpoint exists
(none does in this environment); --hierarchical enables the H1 fine pass (the reference
ignores n_importance, render.py:83-86) with --n_importance samples; --chunk renders the frame
in ray chunks (0 = whole frame per call).  Under torchrun every frame is ray-sharded across
the ranks (frames.py) and rank 0 writes the images.
--mode train runs the reference's training loop (run.py:326-347 -> src/train.py) on the nerfmi
kernels (nerfmi.train.train_nerf; the nerf_synthetic scene when present, else the
teacher-rendered synthetic scene), data-parallel under torchrun; --iterations overrides
Config.num_iterations; checkpoints go to --save_dir (default 'checkpoints', the reference's
train_nerf default, while its render mode looks for checkpoints_<scene>/ — a reference
inconsistency kept as is).  --use_shader / --shader NAME applies a depth-aware effect of the
reference's PostProcessor on the GPU (nerfmi.PostProcessor: "Fog", "Toon Shader", "Original") to
each frame before it is written, with run.py:248's depth normalisation; the reference's
interactive first-frame editor (tkinter) is not reproduced, so --shader names the effect
(default with --use_shader alone: Fog).  Out of scope: video encoding (--mode
video, --create_video; cv2 is absent).
Camera metadata: data/nerf_synthetic/<scene>/transforms_test.json when present (focal from
camera_angle_x, dataset.py:66); otherwise the public nerf_synthetic value at 800x800.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='NeRF-W runner (nerfmi HIP renderer)')
    p.add_argument('--mode', type=str, default='train', help='Mode: train, render, or video')
    p.add_argument('--scene', type=str, default='hotdog', help='Scene from NeRF synthetic dataset')
    p.add_argument('--checkpoint', type=str, default=None, help='Checkpoint to load for rendering')
    p.add_argument('--output_dir', type=str, default='output', help='Output directory for renders')
    p.add_argument('--use_shader', action='store_true', help='Enable post-processing effects')
    p.add_argument('--create_video', action='store_true', help='Create a video from rendered images')
    p.add_argument('--fps', type=int, default=30, help='Frames per second for the output video')
    p.add_argument('--input_dir', type=str, default=None, help='Input directory for video creation')
    p.add_argument('--output', type=str, default=None, help='Output path for the video file')
    p.add_argument('--pattern', type=str, default='rgb_*.png', help='Image filename pattern')
    p.add_argument('--shader', type=str, default=None, help='Shader to apply to the rendered images')
    p.add_argument('--width', type=int, default=800, help='Output image width')
    p.add_argument('--height', type=int, default=800, help='Output image height')
    p.add_argument('--frames', type=int, default=120, help='Number of frames to render')
    p.add_argument('--quality', type=str, default='high', choices=['preview', 'medium', 'high'])
    p.add_argument('--start_frame', type=int, default=0, help='First frame to render')
    p.add_argument('--end_frame', type=int, default=None, help='Last frame to render')
    p.add_argument('--save_depth', action='store_true', help='Save depth maps along with RGB images')
    p.add_argument('--raw_output', action='store_true', help='Save raw unprocessed renders')
    p.add_argument('--camera_path', type=str, default='circle',
                   choices=['circle', 'spiral', 'hemisphere', 'horizontal_only'])
    p.add_argument('--spiral_loops', type=float, default=2.0, help='Number of loops in the spiral path')
    p.add_argument('--height_range', type=float, nargs=2, default=[-0.5, 0.5])
    # nerfmi additions
    p.add_argument('--random_init', type=int, default=None, help='render a torch.manual_seed(SEED) random-init model')
    p.add_argument('--hierarchical', action='store_true', help='H1 fine pass with --n_importance samples')
    p.add_argument('--n_importance', type=int, default=None, help='fine samples (default Config.num_importance)')
    p.add_argument('--chunk', type=int, default=0, help='rays per render call (0 = whole frame)')
    p.add_argument('--seed', type=int, default=0, help='seed of the in-kernel sampling RNG')
    p.add_argument('--iterations', type=int, default=None, help='training iterations (default Config)')
    p.add_argument('--save_dir', type=str, default='checkpoints',
                   help="training checkpoint directory (the reference's train_nerf default, train.py:13)")
    return p.parse_args(argv)


class SceneInfo:
    """What render_path needs from NeRFDataset (dataset.py:29-83): W, H, focal, near, far and the
    per-image appearance embeddings."""

    def __init__(self, config, n_images=100):
        from nerfmi import cameras
        self.W = self.H = 800
        self.focal = cameras.synthetic_focal(800)
        meta = os.path.join(config.dataset_path, config.scene, 'transforms_test.json')
        if os.path.exists(meta):
            with open(meta) as f:
                js = json.load(f)
            first = js['frames'][0]['file_path']
            first = first[2:] if first.startswith('./') else first
            png = os.path.join(config.dataset_path, config.scene, first + '.png')
            if os.path.exists(png):
                from PIL import Image
                with Image.open(png) as img:
                    self.W, self.H = img.size
            if 'camera_angle_x' in js:
                self.focal = 0.5 * self.W / np.tan(0.5 * js['camera_angle_x'])
            n_images = len(js['frames'])
        self.near, self.far = config.near, config.far
        self.appearance_embeddings = torch.randn(n_images, config.appearance_dim)


@torch.no_grad()                                   # the reference renders its path under no_grad (run.py:217)
def render_path(model, scene, config, output_dir, num_frames=120, quality='high', width=800, height=800,
                start_frame=0, end_frame=None, save_depth=False, raw_output=False, camera_path='circle',
                spiral_loops=2.0, height_range=(-0.5, 0.5), hierarchical=False, n_importance=None, chunk=0,
                seed=0, shader=None):
    """run.py:63-282 (render mode) on nerfmi."""
    import torch.distributed as dist
    from nerfmi import cameras, frames
    from nerfmi.render import render_rays
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if rank == 0:
        os.makedirs(output_dir, exist_ok=True)
    if quality == 'preview':                      # run.py:88-100
        n_samples, perturb = config.num_samples // 2, False
    else:
        n_samples, perturb = config.num_samples, True
    n_imp = (n_importance if n_importance is not None else config.num_importance) if quality != 'preview' else 0
    if end_frame is None:
        end_frame = num_frames
    theta, heights, phi = cameras.path_angles(camera_path, num_frames, config.scene, spiral_loops, height_range)
    center, up = cameras.scene_center_up(config.scene)
    focal = scene.focal * (width / scene.W)       # run.py:199-200
    app = scene.appearance_embeddings[0] if config.use_appearance else None
    model.eval()
    for i in range(len(theta)):
        frame_idx = start_frame + i
        cam = cameras.camera_position(camera_path, theta[i], heights[i], phi[i])
        c2w = torch.tensor(cameras.look_at_c2w(cam, center, up), dtype=torch.float32)
        kw = dict(appearance_embedding=app, perturb=perturb, hierarchical=hierarchical)
        if world > 1 or not chunk:
            rgb, depth = frames.render_path_frames(model, [c2w], height, width, focal, scene.near, scene.far,
                                                   n_samples, n_imp, seed=seed + frame_idx, **kw)
            rgb, depth = rgb[0], depth[0]
        else:
            from nerfmi import get_rays
            o, d = get_rays(height, width, focal, c2w.cuda())
            o, d = o.reshape(-1, 3), d.reshape(-1, 3)
            outs = [render_rays(model, o[j:j + chunk], d[j:j + chunk], scene.near, scene.far, n_samples, n_imp,
                                seed=seed + frame_idx, ray_offset=j, **kw)[:2]
                    for j in range(0, o.shape[0], chunk)]
            rgb = torch.cat([r for r, _ in outs]).reshape(height, width, 3)
            depth = torch.cat([dd for _, dd in outs]).reshape(height, width)
        if rank != 0:
            continue
        write_frame(output_dir, frame_idx, rgb, depth, save_depth, raw_output, shader)
    if rank == 0:
        print(f"Rendered {len(theta)} frames to {output_dir}")


def write_frame(output_dir, frame_idx, rgb, depth, save_depth=False, raw_output=False, shader=None):
    """Outputs of run.py:233-275 from the frame's device tensors; with `shader`, the effect is
    applied to the written rgb image (not the raw one) after run.py:248's depth normalisation, both
    on the GPU (Fog: nerf_frame_fog, straight from the render outputs)."""
    from PIL import Image
    fogged = None
    if shader == "Fog" and not raw_output:                    # run.py:233 + :248 + Fog in one GPU pass
        from nerfmi.post_processor import PostProcessor, frame_fog
        fogged = frame_fog(rgb, depth, PostProcessor().params["fog_start"]).cpu().numpy()
    rgb, depth = rgb.cpu(), depth.cpu()
    rgb_img = (rgb * 255).numpy().astype(np.uint8)            # truncation, run.py:233
    depth_img = depth.numpy()
    raw_dir = os.path.join(output_dir, 'raw')
    if raw_output or save_depth:
        os.makedirs(raw_dir, exist_ok=True)
    if raw_output:
        Image.fromarray(rgb_img).save(os.path.join(raw_dir, f'rgb_{frame_idx:03d}.png'))
    if save_depth:
        np.save(os.path.join(raw_dir, f'depth_{frame_idx:03d}.npy'), depth_img)
    if fogged is not None:
        rgb_img = fogged
    elif shader and not raw_output:                           # run.py:247-262
        from nerfmi.post_processor import PostProcessor, normalize_depth
        processor = PostProcessor()
        processor.current_effect = shader
        rgb_img = processor.apply_effect(rgb_img, normalize_depth(depth_img))
    Image.fromarray(rgb_img).save(os.path.join(output_dir, f'rgb_{frame_idx:03d}.png'))
    import matplotlib
    matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    h, w = depth_img.shape
    plt.figure(figsize=(w / 100, h / 100), dpi=100)
    plt.imshow(depth_img, cmap='viridis')
    plt.axis('off')
    plt.savefig(os.path.join(output_dir, f'depth_{frame_idx:03d}.png'), bbox_inches='tight', pad_inches=0)
    plt.close()


def model_dimension_check(config):
    """run.py:327-345: the model on 10 random points, without and (with gradients enabled, as the
    reference calls it) with an appearance embedding."""
    import torch.nn.functional as F
    import nerfmi
    model = nerfmi.NeRF(config).cuda()
    x = torch.randn(10, 3).cuda()
    d = F.normalize(torch.randn(10, 3), dim=-1).cuda()
    with torch.no_grad():
        rgb, sigma = model(x, d)
    print(f"Test passed! Output shapes: rgb={tuple(rgb.shape)}, sigma={tuple(sigma.shape)}")
    if config.use_appearance:
        rgb, sigma = model(x, d, torch.randn(1, config.appearance_dim).cuda())
        print(f"Appearance test passed! Output shapes: rgb={tuple(rgb.shape)}, sigma={tuple(sigma.shape)}")
    return rgb, sigma


def main(argv=None):
    args = parse_args(argv)
    import nerfmi
    config = nerfmi.Config()
    config.scene = args.scene
    if args.mode == 'video' or args.create_video:
        print("nerfmi: video encoding is out of scope (post-processing, SURVEY.md §2; cv2 is absent)")
        if args.mode == 'video':
            return 2
    shader = args.shader or ('Fog' if args.use_shader else None)
    if shader:
        from nerfmi.post_processor import PostProcessor
        if shader not in PostProcessor().effects:
            print(f"nerfmi: effect {shader!r} is not on the GPU path; available: {sorted(PostProcessor().effects)}")
            return 2
    import torch.distributed as dist
    from nerfmi import launch
    # under a launcher (WORLD_SIZE set, 1 included): one rank per GPU, RCCL group for the frame
    # all-gather / gradient all-reduce
    world, rank, _, group = launch.init_ranks('nccl')
    if args.mode == 'train':                                           # run.py:326-347
        from nerfmi.dataset import make_dataset
        from nerfmi.train import train_nerf
        np.random.seed(args.seed + rank)
        dataset = make_dataset(config)
        model_dimension_check(config)                                  # run.py:327-345
        torch.manual_seed(args.random_init or 0)
        model = train_nerf(config, dataset, save_dir=args.save_dir, num_iterations=args.iterations,   # run.py:347
                           group=group)
        if group is not None:
            dist.destroy_process_group()
        return 0
    checkpoint = args.checkpoint
    if not checkpoint and args.random_init is None:
        default = f"checkpoints_{args.scene}/checkpoint_final.pt"     # run.py:351-359
        if os.path.exists(default):
            checkpoint = default
            print(f"Using default checkpoint: {checkpoint}")
        else:
            print(f"No checkpoint specified and default not found at {default}")
            print("Please specify a checkpoint file using --checkpoint (or --random_init SEED)")
            return 1
    torch.manual_seed(args.random_init or 0)
    model = nerfmi.NeRF(config)
    scene = SceneInfo(config)
    if checkpoint:
        ckpt = torch.load(checkpoint, map_location='cpu', weights_only=True)
        model.load_state_dict(ckpt['model_state_dict'])                # run.py:361-366
        if config.use_appearance and ckpt.get('appearance_embeddings') is not None:
            scene.appearance_embeddings = ckpt['appearance_embeddings']
    model = model.cuda()
    with torch.no_grad():
        render_path(model, scene, config, args.output_dir, num_frames=args.frames, quality=args.quality,
                    width=args.width, height=args.height, start_frame=args.start_frame, end_frame=args.end_frame,
                    save_depth=args.save_depth, raw_output=args.raw_output, camera_path=args.camera_path,
                    spiral_loops=args.spiral_loops, height_range=args.height_range,
                    hierarchical=args.hierarchical, n_importance=args.n_importance, chunk=args.chunk,
                    seed=args.seed, shader=shader)
    if group is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
