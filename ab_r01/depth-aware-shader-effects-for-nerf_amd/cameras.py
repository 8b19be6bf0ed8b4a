"""Camera poses for the render driver: look-at c2w matrices and camera paths.

Restates the host-side pose logic of ``/root/reference/run.py``:
  * scene look-at centre / up vector          run.py:106-116
  * circle / spiral / horizontal_only / hemisphere paths   run.py:118-147
  * radius 4.0                                 run.py:149
  * camera position per frame                  run.py:168-180
  * look-at basis and c2w assembly             run.py:182-197
The arithmetic stays in float64 numpy exactly as the reference does and is cast
to float32 only when the matrix becomes a tensor (run.py:197).

There is no dataset in this environment.  The focal length of
the public nerf_synthetic scenes follows ``dataset.py:66`` with the published
``camera_angle_x``; ``synthetic_focal`` restates it.
"""
import numpy as np
import torch

# transforms_*.json "camera_angle_x" of the Blender nerf_synthetic scenes.
NERF_SYNTHETIC_CAMERA_ANGLE_X = 0.6911112070083618
RADIUS = 4.0  # run.py:149


def synthetic_focal(width=800, camera_angle_x=NERF_SYNTHETIC_CAMERA_ANGLE_X):
    """focal = 0.5 W / tan(0.5 camera_angle_x)   (dataset.py:66)."""
    return 0.5 * width / np.tan(0.5 * camera_angle_x)


def scene_center_up(scene):
    """Look-at centre and up vector per scene (run.py:106-116)."""
    center = np.array([0, 0, 0])
    up = np.array([0, 1, 0])
    if scene == 'lego':
        center = np.array([0, 0.5, 0])
        up = np.array([0, 0, 1])
    elif scene == 'chair':
        center = np.array([0, 0.5, 0])
    return center, up


def path_angles(camera_path, num_frames, scene, spiral_loops=2.0,
                height_range=(-0.5, 0.5)):
    """(theta, heights, phi) arrays of a camera path (run.py:118-147)."""
    if camera_path == 'circle':
        theta = np.linspace(0, 2 * np.pi, num_frames)
        heights = np.zeros_like(theta) + 0.5 if scene == 'lego' else np.zeros_like(theta)
        phi = np.zeros_like(theta)
    elif camera_path == 'spiral':
        theta = np.linspace(0, 2 * np.pi * spiral_loops, num_frames)
        if scene == 'lego':
            height_range = [0.3, 0.7]
        heights = np.linspace(height_range[0], height_range[1], num_frames)
        phi = np.zeros_like(theta)
    elif camera_path == 'horizontal_only':
        theta = np.linspace(0, 2 * np.pi * spiral_loops, num_frames)
        heights = np.full_like(theta, 0.5)
        phi = np.zeros_like(theta)
    elif camera_path == 'hemisphere':
        indices = np.arange(0, num_frames, dtype=float) + 0.5
        phi = np.arccos(1 - 2 * indices / num_frames) - np.pi / 2
        theta = np.pi * (1 + 5 ** 0.5) * indices
        heights = np.zeros_like(theta)
    else:
        raise ValueError(f"unknown camera_path {camera_path!r}")
    return theta, heights, phi


def camera_position(camera_path, angle, height, phi, radius=RADIUS):
    """run.py:168-180."""
    if camera_path in ('circle', 'spiral', 'horizontal_only'):
        return np.array([radius * np.sin(angle), height, radius * np.cos(angle)])
    return np.array([radius * np.cos(phi) * np.sin(angle),
                     radius * np.sin(phi),
                     radius * np.cos(phi) * np.cos(angle)])


def look_at_c2w(cam_pos, center, up):
    """4x4 float64 camera-to-world matrix (run.py:182-195)."""
    forward = center - cam_pos
    forward = forward / np.linalg.norm(forward)
    right = np.cross(forward, up)
    right = right / np.linalg.norm(right)
    camera_up = np.cross(right, forward)
    camera_up = camera_up / np.linalg.norm(camera_up)
    c2w = np.eye(4)
    c2w[:3, 0] = right
    c2w[:3, 1] = camera_up
    c2w[:3, 2] = -forward
    c2w[:3, 3] = cam_pos
    return c2w


def frame_c2w(scene, camera_path='circle', frame=0, num_frames=120,
              spiral_loops=2.0, height_range=(-0.5, 0.5)):
    """float32 c2w tensor of one frame of a render path (run.py:165-197)."""
    theta, heights, phi = path_angles(camera_path, num_frames, scene,
                                      spiral_loops, height_range)
    center, up = scene_center_up(scene)
    cam_pos = camera_position(camera_path, theta[frame], heights[frame], phi[frame])
    return torch.tensor(look_at_c2w(cam_pos, center, up), dtype=torch.float32)
