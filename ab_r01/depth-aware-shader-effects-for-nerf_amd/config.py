"""Hyper-parameters that fix the hot path's shapes.

Mirrors ``/root/reference/config.py:3-36`` attribute for attribute (class
attributes, overridable per instance), so ``NeRF(Config())`` builds the same
layer stack and ``volume_render`` sees the same near/far/sample counts.
"""
import torch


class Config:
    # Dataset parameters (config.py:5-7)
    dataset_type = 'nerf_synthetic'
    dataset_path = 'data/nerf_synthetic'
    scene = 'lego'

    # Model parameters (config.py:10-14)
    hidden_dim = 256
    num_layers = 8
    skip_connect_layers = [4]
    num_samples = 64        # coarse samples per ray
    num_importance = 64     # fine samples per ray (BASELINE.json quotes 128)

    # Appearance embedding (config.py:17-18)
    use_appearance = True
    appearance_dim = 32

    # Training parameters (config.py:21-25)
    batch_size = 1024
    learning_rate = 5e-4
    num_iterations = 30000
    scheduler_step_size = 10000
    scheduler_gamma = 0.5

    # Bounds for synthetic scenes (config.py:28-29)
    near = 2.0
    far = 6.0

    # Encoding parameters (config.py:32-33)
    pos_enc_levels = 10
    dir_enc_levels = 4

    # Device (config.py:36).  Counting devices does not initialise HIP.
    device = torch.device("cuda" if torch.cuda.device_count() > 0 else "cpu")
