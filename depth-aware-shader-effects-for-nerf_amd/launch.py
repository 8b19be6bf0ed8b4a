"""One process per GPU for the benches: `python bench.py --gpus N` starts its own N ranks.

The driver launches the N-GPU bench as `python -m torch.distributed.run --nproc-per-node N ...
bench.py --gpus N` (WORLD_SIZE set by the launcher); run by hand as `python bench.py --gpus N`, the
bench starts that same launcher as a child process and exits with its status.  The parent never
initialises the GPU (no HIP call before the child exists; counting devices does not initialise it
on this image), so nothing is exec'd from a process that holds the device.
"""
import os
import socket
import subprocess
import sys


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def under_launcher():
    """True when a launcher started this process: WORLD_SIZE plus a rendezvous marker
    (torch.distributed.run's TORCHELASTIC_RUN_ID, or MASTER_ADDR and MASTER_PORT).  A WORLD_SIZE left
    over in the environment without one (a scheduler export, a parent shell) does not count: the
    process runs alone instead of waiting on an env:// rendezvous nobody serves."""
    if os.environ.get("WORLD_SIZE") is None:
        return False
    if os.environ.get("TORCHELASTIC_RUN_ID") or (os.environ.get("MASTER_ADDR") and os.environ.get("MASTER_PORT")):
        return True
    sys.stderr.write("nerfmi.launch: WORLD_SIZE is set but no launcher marker (TORCHELASTIC_RUN_ID or "
                     "MASTER_ADDR/MASTER_PORT) is: running as a single process without a process group\n")
    return False


def world_or_launch(gpus, script, argv, check_devices=True):
    """Return None when this process is a rank that should run (WORLD_SIZE == gpus, or a 1-GPU run),
    or an exit status: the launched ranks' status, or 2 when --gpus contradicts WORLD_SIZE or the
    node has fewer GPUs than asked for."""
    env_world = os.environ.get("WORLD_SIZE") if under_launcher() else None
    if env_world is not None:
        if int(env_world) != gpus:
            sys.stderr.write(f"{os.path.basename(script)}: --gpus {gpus} but WORLD_SIZE={env_world}: "
                             f"the launcher and the flag must agree\n")
            return 2
        return None
    if gpus <= 1:
        return None
    if check_devices:
        import torch
        have = torch.cuda.device_count()
        if have < gpus:
            sys.stderr.write(f"{os.path.basename(script)}: --gpus {gpus} but {have} GPU(s) visible\n")
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", script] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def init_ranks(backend="nccl"):
    """(world, rank, local_rank, group) of this process.  Under a launcher (`under_launcher()`, world 1
    included) the device is set to LOCAL_RANK and the process group is initialised on `backend`
    ("nccl" = RCCL over xGMI on ROCm), so the collectives of the benches and the CLI run on the
    device even on one GPU; a plain `python bench.py` has no group (None) and runs no collective."""
    import torch
    import torch.distributed as dist
    if not under_launcher():
        return 1, 0, 0, None
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return world, rank, local, dist.group.WORLD


def rank_list(group):
    """Every rank's global rank as the group sees it (all_gather_object): [0] alone."""
    if group is None:
        return [0]
    import torch.distributed as dist
    got = [None] * dist.get_world_size(group)
    dist.all_gather_object(got, dist.get_rank(), group=group)
    return got
