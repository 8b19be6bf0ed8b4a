"""The RCCL code paths of configs 4 and 5 on the device, at world size 1.

Every multi-GPU collective (frames.py's all_gather_into_tensor of the frame, the trainer's gradient
all_reduce and rank-0 broadcast, the benches' barriers and max-over-ranks timing) runs whenever a
launcher created the process group, world size 1 included (nerfmi.launch.init_ranks).  These tests
start the real launcher (`python -m torch.distributed.run --nproc-per-node 1`) as a child process, so
the "nccl" backend (RCCL on ROCm) initialises on the GPU and carries each collective:
  * bench.py and bench_train.py under the launcher exit 0 and report n_gpus 1, ranks [0] and the
    RCCL group (the driver's N-GPU command line, at N = 1);
  * tests/rccl_world1.py: a hotdog frame (64 + 128 H1, perturbed) gathered through the RCCL group is
    torch.equal to the same frame reassembled without a collective, and Trainer.all_reduce leaves the
    gradients bit-identical (reference: run.py:212-231's chunk loop, src/train.py:77-92)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(args, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}"] + args
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    return p.stdout


def _json_line(stdout, prefix="{"):
    lines = [ln for ln in stdout.splitlines() if ln.startswith(prefix)]
    assert lines, stdout[-2000:]
    return json.loads(lines[-1] if prefix == "{" else lines[-1][len(prefix):])


def test_bench_under_launcher_runs_on_rccl():
    line = _json_line(_torchrun(["bench.py", "--gpus", "1", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]))
    assert line["n_gpus"] == 1 and line["ranks"] == [0], line
    assert line["process_group"] == "nccl (RCCL)" and line["value"] > 0


def test_bench_train_under_launcher_runs_on_rccl():
    line = _json_line(_torchrun(["bench_train.py", "--gpus", "1", "--steps", "2", "--warmup", "1",
                                 "--no-cpu-baseline"]))
    assert line["n_gpus"] == 1 and line["ranks"] == [0], line
    assert line["process_group"] == "nccl (RCCL)" and line["value"] > 0


def test_frame_gather_and_gradient_allreduce_on_rccl():
    r = _json_line(_torchrun([os.path.join("tests", "rccl_world1.py")]), prefix="RCCL_CHECK ")
    assert r["world"] == 1 and r["ranks"] == [0], r
    assert r["frame_finite"] and r["frame_equal"], r
    assert r["grad_nonzero"] and r["allreduce_equal"], r
