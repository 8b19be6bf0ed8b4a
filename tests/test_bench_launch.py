"""The benches start their own ranks: `python bench.py --gpus N` (WORLD_SIZE unset) launches N
processes through torch.distributed.run before touching a GPU, and a --gpus that contradicts the
launcher's WORLD_SIZE is an error (nerfmi/launch.py).  Rehearsed on the CPU with --dry-run (gloo
process group, the benches' own shard plan / gradient all-reduce, max-over-ranks timing)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO


def _run(script, *args, world=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    if world is not None:
        env["WORLD_SIZE"] = str(world)
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(REPO, script), *args], capture_output=True, text=True,
                          env=env, timeout=240, cwd="/tmp")


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_bench_gpus_2_launches_two_ranks(scaling):
    r = _run("bench.py", "--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--scaling", scaling)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2 and line["ranks"] == [0, 1] and line["reassembly_ok"]
    assert line["dry_run"] is True and line["scaling"] == scaling


def test_bench_train_gpus_2_launches_two_ranks():
    r = _run("bench_train.py", "--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2 and line["ranks"] == [0, 1] and line["allreduce_ok"]


@pytest.mark.parametrize("script", ["bench.py", "bench_train.py"])
def test_gpus_must_match_world_size(script):
    r = _run(script, "--gpus", "2", "--dry-run", world=1)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
