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


def _run(script, *args, world=None, marker=True, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    if world is not None:
        env["WORLD_SIZE"] = str(world)
        if marker:                     # as a launcher sets it
            env["MASTER_ADDR"], env["MASTER_PORT"] = "127.0.0.1", "29999"
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(REPO, script), *args], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd="/tmp")


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


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_bench_gpus_8_plan(scaling):
    """The driver's 8-GPU SCALE run, rehearsed: 8 gloo ranks through the real launcher, 800x800
    frames, bench.workload's poses and frames.render_frames_sharded's plan.  Strong scaling (BASELINE
    config 4) gives every rank 100 rows of the one frame; weak scaling one whole frame per rank; the
    reassembled frames are bit-exact in ray order on every rank (the stand-in renderer's depth is the
    global ray index mod 997)."""
    r = _run("bench.py", "--gpus", "8", "--dry-run", "--dry-size", "800", "--steps", "1", "--warmup", "1",
             "--scaling", scaling, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 8 and line["ranks"] == list(range(8)) and line["reassembly_ok"]
    assert len(line["rank_ms"]) == 8 and line["ms_per_step"] == pytest.approx(max(line["rank_ms"]))
    if scaling == "strong":
        assert line["rows_per_rank"] == [100.0] * 8
        assert line["shards"] == [[k * 80_000, (k + 1) * 80_000] for k in range(8)]
    else:
        assert line["rows_per_rank"] == [800.0] * 8
        assert line["shards"] == [[k * 640_000, (k + 1) * 640_000] for k in range(8)]


def test_bench_train_gpus_8_plan():
    r = _run("bench_train.py", "--gpus", "8", "--dry-run", "--steps", "2", "--warmup", "1", timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 8 and line["ranks"] == list(range(8)) and line["allreduce_ok"]
    assert len(line["rank_ms"]) == 8


def test_leftover_world_size_runs_alone():
    """A WORLD_SIZE left in the environment without a launcher's rendezvous marker does not make the
    bench wait on an env:// rendezvous: it runs as one process (nerfmi.launch.under_launcher)."""
    r = _run("bench.py", "--gpus", "1", "--dry-run", "--steps", "1", "--warmup", "0", world=1, marker=False)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "no launcher marker" in r.stderr
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 1 and line["ranks"] == [0]
