"""Generate tests/golden/f9_fog.npz: the reference's own Fog effect on synthetic frames.

Runs ONLY in the build container, where the reference is mounted read-only at /root/reference.
src/post_processor.py imports cv2 and tkinter at module level (post_processor.py:2-4), neither of
which is installed, so the module cannot be imported.  Its Fog effect (`_effect_fog`,
post_processor.py:451-493) uses numpy alone: this script parses the module with `ast`, compiles
that one method by itself in a namespace holding only numpy, and calls it on a stand-in `self` that
carries the reference's default parameter table (post_processor.py:33-55, read from the same
parse).  Nothing else of the module is executed.  What gets committed is data: the inputs and the
reference's outputs, never reference code.

    python tests/golden/make_post_golden.py         # rewrites tests/golden/f9_fog.npz

Cases (uint8 RGB frame, float32 depth; params = the reference defaults unless noted):
  norm    depth already in [0, 1] (run.py:248's normalisation), fog_start 0.1
  raw     raw depth (max > 1: the method divides by its max)
  chan    raw depth with 3 channels (the method takes channel 0)
  edges   depth exactly 0, fog_start, 1 and their float32 neighbours
  start0  fog_start 0.0
  start35 fog_start 0.35
  none    depth None (the uniform 5 % visibility branch)
Also stored per depth case: `cube_differs`, the pixels where this host's numpy float32 pow
(`adjusted ** 3.0`, post_processor.py:480) differs from the correctly rounded cube the kernel
computes (oracle/post_oracle.py cube_rn): only there may a kernel value differ from the reference's.
"""
import ast
import contextlib
import io
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
REF_FILE = "/root/reference/src/post_processor.py"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import post_oracle as P     # noqa: E402  (cube_rn and the restated normalisation)


def reference_fog_and_params():
    tree = ast.parse(open(REF_FILE).read(), REF_FILE)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "PostProcessor")
    fog = next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "_effect_fog")
    init = next(n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "__init__")
    params = None
    for node in ast.walk(init):
        if (isinstance(node, ast.Assign) and isinstance(node.targets[0], ast.Attribute)
                and node.targets[0].attr == "params"):
            params = ast.literal_eval(node.value)
    ns = {"np": np}
    exec(compile(ast.Module(body=[fog], type_ignores=[]), REF_FILE, "exec"), ns)
    return ns["_effect_fog"], params


class _Self:
    def __init__(self, params):
        self.params = params


def frame(H, W, seed):
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.stack([(xx / W) * 255, (yy / H) * 255, 128 + 100 * np.sin(xx / 7 + yy / 11)], -1)
    img = np.clip(img + g.normal(0, 6, img.shape), 0, 255).astype(np.uint8)
    img.reshape(-1, 3)[:256, 0] = np.arange(256, dtype=np.uint8)          # every byte value
    depth = (2.5 + 1.5 * g.random((H, W))).astype(np.float32)
    depth[H // 4: 3 * H // 4, W // 3: 2 * W // 3] = 2.2
    return img, depth


def adjusted(depth, start):
    """post_processor.py:470-477 up to the cube, as the oracle restates it."""
    d = np.array(depth, np.float32)
    if d.ndim > 2:
        d = d[:, :, 0]
    if d.max() > 1.0:
        d = d / d.max()
    a = np.maximum(d - np.float32(start), np.float32(0.0)) / np.float32(1.0 - start)
    return np.clip(a, np.float32(0.0), np.float32(1.0))


def main():
    fog, defaults = reference_fog_and_params()
    H, W = 48, 64
    out = {}
    cases = []
    img, depth = frame(H, W, 0)
    cases.append(("norm", img, P.depth_normalize(depth), defaults["fog_start"]))
    img, depth = frame(H, W, 1)
    cases.append(("raw", img, depth, defaults["fog_start"]))
    img, depth = frame(H, W, 2)
    cases.append(("chan", img, np.stack([depth, depth * 2, depth * 3], -1).astype(np.float32), defaults["fog_start"]))
    img, _ = frame(H, W, 3)
    f32 = np.float32
    vals = [f32(0), f32(0.1), np.nextafter(f32(0.1), f32(0)), np.nextafter(f32(0.1), f32(1)), f32(1),
            np.nextafter(f32(1), f32(0)), f32(0.5), f32(1e-7)]
    edge = np.resize(np.array(vals, f32), H * W).reshape(H, W)
    cases.append(("edges", img, edge, defaults["fog_start"]))
    img, depth = frame(H, W, 4)
    cases.append(("start0", img, P.depth_normalize(depth), 0.0))
    img, depth = frame(H, W, 5)
    cases.append(("start35", img, P.depth_normalize(depth), 0.35))
    img, _ = frame(H, W, 6)
    cases.append(("none", img, None, defaults["fog_start"]))
    for name, img, depth, start in cases:
        params = dict(defaults, fog_start=start)
        with contextlib.redirect_stdout(io.StringIO()):     # the depth=None branch prints a warning
            ref = fog(_Self(params), img.copy(), None if depth is None else depth.copy())
        assert ref.dtype == np.uint8 and ref.shape == img.shape
        out[f"{name}_img"] = img
        out[f"{name}_out"] = ref
        out[f"{name}_start"] = np.float64(start)
        if depth is not None:
            out[f"{name}_depth"] = depth
            a = adjusted(depth, start)
            out[f"{name}_cube_differs"] = a ** np.float32(3.0) != P.cube_rn(a)
    np.savez_compressed(os.path.join(HERE, "f9_fog.npz"), **out)
    print("wrote f9_fog.npz:", ", ".join(n for n, *_ in cases),
          "| cube differs at", {n: int(out[f"{n}_cube_differs"].sum()) for n, _, d, _ in cases if d is not None})


if __name__ == "__main__":
    main()
