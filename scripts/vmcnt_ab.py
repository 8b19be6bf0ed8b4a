"""Same-box check of the stream waits' counted vmcnt (stream16.h chunk_step): does the count change results?

Each library build given (NERFMI_LIB; '' = the in-tree library) runs in a fresh child process:
  * the trained fixture of tests/test_gpu_accuracy.py (200 Trainer steps, 1,024-ray batches, seed 0);
  * 25 production-size steps (4,096 rays x 64 samples) as in test_training_is_deterministic;
and prints the SHA-256 of the parameter buffer and Adam moments after each.  Builds whose waits are
all correct produce the same bits (the kernels' arithmetic does not depend on the counts); a wait that
returns before its DMA landed shows up as a different hash or as run-to-run differences.

  python scripts/vmcnt_ab.py [--repeat R] lib.so ...
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, REPO)
    import numpy as np
    import torch
    import nerfmi
    from nerfmi.dataset import SyntheticNeRFDataset
    from nerfmi.train import Trainer

    def h(*ts):
        m = hashlib.sha256()
        for t in ts:
            m.update(t.detach().cpu().contiguous().numpy().tobytes())
        return m.hexdigest()[:16]

    out = {}
    cfg = nerfmi.Config()
    for name, n_img, steps, batch in (("fixture200", 8, 200, 1024), ("prod25", 3, 25, 4096)):
        np.random.seed(0)
        torch.manual_seed(0)
        ds = SyntheticNeRFDataset(cfg, n_images=n_img, H=96, W=96)
        torch.manual_seed(0)
        tr = Trainer(cfg, appearance_embeddings=ds.appearance_embeddings)
        losses = []
        for i in range(steps):
            b = ds.get_rays(batch_size=batch)
            losses.append(float(tr.step(b["rays_o"], b["rays_d"], b["rgb"], b["appearance_idx"], seed=i + 1)))
        torch.cuda.synchronize()
        out[name] = {"params": h(tr.flat), "moments": h(tr.exp_avg, tr.exp_avg_sq), "last_loss": losses[-1]}
    print("RESULT " + json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child()
    libs = [""] + a.libs
    for r in range(a.repeat):
        for lib in libs:
            env = dict(os.environ, NERFMI_LIB=lib)
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                               text=True, timeout=600)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")]
            if p.returncode or not line:
                print(p.stdout[-2000:], p.stderr[-4000:])
                return p.returncode or 1
            res = json.loads(line[0][7:])
            print(f"round {r} {os.path.basename(lib) or 'in-tree':28s} " +
                  " ".join(f"{k}: params {v['params']} moments {v['moments']} loss {v['last_loss']:.9g}"
                           for k, v in res.items()), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
