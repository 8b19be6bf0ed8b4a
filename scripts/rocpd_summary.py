"""Kernel statistics from a rocprofv3 rocpd database (rocprofv3 --kernel-trace writes
<dir>/<name>_results.db): per kernel name, calls / total / average / min / max duration, and
optionally one row per (name, grid) so launches of the same kernel on different shapes separate.

    python scripts/rocpd_summary.py gpurun_out/prof_train/run_results.db [--by-grid] [--csv out.csv]
"""
import argparse
import csv
import sqlite3
import sys


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--by-grid", action="store_true")
    p.add_argument("--csv")
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    key = "name, grid_x" if a.by_grid else "name"
    rows = list(c.execute(f"select {key}, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                          f"from kernels group by {key} order by sum(duration) desc"))
    total = sum(r[-4] for r in rows)
    hdr = ["Name"] + (["Grid"] if a.by_grid else []) + ["Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs",
                                                         "Percentage"]
    out = [hdr] + [list(r) + [100.0 * r[-4] / total] for r in rows]
    w = csv.writer(open(a.csv, "w", newline="") if a.csv else sys.stdout)
    for r in out:
        w.writerow([f"{x:.1f}" if isinstance(x, float) else x for x in r])


if __name__ == "__main__":
    main()
