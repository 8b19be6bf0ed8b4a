"""Summarise the PMC passes of scripts/profile_pmc.sh into profiles/<tag>_pmc_summary.json.

Kernels are keyed by their full template instance AND grid size ("nerf::mlp16_kernel<false>|grid=..."):
two instances of one template (mlp16_kernel<false> renders, <true> trains) or two shapes of one
kernel (the coarse and fine launches) are different workloads and are never averaged together.
Per key: the average per dispatch of every counter, the dispatch count, the average duration of
the pass that collected GRBM_GUI_ACTIVE, and
  * hbm_bytes_per_dispatch = (2 x FETCH_SIZE + WRITE_SIZE) KiB -> bytes (gfx950's FETCH_SIZE counts
    half the bytes of a wide coalesced streaming read, MI355X_MICROARCH.md §HBM; WRITE_SIZE is exact
    for 16-byte-per-lane stores) and the same without the x2 (fetch_bytes_raw) for access patterns
    the x2 has not been calibrated on;
  * clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / duration and mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES /
    (1024 SIMDs x GRBM_GUI_ACTIVE / 8), per dispatch from the pass that collected them (its own
    duration), averaged over the dispatches; a dispatch whose derived clock exceeds the part's 2.4
    GHz maximum carries a corrupt counter and is dropped (listed under "notes").
Top-level mlp_* fields describe the render MLP (mlp16s_kernel; mlp16_kernel<false> until round 5; else
mlp_kernel), averaged over
its dispatches of every grid size (bench.py's traffic per average launch)."""
import collections
import csv
import glob
import json
import os
import sys

MAX_CLOCK_GHZ = 2.4


def kernel_name(raw):
    k = raw.split("(")[0]
    return k[5:] if k.startswith("void ") else k


def summarize(src):
    per = collections.defaultdict(lambda: collections.defaultdict(list))   # key -> counter -> values
    # key -> dispatch (file, id) -> {counter: value, "_t": duration}: the pass's own pairing
    disp = collections.defaultdict(lambda: collections.defaultdict(dict))
    files = sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))) or \
        sorted(glob.glob(os.path.join(src, "pass*.csv")))          # (the copies committed under profiles/)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = kernel_name(r["Kernel_Name"])
            if not name.startswith("nerf::"):
                continue
            key = f"{name}|grid={r['Grid_Size']}"
            v = float(r["Counter_Value"])
            per[key][r["Counter_Name"]].append(v)
            d = disp[key][(f, r["Dispatch_Id"])]
            d[r["Counter_Name"]] = v
            d["_t"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    res = {"source": src, "kernels": {}, "notes": []}
    for key, cs in sorted(per.items()):
        kk = {c: sum(v) / len(v) for c, v in cs.items()}
        kk["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in kk and "WRITE_SIZE" in kk:
            kk["hbm_bytes_per_dispatch"] = (2 * kk["FETCH_SIZE"] + kk["WRITE_SIZE"]) * 1024
            kk["fetch_bytes_raw"] = kk["FETCH_SIZE"] * 1024
            kk["write_bytes"] = kk["WRITE_SIZE"] * 1024
            kk["dispatches"] = len(cs["FETCH_SIZE"])
        # clock and MFMA duty per dispatch, from the GRBM_GUI_ACTIVE pass's own rows; a dispatch whose
        # derived clock exceeds the part's maximum has a corrupt counter (an outlier) and is dropped
        good, bad = [], 0
        for d in disp[key].values():
            if "GRBM_GUI_ACTIVE" not in d or d["_t"] <= 0:
                continue
            clk = d["GRBM_GUI_ACTIVE"] / 8 / d["_t"] / 1e9
            if clk > MAX_CLOCK_GHZ:
                bad += 1
                continue
            busy = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 1024) \
                if "SQ_VALU_MFMA_BUSY_CYCLES" in d else None
            good.append((clk, busy, d["_t"]))
        if bad:
            res["notes"].append(f"{key}: {bad} dispatch(es) with a derived clock above {MAX_CLOCK_GHZ} GHz dropped")
        if good:
            kk["clock_ghz"] = sum(g[0] for g in good) / len(good)
            kk["duration_s"] = sum(g[2] for g in good) / len(good)
            if good[0][1] is not None:
                kk["mfma_busy"] = sum(g[1] for g in good) / len(good)
        elif any("GRBM_GUI_ACTIVE" in d for d in disp[key].values()):
            kk["clock_ghz"] = None
        if "TCC_HIT_sum" in kk and "TCC_MISS_sum" in kk:
            kk["l2_hit_rate"] = kk["TCC_HIT_sum"] / max(kk["TCC_HIT_sum"] + kk["TCC_MISS_sum"], 1.0)
        res["kernels"][key] = kk
    # the render MLP over all its grid sizes (dispatch-weighted)
    for mlp in ("nerf::mlp16s_kernel", "nerf::mlp16_kernel<false>", "nerf::mlp_kernel"):
        keys = [k for k in res["kernels"] if k.split("|")[0] == mlp]
        if keys:
            break
    res["mlp_kernel"] = mlp if keys else None

    def wavg(field):
        num = den = 0.0
        for k in keys:
            v, n = res["kernels"][k].get(field), res["kernels"][k].get("dispatches", 0)
            if v is None or not n:
                continue
            num, den = num + v * n, den + n
        return num / den if den else None
    if keys:
        res["mlp_hbm_bytes_per_launch"] = wavg("hbm_bytes_per_dispatch")
        res["mlp_clock_ghz"] = wavg("clock_ghz")
        res["mlp_mfma_busy"] = wavg("mfma_busy")
        res["mlp_l2_hit_rate"] = wavg("l2_hit_rate")
    return res


if __name__ == "__main__":
    src, out = sys.argv[1], sys.argv[2]
    res = summarize(src)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
