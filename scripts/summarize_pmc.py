"""Summarise the PMC passes of scripts/profile_pmc.sh into profiles/<tag>_pmc_summary.json.

Per kernel: average per dispatch of every counter, and for the MLP kernel the HBM-side traffic
per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; gfx950's FETCH_SIZE reads half the
bytes of a wide coalesced stream, MI355X_MICROARCH.md §HBM), the clock (GRBM_GUI_ACTIVE / 8 /
duration) and the MFMA busy fraction; the MLP kernel is mlp16_kernel (f16x3) when present, else mlp_kernel (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles))."""
import collections, csv, glob, json, os, sys

src, out = sys.argv[1], sys.argv[2]
per = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if k.startswith("void "):
            k = k[5:]
        k = k.split("<")[0]            # template instances (nerf::mlp16_kernel<false>) under one name
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
res = {"source": src, "kernels": {}}
for k, cs in per.items():
    if not k.startswith("nerf::"):
        continue
    res["kernels"][k] = {c: sum(v) / len(v) for c, v in cs.items()}
    kk = res["kernels"][k]
    if "FETCH_SIZE" in kk and "WRITE_SIZE" in kk:   # same gfx950 correction as the MLP figure below
        kk["hbm_bytes_per_dispatch"] = (2 * kk["FETCH_SIZE"] + kk["WRITE_SIZE"]) * 1024
        kk["dispatches"] = len(cs["FETCH_SIZE"])   # in the profiled run (all shapes of a templated kernel)
mlp = "nerf::mlp16_kernel" if "nerf::mlp16_kernel" in res["kernels"] else "nerf::mlp_kernel"
res["mlp_kernel"] = mlp
m = res["kernels"].get(mlp, {})
if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    res["mlp_hbm_bytes_per_launch"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
if "GRBM_GUI_ACTIVE" in m:
    ts = [t for (f, _), t in dur[mlp].items() if "/p3/" in f]
    avg_t = sum(ts) / len(ts)
    res["mlp_clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / avg_t / 1e9
    res["mlp_mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
if "TCC_HIT_sum" in m:
    res["mlp_l2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
