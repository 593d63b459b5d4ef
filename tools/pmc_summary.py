"""Summarise rocprofv3 --pmc passes (tools/pmc.sh output) per kernel: mean counter value per
dispatch, and derived HBM bytes (FETCH_SIZE doubled per the gfx950 correction in
MI355X_MICROARCH.md §HBM; WRITE_SIZE as is), both in KB -> converted to bytes.

    python tools/pmc_summary.py gpurun_out/<tag> [out.csv]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "pass*", "*counter_collection.csv"))):
    per = defaultdict(float)
    meta = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            key = (r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            meta[r["Dispatch_Id"]] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for (d, k, c), v in per.items():
        vals[k][c].append(v)
    if "pass1" in f:
        for d, (k, ns) in meta.items():
            dur[k].append(ns)


def short(k):
    return k.split("(")[0].replace("void ", "").replace("marf::", "")[:64]


rows = []
for k, cs in vals.items():
    row = {"kernel": short(k)}
    for c, v in cs.items():
        row[c] = sum(v) / len(v)
    if "FETCH_SIZE" in row:
        row["hbm_read_bytes"] = 2 * row["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in row:
        row["hbm_write_bytes"] = row["WRITE_SIZE"] * 1024
    if dur.get(k):
        row["pmc_avg_ns"] = sum(dur[k]) / len(dur[k])
    # matrix-core utilisation (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over
    # the SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs: / 8 = the dispatch's wall cycles; 1024 SIMDs)
    if row.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in row:
        row["mfma_busy"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / (row["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if row.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in row:
        row["valu_per_mfma"] = row["SQ_INSTS_VALU"] / row["SQ_INSTS_MFMA"]
    rows.append(row)
cols = sorted({c for r in rows for c in r if c != "kernel"})
out = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
if out:
    with open(out, "w", newline="") as fh:
        w = csv.DictWriter(fh, ["kernel"] + cols)
        w.writeheader()
        for r in rows:
            w.writerow(r)
for r in rows:
    print(r["kernel"])
    for c in cols:
        if c in r:
            print(f"    {c:28s} {r[c]:.4g}")

# bench.py reads the HBM bytes per launch of its kernels from profiles/pmc_traffic.json
# (python tools/pmc_summary.py gpurun_out/<tag> profiles/<round>_pmc.csv --traffic c3/bf16x3 <source hash>)
# An entry names the kernel symbol it measured and the marf_source_hash of the library that ran it;
# bench.py reports its traffic only when both match the run (otherwise traffic: null).
if "--traffic" in sys.argv:
    import json
    i = sys.argv.index("--traffic")
    tag, src_hash = sys.argv[i + 1], sys.argv[i + 2]
    tj = os.path.join(os.path.dirname(out) if out else "profiles", "pmc_traffic.json")
    data = json.load(open(tj)) if os.path.exists(tj) else {}
    kernels = {}
    for r in rows:
        k = r["kernel"]
        name = None
        if k.startswith("k_mlp_step") or k.startswith("k_step2") or k.startswith("k_step3"):
            name = "mlp_step"
        elif k.startswith("k_prologue_probe"):
            name = "prologue_probe"
        elif k.startswith("k_wgrad_dma_layers<"):  # every hidden layer in one launch (fused path)
            name = "wgrad_hidden"
        elif k.startswith("k_wgrad_dma<"):
            name = "wgrad_l0" if ", 96" in k else "wgrad_hidden"
        elif k.startswith("k_wgrad<"):
            name = "wgrad_hidden" if ", 2, 4" in k else "wgrad_l0"
        if name and "hbm_read_bytes" in r and "hbm_write_bytes" in r:
            if name in kernels:  # two instantiations of one role in one run: keep the busier one
                if kernels[name]["pmc_avg_ns"] and (r.get("pmc_avg_ns") or 0) <= kernels[name]["pmc_avg_ns"]:
                    continue
            kernels[name] = {"symbol": k, "hbm_read_bytes": r["hbm_read_bytes"], "hbm_write_bytes": r["hbm_write_bytes"],
                             "pmc_avg_ns": r.get("pmc_avg_ns")}
            for c in ("mfma_busy", "valu_per_mfma", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD",
                      "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
                if c in r:
                    kernels[name][c] = r[c]
    data[tag] = {"source_hash": src_hash, "kernels": kernels,
                 "source": (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (+ SQ_INSTS_VALU SQ_INSTS_MFMA "
                            f"SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE) passes over bench.py --steps 2 ({root}); "
                            "read bytes = 2 x FETCH_SIZE (gfx950 correction, MI355X_MICROARCH.md HBM); mfma_busy = "
                            "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)")}
    json.dump(data, open(tj, "w"), indent=1)
    print("wrote", tj)
