"""The committed basin table (profiles/basin_table.json): per precision recipe, how often the seed-3
cat_batch3 C1 run (3000 iterations) lands in the reference's 26 dB basin over the committed one-ulp
init draws (tools/seed_sweep.py --perturb; draw 0 = the unperturbed seed-3 run).  A new recipe must
not fall below the benchmarked one's rate on the same draws.  Built from
the per-draw records under profiles/ (each produced by tools/seed_sweep.py / tools/basin_table.py on
an MI355X; tools/gpu_session.sh basin=... regenerates any of them):

    python tools/make_basin_table.py            -> profiles/basin_table.json (+ a printed table)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
BASIN_DB = 25.5

# recipe -> (description, [(file, precision filter or None)])
SOURCES = {
    "fp32": ("fp32 tile kernel (exact fp32 MFMA), real kernel",
             [("r4i/basin_fp32_p25_64.json", None), ("r7i/basin_p65_104.json", "fp32"), ("r7s/rs_fp32_105.json", None),
              ("r8d/seed3_rule.json", "fp32")]),
    "bf16x3": ("split bf16 (k_step2, the benchmarked recipe; bits pinned by tests/golden/step2_bits.json), real kernel",
               [("r3k_basin/basin_step2_p25_64.json", None), ("r7i/basin_p65_104.json", "bf16x3"),
                ("r7s/rs_x3_105.json", None), ("r8d/seed3_rule.json", "bf16x3")]),
    "bf16x3_split_dz": ("bf16x3 + the hidden dgrad's dz split hi + lo (k_step2dz, MARF_STEP2_DZ=1), real kernel",
                        [("r7s/rs_dzreal.json", None), ("r7s/rs_dz_105.json", None), ("r7u/dz_seed3.json", None)]),
    "fp16x2_e1": ("fp16 forward (fp16 hi + lo weights, fp16 activations) + the split-bf16 dgrad (k_step2h, round 6's "
                  "first build), real kernel", [("r8d/fp16x2.json", None), ("r8a/seed3_fp16x2.json", None)]),
    "fp16x2": ("split-fp16 weights, fp16 activations and dz (k_step2h as committed), real kernel",
               [("r8e/fp16x2.json", None)]),
    "emu_bf16x3": ("bf16x3 emulated in the fp32 kernels (MARF_DIAG_PREC 2221,...,2222)",
                   [("r4j/rs_x3.json", None), ("r4j/rs_x3_b.json", None), ("r7k/rs_x3emu.json", None)]),
    "emu_fp16x2_e1": ("fp16x2_e1 emulated (MARF_DIAG_PREC 42311,4231,4231,4231,4232)",
                      [("r8d/e1_g1.json", None), ("r8d/e1.json", None), ("r8d/e1_extra.json", None)]),
    "emu_fp16x2": ("fp16x2 emulated: every operand fp16, weights hi + lo (MARF_DIAG_PREC 4433,...,4434)",
                   [("r4j/rs_f16s.json", None), ("r4j/rs_f16s_b.json", None), ("r8d/e3.json", None)]),
    "emu_fp16x2_split_dz": ("fp16x2_e1 + the hidden dgrad's dz split (MARF_DIAG_PREC 42311,4232,...), emulated",
                            [("r8d/e2.json", None)]),
}


def load(rel, prec):
    path = os.path.join(P, rel)
    if not os.path.exists(path):
        return {}
    runs = json.load(open(path))
    return {r["perturb"]: r for r in runs if prec is None or r.get("precision") == prec}


def main():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import psnr_rule
    recs = {}
    for name, (desc, files) in SOURCES.items():
        d = {}
        for rel, prec in files:
            d.update(load(rel, prec))
        recs[name] = (desc, d)
    common = sorted(set(recs["bf16x3"][1]) & set(recs["fp32"][1]))
    out = {"note": "seed-3 C1 run, 3000 iterations, one-ulp init draws (tools/seed_sweep.py --perturb, draw 0 = "
                   "unperturbed); basin = mean of the last 10 logged PSNRs >= 25.5 dB (every run lands >= 25.8 or "
                   "<= 25.3); vs_bf16x3 = counts on the draws both recipes ran; seed3 = draw 0's final PSNR and "
                   "mean of the last 10 logged values where run", "recipes": {}}
    for name, (desc, d) in recs.items():
        draws = sorted(k for k in d if k > 0)
        if not draws:
            continue
        basin = sum(d[k]["psnr_mean10"] >= BASIN_DB for k in draws)
        both = [k for k in draws if k in recs["bf16x3"][1]]
        row = {"description": desc, "draws": [min(draws), max(draws)], "n": len(draws), "basin": basin,
               "rate": round(basin / len(draws), 3),
               "sigma": round((basin / len(draws) * (1 - basin / len(draws)) / len(draws)) ** 0.5, 3),
               "within_005dB_of_25.9968": sum(abs(d[k]["psnr"] - 25.9968) <= 0.05 for k in draws),
               "vs_bf16x3": {"n": len(both), "this": sum(d[k]["psnr_mean10"] >= BASIN_DB for k in both),
                             "bf16x3": sum(recs["bf16x3"][1][k]["psnr_mean10"] >= BASIN_DB for k in both)}}
        if 0 in d:
            ok, msg = psnr_rule.psnr_check(d[0]["psnr"], d[0]["psnr_mean10"])
            row["seed3"] = {"final": round(d[0]["psnr"], 4), "mean10": round(d[0]["psnr_mean10"], 4),
                            "psnr_rule": bool(ok), "rule": msg}
        out["recipes"][name] = row
    json.dump(out, open(os.path.join(P, "basin_table.json"), "w"), indent=1)
    print(f"{'recipe':22s} {'basin':>9s} {'rate':>6s}  vs bf16x3 on the same draws   seed-3 draw")
    for name, r in out["recipes"].items():
        v = r["vs_bf16x3"]
        s3 = r.get("seed3")
        print(f"{name:22s} {r['basin']:3d}/{r['n']:<4d} {r['rate']:6.3f}  {v['this']:3d} vs {v['bf16x3']:3d} of {v['n']:3d}"
              f"          {'' if not s3 else '%.3f / %.3f %s' % (s3['final'], s3['mean10'], 'rule ok' if s3['psnr_rule'] else 'rule FAILS')}")


if __name__ == "__main__":
    main()
