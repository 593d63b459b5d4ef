"""Bit images (sha1 per output tensor) of one fused step + two training iterations of a recipe, as
tests/step_bits.py computes them, for the library loaded now (MARF_LIB): the A/B check that a
kernel change is bit-neutral for a recipe whose bits no golden file pins (fp16x2).

    MARF_LIB=... python tools/recipe_bits.py --precision fp16x2 OUT.json [case ...]   (GPU)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp16x2")
    ap.add_argument("out")
    ap.add_argument("cases", nargs="*", default=["c1", "c3x2", "c3x3-L10", "L13", "L16-1tile", "c3x64"])
    a = ap.parse_args()
    import torch
    import marf_hip
    import step_bits
    res = {"source_hash": marf_hip.lib().marf_source_hash().decode(), "precision": a.precision, "cases": {}}
    for c in a.cases:
        m, var = step_bits.build_case(c, precision=a.precision)
        kernel = m.graph.neural_image.engine(torch.device(step_bits.DEV)).net.step_kernel
        out = step_bits.run_case(m, var)
        res["cases"][c] = {"kernel": kernel, "bits": {k: step_bits._digest(v) for k, v in out.items()}}
        print(c, kernel, flush=True)
    json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
