"""Write the bit images of the split-bf16 fused step (tests/step_bits.py) computed by the library
loaded now:  python tools/make_step2_bits.py OUT.json [case ...]   (GPU; default: every case)

The committed tests/golden/step2_bits.json was written by this script from the library named in
its "source_hash" / "commit" fields; the GPU test test_step2_bits_unchanged compares later builds
against it."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
os.environ.setdefault("MARF_STEP3", "0")  # (libraries that still had k_step3: the k_step2 bits)


def main():
    import marf_hip
    import step_bits
    out = sys.argv[1]
    cases = sys.argv[2:] or list(step_bits.CASES)
    try:
        commit = subprocess.run(["git", "rev-parse", "HEAD"], cwd=ROOT, capture_output=True, text=True).stdout.strip()
    except OSError:
        commit = ""
    res = {"source_hash": marf_hip.lib().marf_source_hash().decode(), "commit": commit or None, "cases": {}}
    for c in cases:
        res["cases"][c] = step_bits.case_bits(c)
        print(c, res["cases"][c]["kernel"], flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", out)


if __name__ == "__main__":
    main()
