#!/bin/bash
# Bit-for-bit A/B of the step kernel against a reference build (lib/libmarf_old.so), then a short
# bench of the current build.  bash tools/ab_check.sh <tag>
set -o pipefail
TAG=${1:-ab}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
LIBD=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib
for cfg in "bf16x3 8" "bf16x3 12" "bf16x3 4" "bf16 8"; do
  set -- $cfg
  MARF_LIB=$LIBD/libmarf_old.so timeout -k 10 120 python tools/ab_grads.py $OUT/old_$1_$2.npz $1 $2 > $OUT/old_$1_$2.log 2>&1 || { echo "old $cfg failed"; tail -5 $OUT/old_$1_$2.log; exit 1; }
  timeout -k 10 120 python tools/ab_grads.py $OUT/new_$1_$2.npz $1 $2 > $OUT/new_$1_$2.log 2>&1 || { echo "new $cfg failed"; tail -5 $OUT/new_$1_$2.log; exit 1; }
  echo "== $cfg"; python tools/ab_grads.py --compare $OUT/old_$1_$2.npz $OUT/new_$1_$2.npz | tail -4; rm -f $OUT/*.npz
done
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.4g px/s  ms/step %.3f  frac %.4f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"]))
for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["launches_per_step"])[:5]:
    print("  %-20s %8.3f ms x %.0f" % (k, v["avg_ms"], v["launches_per_step"]))
PY
