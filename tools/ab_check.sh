#!/bin/bash
# Bit-for-bit A/B of the step kernel against a reference build (lib/libmarf_old.so, e.g. built from
# the last commit:  git archive HEAD <pkg>/csrc <pkg>/build_lib.py include | tar -x -C /tmp/old &&
# (cd /tmp/old/<pkg> && python build_lib.py --variant libmarf_old.so), copied into lib/), then a short
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
# the reference build and the current one benched on the same box, alternating
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=$LIBD/libmarf_old.so; else L=""; fi
    MARF_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v failed"; tail -5 $OUT/bench_$v.err; exit 1; }
    python - $OUT/bench_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print("%-4s value %.4g px/s  ms/step %.3f  mlp_step %.3f ms  wgrad_hidden %.3f ms" % (sys.argv[2], d["value"], d["ms_per_step"], k["mlp_step"]["avg_ms"], k["wgrad_hidden"]["avg_ms"]))
PY
  done
done
