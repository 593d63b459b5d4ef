#!/bin/bash
# Secondary bench lines (BASELINE configs other than the headline C3): C1 in fp32 and bf16x3, C5
# (8 x 512, plain bf16) with c2f on and off, C3 strong-scaling shape (--strong 512 on one GPU).
# bash tools/bench_configs.sh <tag>
set -o pipefail
TAG=${1:-cfg}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-alt-recipe "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; return 1; }
  python - $OUT/$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%-14s %.4g px/s  %.3f ms/step  dtype %s  %s %.3f ms  frac %.4f" % (sys.argv[2], d["value"], d["ms_per_step"], d["dtype"], r["kernel"], r["avg_launch_ms"], r["frac"]))
PY
}
run c1_fp32 --config c1 --precision fp32 && run c1_bf16x3 --config c1 --precision bf16x3 && \
run c5 --config c5 --no-render && run c5_noc2f --config c5 --no-c2f --no-render
