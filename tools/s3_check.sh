#!/bin/bash
# Two-waves-per-SIMD step kernel (marf_step3.hip): bf16x3 parity tests, then bench lines against the
# one-wave kernel (default).   bash tools/s3_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-s3}
K=${2:-"bf16x3 and not 3000 and not train"}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
MARF_STEP3=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "$K" > $OUT/tests.log 2>&1
RC=$?
tail -25 $OUT/tests.log
case $RC in 0|1) ;; *) echo "pytest died ($RC): stopping"; exit $RC;; esac
b() {  # b <name> [env...]
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$n.json 2> $OUT/bench_$n.err \
    || { echo "bench $n failed"; tail -5 $OUT/bench_$n.err; exit 1; }
  python tools/bench_summary.py $OUT/bench_$n.json | head -6
  python -c "import json; d=json.loads(open('$OUT/bench_$n.json').read().strip().splitlines()[-1]); print('render px/s', d['config']['render_pixels_per_s'])"
}
b s3 MARF_STEP3=1
b s2 MARF_STEP3=0
exit $RC
