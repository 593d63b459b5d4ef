#!/bin/bash
# Split-dz dgrad (MARF_DZSPLIT=1) of the two-wave kernel: bf16x3 parity tests, bench line, the
# 3000-step seed-3 test and a 40-draw seed-3 basin sweep.   bash tools/dzs_check.sh <tag>
set -o pipefail
TAG=${1:-dzs}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export MARF_STEP3=1 MARF_DZSPLIT=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "bf16x3 and not 3000 and not train" > $OUT/tests.log 2>&1
RC=$?; tail -2 $OUT/tests.log
[ $RC -eq 0 ] || { echo "tests failed"; grep -B5 Error $OUT/tests.log | head -30; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
python tools/bench_summary.py $OUT/bench.json | head -3
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "3000 and bf16x3" > $OUT/tests3000.log 2>&1
echo "3000-step test exit $?"; grep -h "final PSNR" $OUT/tests3000.log | head -3
timeout -k 10 600 python -u tools/seed_sweep.py --precisions bf16x3 --seeds 3 --perturb $(seq 25 64) \
  --out $OUT/basin.json > $OUT/sweep.log 2>&1
echo "sweep exit $?"; tail -1 $OUT/sweep.log
