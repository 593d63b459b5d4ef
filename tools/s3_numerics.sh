#!/bin/bash
# Two-waves-per-SIMD kernel, numerics: quick bf16x3 parity tests + bench (s3_check.sh), the 3000-step
# seed-3 tests, then the 25-draw seed-3 basin sweep.   bash tools/s3_numerics.sh <tag>
set -o pipefail
TAG=${1:-s3n}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
bash tools/s3_check.sh $TAG || exit $?
MARF_STEP3=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "3000 and bf16x3 or train_py and bf16x3" > $OUT/tests3000.log 2>&1
echo "3000-step tests exit $?"; grep -h "final PSNR\|passed\|failed" $OUT/tests3000.log | head -6
MARF_STEP3=1 timeout -k 10 600 python -u tools/seed_sweep.py --precisions bf16x3 --seeds 3 --perturb $(seq 0 24) \
  --out $OUT/basin_step3.json > $OUT/sweep.log 2>&1
echo "sweep exit $?"; tail -2 $OUT/sweep.log
