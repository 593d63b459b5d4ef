#!/bin/bash
# Same-box seed-3 basin A/B of the two split-bf16 step kernels: k_step2 (MARF_STEP3=0) and k_step3
# (MARF_STEP3=1), the same one-ulp init perturbation draws.   bash tools/basin_ab.sh <tag> <first> <last>
set -o pipefail
TAG=${1:-bab}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
for k in 0 1; do
  MARF_STEP3=$k timeout -k 10 500 python -u tools/seed_sweep.py --precisions bf16x3 --seeds 3 --perturb $(seq ${2:-25} ${3:-64}) \
    --out $OUT/basin_step$((k + 2)).json > $OUT/sweep_step$((k + 2)).log 2>&1 || { echo "sweep $k failed"; tail -3 $OUT/sweep_step$((k + 2)).log; exit 1; }
  tail -1 $OUT/sweep_step$((k + 2)).log
done
