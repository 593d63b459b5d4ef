#!/bin/bash
# Basin sweeps of emulated precision recipes (numerics experiments): the fp32 kernels of the
# MARF_DIAG_RT build round each operand class per layer as the recipe would (MARF_DIAG_PREC codes,
# marf_common.h diag_round), 24 one-ulp perturbations of the seed-3 C1 init each.
#   bash tools/recipe_sweep.sh name=WTAD,WTAD,... [name=...]
# Build first (CPU): python build_lib.py --variant libmarf_diagrt.so -DMARF_DIAG_RT
LIB=${MARF_RT_LIB:-$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_diagrt.so}
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%=*}; code=${spec#*=}
  MARF_LIB=$LIB MARF_DIAG_PREC=$code timeout -k 10 ${SWEEP_TIMEOUT:-420} python -u tools/seed_sweep.py --seeds 3 --precisions fp32 \
    --perturb ${PERTURB:-$(seq -s ' ' 0 23)} --out gpurun_out/rs_$name.json > gpurun_out/rs_$name.log 2>&1
  rc=$?
  echo "$name ($code): $(tail -1 gpurun_out/rs_$name.log)"
  case $rc in 0) ;; *) echo "recipe $name failed ($rc): stopping"; exit $rc;; esac
done
