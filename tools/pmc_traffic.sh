#!/bin/bash
# HBM traffic and matrix-core counters of the timed kernels: rocprofv3 FETCH_SIZE, WRITE_SIZE and
# SQ_INSTS_VALU / SQ_INSTS_MFMA / SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_VMEM_RD / GRBM_GUI_ACTIVE passes (each its own process,
# kernel-trace only) over a short bench.py run of <config>, summarised into profiles/pmc_traffic.json
# under "<config>/<precision>" with the kernel symbols and the loaded library's source hash
# (gpurun_out/<tag>/pmc_traffic.json: copy it to profiles/).
#   bash tools/pmc_traffic.sh <tag> <config> <precision> [extra bench args]
set -o pipefail
TAG=$1; CFG=$2; PREC=$3; shift 3
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
HASH=$(python -c "import sys; sys.path.insert(0, 'masking-bundle-adjusting-neural-radiance-fields_amd'); import build_lib; print(build_lib.embedded_hash(build_lib.LIB))") || exit 1
export TMPDIR=/tmp
i=0
for CTR in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $OUT/pass$i -o run \
     --kernel-include-regex "k_mlp|k_wgrad|k_step2|k_step3|k_prologue" -- python3 $ROOT/bench.py --config $CFG --precision $PREC \
     --steps 2 --warmup 1 --no-cpu-baseline --no-render --no-alt-recipe "$@" > $OUT/pass$i.log 2>&1) || { echo "pass $i ($CTR) failed"; tail -5 $OUT/pass$i.log; exit 1; }
done
# (profiles/ does not come back from a GPU box: the updated json lands in $OUT, copied back by hand)
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json 2>/dev/null
python tools/pmc_summary.py $OUT $OUT/pmc.csv --traffic $CFG/$PREC $HASH
