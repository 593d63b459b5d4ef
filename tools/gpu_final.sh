#!/bin/bash
# Round-end style GPU session: every GPU test, smoke(), the headline bench (CPU baseline included),
# the fp16 / bf16 bench lines, rocprofv3 kernel stats of the headline bench, PMC passes.
#   bash tools/gpu_final.sh <tag>
set -o pipefail
T=${1:-final}
OUT=$PWD/gpurun_out/$T
mkdir -p $OUT
bash tools/gpu_r3.sh $T || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
echo "smoke exit $?"; tail -2 $OUT/smoke.log
bash tools/pmc.sh $T/pmc > $OUT/pmc.log 2>&1; tail -6 $OUT/pmc.log
