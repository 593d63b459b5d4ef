#!/bin/bash
# Pipelined weight gradients: the pipeline tests, then bench lines with the pipeline off / on at
# several weight-gradient CU counts (MARF_PIPE_WG) on one box.   bash tools/pipe_ab.sh <tag> [wg ...]
set -o pipefail
TAG=${1:-pipe}
shift
WGS=${@:-20 28 36}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "pipelined or tile_grouping or c3_linearity" > $OUT/tests.log 2>&1
RC=$?
tail -5 $OUT/tests.log
[ $RC -eq 0 ] || { echo "tests failed ($RC): stopping"; exit $RC; }
b() {  # b <name> [env...]
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > $OUT/bench_$n.json 2> $OUT/bench_$n.err \
    || { echo "bench $n failed"; tail -5 $OUT/bench_$n.err; exit 1; }
  python tools/bench_summary.py $OUT/bench_$n.json | head -12
}
b off MARF_PIPE=0
for w in $WGS; do b wg$w MARF_PIPE_WG=$w; done
b off2 MARF_PIPE=0
