#!/bin/bash
# One GPU session: parity tests, bench (with CPU baseline), rocprofv3 kernel trace of the bench.
# Usage (from the repo root, on the GPU box): bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r1}
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
RC=$?
echo "pytest exit $RC" >> $OUT/gpu_tests_$TAG.log
tail -3 $OUT/gpu_tests_$TAG.log
# a crash / abort / timeout (not plain test failures) ends the GPU session here
case $RC in 124|134|137|139) echo "pytest died ($RC): stopping"; exit $RC;; esac
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -5 $OUT/bench_$TAG.err; exit 1; }
tail -1 $OUT/bench_$TAG.json | cut -c1-600
export TMPDIR=/tmp
ROOT=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > $OUT/prof_$TAG.log 2>&1
echo "rocprof exit $?"
find $OUT/prof_$TAG -name "*stats*" | head
