#!/bin/bash
# Round-3 GPU session: parity tests, bench lines (bf16x3 headline + fp16 / bf16 beside it), rocprofv3
# kernel stats of the headline bench.   bash tools/gpu_r3.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-r3}
K=${2:-}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread "${KARG[@]}" > $OUT/gpu_tests.log 2>&1
RC=$?
echo "pytest exit $RC" >> $OUT/gpu_tests.log
tail -4 $OUT/gpu_tests.log
case $RC in 0|1) ;; *) echo "pytest died ($RC): stopping"; exit $RC;; esac
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
python tools/bench_summary.py $OUT/bench.json
for p in fp16 bf16; do
  timeout -k 10 300 python bench.py --precision $p --no-cpu-baseline --steps 10 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || { echo "bench $p failed $?"; exit 1; }
  python tools/bench_summary.py $OUT/bench_$p.json
done
export TMPDIR=/tmp
ROOT=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > $OUT/prof.log 2>&1
echo "rocprof exit $?"
exit $RC
