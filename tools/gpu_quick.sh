#!/bin/bash
# Quick GPU check: parity tests (stop at first failure) then a short bench without CPU baseline.
# Usage on the box from the repo root: bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-q}
K=${2:-}
OUT=$PWD/gpurun_out
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > $OUT/gpu_tests_$TAG.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
fi
RC=$?
tail -15 $OUT/gpu_tests_$TAG.log
case $RC in 0|1) ;; *) echo "pytest died ($RC): stopping"; exit $RC;; esac
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -5 $OUT/bench_$TAG.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/bench_$TAG.json').read().strip().splitlines()[-1])
print('value %.4g px/s  ms/step %.3f  roof %s' % (d['value'], d['ms_per_step'], d['roofline']))
for k,v in sorted(d['kernels'].items(), key=lambda kv:-kv[1]['avg_ms']*kv[1]['launches_per_step']): print('  %-20s %8.3f ms x %.0f' % (k, v['avg_ms'], v['launches_per_step']))
"
exit $RC
