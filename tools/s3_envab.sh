#!/bin/bash
# bf16x3 parity tests under an environment setting, then bench lines with and without it, alternating.
#   bash tools/s3_envab.sh <tag> VAR=value [VAR2=value ...]
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
env "$@" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "bf16x3 and not 3000 and not train" > $OUT/tests.log 2>&1
rc=$?
echo "tests ($*): rc $rc: $(tail -1 $OUT/tests.log)"
case $rc in 0) ;; 1) tail -30 $OUT/tests.log; exit 1;; *) echo "pytest died ($rc): stopping"; tail -30 $OUT/tests.log; exit $rc;; esac
for rep in 1 2; do
  for arm in base env; do
    if [ $arm = env ]; then E="$*"; else E="MARF_AB_NONE=1"; fi
    env $E timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_${arm}_$rep.json 2> $OUT/bench_${arm}_$rep.err \
      || { echo "bench $arm failed"; tail -5 $OUT/bench_${arm}_$rep.err; exit 1; }
    echo "== $arm (rep $rep)"
    python tools/bench_summary.py $OUT/bench_${arm}_$rep.json | head -2
  done
done
