# round-end rehearsal on the committed tree: the driver's GPU suite, smoke() and the default bench line
set -o pipefail
OUT=$PWD/gpurun_out/r5h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
RC=$?; tail -2 $OUT/gpu_tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-300
