# round-4 record on the committed library: GPU suite, smoke, headline bench (+ CPU baseline), rocprofv3
# kernel stats, PMC traffic of the timed kernels (C3 bf16x3, C5 bf16), C5 and C1 bench lines
set -o pipefail
T=${1:-r4l}
OUT=$PWD/gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
RC=$?; tail -2 $OUT/gpu_tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
bash tools/pmc_traffic.sh $T/pmc_c3 c3 bf16x3 > $OUT/pmc_c3.log 2>&1 || { echo "pmc c3 failed"; tail -5 $OUT/pmc_c3.log; exit 1; }
cp $OUT/pmc_c3/pmc_traffic.json profiles/pmc_traffic.json
bash tools/pmc_traffic.sh $T/pmc_c5 c5 bf16 > $OUT/pmc_c5.log 2>&1 || { echo "pmc c5 failed"; tail -5 $OUT/pmc_c5.log; exit 1; }
cp $OUT/pmc_c5/pmc_traffic.json profiles/pmc_traffic.json
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-200
ROOT=$PWD
(cd /tmp && TMPDIR=/tmp timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > $OUT/prof.log 2>&1) || { echo "rocprof failed"; exit 1; }
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "bench c5 failed"; tail -5 $OUT/bench_c5.err; exit 1; }
timeout -k 10 400 python bench.py --config c1 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c1.json 2> $OUT/bench_c1.err || { echo "bench c1 failed"; tail -5 $OUT/bench_c1.err; exit 1; }
for f in bench bench_c5 bench_c1; do python -c "
import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', '%.4g px/s' % d['value'], '%.3f ms/step' % d['ms_per_step'], r['kernel'], '%.3f ms' % r['avg_launch_ms'], 'frac %.3f' % r['frac'], 'traffic', r['traffic'])"; done
