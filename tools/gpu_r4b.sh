set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread -k "step3_bitwise or c3_two_patch" -s > gpurun_out/t_r4b.log 2>&1
RC=$?
grep -E "differs|passed|failed|PASS|FAIL" gpurun_out/t_r4b.log | tail -30
case $RC in 0|1) ;; *) echo "pytest died ($RC)"; exit $RC;; esac
MARF_STEP3=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > gpurun_out/bench_r4b_s3.json 2> gpurun_out/bench_r4b_s3.err || { echo bench failed; tail -5 gpurun_out/bench_r4b_s3.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_r4b_s3.json').read().strip().splitlines()[-1])
print('value %.4g px/s  ms/step %.3f kernel %s' % (d['value'], d['ms_per_step'], d['config']['step_kernel']), d['roofline']['avg_launch_ms'])
"
