# the full GPU suite and the headline bench after the k_step2 specializations became the default at
# every size; phase stamps of the specialized k_step2 at C3
set -o pipefail
mkdir -p gpurun_out/r4t
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4t/gpu_tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4t/gpu_tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
timeout -k 10 400 python bench.py > gpurun_out/r4t/bench.json 2> gpurun_out/r4t/bench.err || { echo "bench failed"; tail -5 gpurun_out/r4t/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r4t/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('%.4g px/s %.3f ms/step %s %.3f ms frac %.3f' % (d['value'], d['ms_per_step'], d['config']['step_kernel'], r['avg_launch_ms'], r['frac']))"
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 300 python tools/step2_phases.py --kernel step2 > gpurun_out/r4t/phases_step2.txt 2>&1 || { echo "phases failed"; exit 1; }
cat gpurun_out/r4t/phases_step2.txt
