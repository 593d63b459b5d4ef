set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
for k in 0 1; do
  MARF_STEP3=$k timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 --no-cpu-baseline --no-render > gpurun_out/c1_s${k}_${round}.json 2> gpurun_out/c1_err || { tail -3 gpurun_out/c1_err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/c1_s${k}_${round}.json').read().strip().splitlines()[-1])
print('c1 MARF_STEP3=$k %.4g px/s %.3f ms/step %s %.3f ms' % (d['value'], d['ms_per_step'], d['config']['step_kernel'], d['roofline']['avg_launch_ms']))
"
done
done
