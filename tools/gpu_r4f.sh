set -o pipefail
mkdir -p gpurun_out
for B in 2 4 8 16 32; do
for k in 0 1; do
  MARF_STEP3=$k timeout -k 10 300 python bench.py --config c3 --strong $B --steps 20 --warmup 3 --no-cpu-baseline --no-render > gpurun_out/x_${B}_${k}.json 2> gpurun_out/x_err || { tail -3 gpurun_out/x_err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/x_${B}_${k}.json').read().strip().splitlines()[-1])
print('B=$B MARF_STEP3=$k %.4g px/s %.3f ms/step %s %.3f ms' % (d['value'], d['ms_per_step'], d['config']['step_kernel'], d['roofline']['avg_launch_ms']))
"
done
done
