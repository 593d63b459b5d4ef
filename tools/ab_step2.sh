set -o pipefail
for cfg in "bf16 0 0" "bf16 1 1" "bf16x3 1 0"; do
  set -- $cfg
  MARF_STEP2=$2 MARF_STEP2_NW4=$3 timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --precision $1 > gpurun_out/b_$1_$2_$3.json 2> gpurun_out/b_$1_$2_$3.err || { echo "fail $cfg"; tail -3 gpurun_out/b_$1_$2_$3.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/b_$1_$2_$3.json').read().strip().splitlines()[-1])
print('$cfg', 'value %.4g px/s  ms/step %.3f' % (d['value'], d['ms_per_step']), ' '.join('%s=%.3f' % (k, v['avg_ms']*v['launches_per_step']) for k,v in sorted(d['kernels'].items(), key=lambda kv:-kv[1]['avg_ms']*kv[1]['launches_per_step'])[:4]))
"
done
