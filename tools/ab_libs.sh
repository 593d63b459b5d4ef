#!/bin/bash
# A/B the bf16x3 bench over library variants: bash tools/ab_libs.sh <variant> ...  ("default" = lib/libmarf.so)
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = default ]; then unset MARF_LIB; else export MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_$v.so; fi
  timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "fail $v"; tail -3 gpurun_out/ab_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1])
print('$v', 'value %.4g px/s  ms/step %.3f' % (d['value'], d['ms_per_step']), ' '.join('%s=%.3f' % (k, v['avg_ms']*v['launches_per_step']) for k,v in sorted(d['kernels'].items(), key=lambda kv:-kv[1]['avg_ms']*kv[1]['launches_per_step'])[:3]))
"
done
