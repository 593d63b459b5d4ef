# same-box A/B of step kernels: bash tools/ab_r4.sh <tag> "<name>=<env>|<lib>" ...  (lib empty: default)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}; envs=${rest%%|*}; lib=${rest#*|}
    if [ -n "$lib" ]; then L="MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/$lib"; else L=""; fi
    env $envs $L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render $AB_ARGS > gpurun_out/ab_${TAG}_${name}_$round.json 2> gpurun_out/ab_${TAG}_${name}_$round.err || { echo "$name failed"; tail -3 gpurun_out/ab_${TAG}_${name}_$round.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab_${TAG}_${name}_$round.json').read().strip().splitlines()[-1])
kk = d.get('kernels', {}); wg = ' '.join('%s %.3f' % (k, v['avg_ms']) for k, v in sorted(kk.items()) if k.startswith('wgrad'))
print('%-10s r$round %.4g px/s  %.3f ms/step  %s %.3f ms  [%s]  loss %.9g' % ('$name', d['value'], d['ms_per_step'], d['config']['step_kernel'], d['roofline']['avg_launch_ms'], wg, d['config']['loss_rgb_last']))
"
  done
done
