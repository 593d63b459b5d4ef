#!/bin/bash
# C5 (8 x 512, plain bf16) tile width A/B: k_mlp_step at TP = 64 (2 blocks / CU) vs 128 (1 block / CU).
# bash tools/c5_tp.sh <tag>
set -o pipefail
TAG=${1:-c5tp}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
MARF_STEP_TP=128 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "c5_shape or wgrad_dma_wide" \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/tests_tp128.log 2>&1 || { echo "tests failed"; tail -5 $OUT/tests_tp128.log; exit 1; }
tail -1 $OUT/tests_tp128.log
for r in 1 2; do
  for tp in 64 128; do
    MARF_STEP_TP=$tp timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-render \
      > $OUT/c5_tp${tp}_$r.json 2> $OUT/c5_tp${tp}_$r.err || { echo "bench tp$tp failed"; tail -3 $OUT/c5_tp${tp}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], '%.4g px/s %.2f ms %s %.2f ms frac %.4f' % (d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac']))" $OUT/c5_tp${tp}_$r.json tp$tp
  done
done
