set -o pipefail
O=gpurun_out/g2
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_fp16x2.py -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1; rc=$?
echo "pytest fp16x2 rc $rc"; tail -15 $O/t.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --precision fp16x2 --steps 10 --warmup 2 --no-cpu-baseline --no-render > $O/b_h.json 2> $O/b_h.err || exit 3
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > $O/b_x3.json 2> $O/b_x3.err || exit 4
  python -c "import json;[print(f, (lambda d:(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac']))(json.loads(open('$O/'+f).read().strip().splitlines()[-1]))) for f in ('b_h.json','b_x3.json')]"
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "bits_unchanged or headline or grouping or captured" -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_bits.log 2>&1; echo "bits rc $?"; tail -5 $O/t_bits.log
fi
