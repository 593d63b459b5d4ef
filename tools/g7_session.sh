set -o pipefail
O=gpurun_out/g7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "bits_unchanged or headline or captured or wide_skip" -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_bits.log 2>&1; rc=$?
echo "bits rc $rc"; tail -2 $O/t_bits.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp16x2.py -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1; rc=$?
echo "fp16x2 tests rc $rc"; grep -E "^fp16x2 \{|passed|failed|headline" $O/t.log | tail -12; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u tools/basin_table.py --draws 0,25-144 --workers 3 --chunk 11 --deadline 500 --hard-deadline 780 \
  --out $O/basin "fp16x2=fp16x2" > $O/basin.log 2>&1; rc=$?
tail -2 $O/basin.log; grep "perturb 0:" $O/basin/*.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --precision fp16x2 --steps 10 --warmup 2 --no-cpu-baseline --no-render > $O/b_h$rep.json 2> $O/b_h$rep.err || exit 3
done
python -c "
import json
for f in ('b_h1','b_h2'):
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); r=d['roofline']
    print(f, '%.4g px/s %.3f ms/step kernel %.3f ms frac %.3f' % (d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac']), {k: round(v['avg_ms']*v['launches_per_step'],3) for k,v in d['kernels'].items() if v['avg_ms']*v['launches_per_step']>0.02})
"
