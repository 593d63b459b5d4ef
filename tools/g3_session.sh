set -o pipefail
O=gpurun_out/g3
mkdir -p $O
LIBD=masking-bundle-adjusting-neural-radiance-fields_amd/lib
for SH in c3x2 c1; do
  EMU_SHAPE=$SH MARF_LIB=$PWD/$LIBD/libmarf_rtg.so timeout -k 10 300 python -u tools/emu_grad_err.py base=0000 x3=22211,2221,2221,2221,2222 \
    e1=42311,4231,4231,4231,4232 e1_l0lo=44311,4231,4231,4231,4232 e1_hidlo=42311,4241,4241,4241,4242 e1_wbf=22311,2231,2231,2231,2232 \
    > $O/emu_$SH.log 2>&1 || { echo "emu $SH failed"; tail -5 $O/emu_$SH.log; exit 1; }
  grep "^$SH" $O/emu_$SH.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "bits_unchanged or headline or captured" -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_bits.log 2>&1; rc=$?
echo "bits rc $rc"; tail -3 $O/t_bits.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_fp16x2.py -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1; rc=$?
echo "pytest fp16x2 rc $rc"; grep -E "passed|failed" $O/t.log | tail -3
[ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --precision fp16x2 --steps 10 --warmup 2 --no-cpu-baseline --no-render > $O/b_h$rep.json 2> $O/b_h$rep.err || exit 3
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render > $O/b_x3$rep.json 2> $O/b_x3$rep.err || exit 4
done
python -c "
import json
for f in ('b_h1','b_x31','b_h2','b_x32'):
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); r=d['roofline']
    print(f, '%.4g px/s %.3f ms/step kernel %.3f ms frac %.3f' % (d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac']), {k: round(v['avg_ms']*v['launches_per_step'],3) for k,v in d['kernels'].items() if v['avg_ms']*v['launches_per_step']>0.02})
"
