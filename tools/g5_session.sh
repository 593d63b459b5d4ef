set -o pipefail
O=gpurun_out/g5
mkdir -p $O
LIBD=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib
# the real fp16x2 kernel over the 120 committed one-ulp draws, and the emulated recipe (E1) on the
# draws the first emulation sweep did not finish plus the unperturbed seed-3 draw
timeout -k 10 900 python -u tools/basin_table.py --draws 25-144 --workers 3 --chunk 10 --deadline 600 --hard-deadline 840 \
  --out $O/basin "fp16x2=fp16x2" "e1=fp32:MARF_LIB=$LIBD/libmarf_rtg.so,MARF_DIAG_PREC=42311,4231,4231,4231,4232" > $O/basin.log 2>&1; rc=$?
tail -4 $O/basin.log; [ $rc -le 1 ] || exit $rc
MARF_LIB=$LIBD/libmarf_rtg.so MARF_DIAG_PREC=42311,4231,4231,4231,4232 timeout -k 10 200 python -u tools/seed_sweep.py --seeds 3 --precisions fp32 \
  --perturb 0 104 112 --out $O/e1_extra.json > $O/e1_extra.log 2>&1 || exit 5
grep "seed 3" $O/e1_extra.log
for rep in 1 2; do
  for v in default nodma nosave nodma_nosave; do
    if [ $v = default ]; then L=""; TO=""; else L=$LIBD/libmarf_ab_$v.so; TO=1; fi
    MARF_LIB=$L MARF_AB_TIMING_ONLY=$TO timeout -k 10 200 python bench.py --precision fp16x2 --steps 10 --warmup 2 --no-cpu-baseline --no-render \
      > $O/ab_$v$rep.json 2> $O/ab_$v$rep.err || { echo "ab $v failed"; tail -3 $O/ab_$v$rep.err; exit 6; }
  done
done
for c in "bf16x3 --graph" "fp16x2 --graph" "bf16x3"; do
  timeout -k 10 200 python bench.py --config c1 --precision $c --steps 30 --warmup 3 --no-cpu-baseline --no-render > "$O/c1_${c// /}.json" 2>&1 || exit 7
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/g5/ab_*.json")) + sorted(glob.glob("gpurun_out/g5/c1_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); r = d["roofline"] or {}
    print(f.split("/")[-1], "%.4g px/s %.3f ms/step kernel %.3f ms" % (d["value"], d["ms_per_step"], r.get("avg_launch_ms", 0)))
PY
