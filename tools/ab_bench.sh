#!/bin/bash
# A/B of library variants on the bench: bash tools/ab_bench.sh <tag> lib1.so lib2.so ... ("default" = libmarf.so)
TAG=$1; shift
OUT=$PWD/gpurun_out; mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = default ]; then L=""; else L=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/$v; fi
  MARF_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/ab_${TAG}_$v.json 2> $OUT/ab_${TAG}_$v.err || { echo "$v failed"; tail -3 $OUT/ab_${TAG}_$v.err; exit 1; }
  python - $OUT/ab_${TAG}_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print("%-16s %.4g px/s  %.3f ms/step  " % (sys.argv[2], d["value"], d["ms_per_step"]) +
      "  ".join("%s %.3f" % (n, k[n]["avg_ms"]) for n in ("mlp_step", "wgrad_hidden", "wgrad_l0") if n in k))
PY
done
