#!/bin/bash
# A/B of environment settings on the bench: bash tools/ab_env.sh <tag> "ENV=1 ENV2=x" "" ...  ("" = defaults)
TAG=$1; shift
OUT=$PWD/gpurun_out; mkdir -p $OUT
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/abe_${TAG}_$i.json 2> $OUT/abe_${TAG}_$i.err || { echo "[$e] failed"; tail -3 $OUT/abe_${TAG}_$i.err; exit 1; }
  python - $OUT/abe_${TAG}_$i.json "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print("%-24s %.4g px/s  %.3f ms/step  " % (sys.argv[2] or "default", d["value"], d["ms_per_step"]) +
      "  ".join("%s %.3f" % (n, k[n]["avg_ms"]) for n in ("mlp_step", "wgrad_hidden", "wgrad_l0") if n in k))
PY
done
