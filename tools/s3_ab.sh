#!/bin/bash
# Timing A/B of library variants (built here: python build_lib.py --variant libmarf_<x>.so "<flags>"):
# one bench line each, alternating, no tests.   bash tools/s3_ab.sh <tag> <variant.so|default> ...
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
LIBD=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib
for rep in 1 2; do
  for v in "$@"; do
    n=${v%.so}
    if [ "$v" = default ]; then L=$LIBD/libmarf.so; else L=$LIBD/$v; fi
    AB=1; [ "$v" = default ] && AB=0
    MARF_AB_TIMING_ONLY=$AB MARF_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_${n}_$rep.json 2> $OUT/bench_${n}_$rep.err \
      || { echo "bench $n failed"; tail -5 $OUT/bench_${n}_$rep.err; exit 1; }
    echo "== $n (rep $rep)"
    python tools/bench_summary.py $OUT/bench_${n}_$rep.json | head -4
  done
done
