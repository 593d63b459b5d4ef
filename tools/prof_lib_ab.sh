#!/bin/bash
# rocprofv3 kernel traces of a short C3 (or $CFG) bench for the product library and lib/libmarf_<v>.so
# variants, one process each:  bash tools/prof_lib_ab.sh <tag> <v1> [v2 ...]   ("default" = lib/libmarf.so)
TAG=$1; shift
ROOT=$PWD; OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
LIBD=$ROOT/masking-bundle-adjusting-neural-radiance-fields_amd/lib
for v in "$@"; do
  if [ "$v" = default ]; then L=""; else L=$LIBD/libmarf_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && MARF_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- \
     python3 $ROOT/bench.py --config ${CFG:-c3} --steps 6 --warmup 2 --no-cpu-baseline --no-render > $OUT/$v.log 2>&1) || { echo "prof $v failed"; tail -5 $OUT/$v.log; exit 1; }
done
