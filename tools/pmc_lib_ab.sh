#!/bin/bash
# One SQ counter pass (LDS bank conflicts, LDS waits, issue stalls, instruction counts) over a short
# C3 bench for the product library and lib/libmarf_<v>.so variants, restricted to kernels matching
# $PMC_REGEX (default: the hidden-layer weight gradients):
#   bash tools/pmc_lib_ab.sh <tag> <v1> [v2 ...]   ("default" = lib/libmarf.so)
TAG=$1; shift
ROOT=$PWD; OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT; LIBD=$ROOT/masking-bundle-adjusting-neural-radiance-fields_amd/lib
for v in "$@"; do
  if [ "$v" = default ]; then L=""; else L=$LIBD/libmarf_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && MARF_LIB=$L timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/pmc_$v -o run --kernel-include-regex "${PMC_REGEX:-k_wgrad_dma_layers}" -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $OUT/pmc_$v.log 2>&1) || { echo "pmc $v failed"; tail -3 $OUT/pmc_$v.log; exit 1; }
done
