#!/bin/bash
# PMC counter passes over a short bench run (each pass its own rocprofv3 process, kernel-trace only).
# Usage on the GPU box from the repo root: bash tools/pmc.sh <tag>   (PMC_BENCH_ARGS: extra bench.py args)
TAG=${1:-pmc}
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/pass$i -o run \
     --kernel-include-regex "${PMC_REGEX:-k_mlp|k_wgrad|k_step2|k_step3|k_prologue}" -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render $PMC_BENCH_ARGS > $OUT/pass$i.log 2>&1
  rc=$?
  echo "pass $i ($CTRS): exit $rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/pass$i.log; break; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
LIST
