#!/bin/bash
# LDS / texture-address-unit occupancy of k_step3 (one rocprofv3 --pmc pass per counter set).
#   bash tools/pmc_lds.sh <tag>
TAG=${1:-pmclds}
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -oE "\b(SQ_LDS[A-Z_]*|SQ_INST_CYCLES_[A-Z_]*|SQ_INSTS_[A-Z_]*|TA_[A-Z_]*BUSY[A-Z_]*|TA_[A-Z_]*STALL[A-Z_]*|TD_[A-Z_]*BUSY[A-Z_]*|SQ_WAIT[A-Z_]*|SQ_IFETCH[A-Z_]*|SQC_[A-Z_]*MISS[A-Z_]*)\b" $OUT/counters.txt | sort -u > $OUT/names.txt
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/pass$i -o run \
     --kernel-include-regex "k_step3" -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $OUT/pass$i.log 2>&1
  rc=$?
  echo "pass $i ($CTRS): exit $rc"
  [ $rc -ne 0 ] && { tail -3 $OUT/pass$i.log; }
done <<'LIST'
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
TA_TA_BUSY_sum TA_BUSY_avr
SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_IFETCH
LIST
