#!/bin/bash
# PMC passes on the vector-memory path of the step kernel (TA / TD / TCP busy and stall cycles, SQ
# FIFO-full counts): is the CU's address / data path the bound?  Each pass its own rocprofv3 run,
# kernel-trace only.  Usage on the GPU box from the repo root: bash tools/pmc_vmem.sh <tag>
TAG=${1:-vmem}
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/pass$i -o run \
     --kernel-include-regex "k_step2" -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $OUT/pass$i.log 2>&1
  rc=$?
  echo "pass $i ($CTRS): exit $rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/pass$i.log; break; }
done <<'LIST'
SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_LDS_DATA_FIFO_FULL SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE
TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE
LIST
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(out + "/pass*/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(float)
    for r in rows:
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, n), v in per.items():
        acc[n].append(v)
for n in sorted(acc):
    v = acc[n]
    print("%-40s %.4g (mean over %d dispatches)" % (n, sum(v) / len(v), len(v)))
PY
