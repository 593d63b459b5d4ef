#!/bin/bash
# PMC passes on instruction supply and issue of the step kernel: I-cache requests / misses, the
# instruction mix and the wave-cycle split.  bash tools/pmc_ifetch.sh <tag>
TAG=${1:-ifetch}
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
SQC_ICACHE_MISSES SQC_ICACHE_REQ GRBM_GUI_ACTIVE
SQC_ICACHE_HITS SQC_TC_INST_REQ SQC_TC_STALL GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
LIST
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(out + "/pass*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, n), v in per.items():
        acc[n].append(v)
for n in sorted(acc):
    v = acc[n]
    print("%-32s %.4g" % (n, sum(v) / len(v)))
PY
