#!/bin/bash
# One GPU session for the two-waves-per-SIMD kernel: quick bf16x3 parity tests, bench lines (new /
# old kernel), per-phase stamps (libmarf_stamps.so), two PMC passes, then the 25-draw seed-3 basin
# sweep.   bash tools/s3_session.sh <tag> [sweep: 0/1]
set -o pipefail
TAG=${1:-s3s}
SWEEP=${2:-1}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
bash tools/s3_check.sh $TAG || exit $?
MARF_STEP3=1 MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 200 \
  python tools/step2_phases.py --kernel step3 > $OUT/phases.txt 2>&1 || { echo "phases failed"; tail -5 $OUT/phases.txt; exit 1; }
cat $OUT/phases.txt | grep -v amdgpu.ids
export TMPDIR=/tmp
ROOT=$PWD
i=0
while read -r CTRS; do
  i=$((i+1))
  (cd /tmp && MARF_STEP3=1 timeout -k 10 200 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT/pmc/pass$i -o run \
     --kernel-include-regex "k_step" -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $OUT/pmc_pass$i.log 2>&1) \
     || { echo "pmc pass $i failed"; tail -3 $OUT/pmc_pass$i.log; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
LIST
python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt 2>&1; cat $OUT/pmc_summary.txt
[ "$SWEEP" = "1" ] || exit 0
MARF_STEP3=1 timeout -k 10 600 python -u tools/seed_sweep.py --precisions bf16x3 --seeds 3 --perturb $(seq 0 24) \
  --out $OUT/basin_step3.json > $OUT/sweep.log 2>&1
echo "sweep exit $?"; tail -3 $OUT/sweep.log
