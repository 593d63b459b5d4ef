set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread -k "step3_bitwise or odd_width or c3_two_patch" -s > gpurun_out/t_r4c.log 2>&1
RC=$?
grep -E "differs|passed|failed" gpurun_out/t_r4c.log | tail -30
case $RC in 0|1) ;; *) echo "pytest died ($RC)"; exit $RC;; esac
for k in step3 step2; do
  if [ $k = step3 ]; then export MARF_STEP3=1; else unset MARF_STEP3; fi
  MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 300 python tools/step2_phases.py --kernel $k > gpurun_out/phases_r4c_$k.txt 2>&1 || { echo "phases $k failed"; tail -5 gpurun_out/phases_r4c_$k.txt; exit 1; }
  cat gpurun_out/phases_r4c_$k.txt
done
export MARF_STEP3=1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_r4c/p1 -o run --kernel-include-regex "k_step" -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $GRAFT_REPO_ROOT/gpurun_out/pmc_r4c_p1.log 2>&1
echo "pmc p1 exit $?"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_r4c/p2 -o run --kernel-include-regex "k_step" -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $GRAFT_REPO_ROOT/gpurun_out/pmc_r4c_p2.log 2>&1
echo "pmc p2 exit $?"
