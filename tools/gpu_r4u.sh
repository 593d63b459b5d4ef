# deferred last-row-tile epilogues in the specialized k_step2: GPU parity suite subset, same-box A/B, phase stamps
set -o pipefail
mkdir -p gpurun_out/r4u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "bitwise or c3_two_patch or odd_width or fused_step or c1_3000 or step2 or dataset_npz" > gpurun_out/r4u/tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4u/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
bash tools/ab_r4.sh defer "base=|libmarf_base.so" "new=|" || exit 1
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 300 python tools/step2_phases.py --kernel step2 > gpurun_out/r4u/phases_step2.txt 2>&1 || { echo "phases failed"; exit 1; }
cat gpurun_out/r4u/phases_step2.txt
