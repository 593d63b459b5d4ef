# layer-0 epilogue as whole pairs per MFMA gap (k_step2): bitwise / parity tests, same-box A/B, layer-0 stamps
set -o pipefail
mkdir -p gpurun_out/r4q
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "bitwise or c3_two_patch or odd_width or fused_step" > gpurun_out/r4q/tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4q/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
bash tools/ab_r4.sh l0pk "base=|libmarf_base.so" "new=|" || exit 1
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stampsl0.so timeout -k 10 300 python tools/step2_phases.py --kernel step2 > gpurun_out/r4q/phases_step2_l0.txt 2>&1 || { echo "phases failed"; exit 1; }
grep -E "layer 0|GEMM bodies|outside|finish|total" gpurun_out/r4q/phases_step2_l0.txt
