# ring-wait accounting fix in k_step2 (layer-0 stages: up to 12 stores + the 3 prologue loads):
# bitwise / parity tests, same-box A/B against the previous build, phase stamps
set -o pipefail
mkdir -p gpurun_out/r4o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "bitwise or c3_two_patch or odd_width or fused_step" > gpurun_out/r4o/tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4o/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
bash tools/ab_r4.sh wait "base=|libmarf_base.so" "new=|" || exit 1
for k in step2 step3; do
  MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 300 python tools/step2_phases.py --kernel $k > gpurun_out/r4o/phases_$k.txt 2>&1 || { echo "phases $k failed"; tail -5 gpurun_out/r4o/phases_$k.txt; exit 1; }
done
cat gpurun_out/r4o/phases_step2.txt
