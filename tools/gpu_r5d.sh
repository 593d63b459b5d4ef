# exposed epilogue steps freely scheduled in the specialized k_step2: forward only (default build)
# and forward + dgrad (libmarf_free2.so): parity / bitwise tests on each, same-box A/B, stamps
set -o pipefail
mkdir -p gpurun_out/r5d
for L in "" libmarf_fwd.so; do
  if [ -n "$L" ]; then export MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/$L; fi
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
     -k "bitwise or c3_two_patch or odd_width or fused_step or c1_3000 or step2 or dataset_npz" > gpurun_out/r5d/tests_${L:-default}.log 2>&1
  RC=$?; tail -1 gpurun_out/r5d/tests_${L:-default}.log
  case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
  unset MARF_LIB
done
bash tools/ab_r4.sh free "base=|libmarf_base.so" "fwd=|libmarf_fwd.so" "both=|" || exit 1
