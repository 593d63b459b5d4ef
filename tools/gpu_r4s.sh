# k_step2 compile-time instantiations for the adjoint / dW_last too, and (3, 2), (4, 2) for L = 8..12:
# parity / bitwise tests, same-box A/B at C3, then the k_step2 / k_step3 crossover again (C3-shaped
# batches of 2..64 patches, and C1)
set -o pipefail
mkdir -p gpurun_out/r4s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "bitwise or c3_two_patch or odd_width or fused_step or c1_3000 or step2 or dataset_npz" > gpurun_out/r4s/tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4s/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
bash tools/ab_r4.sh adj "base=|libmarf_base.so" "new=|" || exit 1
for B in 2 4 8 16 32 64; do
for k in 0 1; do
  MARF_STEP3=$k timeout -k 10 300 python bench.py --config c3 --strong $B --steps 20 --warmup 3 --no-cpu-baseline --no-render > gpurun_out/r4s/x_${B}_${k}.json 2> gpurun_out/r4s/x_err || { tail -3 gpurun_out/r4s/x_err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r4s/x_${B}_${k}.json').read().strip().splitlines()[-1])
print('B=$B MARF_STEP3=$k %.4g px/s %.3f ms/step %s %.3f ms' % (d['value'], d['ms_per_step'], d['config']['step_kernel'], d['roofline']['avg_launch_ms']))"
done
done
for k in 0 1; do
  MARF_STEP3=$k timeout -k 10 300 python bench.py --config c1 --steps 20 --warmup 3 --no-cpu-baseline --no-render > gpurun_out/r4s/c1_${k}.json 2> gpurun_out/r4s/x_err || { tail -3 gpurun_out/r4s/x_err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r4s/c1_${k}.json').read().strip().splitlines()[-1])
print('C1 MARF_STEP3=$k %.4g px/s %.3f ms/step %s %.3f ms' % (d['value'], d['ms_per_step'], d['config']['step_kernel'], d['roofline']['avg_launch_ms']))"
done
