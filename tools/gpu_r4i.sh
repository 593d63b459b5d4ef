# GPU suite + bench on the library with the 64-row layer-0 weight-gradient stages; fp32 basin draws 25-64
set -o pipefail
mkdir -p gpurun_out/r4i
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4i/gpu_tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4i/gpu_tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
timeout -k 10 400 python bench.py > gpurun_out/r4i/bench.json 2> gpurun_out/r4i/bench.err || { echo "bench failed"; tail -5 gpurun_out/r4i/bench.err; exit 1; }
tail -1 gpurun_out/r4i/bench.json | cut -c1-300
timeout -k 10 720 python -u tools/seed_sweep.py --precisions fp32 --seeds 3 --perturb $(seq 25 64) \
    --out gpurun_out/r4i/basin_fp32_p25_64.json > gpurun_out/r4i/sweep_fp32.log 2>&1 || { echo "sweep failed"; tail -3 gpurun_out/r4i/sweep_fp32.log; exit 1; }
tail -1 gpurun_out/r4i/sweep_fp32.log
