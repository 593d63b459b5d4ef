# PMC passes (SQ busy / MFMA / LDS / VMEM, FETCH / WRITE, L2 hit) of the committed library's C3 step
set -o pipefail
PMC_REGEX="k_step2|k_wgrad" bash tools/pmc.sh r5c_pmc > gpurun_out/r5c_pmc.log 2>&1; tail -6 gpurun_out/r5c_pmc.log
