# round-4 validation: GPU suite + bench + rocprof stats (gpu_round.sh), smoke, feat_0 recompute A/B
set -o pipefail
bash tools/gpu_round.sh r4g || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r4g.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_r4g.log; exit 1; }
tail -1 gpurun_out/smoke_r4g.log
bash tools/ab_r4.sh f0 "rec1=MARF_F0_RECOMPUTE=1|" "rec0=MARF_F0_RECOMPUTE=0|"
bash tools/ab_r4.sh wg "base=|" "nt=|libmarf_wgnt.so" "sp64=|libmarf_sp64.so" "ntsp64=|libmarf_ntsp64.so"
PMC_REGEX="k_mlp_step" PMC_BENCH_ARGS="--config c5" bash tools/pmc.sh r4g_c5pmc > gpurun_out/r4g_c5pmc.log 2>&1; tail -6 gpurun_out/r4g_c5pmc.log
