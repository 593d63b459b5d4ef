export TMPDIR=/tmp
ROOT=$PWD
OUT=$PWD/gpurun_out/ifetch
mkdir -p $OUT
timeout -k 5 30 ./tools/glds_offset_probe > $OUT/probe.txt 2>&1; echo probe $?
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pass1 -o run --kernel-include-regex "k_step2" -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $OUT/pass1.log 2>&1; echo pmc $?
