#!/bin/bash
# C5 (128 patches x 256^2 per GPU, 8 x 512 MLP, plain bf16) bench lines: the fused tile step at one
# 512-thread block per CU and TP = 128 (default) against two 4-wave blocks at TP = 64
# (MARF_STEP_NW=4), c2f on and off.   bash tools/c5_ab.sh <tag>
OUT=$PWD/gpurun_out/${1:-c5}
mkdir -p $OUT
for nw in 8 4; do
  for c2f in on off; do
    extra=""; [ $c2f = off ] && extra="--no-c2f"
    MARF_STEP_NW=$nw timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-render $extra \
      > $OUT/c5_nw${nw}_$c2f.json 2> $OUT/c5_nw${nw}_$c2f.err || { echo "c5 nw$nw $c2f failed $?"; tail -3 $OUT/c5_nw${nw}_$c2f.err; exit 1; }
    echo "nw$nw c2f $c2f: $(python tools/bench_summary.py $OUT/c5_nw${nw}_$c2f.json | head -2 | tr '\n' ' ')"
  done
done
