# round 6: the dW_last restructure (libmarf.so) against the previous library (libmarf_prev.so):
# the GPU suite on the new library, then C3 benches of both libraries alternating, bf16x3 and fp16x2
set -o pipefail
O=gpurun_out/g9
mkdir -p $O
LIBD=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib
bash tools/gpu_session.sh g9 tests || exit 1
for rep in 1 2; do
  for P in bf16x3 fp16x2; do
    for v in prev new; do
      if [ $v = prev ]; then L=$LIBD/libmarf_prev.so; else L=""; fi
      MARF_LIB=$L timeout -k 10 200 python bench.py --precision $P --steps 10 --warmup 2 --no-cpu-baseline --no-render > $O/b_${P}_${v}_$rep.json 2> $O/b_${P}_${v}_$rep.err || { echo "bench $P $v failed"; tail -5 $O/b_${P}_${v}_$rep.err; exit 1; }
      python tools/bench_summary.py $O/b_${P}_${v}_$rep.json 2>/dev/null || tail -c 300 $O/b_${P}_${v}_$rep.json
    done
  done
done
