# multi-rank bench rehearsal on a one-GPU box: ranks share cuda:0 and exchange over gloo (RCCL needs
# one GPU per rank); exercises the per-layer bucketed all-reduce path of bench.py / Model
set -o pipefail
mkdir -p gpurun_out/r4m
for N in 2 4; do
  MARF_BENCH_ONE_DEVICE=1 MARF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 5 --warmup 2 \
    --strong 64 --no-render > gpurun_out/r4m/bench_n$N.json 2> gpurun_out/r4m/bench_n$N.err || { echo "N=$N failed"; tail -5 gpurun_out/r4m/bench_n$N.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r4m/bench_n$N.json').read().strip().splitlines()[-1])
print('N=$N', d['n_gpus'], '%.4g px/s' % d['value'], '%.2f ms/step' % d['ms_per_step'], d['scaling'], d['config']['parallelism'], 'loss %.9g' % d['config']['loss_rgb_last'])"
done
