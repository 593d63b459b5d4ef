"""Multi-process plumbing of the patch-sharded data parallelism, on CPU with gloo (world size 2):
rank -> patch range, the global masked-MSE denominator, the MLP-gradient all-reduce over the flat
gradient buffer, and the gather of rank-local warp rows.  No kernels run here."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, q):
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import options
        from model import planar
        from util import EasyDict as edict
        opt = options.load_options("options/planar.yaml")
        opt = options.override_options(opt, edict({"model": "planar", "yaml": "planar", "seed": 3,
                                                    "barf_c2f": [0, 0.4], "batch_size": B,
                                                    "arch": {"layers": [None, 32, 32, 3], "skip": [],
                                                             "posenc": {"L_2D": 4}}}))
        opt.device = "cpu"
        opt.output_path = f"/tmp/marf_dist_test_{port}_{rank}"
        torch.manual_seed(3)
        m = planar.Model(opt)
        masks = torch.zeros(B, 1, 18, 24)
        masks[:, :, ::2] = 1
        m.images = edict(rgb=torch.rand(B, 3, 18, 24), masks=masks)
        m.build_networks()
        g = m.graph
        ps = g.neural_image._params()  # MLP parameters become views of one flat buffer
        for i, p in enumerate(ps):
            p.grad = torch.full_like(p, float(rank + 1))
        # make the grads views of one flat buffer too, as the backward kernel produces them
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        off = 0
        for p in ps:
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        m.all_reduce_grads()
        b0, b1 = g.shard
        g.warp_param.weight.data[b0:b1] = rank + 1
        w = m.gathered_warps()
        q.put((rank, g.shard, float(g.loss_denominator), float(flat.min()), float(flat.max()), w.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("B", [4, 5])
def test_two_rank_sharding_and_allreduce(B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, d0, lo0, hi0, w0), (r1, s1, d1, lo1, hi1, w1) = res
    assert s0 == (0, B // 2) and s1 == (B // 2, B)
    assert d0 == d1 == 3 * B * 9 * 24  # global 3 * sum(mask), identical on both ranks
    assert lo0 == hi0 == lo1 == hi1 == 3.0  # 1 + 2 summed over ranks
    assert w0 == w1
    for b in range(B):
        assert w0[b] == [1.0 if b < B // 2 else 2.0] * 8


def _bench(args, **env_over):
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                                "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env.update(MARF_BENCH_ONE_DEVICE="1", MARF_BENCH_BACKEND="gloo", **env_over)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return r.returncode, lines, r.stderr


def test_bench_gpus_flag_launches_the_ranks():
    """`bench.py --gpus 2` outside a launcher starts two ranks itself (torch.distributed.run child,
    before any GPU call) and the JSON line reports the world size the process group has and its
    backend; a launcher whose WORLD_SIZE disagrees with --gpus is refused (bench.py main)."""
    rc, lines, err = _bench(["--gpus", "2", "--launch-check"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines  # rank 0 prints the one line
    d = lines[0]
    assert d["n_gpus"] == 2 and d["dist"]["world_size"] == 2 and d["dist"]["backend"] == "gloo", d
    assert "torch.distributed.run" in d["dist"]["launcher"], d
    rc, lines, err = _bench(["--gpus", "2", "--launch-check"], WORLD_SIZE="1")
    assert rc != 0 and not lines and "WORLD_SIZE" in err
    rc, lines, err = _bench(["--launch-check"])
    assert rc == 0 and lines[0]["n_gpus"] == 1 and lines[0]["dist"]["world_size"] == 1, (rc, lines, err[-500:])
