"""Throughput of the planar bundle-adjustment training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c1|c5] [--precision bf16x3|fp16x2|bf16|fp16|fp32]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step is one full Model.train_iteration of the product (model/planar.py): fused
grid->warp->posenc->MLP forward, masked MSE, backward (dgrad chain, warp adjoint, weight
gradients), the RCCL all-reduce of the MLP gradient (N > 1), Adam, progress update, fix_first.
Workload (BASELINE.json configs[2]): per GPU 64 patches of 256x256 pixels cropped
from a 512x512 canvas, L=16 posenc, MLP 66-256-256-256-256-3, c2f [0,0.4] at progress 0.2, in
the precision recipe that carries the seed-3 end-to-end contract: bf16x3 (split-bf16 hi+lo MFMA
operands with fp32 accumulation: forward hi*hi+hi*lo+lo*hi, dgrad W_hi^T dz + W_lo^T dz; DESIGN.md
§4).  --precision bf16 (plain bf16 MFMA) and fp32 are the other recipes.  Synthetic targets (smooth procedural RGB, seed 0), Bernoulli(0.85) masks (seed 1),
warps ~ N(0, 0.01^2) (seed 2, patch 0 fixed).  Weak scaling: 64 patches per GPU at every N.

Prints one JSON line (rank 0).  `value` = pixels processed by all ranks per second.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "masking-bundle-adjusting-neural-radiance-fields_amd")
sys.path.insert(0, PKG)

METRIC = "warped+encoded+MLP pixels/s/GPU; final PSNR vs ref (seed=3)"
PEAK_BF16 = 2.5e15   # dense bf16 MFMA, MI355X_MICROARCH.md
PEAK_FP32 = 157.3e12  # fp32 MFMA = vector rate
PEAK_HBM = 8.0e12
RECIPES = {"bf16x3": "bf16x3 recipe (split-bf16 hi+lo MFMA operands, fp32 accumulate; seed-3 parity)",
           "fp16x2": "fp16x2 recipe (fp16 hi+lo weights x fp16 activations / dz, 2 MFMAs per MAC; fp32 accumulate)",
           "bf16": "plain bf16 MFMA (fp32 accumulate)", "fp16": "plain fp16 MFMA (fp32 accumulate)", "fp32": "fp32"}

CONFIGS = {
    # name: (canvas, crop, patches per GPU, L, hidden layers)
    "c3": (512, 256, 64, 16, [256, 256, 256, 256]),
    "c1": (None, None, 5, 8, [256, 256, 256, 256]),
    "c5": (512, 256, 128, 16, [512] * 8),
}


def flops_per_px(dims):
    """Algorithmic FLOPs of one pixel through a training step: 6 * sum k_in*k_out (fwd 2, dgrad 2,
    wgrad 2 per MAC)."""
    return 6 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))


def step_kernel_bytes(S, Kp0, hidden, elem):
    """Algorithmic HBM bytes per launch of the store-activations decomposition (each value moved
    once): the fused step reads targets + masks (16 B/px, fp32) and its own ReLU-mask records back,
    and writes rgb (12 B/px), every saved layer input feat_0..feat_{n-2}, every dz_1..dz_{n-1} (elem bytes per
    feature), the ReLU-mask records (1 bit per hidden feature) and the per-tile last-layer gradient
    partials; each weight-gradient kernel reads dz_{l+1} and feat_l once."""
    n_h = len(hidden)
    masks = S * sum(hidden) // 8
    feat = S * elem * (Kp0 + sum(hidden[:-1]))
    dz = S * elem * sum(hidden)
    wlast = (S // 128) * 4 * 3 * hidden[-1]
    return {
        "mlp_step": 16 * S + 12 * S + masks + feat + dz + wlast + masks,
        "wgrad_hidden": S * elem * (hidden[0] + hidden[0]) if n_h > 1 else 0,
        "wgrad_l0": S * elem * (Kp0 + hidden[0]),
    }


def pmc_traffic(cfg, precision, kernel, symbol_prefix):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py --traffic), or None unless the entry
    was measured on the library loaded now (same marf_source_hash) and on the same kernel
    instantiation kind (its symbol starts with `symbol_prefix`, e.g. the step kernel this size
    picked): a number from another build or kernel is never reported as this run's traffic."""
    import marf_hip
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))[f"{cfg}/{precision}"]
        e = d["kernels"][kernel]
        if d["source_hash"] != marf_hip.lib().marf_source_hash().decode():
            return None
        if symbol_prefix and not e["symbol"].startswith(symbol_prefix):
            return None
        return (e["hbm_read_bytes"] + e["hbm_write_bytes"], f"{d['source']}; {e['symbol']}; source hash {d['source_hash']}",
                {k: e.get(k) for k in ("mfma_busy", "valu_per_mfma", "SQ_INSTS_VMEM_RD")})
    except (OSError, KeyError, ValueError, TypeError):
        return None


def make_opt(cfg, precision, B_total, c2f=True):
    import options
    from util import EasyDict as edict
    canvas, crop, _, L, hidden = CONFIGS[cfg]
    opt = options.load_options("options/planar.yaml")
    over = {"model": "planar", "yaml": "planar", "seed": 3, "barf_c2f": [0, 0.4] if c2f else None, "batch_size": B_total,
            "precision": precision, "use_edges": False, "max_iter": 3000,
            "arch": {"layers": [None] + hidden + [3], "skip": [], "posenc": {"L_2D": L}}}
    if canvas:
        over.update(H=canvas, W=canvas, patch_H=crop, patch_W=crop)
    opt = options.override_options(opt, edict(over))
    opt.output_path = os.path.join(ROOT, "output", "bench")
    return opt


def synthetic_inputs(B_total, h, w, device):
    g0 = torch.Generator().manual_seed(0)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, h), torch.linspace(0, 1, w), indexing="ij")
    phase = torch.rand(B_total, 3, 1, 1, generator=g0) * 6.28
    freq = 1 + 3 * torch.rand(B_total, 3, 2, generator=g0)
    rgb = 0.5 + 0.4 * torch.sin(2 * np.pi * (freq[..., 0, None, None] * xx + freq[..., 1, None, None] * yy) + phase)
    g1 = torch.Generator().manual_seed(1)
    mask = (torch.rand(B_total, 1, h, w, generator=g1) < 0.85).float()
    g2 = torch.Generator().manual_seed(2)
    warp = torch.randn(B_total, 8, generator=g2) * 0.01
    warp[0] = 0
    return rgb.to(device), mask.to(device), warp.to(device)


def cpu_baseline(cfg, sample_patches):
    """SURVEY.md §8(d) CPU baseline: oracle/cpu_ref.py (op-for-op torch-CPU fp32 restatement of the
    reference step, pinned to the reference's fixtures by tests/test_cpu_ref.py) on a bounded slice
    of the same workload: `sample_patches` patches of the config, reference init (seed 3), c2f at
    progress 0.2, torch threads = every core this process may run on, 2 warm-up + >= 5 timed
    steps.  Pixels/s."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref
    cores = cpu_ref.set_threads()
    canvas, crop, _, L, hidden = CONFIGS[cfg]
    if canvas is None:
        canvas_h, canvas_w, ch, cw = 360, 480, 180, 240
    else:
        canvas_h = canvas_w = canvas
        ch = cw = crop
    D = 2 + 4 * L
    torch.manual_seed(3)
    params, k_in = [], D
    for li, k_out in enumerate(hidden + [3]):  # RNG-ordered reference init (model/planar.py:410-427)
        lin = torch.nn.Linear(k_in, k_out)
        if li == 0:
            lin.weight.data *= np.sqrt(D / 2.)
            lin.bias.data *= np.sqrt(D / 2.)
        params.append((lin.weight.detach().numpy().copy(), lin.bias.detach().numpy().copy()))
        k_in = k_out
    rgb, mask, warp = synthetic_inputs(sample_patches, ch, cw, torch.device("cpu"))
    c = dict(H=canvas_h, W=canvas_w, patch_H=ch, patch_W=cw, L=L, c2f=[0, 0.4], max_iter=10 ** 9, lr=1e-3,
             lr_warp=1e-3, fix_first=True, use_edges=False, alpha_initial=0.0, alpha_final=1.0)
    st = cpu_ref.CpuRefStep(c, params, warp.numpy(), rgb.numpy(), mask.numpy())
    times = []
    for i in range(7):
        st.progress.data.fill_(0.2)
        t0 = time.perf_counter()
        st.step()
        if i >= 2:
            times.append(time.perf_counter() - t0)
    px = sample_patches * ch * cw
    cpu = "unknown CPU"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": px / float(np.mean(times)), "unit": "pixels/s", "cores": int(cores), "kind": "port", "cpu": cpu,
            "sample": f"{sample_patches} patches x {ch}x{cw} px of {cfg}, 2 warm-up + {len(times)} timed "
                      f"oracle/cpu_ref.py steps (torch-CPU fp32, autograd, Adam), mean {np.mean(times):.2f} s/step"}


def prologue_rate(graph, var, L, c2f, n=20):
    """Achieved HBM rate of the step's input side (16 B/px target + mask reads),
    from a prologue-only launch (marf_prologue_probe) timed with HIP events on torch's stream, the
    stream the library launches on."""
    import marf_hip
    w = graph.warp_param.weight.detach()
    eng = graph.neural_image.engine(w.device)
    b0, b1 = graph.shard if graph.shard else (0, w.shape[0])
    Hm = marf_hip.sl3_to_SL3(w[b0:b1].contiguous())
    gt = var.images.rgb[b0:b1]
    mask = var.images.masks[b0:b1]
    prog = graph.neural_image.progress
    args = (gt, mask, Hm, eng.H, eng.W, eng.patch_H, eng.patch_W, L, prog, c2f)
    marf_hip.prologue_probe(*args)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        marf_hip.prologue_probe(*args)
    e1.record()
    e1.synchronize()
    s = e0.elapsed_time(e1) / n / 1e3
    nbytes = 16 * gt.shape[0] * gt.shape[2] * gt.shape[3]
    return {"kernel": "prologue_probe", "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": s * 1e3,
            "achieved": nbytes / s / 1e9, "unit": "GB/s", "peak": PEAK_HBM / 1e9, "frac": nbytes / s / PEAK_HBM}


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n):
    """Run this script on n ranks: python -m torch.distributed.run --nnodes=1 --nproc-per-node n
    --master-addr 127.0.0.1 (the driver's own launch line) as a child process; its exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MARF_BENCH_LAUNCHER="bench.py --gpus (torch.distributed.run child)")
    return subprocess.run(cmd, env=env).returncode


def alt_recipe(args, dev, precision="fp16x2"):
    """A second bench leg on one GPU (rank 0, world 1): the same workload in another recipe, timed the
    same way (warm-up, then args.steps steps between synchronizations, HIP events around the step
    kernel only), with its row of the committed basin table (profiles/basin_table.json).  The
    headline stays the recipe that carries the seed-3 contract; this reports what the
    faster recipe measures on the same box."""
    import marf_hip
    from model import planar
    from util import EasyDict as edict
    canvas, crop, per_gpu, L, hidden = CONFIGS[args.config]
    opt = make_opt(args.config, precision, per_gpu)
    opt.device = str(dev)
    torch.manual_seed(opt.seed)
    m = planar.Model(opt)
    rgb, mask, warp = synthetic_inputs(per_gpu, opt.patch_H, opt.patch_W, dev)
    m.images = edict(rgb=rgb, masks=mask, masks_eroded=mask, edges=None, gt_hom=None, gt=None)
    m.build_networks()
    m.graph.warp_param.weight.data.copy_(warp)
    m.graph.neural_image.progress.data.fill_(0.2)
    m.setup_optimizer()
    g = m.graph
    g.need_edges = False
    var = edict(idx=torch.arange(per_gpu), images=m.images)

    def step():
        m.optim.zero_grad()
        v = g.forward(var, mode="train")
        loss = m._loss_sum(g.compute_loss(v, mode="train"))
        loss.all.backward()
        m.optim.step()
        g.neural_image.progress.data.fill_(0.2)
        g.warp_param.weight.data[0] = 0
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    marf_hip.profile_reset()
    marf_hip.profile_filter(["mlp_step"])
    marf_hip.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    marf_hip.profile_enable(False)
    prof = marf_hip.profile_read()
    px = per_gpu * opt.patch_H * opt.patch_W
    dims = [2 + 4 * L] + hidden + [3]
    sum_mac = sum(a * b for a, b in zip(dims[:-1], dims[1:]))
    out = {"precision": precision, "recipe": RECIPES[precision], "value": px / (elapsed / args.steps),
           "unit": "pixels/s", "ms_per_step": elapsed / args.steps * 1e3,
           "loss_rgb_last": float(loss.rgb.detach()), "step_kernel": g.neural_image.engine(dev).net.step_kernel}
    if "mlp_step" in prof:
        avg_s = prof["mlp_step"][0] / prof["mlp_step"][1] / 1e3
        alg = px * (4 * sum_mac + 6 * dims[-2])
        out.update(kernel_avg_launch_ms=avg_s * 1e3, roofline_frac=alg / avg_s / PEAK_BF16)
        tr = pmc_traffic(args.config, precision, "mlp_step", out["step_kernel"])
        out.update(traffic=tr[0] if tr else None, mfma_busy=tr[2].get("mfma_busy") if tr else None,
                   valu_per_mfma=tr[2].get("valu_per_mfma") if tr else None)
    bt = os.path.join(ROOT, "profiles", "basin_table.json")
    if os.path.exists(bt):
        rows = json.load(open(bt))["recipes"]
        for name in (precision, "bf16x3"):
            if name in rows:
                r = rows[name]
                out[f"basin_{name}"] = {"basin": r["basin"], "draws": r["n"],
                                        "seed3_psnr_rule": (r.get("seed3") or {}).get("psnr_rule")}
    del m, g, var
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=list(CONFIGS))
    ap.add_argument("--precision", default=None, choices=["bf16x3", "fp16x2", "bf16", "fp16", "fp32"],
                    help="default bf16x3 (the seed-3 parity recipe); c5's 512-wide layers: bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c2f", action="store_true", help="barf_c2f None (BASELINE config 5: c2f on vs off)")
    ap.add_argument("--strong", type=int, default=0, metavar="PATCHES",
                    help="strong scaling: PATCHES in total split over the ranks (SURVEY §8d: 512)")
    ap.add_argument("--cpu-sample-patches", type=int, default=4)
    ap.add_argument("--no-render", action="store_true",
                    help="skip the forward-only render rate (PMC passes: its launches share the step kernel's name)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the whole iteration (forward, loss, backward, Adam, progress, fix_first) as one "
                         "captured HIP graph (Model.captured_step); "
                         "the per-kernel times and the roofline then come from eager steps")
    ap.add_argument("--no-alt-recipe", action="store_true",
                    help="skip the second leg (one GPU, c3, bf16x3 only): the same workload in the fp16x2 recipe")
    ap.add_argument("--launch-check", action="store_true",
                    help="set up the ranks and print the JSON line's world size / backend only (no GPU work)")
    args = ap.parse_args()
    if args.precision is None:  # split-bf16 keeps 256-wide activations in registers: c5 runs plain bf16
        args.precision = "bf16" if max(CONFIGS[args.config][4]) > 256 else "bf16x3"

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` outside a launcher: start the N ranks (one process per GPU) through
        # torch.distributed.run as a child, before anything here touches the GPU, and exit with its code
        sys.exit(_self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks (WORLD_SIZE)")
    # rehearsal knobs for a one-GPU box (never set by the driver): every rank on cuda:0, gloo
    if os.environ.get("MARF_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("MARF_BENCH_BACKEND", "nccl")  # "nccl" is RCCL on ROCm
    if args.launch_check:
        dev = None
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend)
        world = torch.distributed.get_world_size()  # what the process group reports, not the env
    dist = {"world_size": world, "backend": torch.distributed.get_backend() if world > 1 else None,
            "launcher": os.environ.get("MARF_BENCH_LAUNCHER", "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ
                                       else ("env" if "WORLD_SIZE" in os.environ else "single process"))}
    if args.launch_check:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "n_gpus": world, "dist": dist, "launch_check": True}), flush=True)
        if world > 1:
            torch.distributed.barrier()
            torch.distributed.destroy_process_group()
        return

    import marf_hip
    from model import planar
    from util import EasyDict as edict

    canvas, crop, per_gpu, L, hidden = CONFIGS[args.config]
    if args.strong:
        if args.strong % world:
            raise SystemExit(f"--strong {args.strong} patches do not split over {world} ranks")
        per_gpu = args.strong // world
    B_total = per_gpu * world
    opt = make_opt(args.config, args.precision, B_total, c2f=not args.no_c2f)
    opt.device = str(dev)
    h, w = opt.patch_H, opt.patch_W
    torch.manual_seed(opt.seed)
    m = planar.Model(opt)
    rgb, mask, warp = synthetic_inputs(B_total, h, w, dev)
    m.images = edict(rgb=rgb, masks=mask, masks_eroded=mask, edges=None, gt_hom=None, gt=None)
    m.build_networks()
    m.graph.warp_param.weight.data.copy_(warp)
    m.graph.neural_image.progress.data.fill_(0.2)
    m.setup_optimizer()
    graph = m.graph
    graph.need_edges = False
    var = edict(idx=torch.arange(B_total), images=m.images)
    b0, b1 = graph.shard if graph.shard else (0, B_total)
    px_local = (b1 - b0) * h * w

    if args.graph and not m.graph_capable():
        raise SystemExit("--graph: the step cannot be captured here (one process, use_edges off)")

    def step(eager=False):
        if args.graph and not eager:
            # the whole iteration replayed: forward, loss, backward, Adam, progress, fix_first
            v, loss = m.captured_step(var)
            graph.neural_image.progress.data.fill_(0.2)  # keep c2f partially on
            return loss
        m.optim.zero_grad()
        v = graph.forward(var, mode="train")
        loss = m._loss_sum(graph.compute_loss(v, mode="train"))  # summarize_loss without host syncs
        loss.all.backward()
        m.all_reduce_grads()
        m.optim.step()
        graph.neural_image.progress.data.fill_(0.2)  # keep c2f partially on
        graph.warp_param.weight.data[0] = 0
        return loss

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        loss = step()
    barrier()
    # timed region: HIP events around the dominant kernel only (the fused step's launches; every
    # event pair adds a few microseconds between launches, so the other kernels are timed after)
    marf_hip.profile_reset()
    marf_hip.profile_filter(["mlp_step"])
    marf_hip.profile_enable(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    barrier()
    elapsed = time.perf_counter() - t0
    marf_hip.profile_enable(False)
    prof = marf_hip.profile_read()
    # per-kernel breakdown: a separate pass of the same step with every kernel timed (eager: a
    # replayed graph records no events)
    n_break = max(3, args.steps // 4)
    marf_hip.profile_reset()
    marf_hip.profile_filter(None)
    marf_hip.profile_enable(True)
    for _ in range(n_break):
        step(eager=True)
    barrier()
    marf_hip.profile_enable(False)
    prof_all = marf_hip.profile_read()
    if args.graph:  # the dominant kernel's duration from the eager steps
        prof = {k: (v[0] * args.steps / n_break, v[1] * args.steps // n_break) for k, v in prof_all.items()}
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t)
    loss_v = float(loss.rgb.detach())
    timing_only = os.environ.get("MARF_AB_TIMING_ONLY") == "1"  # A/B builds whose results are wrong on purpose
    assert np.isfinite(loss_v) or timing_only, "loss is not finite"
    step_kernel = graph.neural_image.engine(dev).net.step_kernel

    # ---- forward-only render rate (reported beside the step): Graph.forward without
    #      grad = grid -> warp -> posenc -> MLP -> rgb over the same patches (k_mlp_fwd, no saves)
    render_pps = None
    with torch.no_grad():
        for _ in range(0 if args.no_render else 2):
            graph.forward(var, mode="eval")
        if not args.no_render:
            barrier()
            t0 = time.perf_counter()
            n_render = max(5, args.steps // 2)
            for _ in range(n_render):
                graph.forward(var, mode="eval")
            barrier()
            tr = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
            if world > 1:
                torch.distributed.all_reduce(tr, op=torch.distributed.ReduceOp.MAX)
            render_pps = world * px_local * n_render / float(tr)

    # ---- roofline of the dominant kernel (HIP-event durations measured above, same stream).
    #      the governing roof is bf16 MFMA; achieved = ALGORITHMIC FLOPs of one
    #      launch (the fp32 reference's multiply-adds, 2 per MAC) / its average duration.  The split
    #      recipe issues 3 MFMAs per forward MAC and 2 per dgrad MAC: that count is reported beside it
    #      (mfma_*), not in `achieved`.  HBM: algorithmic 16 B/px (target + mask) + 12 B/px (rgb
    #      out); the saved layer inputs / pre-activation gradients the weight-gradient kernels read
    #      back are the design's own traffic (design_bytes_per_launch), not algorithmic.
    dims = [2 + 4 * L] + hidden + [3]
    Kp0 = (dims[0] + 31) // 32 * 32
    S = (b1 - b0) * ((h * w + 127) // 128 * 128)
    sum_mac = sum(a * b for a, b in zip(dims[:-1], dims[1:]))
    fwd_mult, bwd_mult = {"bf16x3": (3, 2), "fp16x2": (2, 2)}.get(args.precision, (1, 1))
    kflops = {  # (algorithmic, MFMA-issued) FLOPs per launch
        # fused step: forward + dgrad chain (incl. layer 0, for the warp gradient) + last-layer wgrad
        "mlp_step": (px_local * (4 * sum_mac + 6 * dims[-2]),
                     px_local * ((2 * fwd_mult + 2 * bwd_mult) * sum_mac + 6 * dims[-2])),
        "wgrad_hidden": (px_local * 2 * hidden[0] * hidden[0],) * 2,
        "wgrad_l0": (px_local * 2 * dims[0] * dims[1],) * 2,
    }
    per_kernel = {k: {"avg_ms": v[0] / v[1], "launches_per_step": v[1] / n_break} for k, v in prof_all.items()}
    # scopes named *_side run on the library's side stream beside the others (their event span
    # includes waiting for free CUs): reported, not summed
    step_kernel_ms = sum(v[0] for k, v in prof_all.items() if not k.endswith("_side")) / n_break
    dom = max(prof.items(), key=lambda kv: kv[1][0])[0] if prof else None
    peak = PEAK_FP32 if args.precision == "fp32" else PEAK_BF16
    roof = None
    if dom in kflops:
        # per step: a pipelined step (marf_net_set_pipeline) runs the step kernel in several
        # launches (pieces of the tiles); FLOPs and bytes are the step's, the time their sum
        avg_s = prof[dom][0] / args.steps / 1e3
        alg, issued = kflops[dom]
        alg_bytes = 28 * px_local if dom == "mlp_step" else None
        design = step_kernel_bytes(S, Kp0, hidden, 2 if args.precision != "fp32" else 4).get(dom)
        tr = pmc_traffic(args.config, args.precision, dom, step_kernel if dom == "mlp_step" else "k_wgrad")
        roof = {"bound": "mfma", "achieved": alg / avg_s / 1e12, "peak": peak / 1e12, "unit": "TFLOP/s",
                "frac": alg / avg_s / peak, "traffic": tr[0] if tr else None,
                "kernel": dom, "launches_per_step": prof[dom][1] / args.steps,
                "kernel_ms_per_step": avg_s * 1e3, "avg_launch_ms": prof[dom][0] / prof[dom][1],
                "algorithmic_flops_per_launch": alg * args.steps / prof[dom][1],
                "algorithmic_flops_per_step": alg,
                "mfma_flops_per_launch": issued * args.steps / prof[dom][1], "mfma_flops_per_step": issued,
                "mfma_tflops": issued / avg_s / 1e12, "mfma_frac": issued / avg_s / peak,
                "algorithmic_bytes_per_launch": alg_bytes, "design_bytes_per_launch": design,
                "traffic_ratio": (tr[0] / alg_bytes) if (tr and alg_bytes) else None,
                "traffic_source": tr[1] if tr else None,
                # matrix-core counters of the same kernel on the same library (PMC pass, null otherwise)
                "mfma_busy": tr[2].get("mfma_busy") if tr else None,
                "valu_per_mfma": tr[2].get("valu_per_mfma") if tr else None,
                "vmem_rd_insts_per_launch": tr[2].get("SQ_INSTS_VMEM_RD") if tr else None}
    prologue = prologue_rate(graph, var, L, opt.barf_c2f) if world == 1 or rank == 0 else None
    ms = elapsed / args.steps * 1e3
    value = world * px_local / (elapsed / args.steps)
    F = flops_per_px(dims)
    out = {
        "metric": METRIC, "value": value, "unit": "pixels/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None, "dtype": args.precision, "data": "synthetic (procedural targets, Bernoulli masks, random warps; reference-style init)",
        "config": {"workload": f"{args.config}: {per_gpu} patches x {h}x{w} px per GPU, L={L}, MLP "
                               f"{'-'.join(map(str, dims))}, {RECIPES[args.precision]}, "
                               + ("c2f off" if args.no_c2f else "c2f [0,0.4] at progress 0.2"),
                   "patches_per_gpu": per_gpu, "pixels_per_step_per_gpu": px_local,
                   "pixels_per_s_per_gpu": value / world, "parallelism": f"dp{world} (patches)",
                   "algorithmic_flops_per_px": F,
                   "step_tflops_per_gpu": value / world * F / 1e12,
                   "step_frac_of_peak": value / world * F / peak,
                   "loss_rgb_last": loss_v,
                   "step_kernel": step_kernel,
                   "render_pixels_per_s": render_pps},
        "roofline": roof,
        "prologue": prologue,
        "dist": dist,
        "kernels": per_kernel,
        "kernel_ms_per_step": step_kernel_ms,
        "kernels_note": f"per-kernel HIP-event durations from {n_break} further eager steps with every kernel "
                        "timed (*_side: side-stream kernels overlapping the others, not in kernel_ms_per_step; "
                        "the timed region times the dominant kernel only"
                        + ("; with --graph it replays a captured graph and the roofline uses these eager steps)"
                           if args.graph else ")"),
        "graph": bool(args.graph),
    }
    if timing_only:
        out["timing_only"] = True  # never a headline: the build under test computes wrong results
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_sample_patches)
    if (world == 1 and args.config == "c3" and args.precision == "bf16x3" and not args.no_alt_recipe
            and not args.strong and not args.no_c2f and not args.graph and not timing_only):
        del m, graph, var, loss
        torch.cuda.empty_cache()
        out["alt_recipe"] = alt_recipe(args, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
