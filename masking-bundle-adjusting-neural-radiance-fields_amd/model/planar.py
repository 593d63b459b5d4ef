"""Planar bundle adjustment with a neural image (the reference's model/planar.py surface).

Same classes, attributes, state-dict keys and training-step order as the reference:
  Model                 lifecycle load_dataset / build_networks / setup_optimizer /
                        setup_visualizer / train (model/planar.py:31-291)
  Graph                 warp_param Embedding(B, 8), forward -> rgb_prediction(_map),
                        compute_loss -> edict(render, rgb, mask, edge), mse_loss (:296-391)
  NeuralImageFunction   mlp ModuleList of nn.Linear, progress Parameter, forward(coord_2d),
                        positional_encoding(coord_2d) (:395-471)
The arithmetic of the step runs in libmarf.so (marf_hip): Graph.forward is one fused HIP
prologue+MLP kernel per tile, its backward the dgrad / warp-adjoint / weight-gradient kernels,
the loss and Adam are HIP kernels too.  Patches shard over ranks (one process per GPU); the
shared MLP gradient is summed with one RCCL all-reduce per step.
"""
import json
import os
import shutil
import time

import numpy as np
import torch
import tqdm

import inputs
import marf_hip
import util
from util import EasyDict as edict
from util import log
from warp import Lie, Warp


def _const_zero(t):
    """The integer zeros compute_loss puts in for the absent mask / edge terms (torch.tensor(0) on
    the CPU, as model/planar.py:374-378 does) -- never a computed loss (those are float tensors)."""
    return (torch.is_tensor(t) and t.device.type == "cpu" and t.dim() == 0 and not t.is_floating_point()
            and not t.requires_grad and int(t) == 0)


def lin_comb(terms, start_zero=False):
    """sum_i c_i * t_i in order ((start_zero: 0. + ...), the expression of model/planar.py:377 /
    :180-183), without the operations that are exact identities in IEEE arithmetic: a factor of
    exactly 1.0 (x * 1.0 == x), a term that is one of compute_loss's integer zero constants, and the
    leading 0. + (x + 0 == x for every x but -0.0; these losses are >= +0 or NaN).  Same values, same
    dtypes (fp32 * python float stays fp32; an int zero never promotes) and same gradients (d(x * 1)
    = d(x + 0) = the upstream gradient), without one GPU launch per identity: 14 launches of scalar
    arithmetic per training step become 3 (one add forward, the seed and one accumulation backward)."""
    acc = None
    for c, t in terms:
        if _const_zero(t):
            continue
        x = t if (isinstance(c, (int, float)) and float(c) == 1.0) else c * t
        acc = x if acc is None else acc + x
    if acc is None:  # every term a constant zero: the plain expression
        acc = 0. if start_zero else 0
        for c, t in terms:
            acc = acc + c * t
    elif start_zero and not torch.is_tensor(acc):
        acc = 0. + acc
    return acc


def _precision(opt):
    p = str(opt.get("precision", "fp32")).lower()
    if p in ("fp32", "float32", "f32"):
        return marf_hip.MARF_FP32
    if p in ("bf16", "bfloat16"):
        return marf_hip.MARF_BF16
    if p in ("bf16x3", "split-bf16"):
        return marf_hip.MARF_BF16X3
    if p in ("fp16", "float16", "half"):
        return marf_hip.MARF_FP16
    if p in ("fp16x2", "split-fp16"):
        return marf_hip.MARF_FP16X2
    raise ValueError(f"precision must be fp32, fp16, bf16, bf16x3 or fp16x2, got {p}")


def _dist():
    return torch.distributed.is_available() and torch.distributed.is_initialized()


class Model(torch.nn.Module):
    """Planar BARF engine (model/planar.py:31-291)."""

    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.batch_size = opt.batch_size
        self.dataset = opt.dataset
        os.makedirs(opt.output_path, exist_ok=True)
        self.warp = Warp(opt)
        self.images = None
        self.graph = None
        self.optim = None
        self.sched = None
        self.tb = None
        self.metrics_file = None
        self.box_colors = None
        self.vis_path = None
        self.video_fname = None
        self.timer = None
        self.warp_pert = None
        self.ep = self.it = self.vis_it = 0
        self.lie = Lie()
        self.rank = torch.distributed.get_rank() if _dist() else 0
        self.world = torch.distributed.get_world_size() if _dist() else 1
        self.exchange_counts = {"bucketed": 0, "flat": 0}  # which gradient exchange each step took
        self._step_graph = None  # (HIP graph, var, loss) of captured_step

    # ------------------------------------------------------------------ data
    def load_dataset(self):
        log.info("loading dataset...")
        opt = self.opt
        if opt.get("dataset_npz"):
            # pre-decoded inputs (uint8 rgb [B,3,h,w], uint8 mask [B,1,h,w]) -- no PIL needed
            z = np.load(opt.dataset_npz, allow_pickle=False)
            rgb = torch.from_numpy(z["rgb"][:self.batch_size].astype(np.float32)).div(255)
            mask = torch.from_numpy(z["mask"][:self.batch_size].astype(np.float32))
            self.images = edict(gt=None, rgb=rgb.to(opt.device), masks=mask.to(opt.device),
                                masks_eroded=inputs.erode_images(mask, opt.device), gray=None, gt_hom=None)
            self.images.edges = None
            return
        root = os.path.join(opt.get("data_root", "data/planar"), self.dataset)
        self.images = inputs.prepare_images(
            opt,
            fps_images=[f"{root}/{i}.png" for i in range(self.batch_size)],
            fps_masks=[f"{root}/{i}-m.png" for i in range(self.batch_size)] if opt.use_masks else None,
            fp_gt=f"{root}/gt.png",
            fps_hom=[f"{root}/H_0_{i}.mat" for i in range(1, self.batch_size)] if opt.use_homographies else None,
            edges=True if opt.use_edges else None)

    # ------------------------------------------------------------------ networks
    def build_networks(self):
        log.info("building networks...")
        self.graph = Graph(self.opt).to(self.opt.device)
        if self.world > 1:
            self.graph.set_shard(self.rank, self.world, self.images)
            if self.opt.device != "cpu":
                self._grad_engine()  # arm the per-layer gradient events before the first backward

    def setup_optimizer(self):
        log.info("setting up optimizers...")
        opt = self.opt
        groups = [dict(params=self.graph.neural_image.parameters(), lr=opt.optim.lr),
                  dict(params=self.graph.warp_param.parameters(), lr=opt.optim.lr_warp)]
        if opt.use_implicit_mask:
            raise NotImplementedError("the implicit-mask branch is outside this implementation")
        if opt.optim.algo == "Adam":
            self.optim = marf_hip.Adam(groups)
        else:
            self.optim = getattr(torch.optim, opt.optim.algo)(groups)
        if opt.optim.sched:
            sched = getattr(torch.optim.lr_scheduler, opt.optim.sched.type)
            self.sched = sched(self.optim, **{k: v for k, v in opt.optim.sched.items() if k != "type"})

    def setup_visualizer(self):
        log.info("setting up visualizers...")
        opt = self.opt
        if opt.tb is not None and self.rank == 0:
            try:
                from torch.utils.tensorboard import SummaryWriter
                self.tb = SummaryWriter(log_dir=opt.output_path, flush_secs=10)
            except Exception:
                self.tb = None
            self.metrics_file = open(os.path.join(opt.output_path, "metrics.jsonl"), "a")
        colors = ["#FF0000", "#00FF00", "#0000FF", "#FFFF00", "#00FFFF", "#FF00FF", "#800000", "#808000",
                  "#008080", "#800080", "#808080"]
        self.box_colors = np.array([util.colorcode_to_number(c) for c in colors[:self.batch_size]]).astype(int)
        self.vis_path = f"{opt.output_path}/vis"
        os.makedirs(self.vis_path, exist_ok=True)
        self.video_fname = f"{opt.output_path}/vis.mp4"

    # ------------------------------------------------------------------ training
    def train(self, mode=True):
        log.title("TRAINING START")
        self.timer = edict(start=time.time(), it_mean=None)
        self.graph.train()
        var = edict(idx=torch.arange(self.batch_size))
        var.images = self.images
        var = util.move_to_device(var, self.opt.device)
        loader = tqdm.trange(self.opt.max_iter, desc="Training", leave=False, disable=self.rank != 0)
        with torch.no_grad():  # the frame-0 render only (visualize re-renders the canvas)
            var = self.graph.forward(var)
        self.visualize(var, step=0)
        for _ in loader:
            self.train_iteration(var, loader)
            if self.opt.warp.fix_first:
                self.graph.warp_param.weight.data[0] = 0
        if self.rank == 0 and shutil.which("ffmpeg"):
            os.system(f"ffmpeg -y -loglevel error -framerate 30 -i {self.vis_path}/%d.png "
                      f"-pix_fmt yuv420p {self.video_fname}")
        if self.tb:
            self.tb.flush()
            self.tb.close()
        if self.metrics_file:
            self.metrics_file.close()
        log.title("TRAINING DONE")

    def summarize_loss(self, loss):
        """all = sum_k 10^w_k loss_k with NaN / Inf checks (model/planar.py:172-185)."""
        assert "all" not in loss
        for key in loss:
            assert key in self.opt.loss_weight
            assert loss[key].shape == ()
            if self.opt.loss_weight[key] is not None:
                assert not torch.isinf(loss[key]), f"loss {key} is Inf"
                assert not torch.isnan(loss[key]), f"loss {key} is NaN"
        return self._loss_sum(loss)

    def _loss_sum(self, loss):
        """summarize_loss's weighted sum without its host-side NaN / Inf asserts (each one waits for
        the GPU: a captured step must not synchronise; train_iteration checks at logging steps).
        0. + sum_k 10^w_k loss_k in key order, through lin_comb: the same values and gradients."""
        terms = [(10 ** float(self.opt.loss_weight[key]), loss[key]) for key in loss
                 if self.opt.loss_weight[key] is not None]
        loss.update(all=lin_comb(terms, start_zero=True))
        return loss

    def graph_capable(self):
        """A whole iteration can be captured when it has no host-dependent value per step: one
        process, the fused step, no edge term (its alpha = it / max_iter is a host value), no
        learning-rate scheduler, the library's Adam (its per-step scalars come from a device table)."""
        return (self.world == 1 and not self.opt.use_edges and self.opt.get("fused_step", True)
                and str(self.opt.device).startswith("cuda") and not self.sched
                and isinstance(self.optim, marf_hip.Adam))

    def _capture_ident(self, var):
        return (tuple(int(i) for i in var.idx.tolist()) if torch.is_tensor(var.idx) else tuple(var.idx),
                var.images.rgb.data_ptr(), var.images.masks.data_ptr() if torch.is_tensor(var.images.get("masks")) else 0,
                self.graph.neural_image.mlp[0].weight.data_ptr(), self.graph.warp_param.weight.data_ptr())

    def captured_step(self, var):
        """One whole training iteration (model/planar.py:187-209 and the loop's fix_first, :154-158)
        as a replayed HIP graph (torch.cuda.CUDAGraph): Graph.forward + compute_loss + the weighted
        loss sum + backward + Adam + the progress update + fix_first.  Adam's per-step scalars
        (bias corrections) come from a device table indexed by a device step counter
        (marf_adam_step_sched), the progress from a device table of it / max_iter (both computed on
        the host exactly as the eager step computes them), so every replay is the eager iteration's
        launches on the same buffers: the same bits (test_captured_step_matches_eager).
        The first call runs two eager warm-up passes (every buffer and kernel attribute set up),
        creates the optimizer state and records once; every call replays.  Host bookkeeping per
        replay: Graph.it, each parameter's Adam step.  The graph is bound to the batch it was
        recorded with: another var raises.  Returns (var, loss) with the graph's static tensors."""
        cap = self._step_graph
        if cap is not None and max(self.it, cap["adam_step"]) + 1 >= cap["limit"]:
            cap = self._step_graph = None  # past the recorded tables: record again with longer ones
        if cap is None:
            if not self.graph_capable():
                raise RuntimeError("captured_step: needs one process, the fused step, use_edges off, no scheduler "
                                   "and the library's Adam")
            dev = torch.device(self.opt.device)
            it0 = self.graph.it
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    self.optim.zero_grad(set_to_none=True)
                    v = self.graph.forward(var, mode="train")
                    self._loss_sum(self.graph.compute_loss(v, mode="train")).all.backward()
                # the optimizer state (zeros) exists before the recording
                for group in self.optim.param_groups:
                    self.optim._segments(group, advance=False)
            torch.cuda.current_stream(dev).wait_stream(side)
            self._drop_autograd(var)  # (no warm-up graph, whose gradient nodes live on `side`, stays alive)
            self.graph.neural_image.engine(dev)._packed_version = None  # the repack must be recorded
            steps = {st["step"] for st in self.optim.state.values() if "step" in st}
            if len(steps) > 1:
                raise RuntimeError(f"captured_step: parameters at different Adam steps {sorted(steps)}")
            adam_step = steps.pop() if steps else 0
            limit = max(int(self.opt.max_iter), self.it, adam_step) + 1024
            tabs = self.optim.schedule_tables(limit, dev)
            # it / max_iter in python float64, then float32: progress.data.fill_ of the eager step
            ptab = torch.tensor([k / self.opt.max_iter for k in range(limit + 1)], dtype=torch.float32, device=dev)
            c_adam = torch.tensor([adam_step], dtype=torch.int32, device=dev)
            c_it = torch.tensor([self.it], dtype=torch.int32, device=dev)
            progress = self.graph.neural_image.progress
            fix_first = bool(self.opt.warp.fix_first)
            self.optim.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                v = self.graph.forward(var, mode="train")
                loss = self._loss_sum(self.graph.compute_loss(v, mode="train"))
                loss.all.backward()
                self.optim.step_scheduled(c_adam, tabs, adam_step + 1)
                c_adam.add_(1)
                c_it.add_(1)
                progress.data.copy_(ptab.index_select(0, c_it.long()).view(()))
                if fix_first:
                    self.graph.warp_param.weight.data[0] = 0
            for k in list(loss.keys()):
                if torch.is_tensor(loss[k]):
                    loss[k] = loss[k].detach()
            self._drop_autograd(v)
            self.graph.it = it0
            # (after the warm-up: the first forward moves the MLP parameters into the engine's flat buffer)
            cap = self._step_graph = dict(graph=g, var=v, loss=loss, ident=self._capture_ident(var), limit=limit,
                                          counters=(c_adam, c_it),
                                          tables=(tabs, ptab), adam_step=adam_step)
        elif cap["ident"] != self._capture_ident(var):
            raise RuntimeError("captured_step: the graph was recorded for another batch (var.idx / images / "
                               "parameters changed); build a new Model step or turn opt.cuda_graph off")
        cap["graph"].replay()
        cap["adam_step"] += 1
        self.graph.it += 1  # Graph.compute_loss's counter (model/planar.py:379), not run on a replay
        self.optim.advance_steps()
        return cap["var"], cap["loss"]

    @staticmethod
    def _drop_autograd(var):
        """Detach the prediction fields of a var bundle (their autograd graph is released)."""
        for k in ("rgb_prediction", "rgb_prediction_map", "edge_prediction"):
            if torch.is_tensor(var.get(k)):
                var[k] = var[k].detach()
        var.fused_loss = None

    def _grad_engine(self):
        """The neural image's engine, with per-layer gradient events armed for a bucketed exchange
        (MARF_GRAD_BUCKETS=0: the flat all-reduce after the whole backward)."""
        eng = self.graph.neural_image.engine(torch.device(self.opt.device))
        if eng.grad_events is None and os.environ.get("MARF_GRAD_BUCKETS", "1") != "0":
            eng.grad_events = marf_hip.GradEvents(len(eng.net.layer_spans), torch.device(self.opt.device))
        return eng

    def all_reduce_grads(self):
        """Sum the shared MLP gradient over ranks (RCCL over xGMI); warp rows are rank-local.

        Bucketed per layer: the fused step's backward marks each layer's gradient
        final as it finishes (last layer first, marf_step_backward_ev), and that layer's all-reduce
        starts on a side stream right then, overlapping the weight gradients still running; the
        step's stream waits for the last bucket before the optimizer reads the sums.  The flat path
        (one all-reduce of the whole vector) covers the unfused step and MARF_GRAD_BUCKETS=0.
        MARF_GRAD_COMM=marf exchanges through the C ABI's own RCCL communicator (marf_comm_*) instead
        of torch.distributed's."""
        if self.world <= 1:
            return
        grads = [p.grad for p in self.graph.neural_image.mlp.parameters()]
        flat = marf_hip.flat_view(grads)
        eng = self._grad_engine() if flat is not None and flat.is_cuda else None  # (gloo on CPU: flat)
        bucketed = eng is not None and eng.grad_events is not None and eng.events_for == flat.data_ptr()
        if eng is not None:
            eng.events_for = None  # the events mark this gradient only: never reused for a later one
        self.exchange_counts["bucketed" if bucketed else "flat"] += 1
        if flat is not None and os.environ.get("MARF_GRAD_COMM") == "marf":
            if getattr(self, "_marf_comm", None) is None:
                uid = [marf_hip.Comm.unique_id() if self.rank == 0 else None]
                torch.distributed.broadcast_object_list(uid, src=0)
                self._marf_comm = marf_hip.Comm(uid[0], self.world, self.rank, flat.device.index)
            if bucketed:
                self._marf_comm.allreduce_layers(eng.net, flat, eng.grad_events)
            else:
                self._marf_comm.allreduce(flat)
            return
        if bucketed:
            if getattr(self, "_comm_stream", None) is None:
                self._comm_stream = torch.cuda.Stream(flat.device)
            side, works = self._comm_stream, []
            for l in reversed(range(len(eng.net.layer_spans))):
                off, n = eng.net.layer_spans[l]
                side.wait_event(eng.grad_events.events[l])
                with torch.cuda.stream(side):
                    works.append(torch.distributed.all_reduce(flat[off:off + n], async_op=True))
            for w in works:
                w.wait()
            torch.cuda.current_stream(flat.device).wait_stream(side)
            return
        if flat is not None:
            torch.distributed.all_reduce(flat)
        else:
            for g in grads:
                torch.distributed.all_reduce(g)

    def train_iteration(self, var, loader):
        """One optimisation step in the reference's order (model/planar.py:187-209)."""
        t_start = time.time()
        log_now = (self.it + 1) % self.opt.freq.scalar == 0
        # the edge term is evaluated every step, as the reference's Graph.forward does
        # (model/planar.py:336, 366-369): it carries no gradient, but loss.render / loss.all hold it
        self.graph.need_edges = bool(self.opt.use_edges)
        captured = bool(self.opt.get("cuda_graph")) and self.graph_capable()
        if captured:  # the whole iteration, optimizer, progress and fix_first included
            var, loss = self.captured_step(var)
            if log_now:
                self.summarize_loss({k: v for k, v in loss.items() if k != "all"})  # the NaN / Inf asserts
        else:
            self.optim.zero_grad()
            var = self.graph.forward(var, mode="train")
            loss = self.graph.compute_loss(var, mode="train")
            loss = self.summarize_loss(loss)
            loss.all.backward()
            self.all_reduce_grads()
            self.optim.step()
            if self.sched:
                self.sched.step()
        if log_now:
            self.log_scalars(loss, var, step=self.it + 1, split="train")
        if (self.it + 1) % self.opt.freq.vis == 0:
            self.visualize(var, step=self.it + 1, split="train")
        self.it += 1
        if log_now:
            loader.set_postfix(it=self.it, loss=f"{float(loss.all):.3f}")
        self.timer.it = time.time() - t_start
        self.timer.it_mean = self.timer.it if self.timer.it_mean is None else 0.99 * self.timer.it_mean + 0.01 * self.timer.it
        if not captured:  # (the captured iteration updated it on the device)
            self.graph.neural_image.progress.data.fill_(self.it / self.opt.max_iter)
        return loss

    @torch.no_grad()
    def predict_entire_image(self):
        """Full-canvas render on the unwarped grid (model/planar.py:211-217)."""
        xy_grid = self.warp.get_normalized_pixel_grid()[:1]
        rgb = self.graph.neural_image.forward(xy_grid)
        return rgb.view(self.opt.H, self.opt.W, 3).detach().cpu().permute(2, 0, 1)

    def homography_error(self, pred_hom, gt_hom):
        if self.opt.warp.type == "se2":
            pred_hom = marf_hip.se2_to_sl3(pred_hom)
        pred_h = self.lie.sl3_to_SL3(pred_hom)
        return torch.norm((pred_h - gt_hom) ** 2).mean()

    def gathered_warps(self):
        w = self.graph.warp_param.weight.detach().clone()
        if self.world > 1:
            b0, b1 = self.graph.shard
            mine = torch.zeros_like(w)
            mine[b0:b1] = w[b0:b1]
            torch.distributed.all_reduce(mine)
            w = mine
        return w

    @torch.no_grad()
    def log_scalars(self, loss, var, metric=None, step=0, split="train"):
        vals = {}
        for key, value in loss.items():
            if key == "all" or self.opt.loss_weight[key] is None:
                continue
            v = value.detach().to(torch.float64).reshape(())
            if self.world > 1 and key in ("rgb", "render"):
                v = v.to(self.opt.device)
                torch.distributed.all_reduce(v)
            vals[f"{split}/loss_{key}"] = float(v)
        for key, value in (metric or {}).items():
            vals[f"{split}/{key}"] = float(value)
        if self.opt.use_homographies and self.images.get("gt_hom") is not None:
            vals[f"{split}/Homography_Error"] = float(self.homography_error(self.gathered_warps(), self.images.gt_hom))
        vals[f"{split}/PSNR"] = -10 * np.log10(vals[f"{split}/loss_rgb"]) if vals.get(f"{split}/loss_rgb") else None
        if self.rank == 0:
            if self.tb:
                for k, v in vals.items():
                    if v is not None:
                        self.tb.add_scalar(k, v, step)
            if self.metrics_file:
                self.metrics_file.write(json.dumps(dict(step=step, **vals)) + "\n")
                self.metrics_file.flush()
        return vals

    @torch.no_grad()
    def visualize(self, var, step=0, split="train"):
        if self.rank != 0:
            self.vis_it += 1
            return
        frame = self.predict_entire_image()
        img = (frame * 255).byte().permute(1, 2, 0).numpy()
        try:
            import PIL.Image
            PIL.Image.fromarray(img).save(f"{self.vis_path}/{self.vis_it}.png")
        except Exception:
            np.save(f"{self.vis_path}/{self.vis_it}.npy", img)
        self.vis_it += 1


# ============================================================================ Graph

class Graph(torch.nn.Module):
    """Per-patch homographies + neural image + masked loss (model/planar.py:296-391)."""

    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.batch_size = opt.batch_size
        self.neural_image = NeuralImageFunction(opt)
        self.warp = Warp(opt)
        self.warp_param = torch.nn.Embedding(self.batch_size, opt.warp.dof).to(opt.device)
        torch.nn.init.zeros_(self.warp_param.weight)
        self.h = opt.patch_H if opt.use_cropped_images else opt.H
        self.w = opt.patch_W if opt.use_cropped_images else opt.W
        self.max_iter = opt.max_iter
        self.it = 0
        if opt.use_implicit_mask:
            raise NotImplementedError("the implicit-mask branch is outside this implementation")
        # warp.py:72-80 has the 8-dof sl(3) homography only; "se2" (3 dof: tx, ty, theta) is this
        # implementation's extension (north_star "sl(3)/SE(2)"): its generator is embedded in the
        # sl(3) parameters on the GPU (marf_hip.se2_to_sl3), so every kernel path is shared
        if (opt.warp.type, opt.warp.dof) not in (("homography", 8), ("se2", 3)):
            raise AssertionError(f"warp {opt.warp.type} with {opt.warp.dof} dof: homography / 8 (warp.py:72-80) "
                                 "or se2 / 3 (extension)")
        self.shard = None
        self.loss_denominator = None
        self.edge_denominator = None
        self.need_edges = True

    def warp_h(self):
        """The warps as the reference's sl(3) parameters [B, 8] (se2: the embedded generators)."""
        w = self.warp_param.weight
        return marf_hip.se2_to_sl3(w) if self.opt.warp.type == "se2" else w

    def set_shard(self, rank, world, images):
        """Own patches [rank*B/world, (rank+1)*B/world); the masked-MSE denominator 3*sum(mask)
        is made global once (masks are fixed inputs)."""
        B = self.batch_size
        b0, b1 = (rank * B) // world, ((rank + 1) * B) // world
        if b1 <= b0:
            raise ValueError(f"{world} ranks for {B} patches: every rank needs at least one patch")
        self.shard = (b0, b1)
        if images is not None and images.get("masks") is not None:
            d = (images.masks.sum().to(torch.float32) * 3).reshape(1).to(self.opt.device)
        else:
            d = torch.tensor([3.0 * B * self.h * self.w], device=self.opt.device)
        self.loss_denominator = d  # global (all patches are loaded on every rank)
        me = images.get("masks_eroded") if images is not None else None
        # the (logging-only) edge term's denominator 3*sum(masks_eroded), global as well
        self.edge_denominator = None if me is None else (me.sum().to(torch.float64) * 3).to(self.opt.device)

    def _range(self):
        return self.shard if self.shard is not None else (0, self.batch_size)

    def forward(self, var, mode=None):
        b0, b1 = self._range()
        imgs = var.get("images")
        var.fused_loss = None
        if (torch.is_grad_enabled() and self.opt.get("fused_step", True) and imgs is not None
                and imgs.get("rgb") is not None and self.opt.loss_weight.render is not None):
            # training forward: the target is known, so the loss and the whole backward are
            # computed in the same pass (marf_step_forward); compute_loss picks the loss up
            masks = imgs.masks[b0:b1] if imgs.get("masks") is not None else None
            denom = self.loss_denominator if self.shard is not None else None
            rgb, loss_rgb = self.neural_image.render_step(self.warp_h(), imgs.rgb[b0:b1], masks, denom, b0, b1)
            var.fused_loss = (loss_rgb, imgs.rgb, imgs.get("masks"))
        else:
            rgb = self.neural_image.render(self.warp_h(), b0, b1)  # [Bl, h*w, 3]
        var.rgb_prediction = rgb
        var.rgb_prediction_map = rgb.view(b1 - b0, int(self.h), int(self.w), 3).permute(0, 3, 1, 2)
        if self.opt.use_edges and self.need_edges:
            var.edge_prediction = inputs.compute_edges(var.rgb_prediction_map, self.opt.device)
        else:
            var.edge_prediction = None
        return var

    def compute_loss(self, var, mode=None):
        loss = edict()
        alpha = (self.opt.alpha_initial + (self.opt.alpha_final - self.opt.alpha_initial) * (self.it / self.max_iter)
                 if self.opt.use_edges else 0)
        b0, b1 = self._range()
        imgs = var.images
        if self.opt.loss_weight.render is not None:
            masks = imgs.masks[b0:b1] if imgs.get("masks") is not None else None
            fused = var.get("fused_loss")
            if fused is not None and fused[1] is imgs.rgb and fused[2] is imgs.get("masks"):
                rgb_loss = fused[0]  # from the fused training forward (same prediction, target, mask)
            else:
                rgb_loss = self.mse_loss(var.rgb_prediction_map, imgs.rgb[b0:b1], masks)
            if self.opt.use_edges:
                if var.get("edge_prediction") is not None and imgs.get("edges") is not None:
                    me = imgs.masks_eroded[b0:b1] if imgs.get("masks_eroded") is not None else None
                    if self.shard is not None and me is not None and self.edge_denominator is not None:
                        # this rank's share of the global masked MSE: the per-rank terms sum to it
                        diff = (var.edge_prediction - imgs.edges[b0:b1]) * me
                        edge_loss = (diff ** 2).sum() / self.edge_denominator
                    elif self.shard is not None and me is None:
                        # unmasked: this rank's share of the global mean over all B patches
                        diff = var.edge_prediction - imgs.edges[b0:b1]
                        edge_loss = (diff ** 2).sum() / (self.batch_size * diff[0].numel())
                    else:
                        edge_loss = self.mse_loss(var.edge_prediction, imgs.edges[b0:b1], me)
                else:  # no edge maps (a caller that turned need_edges off, or no edge targets)
                    edge_loss = torch.zeros((), dtype=torch.float64, device=rgb_loss.device)
            else:
                edge_loss = torch.tensor(0)
            mask_loss = torch.tensor(0)
            loss.render = lin_comb([(1 - alpha, rgb_loss), (0.5, mask_loss), (alpha, edge_loss)])
            loss.rgb = rgb_loss
            loss.mask = mask_loss
            loss.edge = edge_loss
        self.it += 1
        return loss

    def mse_loss(self, pred, labels, masks=None):
        """Masked MSE sum((pred-labels)*m)^2 / (3 sum m), or the plain mean without masks
        (model/planar.py:382-391).  fp32 GPU inputs run the HIP kernel; the float64 edge maps
        (logging only) use tensor ops."""
        if pred.dtype == torch.float32 and labels.dtype == torch.float32 and pred.is_cuda and pred.shape[1] == 3:
            B = pred.shape[0]
            pred_bn3 = pred.permute(0, 2, 3, 1).reshape(B, -1, 3)
            gt = labels.reshape(B, 3, -1)
            m = None if masks is None else masks.reshape(B, 1, -1)
            denom = self.loss_denominator if self.shard is not None else None
            return marf_hip.masked_mse(pred_bn3, gt, m, denom)
        diff = pred.contiguous() - labels
        if masks is None:
            return (diff ** 2).mean()
        return ((diff * masks) ** 2).sum() / (masks.sum() * 3)


# ============================================================================ neural image

class NeuralImageFunction(torch.nn.Module):
    """Coordinate MLP image with BARF coarse-to-fine posenc (model/planar.py:395-471)."""

    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.define_network()
        self.progress = torch.nn.Parameter(torch.tensor(0.))
        self._engines = {}

    @property
    def L(self):
        return int(self.opt.arch.posenc.L_2D) if self.opt.arch.posenc else 0

    @property
    def input_dim(self):
        return 2 + 4 * self.L if self.opt.arch.posenc else 2

    @property
    def skip(self):
        return [int(s) for s in (self.opt.arch.skip or [])]

    def define_network(self):
        """Linear layers in module order (this order is the RNG order of the init), layer 0
        rescaled by sqrt(D_in / 2) when coarse-to-fine is on; a skip layer takes the posenc
        features beside its input (k_in + D, model/planar.py:419-420)."""
        widths = list(self.opt.arch.layers)
        widths[0] = self.input_dim
        self.mlp = torch.nn.ModuleList()
        for li, (k_in, k_out) in enumerate(util.get_layer_dims(widths)):
            if li in self.skip:
                k_in += self.input_dim
            layer = torch.nn.Linear(k_in, k_out)
            if self.opt.barf_c2f and li == 0:
                s = np.sqrt(self.input_dim / 2.)
                layer.weight.data *= s
                layer.bias.data *= s
            self.mlp.append(layer)

    # ---- library state
    def _params(self):
        """MLP parameters as consecutive views of one flat fp32 buffer (re-flattened after a
        device move); the library reads them through that single pointer."""
        ps = list(self.mlp.parameters())
        if marf_hip.flat_view(ps) is None:
            flat = torch.cat([p.detach().reshape(-1) for p in ps]).contiguous()
            off = 0
            for p in ps:
                n = p.numel()
                p.data = flat[off:off + n].view_as(p)
                off += n
        return ps

    def engine(self, device):
        key = str(device)
        e = self._engines.get(key)
        if e is None:
            o = self.opt
            dims = [self.input_dim] + [int(d) for d in list(o.arch.layers)[1:]]
            ph, pw = (o.patch_H, o.patch_W) if o.use_cropped_images else (o.H, o.W)
            # the fused step's pixels on this GPU (this rank's patches), for the library's kernel choice
            world = torch.distributed.get_world_size() if _dist() else 1
            hint = -(-int(o.batch_size) // world) * ph * pw
            e = marf_hip.Engine(dims, self.L, _precision(o), list(o.barf_c2f) if o.barf_c2f else None,
                                o.H, o.W, ph, pw, lie_batch=int(o.batch_size), crop=bool(o.use_cropped_images),
                                pixels_hint=hint, skip=self.skip)
            self._engines[key] = e
        return e

    def render(self, warp_weight, b0=0, b1=None):
        """Fused training forward over the crop pixels of patches [b0, b1)."""
        ps = self._params()
        return marf_hip.render_train(warp_weight, self.progress.detach(), self.engine(warp_weight.device), ps, b0, b1)

    def render_step(self, warp_weight, gt, masks, denom=None, b0=0, b1=None):
        """Fused training forward + masked MSE (+ the backward of both, applied when the loss is
        differentiated): returns (rgb [Bl, h*w, 3], loss_rgb)."""
        ps = self._params()
        return marf_hip.render_step(warp_weight, self.progress.detach(), self.engine(warp_weight.device), ps, gt, masks,
                                    denom, b0, b1)

    def forward(self, coord_2d):
        """rgb = MLP(cat[coord, posenc(coord)]) for explicit coordinates [..., 2] (:429-449)."""
        ps = self._params()
        return marf_hip.mlp_forward(coord_2d, self.progress.detach(), self.engine(coord_2d.device), ps)

    def positional_encoding(self, coord_2d):
        """[..., 2] -> [..., 4L] sin/cos bands with c2f weights (:451-471)."""
        c2f = list(self.opt.barf_c2f) if self.opt.barf_c2f is not None else None
        return marf_hip.posenc(coord_2d, self.L, self.progress.detach(), c2f)
