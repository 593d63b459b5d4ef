"""Training entry point with the reference's CLI (train.py:11-31):

    python train.py --group=<GROUP> --model=planar --yaml=planar --name=<NAME> --seed=3 --barf_c2f=[0,0.4]

Multi-GPU (patches sharded over ranks, one process per GPU):
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 train.py ...
"""
import importlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import torch  # noqa: E402

import options  # noqa: E402
from util import log  # noqa: E402


def main(argv=None):
    log.process(os.getpid())
    log.title(f"[{sys.argv[0]}] (MI355X planar bundle adjustment)")
    opt_cmd = options.parse_arguments(sys.argv[1:] if argv is None else argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not torch.distributed.is_initialized():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        torch.distributed.init_process_group("nccl")
    opt = options.set_opt(opt_cmd=opt_cmd)
    if int(os.environ.get("RANK", "0")) == 0:
        options.save_options_file(opt)
    if not opt.device.startswith("cuda"):
        raise RuntimeError("this implementation runs on a ROCm GPU only (no CPU path)")
    with torch.cuda.device(opt.device):
        model = importlib.import_module(f"model.{opt.model}")
        m = model.Model(opt)
        m.load_dataset()
        m.build_networks()
        m.setup_optimizer()
        m.setup_visualizer()
        m.train()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
