"""Options: YAML + dotted command-line overrides, same syntax and semantics as the reference
(options.py:14-150):

    --key1.key2=value   value parsed with yaml.safe_load
    --key1.key2=        None
    --key1.key2         True
    --key1.key2!        False

Differences, all for unattended runs: an override of a key absent from the yaml is added with a
warning instead of an interactive y/n prompt, and an existing different options.yaml in the output
directory is overwritten with a warning.
"""
import os
import random
import string

import numpy as np
import torch
import yaml

from util import EasyDict as edict
from util import log, plain_dict

_HERE = os.path.dirname(os.path.abspath(__file__))


def parse_arguments(args):
    opt_cmd = {}
    for arg in args:
        assert arg.startswith("--"), arg
        if "=" not in arg[2:]:
            key_str, value = (arg[2:-1], "false") if arg[-1] == "!" else (arg[2:], "true")
        else:
            key_str, value = arg[2:].split("=", 1)
        keys_sub = key_str.split(".")
        opt_sub = opt_cmd
        for k in keys_sub[:-1]:
            opt_sub = opt_sub.setdefault(k, {})
        assert keys_sub[-1] not in opt_sub, keys_sub[-1]
        opt_sub[keys_sub[-1]] = yaml.safe_load(value)
    return edict(opt_cmd)


def _yaml_path(name):
    if os.path.isabs(name) or os.path.exists(name):
        return name
    return os.path.join(_HERE, name)


def load_options(fname):
    with open(_yaml_path(fname)) as f:
        opt = edict(yaml.safe_load(f))
    if "_parent_" in opt:
        parents = opt.pop("_parent_")
        if isinstance(parents, str):
            parents = [parents]
        for pf in parents:
            base = load_options(pf)
            opt = override_options(base, opt, key_stack=[])
    return opt


def override_options(opt, opt_over, key_stack=None, safe_check=False):
    key_stack = key_stack or []
    for key, value in opt_over.items():
        if isinstance(value, dict):
            opt[key] = override_options(opt.get(key, edict()), value, key_stack=key_stack + [key], safe_check=safe_check)
        else:
            if safe_check and key not in opt:
                print(f'warning: "{".".join(key_stack + [key])}" not found in the yaml, adding it')
            opt[key] = value
    return edict(opt)


def set_opt(opt_cmd=None, make_dirs=True):
    opt_cmd = opt_cmd or edict()
    log.info("setting configurations...")
    assert "model" in opt_cmd
    assert "yaml" in opt_cmd
    opt = load_options(f"options/{opt_cmd.yaml}.yaml")
    opt = override_options(opt, opt_cmd, key_stack=[], safe_check=True)
    process_options(opt, make_dirs=make_dirs)
    return opt


def process_options(opt, make_dirs=True):
    """Seeding, run name, output path and device (options.py:99-120).  Multi-GPU: one process per
    GPU launched by torch.distributed.run; LOCAL_RANK selects the device."""
    if opt.seed is not None:
        random.seed(opt.seed)
        np.random.seed(opt.seed)
        torch.manual_seed(opt.seed)
        torch.cuda.manual_seed_all(opt.seed)
        if opt.seed != 0:
            opt.name = str(opt.name) + f"_seed{opt.seed}"
    else:
        opt.name = str(opt.name) + "_" + "".join(random.choice(string.ascii_uppercase) for _ in range(4))
    opt.output_path = f"{opt.output_root}/{opt.group}/{opt.name}"
    if make_dirs:
        os.makedirs(opt.output_path, exist_ok=True)
    assert isinstance(opt.gpu, int)
    local_rank = int(os.environ.get("LOCAL_RANK", opt.gpu))
    opt.device = "cpu" if opt.cpu or not torch.cuda.is_available() else f"cuda:{local_rank}"


def save_options_file(opt):
    fname = f"{opt.output_path}/options.yaml"
    if os.path.isfile(fname):
        with open(fname) as f:
            old = yaml.safe_load(f)
        if old != plain_dict(opt):
            print("existing options file differs; overwriting")
        else:
            print("existing options file found (identical)")
    with open(fname, "w") as f:
        yaml.safe_dump(plain_dict(opt), f, default_flow_style=False, indent=4)
