"""Small host utilities with the reference's names (util.py:44-115): console log, timer,
device moves, layer dims.  No termcolor / ipdb dependency."""
import time

import torch


class EasyDict(dict):
    """Recursive attribute dict (the reference uses the `easydict` package)."""

    def __init__(self, d=None, **kwargs):
        super().__init__()
        for k, v in dict(d or {}, **kwargs).items():
            self[k] = v

    def __setitem__(self, k, v):
        if isinstance(v, dict) and not isinstance(v, EasyDict):
            v = EasyDict(v)
        elif isinstance(v, (list, tuple)):
            v = type(v)(EasyDict(x) if isinstance(x, dict) and not isinstance(x, EasyDict) else x for x in v)
        super().__setitem__(k, v)

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        del self[k]

    def update(self, d=None, **kw):
        for k, v in dict(d or {}, **kw).items():
            self[k] = v


edict = EasyDict


class Log:
    """Console logger (util.py:44-67)."""

    def process(self, pid):
        print(f"Process ID: {pid}")

    def title(self, message):
        print(f"== {message} ==")

    def info(self, message):
        print(message)

    def options(self, opt, level=0):
        for key, value in sorted(opt.items()):
            if isinstance(value, dict):
                print("   " * level + "* " + key + ":")
                self.options(value, level + 1)
            else:
                print("   " * level + "* " + key + ":", value)


log = Log()


def update_timer(opt, timer, ep, it_per_ep):
    """Moving-average iteration timer (util.py:69-79)."""
    if not opt.max_epoch:
        return
    momentum = 0.99
    timer.elapsed = time.time() - timer.start
    timer.it = timer.it_end - timer.it_start
    timer.it_mean = timer.it_mean * momentum + timer.it * (1 - momentum) if timer.it_mean is not None else timer.it
    timer.arrival = timer.it_mean * it_per_ep * (opt.max_epoch - ep)


def move_to_device(x, device):
    """util.py:81-95."""
    if isinstance(x, dict):
        for k, v in x.items():
            x[k] = move_to_device(v, device)
    elif isinstance(x, list):
        for i, e in enumerate(x):
            x[i] = move_to_device(e, device)
    elif isinstance(x, tuple) and hasattr(x, "_fields"):
        return type(x)(**move_to_device(x._asdict(), device))
    elif isinstance(x, torch.Tensor):
        return x.to(device=device)
    return x


def to_dict(d, dict_type=dict):
    d = dict_type(d)
    for k, v in d.items():
        if isinstance(v, dict):
            d[k] = to_dict(v, dict_type)
    return d


def get_layer_dims(layers):
    """[(k_in, k_out), ...] from a layer-width list (util.py:105-108)."""
    return list(zip(layers[:-1], layers[1:]))


def colorcode_to_number(code):
    ords = [ord(c) for c in code[1:]]
    ords = [n - 48 if n < 58 else n - 87 for n in ords]
    return (ords[0] * 16 + ords[1], ords[2] * 16 + ords[3], ords[4] * 16 + ords[5])
