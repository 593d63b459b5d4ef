"""Host helpers the planar engine needs (the reference keeps its equivalents in util.py:44-115):
an attribute dict for options, a plain console logger, a device mover for the `var` bundle, the
layer-width pairing of define_network and the hex colour parser used for the patch boxes."""
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
    """Console logger with the reference's method names (no colour codes)."""

    def process(self, pid):
        print(f"Process ID: {pid}")

    def title(self, message):
        print(f"== {message} ==")

    def info(self, message):
        print(message)

    def options(self, opt, level=0):
        pad = "   " * level
        for key in sorted(opt):
            value = opt[key]
            if isinstance(value, dict):
                print(f"{pad}* {key}:")
                self.options(value, level + 1)
            else:
                print(f"{pad}* {key}: {value}")


log = Log()


def move_to_device(x, device):
    """Recursively move every tensor inside dicts / lists / namedtuples to `device` (dicts and
    lists in place, as the engine's `var` bundle expects)."""
    if torch.is_tensor(x):
        return x.to(device=device)
    if isinstance(x, dict):
        for key in list(x.keys()):
            x[key] = move_to_device(x[key], device)
        return x
    if isinstance(x, list):
        x[:] = [move_to_device(e, device) for e in x]
        return x
    if isinstance(x, tuple) and hasattr(x, "_fields"):
        return type(x)(*(move_to_device(e, device) for e in x))
    return x


def plain_dict(d):
    """Nested attribute dicts -> plain dicts (what yaml.safe_dump accepts)."""
    return {k: plain_dict(v) if isinstance(v, dict) else v for k, v in d.items()}


def get_layer_dims(widths):
    """Consecutive width pairs [(k_in, k_out), ...] of an MLP width list."""
    return [(widths[i], widths[i + 1]) for i in range(len(widths) - 1)]


def colorcode_to_number(code):
    """'#RRGGBB' -> (r, g, b) integers."""
    h = code.lstrip("#")
    return tuple(int(h[i:i + 2], 16) for i in (0, 2, 4))
