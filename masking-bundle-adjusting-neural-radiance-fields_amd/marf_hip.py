"""ctypes binding of libmarf.so (include/marf.h) and the autograd functions built on it.

This is the only module that talks to the HIP library.  PyTorch is used for device memory
(caching allocator), the current HIP stream and autograd bookkeeping; every arithmetic step of
the planar render loop runs in the library's kernels.  There is no CPU or eager-PyTorch fallback:
if the library is missing or the tensors are not on a ROCm device the calls raise.
"""
import ctypes
import os

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# MARF_LIB selects a diagnostic build (lib/libmarf_stamps.so, tools/phase_stamps.py)
LIB_PATH = os.environ.get("MARF_LIB") or os.path.join(_HERE, "lib", "libmarf.so")

MARF_FP32, MARF_BF16, MARF_BF16X3, MARF_FP16, MARF_FP16X2 = 0, 1, 2, 3, 4
GEO_GRID, GEO_COORDS, GEO_CANVAS = 0, 1, 2

_c_int, _c_ll, _c_dbl, _c_vp, _c_sz = ctypes.c_int, ctypes.c_longlong, ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t


class Geometry(ctypes.Structure):
    _fields_ = [("mode", _c_int), ("B", _c_int), ("Np", _c_int), ("H", _c_int), ("W", _c_int),
                ("patch_H", _c_int), ("patch_W", _c_int), ("d_H", _c_vp), ("d_coords", _c_vp)]


class C2f(ctypes.Structure):
    _fields_ = [("d_progress", _c_vp), ("start", _c_dbl), ("end", _c_dbl), ("on", _c_int)]


_SIGS = {
    "marf_last_error": (ctypes.c_char_p, []),
    "marf_version": (_c_int, []),
    "marf_source_hash": (ctypes.c_char_p, []),
    "marf_sl3_to_SL3": (_c_int, [_c_vp, _c_vp, _c_int, _c_int, _c_vp]),
    "marf_sl3_to_SL3_backward": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp]),
    "marf_se2_to_sl3": (_c_int, [_c_vp, _c_vp, _c_int, _c_vp]),
    "marf_se2_to_sl3_backward": (_c_int, [_c_vp, _c_vp, _c_int, _c_vp]),
    "marf_pixel_grid": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_vp, _c_vp]),
    "marf_warp_points": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_vp]),
    "marf_posenc": (_c_int, [_c_vp, _c_ll, _c_int, ctypes.POINTER(C2f), _c_vp, _c_vp]),
    "marf_warp_points_backward": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_int, _c_vp]),
    "marf_posenc_backward": (_c_int, [_c_vp, _c_ll, _c_int, ctypes.POINTER(C2f), _c_vp, _c_vp, _c_vp]),
    "marf_prologue_probe": (_c_int, [ctypes.POINTER(Geometry), ctypes.POINTER(C2f), _c_int, _c_vp, _c_vp, _c_vp, _c_int,
                                     _c_vp]),
    "marf_net_create": (_c_int, [_c_int, ctypes.POINTER(_c_int), _c_int, _c_int, ctypes.POINTER(_c_vp)]),
    "marf_net_create_hint": (_c_int, [_c_int, ctypes.POINTER(_c_int), _c_int, _c_int, _c_ll, ctypes.POINTER(_c_vp)]),
    "marf_net_create_skip": (_c_int, [_c_int, ctypes.POINTER(_c_int), _c_int, _c_int, _c_ll, ctypes.c_uint,
                                      ctypes.POINTER(_c_vp)]),
    "marf_net_destroy": (None, [_c_vp]),
    "marf_net_param_count": (_c_ll, [_c_vp]),
    "marf_net_packed_bytes": (_c_sz, [_c_vp]),
    "marf_net_step_kernel": (ctypes.c_char_p, [_c_vp]),
    "marf_net_pack": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp]),
    "marf_net_set_pipeline": (_c_int, [_c_vp, _c_int, _c_int, _c_int]),
    "marf_saved_bytes": (_c_sz, [_c_vp, ctypes.POINTER(Geometry)]),
    "marf_workspace_bytes": (_c_sz, [_c_vp, ctypes.POINTER(Geometry)]),
    "marf_forward": (_c_int, [_c_vp, ctypes.POINTER(Geometry), ctypes.POINTER(C2f), _c_vp, _c_vp, _c_vp, _c_vp]),
    "marf_backward": (_c_int, [_c_vp, ctypes.POINTER(Geometry), ctypes.POINTER(C2f), _c_vp, _c_vp, _c_int, _c_vp,
                               _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "marf_step_saved_bytes": (_c_sz, [_c_vp, ctypes.POINTER(Geometry)]),
    "marf_render_workspace_bytes": (_c_sz, [_c_vp, ctypes.POINTER(Geometry)]),
    "marf_render": (_c_int, [_c_vp, ctypes.POINTER(Geometry), ctypes.POINTER(C2f), _c_vp, _c_vp, _c_vp, _c_vp]),
    "marf_step_forward": (_c_int, [_c_vp, ctypes.POINTER(Geometry), ctypes.POINTER(C2f), _c_vp, _c_vp, _c_vp, _c_vp,
                                   _c_vp, _c_vp, _c_vp, _c_vp]),
    "marf_step_backward": (_c_int, [_c_vp, ctypes.POINTER(Geometry), _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                                    _c_vp]),
    "marf_step_backward_ev": (_c_int, [_c_vp, ctypes.POINTER(Geometry), _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp,
                                       _c_vp, ctypes.POINTER(_c_vp), _c_vp]),
    "marf_net_layer_count": (_c_int, [_c_vp]),
    "marf_net_layer_span": (_c_int, [_c_vp, _c_int, ctypes.POINTER(_c_ll), ctypes.POINTER(_c_ll)]),
    "marf_comm_unique_id": (_c_int, [_c_vp, _c_sz]),
    "marf_comm_create": (_c_int, [_c_vp, _c_int, _c_int, _c_int, ctypes.POINTER(_c_vp)]),
    "marf_comm_destroy": (None, [_c_vp]),
    "marf_allreduce_grads": (_c_int, [_c_vp, _c_vp, _c_sz, _c_vp]),
    "marf_allreduce_grads_layers": (_c_int, [_c_vp, _c_vp, _c_vp, ctypes.POINTER(_c_vp), _c_vp]),
    "marf_mse_workspace_bytes": (_c_sz, []),
    "marf_edge_map": (_c_int, [_c_vp, _c_int, _c_int, _c_int, _c_vp, _c_vp]),
    "marf_erode_rect": (_c_int, [_c_vp, _c_int, _c_int, _c_int, _c_int, _c_int, _c_vp, _c_vp]),
    "marf_masked_mse": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    "marf_masked_mse_backward": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    "marf_adam_step": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_ll, _c_dbl, _c_dbl, _c_dbl, _c_dbl, _c_ll, _c_vp,
                                _c_vp]),
    "marf_adam_schedule": (_c_int, [_c_dbl, _c_dbl, _c_dbl, _c_ll, _c_ll, _c_vp]),
    "marf_adam_step_sched": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_ll, _c_dbl, _c_dbl, _c_dbl, _c_vp, _c_vp, _c_vp,
                                      _c_vp]),
    "marf_debug_set_stamps": (None, [_c_vp]),
    "marf_profile_enable": (_c_int, [_c_int]),
    "marf_profile_reset": (_c_int, []),
    "marf_profile_filter": (_c_int, [ctypes.c_char_p]),
    "marf_profile_read": (_c_int, [ctypes.c_char_p, _c_int, ctypes.POINTER(_c_dbl), ctypes.POINTER(_c_ll), _c_int]),
}

_lib = None

# Bumped by every in-library parameter update (marf Adam writes through raw pointers, which torch's
# version counters do not see); Engine.packed_for re-packs when it changes.
PARAM_GENERATION = [0]


def _ensure_current():
    """Refuse (or, for the default library, rebuild) a libmarf.so whose embedded source hash does
    not match the sources next to it (build_lib.source_hash)."""
    import build_lib
    default = not os.environ.get("MARF_LIB")
    want = build_lib.source_hash()
    have = build_lib.embedded_hash(LIB_PATH) if os.path.exists(LIB_PATH) else None
    if have == want:
        return
    if not default:
        # an explicitly chosen library (MARF_LIB: A/B and diagnostic builds, possibly of other
        # sources on purpose) is loaded, but never silently
        import sys
        print(f"[marf] warning: MARF_LIB={LIB_PATH} was built from other sources (hash {have}, tree {want})",
              file=sys.stderr, flush=True)
        return
    try:
        # one builder at a time (torchrun ranks, spawned test workers): the lock is held across the
        # re-check and the build, so a process that waited finds the fresh library and loads it
        import fcntl
        os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
        with open(LIB_PATH + ".lock", "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                have = build_lib.embedded_hash(LIB_PATH) if os.path.exists(LIB_PATH) else None
                if have != want:
                    build_lib.build(force=True, verbose=False)
            finally:
                fcntl.flock(lk, fcntl.LOCK_UN)
    except Exception as e:  # pragma: no cover - message path
        raise RuntimeError(f"libmarf.so at {LIB_PATH} is missing or stale and could not be built: {e}") from e


def lib():
    """Load libmarf.so; a library built from other sources than the ones in this tree is rebuilt
    (default path) or loaded with a warning (an explicit MARF_LIB), never loaded silently."""
    global _lib
    if _lib is None:
        _ensure_current()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("MARF_LIB") and not hasattr(L, name):
                continue  # (an explicit older diagnostic build: entry points added since are absent)
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError("libmarf: " + lib().marf_last_error().decode())


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _dev(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"libmarf: {name} must live on a ROCm GPU (got {t.device}); there is no CPU path")
    return t


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _f32(t, name):
    _dev(t, name)
    if t.dtype != torch.float32:
        raise TypeError(f"libmarf: {name} must be float32 (got {t.dtype})")
    return t.contiguous()


def profile_enable(on=True):
    _check(lib().marf_profile_enable(1 if on else 0))


def profile_reset():
    _check(lib().marf_profile_reset())


def profile_filter(names=None):
    """Time only the kernels named (profile names, e.g. ["mlp_step"]); None = every kernel."""
    _check(lib().marf_profile_filter(",".join(names).encode() if names else None))


def profile_read():
    """{kernel name: (total_ms, launches)} recorded with HIP events since the last reset."""
    cap, nl = 64, 64
    names = ctypes.create_string_buffer(cap * nl)
    tot = (_c_dbl * cap)()
    cnt = (_c_ll * cap)()
    n = lib().marf_profile_read(names, nl, tot, cnt, cap)
    out = {}
    for i in range(n):
        nm = names.raw[i * nl:(i + 1) * nl].split(b"\0", 1)[0].decode()
        out[nm] = (tot[i], cnt[i])
    return out


# ====================================================================== Lie / warp / posenc

class _SL3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, lie_batch):
        h = _f32(h, "h")
        B = h.shape[0]
        H = torch.empty(B, 3, 3, device=h.device, dtype=torch.float32)
        _check(lib().marf_sl3_to_SL3(_ptr(h), _ptr(H), B, lie_batch, _stream(h)))
        ctx.save_for_backward(h)
        ctx.lie_batch = lie_batch
        return H

    @staticmethod
    def backward(ctx, dH):
        (h,) = ctx.saved_tensors
        dH = _f32(dH, "dH")
        dh = torch.empty_like(h)
        _check(lib().marf_sl3_to_SL3_backward(_ptr(h), _ptr(dH), _ptr(dh), h.shape[0], ctx.lie_batch, _stream(h)))
        return dh, None


def sl3_to_SL3(h, lie_batch=0):
    """h [..., 8] -> H [..., 3, 3]  (warp.py:98-106), differentiable."""
    shp = h.shape[:-1]
    hb = h.reshape(-1, 8)
    lb = lie_batch if lie_batch > 0 else hb.shape[0]
    return _SL3.apply(hb, lb).reshape(*shp, 3, 3)


class _SE2Embed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p):
        p = _f32(p, "p")
        h = torch.empty(p.shape[0], 8, device=p.device, dtype=torch.float32)
        _check(lib().marf_se2_to_sl3(_ptr(p), _ptr(h), p.shape[0], _stream(p)))
        return h

    @staticmethod
    def backward(ctx, dh):
        dh = _f32(dh, "dh")
        dp = torch.empty(dh.shape[0], 3, device=dh.device, dtype=torch.float32)
        _check(lib().marf_se2_to_sl3_backward(_ptr(dh), _ptr(dp), dh.shape[0], _stream(dh)))
        return dp


def se2_to_sl3(p):
    """se(2) tangent p [..., 3] = (tx, ty, theta) -> the sl(3) parameters [..., 8] of the same
    generator (an extension: the reference has no SE(2), warp.py:72-80), differentiable."""
    shp = p.shape[:-1]
    return _SE2Embed.apply(p.reshape(-1, 3)).reshape(*shp, 8)


def se2_to_SE2(p, lie_batch=0):
    """p [..., 3] -> the SE(2) matrix [..., 3, 3] (the sl(3) exponential of the embedded generator)."""
    return sl3_to_SL3(se2_to_sl3(p), lie_batch)


def pixel_grid(H, W, patch_H, patch_W, crop, device):
    """One copy of Warp.get_normalized_pixel_grid (warp.py:33-68): [h*w, 2]."""
    if crop:
        h = (H // 2 + patch_H // 2) - (H // 2 - patch_H // 2)
        w = (W // 2 + patch_W // 2) - (W // 2 - patch_W // 2)
    else:
        h, w = H, W
    xy = torch.empty(h * w, 2, device=device, dtype=torch.float32)
    _check(lib().marf_pixel_grid(H, W, patch_H, patch_W, 1 if crop else 0, _ptr(xy), _stream(xy)))
    return xy


def _warp_points_fwd(xy, Hm):
    B, n = Hm.shape[0], xy.shape[-2]
    shared = 1 if xy.dim() == 2 or xy.shape[0] == 1 else 0
    if not shared and xy.shape[0] != B:
        raise ValueError("warp_points: batch mismatch")
    uv = torch.empty(B, n, 2, device=xy.device, dtype=torch.float32)
    _check(lib().marf_warp_points(_ptr(xy), _ptr(Hm), _ptr(uv), B, n, shared, _stream(xy)))
    return uv, shared


class _WarpPoints(torch.autograd.Function):
    """uv = (H [x, y, 1])[:2] / ((H [x, y, 1])[2] + 1e-8) and its autograd (warp.py:70-81)."""

    @staticmethod
    def forward(ctx, xy, Hm):
        xy, Hm = _f32(xy, "xy"), _f32(Hm, "H")
        uv, shared = _warp_points_fwd(xy, Hm)
        ctx.save_for_backward(xy, Hm)
        ctx.shared, ctx.xy_shape = shared, xy.shape
        return uv

    @staticmethod
    def backward(ctx, g):
        xy, Hm = ctx.saved_tensors
        g = _f32(g, "d uv")
        B, n = Hm.shape[0], xy.shape[-2]
        dxy = torch.empty(B, n, 2, device=g.device, dtype=torch.float32)
        dH = torch.empty(B, 3, 3, device=g.device, dtype=torch.float32)
        _check(lib().marf_warp_points_backward(_ptr(xy), _ptr(Hm), _ptr(g), _ptr(dxy), _ptr(dH), B, n, ctx.shared,
                                               _stream(g)))
        if ctx.shared:
            dxy = dxy.sum(0).reshape(ctx.xy_shape)
        return dxy, dH


def warp_points(xy, Hm):
    """xy [B or 1, n, 2] warped by Hm [B, 3, 3] -> [B, n, 2] (warp.py:74-78); differentiable in
    both (marf_warp_points_backward)."""
    if torch.is_grad_enabled() and (xy.requires_grad or Hm.requires_grad):
        return _WarpPoints.apply(xy, Hm)
    return _warp_points_fwd(_f32(xy, "xy"), _f32(Hm, "H"))[0]


def make_c2f(progress, c2f):
    c = C2f()
    if c2f is not None and progress is not None:
        c.d_progress = progress.data_ptr()
        c.start, c.end, c.on = float(c2f[0]), float(c2f[1]), 1
    return c


def prologue_probe(gt, mask, Hm, H, W, patch_H, patch_W, L, progress=None, c2f=None, grid=4096):
    """Measurement only: the fused step's input side (16 B/px target + mask reads, grid, warp,
    posenc) as one launch (marf_prologue_probe); returns the per-block partials."""
    B = gt.shape[0]
    geo = grid_geometry(B, H, W, patch_H, patch_W, _f32(Hm, "Hm"))
    out = torch.empty(grid, device=gt.device, dtype=torch.float32)
    cf = make_c2f(progress, c2f)
    _check(lib().marf_prologue_probe(ctypes.byref(geo), ctypes.byref(cf), L, _ptr(_f32(gt, "gt")),
                                     _ptr(None if mask is None else _f32(mask, "mask")), _ptr(out), grid,
                                     _stream(gt)))
    return out


def _posenc_fwd(coord, L, progress, c2f):
    n = coord.numel() // 2
    enc = torch.empty(*coord.shape[:-1], 4 * L, device=coord.device, dtype=torch.float32)
    cf = make_c2f(progress, c2f)
    _check(lib().marf_posenc(_ptr(coord), n, L, ctypes.byref(cf), _ptr(enc), _stream(coord)))
    return enc


class _Posenc(torch.autograd.Function):
    """Positional encoding with BARF c2f weights and its autograd in the coordinates
    (model/planar.py:451-471; progress enters through .data, so it gets no gradient)."""

    @staticmethod
    def forward(ctx, coord, L, progress, c2f):
        coord = _f32(coord, "coord")
        ctx.save_for_backward(coord)
        ctx.L, ctx.progress, ctx.c2f = L, progress, c2f
        return _posenc_fwd(coord, L, progress, c2f)

    @staticmethod
    def backward(ctx, g):
        (coord,) = ctx.saved_tensors
        g = _f32(g, "d enc")
        dc = torch.empty_like(coord)
        cf = make_c2f(ctx.progress, ctx.c2f)
        _check(lib().marf_posenc_backward(_ptr(coord), coord.numel() // 2, ctx.L, ctypes.byref(cf), _ptr(g), _ptr(dc),
                                          _stream(g)))
        return dc, None, None, None


def posenc(coord, L, progress=None, c2f=None):
    """coord [..., 2] -> [..., 4L] (model/planar.py:451-471 layout); differentiable in coord
    (marf_posenc_backward)."""
    if progress is not None:
        progress = progress.detach()
    if torch.is_grad_enabled() and coord.requires_grad:
        return _Posenc.apply(coord, L, progress, c2f)
    return _posenc_fwd(_f32(coord, "coord"), L, progress, c2f)


# ====================================================================== MLP engine

class Net:
    """An MLP shape + padding plan in the library (marf_net).  skip: the layer indices whose input
    is [previous output ; posenc features] (opt.arch.skip, model/planar.py:419-420, 440-441)."""

    def __init__(self, dims, L, dtype, pixels_hint=0, skip=()):
        self.dims = [int(d) for d in dims]
        self.L = int(L)
        self.dtype = dtype
        self.skip = sorted(int(s) for s in skip)
        mask = 0
        for s_ in self.skip:
            if not 0 <= s_ < 32:
                raise ValueError(f"skip layer {s_}")
            mask |= 1 << s_
        arr = (_c_int * len(self.dims))(*self.dims)
        h = _c_vp()
        _check(lib().marf_net_create_skip(len(self.dims) - 1, arr, self.L, dtype, int(pixels_hint), mask, ctypes.byref(h)))
        self._h = h
        self.param_count = lib().marf_net_param_count(h)
        self.packed_bytes = lib().marf_net_packed_bytes(h)
        self.step_kernel = lib().marf_net_step_kernel(h).decode()
        self.layer_spans = []  # (offset, length) of W_l then b_l in the flat parameter vector
        for l in range(lib().marf_net_layer_count(h)):
            off, n = ctypes.c_longlong(), ctypes.c_longlong()
            _check(lib().marf_net_layer_span(h, l, ctypes.byref(off), ctypes.byref(n)))
            self.layer_spans.append((off.value, n.value))

    @property
    def handle(self):
        return self._h

    def __del__(self):
        try:
            if getattr(self, "_h", None) and _lib is not None:
                _lib.marf_net_destroy(self._h)
        except Exception:
            pass

    def pack(self, flat_params, packed):
        _check(lib().marf_net_pack(self._h, _ptr(flat_params), _ptr(packed), _stream(flat_params)))

    def set_pipeline(self, mode=-1, wg_blocks=0, piece_tiles=0):
        """Pipelined weight gradients of the fused step (include/marf.h marf_net_set_pipeline):
        mode 0 off (default: measured slower), 1 on at any size, -1 large steps
        only.  Between steps only."""
        _check(lib().marf_net_set_pipeline(self._h, int(mode), int(wg_blocks), int(piece_tiles)))

    def saved_bytes(self, geo):
        return lib().marf_saved_bytes(self._h, ctypes.byref(geo))

    def workspace_bytes(self, geo):
        return lib().marf_workspace_bytes(self._h, ctypes.byref(geo))


def grid_geometry(B, H, W, patch_H, patch_W, Hm=None, crop=True):
    """Centre-crop pixel grid (crop) or every canvas pixel (use_cropped_images off, warp.py:54-68)."""
    g = Geometry()
    g.mode, g.B, g.H, g.W, g.patch_H, g.patch_W = GEO_GRID if crop else GEO_CANVAS, B, H, W, patch_H, patch_W
    g.d_H = None if Hm is None else Hm.data_ptr()
    return g


def coords_geometry(coords):
    g = Geometry()
    g.mode, g.B, g.Np = GEO_COORDS, 1, coords.shape[0]
    g.d_coords = coords.data_ptr()
    return g


class _Buffers:
    """Per-device cache of the byte buffers the library borrows (reused across steps).  Every get()
    bumps the buffer's generation, so a backward can check that no later forward reused it."""

    def __init__(self):
        self.bufs = {}
        self.gen = {}

    def get(self, name, nbytes, device):
        key = (name, str(device))
        t = self.bufs.get(key)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
            self.bufs[key] = t
        self.gen[key] = self.gen.get(key, 0) + 1
        return t

    def generation(self, name, device):
        return self.gen.get((name, str(device)), 0)


_BUFS = _Buffers()


def _split_grads(flat, shapes):
    out, off = [], 0
    for s in shapes:
        n = 1
        for d in s:
            n *= d
        out.append(flat[off:off + n].view(*s))
        off += n
    return out


class _MLPFunction(torch.autograd.Function):
    """NeuralImageFunction.forward on explicit coordinates (model/planar.py:429-449)."""

    @staticmethod
    def forward(ctx, coords, progress, engine, grad_on, *params):
        coords = _f32(coords, "coord_2d")
        shp = coords.shape[:-1]
        c2 = coords.reshape(-1, 2)
        n = c2.shape[0]
        rgb = torch.empty(n, 3, device=coords.device, dtype=torch.float32)
        need_grad = grad_on and any(ctx.needs_input_grad)
        ctx.empty = n == 0
        if ctx.empty:
            # torch's path on an empty batch: an empty [..., 0, 3] prediction and all-zero gradients
            # (mm over a zero-length axis); nothing to launch.
            ctx.coord_shape = coords.shape
            ctx.shapes = [p.shape for p in params]
            return rgb.view(*shp, 3)
        geo = coords_geometry(c2)
        packed = engine.packed_for(params)
        saved = None
        if need_grad:
            saved = torch.empty(max(engine.net.saved_bytes(geo), 1), dtype=torch.uint8, device=coords.device)
        cf = make_c2f(progress, engine.c2f)
        if need_grad:
            _check(lib().marf_forward(engine.net.handle, ctypes.byref(geo), ctypes.byref(cf), _ptr(packed), _ptr(rgb),
                                      _ptr(saved), _stream(coords)))
        else:
            _render(engine, geo, cf, packed, rgb, _stream(coords))
        if need_grad:
            ctx.save_for_backward(c2, progress, rgb)
            ctx.coord_shape = coords.shape
            ctx.saved_buf, ctx.packed, ctx.engine = saved, packed, engine
            ctx.shapes = [p.shape for p in params]
        return rgb.view(*shp, 3)

    @staticmethod
    def backward(ctx, d_rgb):
        if ctx.empty:
            grads = [torch.zeros(s, device=d_rgb.device, dtype=torch.float32) for s in ctx.shapes]
            dc = torch.zeros(ctx.coord_shape, device=d_rgb.device, dtype=torch.float32) if ctx.needs_input_grad[0] else None
            return (dc, None, None, None, *grads)
        c2, progress, rgb = ctx.saved_tensors
        engine = ctx.engine
        geo = coords_geometry(c2)
        d_rgb = _f32(d_rgb, "d_rgb").reshape(-1, 3)
        ws = _BUFS.get("mlp_ws", engine.net.workspace_bytes(geo), c2.device)
        dflat = torch.empty(engine.net.param_count, device=c2.device, dtype=torch.float32)
        dcoords = torch.empty_like(c2) if ctx.needs_input_grad[0] else None
        cf = make_c2f(progress, engine.c2f)
        _check(lib().marf_backward(engine.net.handle, ctypes.byref(geo), ctypes.byref(cf), _ptr(ctx.packed), None, 0,
                                   _ptr(rgb), _ptr(d_rgb), _ptr(ctx.saved_buf), _ptr(ws), _ptr(dflat), None,
                                   _ptr(dcoords), _stream(c2)))
        grads = _split_grads(dflat, ctx.shapes)
        dc = None if dcoords is None else dcoords.view(ctx.coord_shape)
        return (dc, None, None, None, *grads)


class _PlanarRenderFunction(torch.autograd.Function):
    """Graph.forward for the training batch (model/planar.py:329-335): crop grid -> sl(3) warp ->
    posenc/c2f -> MLP, fused in one kernel; backward = dgrad chain + warp adjoint + weight
    gradients.  Inputs: warp weight [B_all, 8], progress, engine, shard (b0, b1), *mlp params."""

    @staticmethod
    def forward(ctx, warp_weight, progress, engine, b0, b1, *params):
        w = _f32(warp_weight, "warp_param")
        Bl = b1 - b0
        h_local = w[b0:b1].contiguous()
        Hm = torch.empty(Bl, 3, 3, device=w.device, dtype=torch.float32)
        st = _stream(w)
        _check(lib().marf_sl3_to_SL3(_ptr(h_local), _ptr(Hm), Bl, engine.lie_batch(w.shape[0]), st))
        geo = engine.grid_geo(Bl, Hm)
        Np = geo_np(engine)
        rgb = torch.empty(Bl, Np, 3, device=w.device, dtype=torch.float32)
        packed = engine.packed_for(params)
        saved = _BUFS.get("planar_saved", engine.net.saved_bytes(geo), w.device)
        cf = make_c2f(progress, engine.c2f)
        _check(lib().marf_forward(engine.net.handle, ctypes.byref(geo), ctypes.byref(cf), _ptr(packed), _ptr(rgb),
                                  _ptr(saved), st))
        ctx.save_for_backward(w, progress, rgb)
        ctx.Hm, ctx.h_local, ctx.saved_buf, ctx.packed, ctx.engine = Hm, h_local, saved, packed, engine
        ctx.gen = _BUFS.generation("planar_saved", w.device)
        ctx.b0, ctx.b1 = b0, b1
        ctx.shapes = [p.shape for p in params]
        return rgb

    @staticmethod
    def backward(ctx, d_rgb):
        w, progress, rgb = ctx.saved_tensors
        engine = ctx.engine
        if ctx.gen != _BUFS.generation("planar_saved", w.device):
            raise RuntimeError("libmarf: the render's saved activations were reused by a later forward; "
                               "call backward() before the next Graph.forward")
        Bl = ctx.b1 - ctx.b0
        geo = engine.grid_geo(Bl, ctx.Hm)
        d_rgb = _f32(d_rgb, "d_rgb")
        ws = _BUFS.get("planar_ws", engine.net.workspace_bytes(geo), w.device)
        dflat = torch.empty(engine.net.param_count, device=w.device, dtype=torch.float32)
        engine.last_flat_grad = dflat
        dh_local = torch.empty(Bl, 8, device=w.device, dtype=torch.float32)
        cf = make_c2f(progress, engine.c2f)
        _check(lib().marf_backward(engine.net.handle, ctypes.byref(geo), ctypes.byref(cf), _ptr(ctx.packed),
                                   _ptr(ctx.h_local), engine.lie_batch(w.shape[0]), _ptr(rgb), _ptr(d_rgb),
                                   _ptr(ctx.saved_buf), _ptr(ws), _ptr(dflat), _ptr(dh_local), None, _stream(w)))
        if Bl == w.shape[0]:
            dw = dh_local
        else:
            dw = torch.zeros_like(w)
            dw[ctx.b0:ctx.b1] = dh_local
        grads = _split_grads(dflat, ctx.shapes)
        return (dw, None, None, None, None, *grads)


class _PlanarStepFunction(torch.autograd.Function):
    """Graph.forward + Graph.mse_loss of a training step (model/planar.py:329-336, 382-391), fused:
    the target and mask are known when the forward runs, so marf_step_forward runs the forward, the
    masked MSE and the whole backward with a unit upstream gradient in one pass over the pixels,
    and backward() only scales and reduces (marf_step_backward) by the d loss it receives.
    Outputs: rgb [Bl, Np, 3] and loss_rgb (0-d).  If rgb itself receives a gradient (a caller
    differentiating through the prediction other than via this loss), backward falls back to the
    general forward-with-saving + backward path for that part."""

    @staticmethod
    def forward(ctx, warp_weight, progress, engine, b0, b1, gt, mask, denom_override, *params):
        ctx.set_materialize_grads(False)
        w = _f32(warp_weight, "warp_param")
        Bl = b1 - b0
        h_local = w[b0:b1].contiguous()
        Hm = torch.empty(Bl, 3, 3, device=w.device, dtype=torch.float32)
        st = _stream(w)
        _check(lib().marf_sl3_to_SL3(_ptr(h_local), _ptr(Hm), Bl, engine.lie_batch(w.shape[0]), st))
        geo = engine.grid_geo(Bl, Hm)
        Np = geo_np(engine)
        gt = _f32(gt, "labels").reshape(Bl, 3, Np)
        mask = None if mask is None else _f32(mask, "masks").reshape(Bl, 1, Np)
        rgb = torch.empty(Bl, Np, 3, device=w.device, dtype=torch.float32)
        stats = torch.empty(3, device=w.device, dtype=torch.float32)
        packed = engine.packed_for(params)
        saved = _BUFS.get("planar_step", lib().marf_step_saved_bytes(engine.net.handle, ctypes.byref(geo)), w.device)
        cf = make_c2f(progress, engine.c2f)
        _check(lib().marf_step_forward(engine.net.handle, ctypes.byref(geo), ctypes.byref(cf), _ptr(packed), _ptr(gt),
                                       _ptr(mask), _ptr(denom_override), _ptr(rgb), _ptr(stats), _ptr(saved), st))
        ctx.save_for_backward(w, progress, rgb, stats)
        ctx.Hm, ctx.h_local, ctx.saved_buf, ctx.packed, ctx.engine = Hm, h_local, saved, packed, engine
        ctx.gen = _BUFS.generation("planar_step", w.device)
        ctx.gt, ctx.mask = gt, mask
        ctx.b0, ctx.b1 = b0, b1
        ctx.params = params
        ctx.shapes = [p.shape for p in params]
        engine.last_stats = stats  # [loss, denominator, local 3*sum(mask)]
        return rgb, stats[0]

    @staticmethod
    def backward(ctx, d_rgb, d_loss):
        w, progress, rgb, stats = ctx.saved_tensors
        engine = ctx.engine
        n_in = 8 + len(ctx.shapes)
        if d_rgb is None and d_loss is None:
            return (None,) * n_in
        if ctx.gen != _BUFS.generation("planar_step", w.device):
            raise RuntimeError("libmarf: the fused step's saved buffers were reused by a later forward; "
                               "call backward() before the next Graph.forward")
        Bl = ctx.b1 - ctx.b0
        geo = engine.grid_geo(Bl, ctx.Hm)
        alloc = torch.empty if d_loss is not None else torch.zeros  # the step backward writes every element
        engine.events_for = None  # set below only when this backward records the per-layer events
        dflat = alloc(engine.net.param_count, device=w.device, dtype=torch.float32)
        dh_local = alloc(Bl, 8, device=w.device, dtype=torch.float32)
        if d_loss is not None:
            gout = _f32(d_loss.reshape(1).to(torch.float32), "grad")
            ev = engine.grad_events  # per-layer "gradient final" events for a bucketed all-reduce (or None)
            _check(lib().marf_step_backward_ev(engine.net.handle, ctypes.byref(geo), _ptr(ctx.saved_buf),
                                               _ptr(ctx.h_local), engine.lie_batch(w.shape[0]), _ptr(gout), _ptr(stats),
                                               _ptr(dflat), _ptr(dh_local), ev.array if ev is not None else None,
                                               _stream(w)))
            engine.events_for = dflat.data_ptr() if ev is not None and d_rgb is None else None
        if d_rgb is not None:
            # gradient reaching the prediction directly: general path (forward with saving + backward)
            with torch.enable_grad():
                wd = w.detach().requires_grad_()
                ps = [q.detach().requires_grad_() for q in ctx.params]
                r = _PlanarRenderFunction.apply(wd, progress, engine, ctx.b0, ctx.b1, *ps)
                gs = torch.autograd.grad(r, [wd] + ps, d_rgb)
            dh_local = dh_local + gs[0][ctx.b0:ctx.b1]
            dflat = dflat + torch.cat([g.reshape(-1) for g in gs[1:]])
        engine.last_flat_grad = dflat
        if Bl == w.shape[0]:
            dw = dh_local
        else:
            dw = torch.zeros_like(w)
            dw[ctx.b0:ctx.b1] = dh_local
        grads = _split_grads(dflat, ctx.shapes)
        return (dw, None, None, None, None, None, None, None, *grads)


def render_step(warp_weight, progress, engine, params, gt, mask, denom_override=None, b0=0, b1=None):
    b1 = warp_weight.shape[0] if b1 is None else b1
    return _PlanarStepFunction.apply(warp_weight, progress, engine, b0, b1, gt, mask, denom_override, *params)


def geo_np(engine):
    if not engine.crop:
        return engine.H * engine.W
    h = (engine.H // 2 + engine.patch_H // 2) - (engine.H // 2 - engine.patch_H // 2)
    w = (engine.W // 2 + engine.patch_W // 2) - (engine.W // 2 - engine.patch_W // 2)
    return h * w


class Engine:
    """Library-side state of one NeuralImageFunction: net plan, packed weights, c2f, geometry."""

    def __init__(self, dims, L, dtype, c2f, H, W, patch_H, patch_W, lie_batch=0, crop=True, pixels_hint=0, skip=()):
        self.net = Net(dims, L, dtype, pixels_hint, skip)
        self.c2f = c2f
        self.H, self.W, self.patch_H, self.patch_W = H, W, patch_H, patch_W
        self.crop = bool(crop)
        self._lie_batch = lie_batch
        self._packed = None
        self._packed_version = None
        self.last_flat_grad = None
        self.last_stats = None
        self.grad_events = None  # GradEvents: set by the Model for the bucketed gradient all-reduce
        self.events_for = None   # data_ptr of the flat gradient those events last marked

    def lie_batch(self, B):
        return self._lie_batch if self._lie_batch > 0 else B

    def grid_geo(self, B, Hm):
        return grid_geometry(B, self.H, self.W, self.patch_H, self.patch_W, Hm, self.crop)

    def packed_for(self, params):
        """Pack the fp32 master weights into the MFMA operand layouts when they changed (tracked by
        the parameters' in-place version counters, so every optimizer step triggers a re-pack)."""
        ver = (PARAM_GENERATION[0],) + tuple((p.data_ptr(), p._version) for p in params)
        if self._packed is not None and ver == self._packed_version:
            return self._packed
        dev = params[0].device
        flat = flat_view(params)
        if flat is None:
            flat = torch.cat([p.detach().reshape(-1) for p in params])
        _f32(flat, "mlp parameters")
        if self._packed is None or self._packed.device != dev:
            self._packed = torch.empty(self.net.packed_bytes, dtype=torch.uint8, device=dev)
        self.net.pack(flat, self._packed)
        self._packed_version = ver
        return self._packed


class GradEvents:
    """One torch event per MLP layer, handed to marf_step_backward_ev: event l is recorded on the
    step's stream when layer l's gradient is final (last layer first), so each layer's all-reduce can
    start while the weight gradients of the others still run."""

    def __init__(self, n_layers, device):
        self.events = []
        for _ in range(n_layers):
            e = torch.cuda.Event()
            e.record(torch.cuda.current_stream(device))  # (torch creates the HIP event at first record)
            self.events.append(e)
        self.array = (_c_vp * n_layers)(*[e.cuda_event for e in self.events])


class Comm:
    """RCCL communicator of the C ABI (marf_comm_*), for hosts without torch.distributed: rank 0's
    unique_id() bytes go to every rank, each then joins with Comm(uid, world, rank, device)."""

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        _check(lib().marf_comm_unique_id(buf, 128))
        return buf.raw

    def __init__(self, uid, world, rank, device):
        h = _c_vp()
        _check(lib().marf_comm_create(ctypes.c_char_p(bytes(uid)), world, rank, device, ctypes.byref(h)))
        self.handle = h

    def allreduce(self, flat):
        """In-place fp32 sum over ranks on the tensor's current stream."""
        _check(lib().marf_allreduce_grads(self.handle, _ptr(_f32(flat, "gradient")), flat.numel(), _stream(flat)))

    def allreduce_layers(self, net, flat, events):
        """Per-layer sums, each after its layer's event, on the communicator's stream; the current
        stream waits for the last."""
        _check(lib().marf_allreduce_grads_layers(self.handle, net.handle, _ptr(_f32(flat, "gradient")), events.array,
                                                 _stream(flat)))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                lib().marf_comm_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None


def flat_view(tensors):
    """If `tensors` are consecutive views of one contiguous fp32 storage, return the flat 1-D view
    covering them (no copy), else None."""
    if not tensors:
        return None
    t0 = tensors[0]
    st = t0.untyped_storage()
    off = t0.storage_offset()
    total = 0
    for t in tensors:
        if t.untyped_storage().data_ptr() != st.data_ptr() or not t.is_contiguous() or t.storage_offset() != off + total:
            return None
        total += t.numel()
    return torch.empty(0, dtype=t0.dtype, device=t0.device).set_(st, off, (total,), (1,))


def render_train(warp_weight, progress, engine, params, b0=0, b1=None):
    b1 = warp_weight.shape[0] if b1 is None else b1
    if not torch.is_grad_enabled():
        return render_nograd(warp_weight, progress, engine, params, b0, b1)
    return _PlanarRenderFunction.apply(warp_weight, progress, engine, b0, b1, *params)


def render_nograd(warp_weight, progress, engine, params, b0, b1):
    """Graph.forward without autograd (evaluation / render rate): the same fused grid -> warp ->
    posenc -> MLP kernel, nothing saved for a backward."""
    w = _f32(warp_weight, "warp_param")
    Bl = b1 - b0
    h_local = w[b0:b1].contiguous()
    Hm = torch.empty(Bl, 3, 3, device=w.device, dtype=torch.float32)
    st = _stream(w)
    _check(lib().marf_sl3_to_SL3(_ptr(h_local), _ptr(Hm), Bl, engine.lie_batch(w.shape[0]), st))
    geo = engine.grid_geo(Bl, Hm)
    rgb = torch.empty(Bl, geo_np(engine), 3, device=w.device, dtype=torch.float32)
    packed = engine.packed_for(params)
    cf = make_c2f(progress, engine.c2f)
    _render(engine, geo, cf, packed, rgb, st)
    return rgb


def _render(engine, geo, cf, packed, rgb, st):
    """marf_render: forward only in the net's recipe (the split-bf16 pixel-per-wave kernel for
    bf16x3 nets, whose workspace is a small per-device buffer)."""
    nb = lib().marf_render_workspace_bytes(engine.net.handle, ctypes.byref(geo))
    ws = _BUFS.get("render_ws", nb, rgb.device) if nb else None
    _check(lib().marf_render(engine.net.handle, ctypes.byref(geo), ctypes.byref(cf), _ptr(packed), _ptr(rgb), _ptr(ws),
                             st))


def mlp_forward(coords, progress, engine, params):
    return _MLPFunction.apply(coords, progress, engine, torch.is_grad_enabled(), *params)


# ====================================================================== loss

class _MaskedMSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, mask, denom_override):
        pred, gt = _f32(pred, "pred"), _f32(gt, "labels")
        mask = None if mask is None else _f32(mask, "masks")
        B, Np = pred.shape[0], pred.shape[1]
        out = torch.empty(3, device=pred.device, dtype=torch.float32)
        ws = _BUFS.get("mse_ws", lib().marf_mse_workspace_bytes(), pred.device)
        _check(lib().marf_masked_mse(_ptr(pred), _ptr(gt), _ptr(mask), B, Np, _ptr(denom_override), _ptr(out),
                                     _ptr(ws), _stream(pred)))
        ctx.save_for_backward(pred, gt, mask, out)
        return out[0]

    @staticmethod
    def backward(ctx, gout):
        pred, gt, mask, out = ctx.saved_tensors
        gout = _f32(gout.reshape(1), "grad")
        d = torch.empty_like(pred)
        _check(lib().marf_masked_mse_backward(_ptr(pred), _ptr(gt), _ptr(mask), pred.shape[0], pred.shape[1],
                                              _ptr(out[1:2]), _ptr(gout), _ptr(d), _stream(pred)))
        return d, None, None, None


def masked_mse(pred_bn3, gt_b3n, mask_b1n=None, denom_override=None):
    """Graph.mse_loss (model/planar.py:382-391) on the MLP's [B, N, 3] output layout."""
    return _MaskedMSE.apply(pred_bn3, gt_b3n, mask_b1n, denom_override)


def mse_stats(pred_bn3, gt_b3n, mask_b1n=None):
    """(loss, denom, local 3*sum(mask)) without autograd."""
    pred, gt = _f32(pred_bn3, "pred"), _f32(gt_b3n, "labels")
    mask = None if mask_b1n is None else _f32(mask_b1n, "masks")
    out = torch.empty(3, device=pred.device, dtype=torch.float32)
    ws = _BUFS.get("mse_ws", lib().marf_mse_workspace_bytes(), pred.device)
    _check(lib().marf_masked_mse(_ptr(pred), _ptr(gt), _ptr(mask), pred.shape[0], pred.shape[1], None, _ptr(out),
                                 _ptr(ws), _stream(pred)))
    return out


# ====================================================================== edge maps

def edge_map(images):
    """inputs.compute_edges (reference inputs.py:50-67) on the device: [B, C, H, W] (any float layout)
    -> [B, C, H, W] float64 Sobel-magnitude edge maps, Gaussian-blurred (cv2 semantics)."""
    _dev(images, "images")
    x = images.detach().to(torch.float32).contiguous()
    B, C, H, W = x.shape
    out = torch.empty((B, C, H, W), dtype=torch.float64, device=x.device)
    _check(lib().marf_edge_map(_ptr(x), B * C, H, W, _ptr(out), _stream(x)))
    return out


def erode_rect(images, kernel=(5, 5)):
    """erode_images (reference inputs.py:71-85) on the device: [B, C, H, W] float -> float32 of the
    same shape, cv2.erode with a kernel[0] (width) x kernel[1] (height) rectangle."""
    _dev(images, "images")
    x = images.detach().to(torch.float32).contiguous()
    B, C, H, W = x.shape
    out = torch.empty_like(x)
    _check(lib().marf_erode_rect(_ptr(x), B * C, H, W, int(kernel[1]), int(kernel[0]), _ptr(out), _stream(x)))
    return out


# ====================================================================== Adam

def adam_step(p, g, m, v, lr, beta1, beta2, eps, step, grad_scale=None):
    _check(lib().marf_adam_step(_ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), float(lr), float(beta1), float(beta2),
                                float(eps), int(step), _ptr(grad_scale), _stream(p)))


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (model/planar.py:98-99) with the update in one HIP kernel per contiguous
    parameter segment.  Same constructor, param groups, state keys (step, exp_avg, exp_avg_sq).
    Parameters with grad None are skipped, as in torch.  step_scheduled() is the same update with the
    per-step scalars read on the device (a captured training iteration replays it)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, **kw):
        if weight_decay != 0 or amsgrad:
            raise ValueError("marf Adam: weight_decay / amsgrad are not used by the planar model")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        self._flat_state = {}

    def _segments(self, group, advance):
        """(param, grad, exp_avg, exp_avg_sq, step) per launch of the group's parameters that have a
        gradient: one per run of consecutive views (the MLP parameters share one flat buffer), state
        created (zeros) on first use; advance: each parameter's step += 1 first."""
        ps = [p for p in group["params"] if p.grad is not None]
        if not ps:
            return []
        runs, cur = [], [ps[0]]
        for p in ps[1:]:
            if flat_view(cur + [p]) is not None and flat_view([q.grad for q in cur + [p]]) is not None:
                cur.append(p)
            else:
                runs.append(cur)
                cur = [p]
        runs.append(cur)
        out = []
        for run in runs:
            for p in run:
                st = self.state[p]
                if not st:
                    st["step"] = 0
            if advance:
                for p in run:
                    self.state[p]["step"] += 1
            step = self.state[run[0]]["step"]
            if len(run) > 1 and all(self.state[p]["step"] == step for p in run):
                pf = flat_view(run)
                gf = flat_view([p.grad for p in run])
                key = tuple(id(p) for p in run)
                if key not in self._flat_state:
                    m = torch.zeros_like(pf)
                    v = torch.zeros_like(pf)
                    self._flat_state[key] = (m, v)
                    for p, mm, vv in zip(run, _split_grads(m, [q.shape for q in run]),
                                         _split_grads(v, [q.shape for q in run])):
                        self.state[p]["exp_avg"], self.state[p]["exp_avg_sq"] = mm, vv
                m, v = self._flat_state[key]
                out.append((pf, gf.contiguous(), m, v, step))
            else:
                for p in run:
                    st = self.state[p]
                    if "exp_avg" not in st:
                        st["exp_avg"] = torch.zeros_like(p)
                        st["exp_avg_sq"] = torch.zeros_like(p)
                    out.append((p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], st["step"]))
        return out

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p, g, m, v, step in self._segments(group, advance=True):
                adam_step(p, g, m, v, group["lr"], b1, b2, group["eps"], step)
        PARAM_GENERATION[0] += 1
        return loss

    def schedule_tables(self, n_steps, device):
        """Per group: the [n_steps][2] float32 table of (step_size, sqrt(1 - beta2^k)) for steps
        k = 1 .. n_steps, as marf_adam_step computes them (marf_adam_schedule), on the device."""
        tabs = []
        for group in self.param_groups:
            b1, b2 = group["betas"]
            buf = (ctypes.c_float * (2 * n_steps))()
            _check(lib().marf_adam_schedule(float(group["lr"]), float(b1), float(b2), 1, int(n_steps), buf))
            tabs.append(torch.from_numpy(np.ctypeslib.as_array(buf).copy()).to(device))
        return tabs

    @torch.no_grad()
    def step_scheduled(self, index, tables, expect_step):
        """The update of every group with its step's scalars read on the device: row index[0] (device
        int32, = step - 1) of the group's schedule table.  Host state is not advanced (the caller
        does, per replay: advance_steps); expect_step = the step this launch sequence is recorded for
        (every segment's state must be one behind it: one shared index)."""
        for group, tab in zip(self.param_groups, tables):
            b1, b2 = group["betas"]
            for p, g, m, v, step in self._segments(group, advance=False):
                if step + 1 != expect_step:
                    raise RuntimeError(f"Adam.step_scheduled: parameter at step {step}, expected {expect_step - 1}")
                _check(lib().marf_adam_step_sched(_ptr(p), _ptr(g), _ptr(m), _ptr(v), p.numel(), float(b1), float(b2),
                                                  float(group["eps"]), _ptr(tab), _ptr(index), None, _stream(p)))

    def advance_steps(self):
        """Host bookkeeping of one replayed step_scheduled: every parameter with a gradient steps."""
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    self.state[p]["step"] += 1
        PARAM_GENERATION[0] += 1
