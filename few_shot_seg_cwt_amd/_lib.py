"""ctypes binding of libcwt.so (include/cwt.h).

The product path has no CPU fallback: if the library is missing or no GPU is visible,
every call raises.  cffi is not installed in this image, so the binding uses ctypes;
the ABI is plain C and equally bindable from cffi.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# CWT_LIB_PATH selects another build of the library (A/B timing of two builds in one session)
LIB_PATH = os.environ.get("CWT_LIB_PATH") or os.path.join(_HERE, "libcwt.so")

_P = C.c_void_p
_I = C.c_int
_F = C.c_float
_I64 = C.c_int64

# name -> (restype, argtypes); must match include/cwt.h exactly (tests check every symbol)
SIGNATURES = {
    "cwt_version": (C.c_char_p, []),
    "cwt_last_error": (C.c_char_p, []),
    "cwt_ctx_create": (_I, [_I, C.POINTER(_P)]),
    "cwt_ctx_destroy": (_I, [_P]),
    "cwt_backbone_load": (_I, [_P, _I, _I, C.POINTER(C.c_char_p), C.POINTER(_P), C.POINTER(_I64), _F,
                               C.POINTER(_P)]),
    "cwt_backbone_destroy": (_I, [_P]),
    "cwt_backbone_set_precision": (_I, [_P, _I]),
    "cwt_extract_features": (_I, [_P, _P, _P, _I, _I, _P, _P]),
    "cwt_extract_features_train_bn": (_I, [_P, _P, _P, _I, _I, _P, _F, _F, C.c_uint64, _P]),
    "cwt_backbone_read_bn": (_I, [_P, C.c_char_p, _P, _I]),
    "cwt_preprocess_image": (_I, [_P, _P, _I, _I, _I, _I, C.POINTER(_F), C.POINTER(_F), C.POINTER(_F), _I, _I, _P,
                                  _P]),
    "cwt_preprocess_label": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "cwt_workspace_bytes": (C.c_size_t, [_P]),
    "cwt_inner_adapt": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _F, _I, _P, _P]),
    "cwt_inner_adapt_batch": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _I, _P, _P]),
    "cwt_normalize": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P]),
    "cwt_attention_fwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cwt_attention_saved_floats": (C.c_size_t, [_I, _I, _I, _I]),
    "cwt_attention_bwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cwt_attention_fwd_train": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, C.c_uint64,
                                     _P]),
    "cwt_attention_bwd_train": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F,
                                     _F, C.c_uint64, _P]),
    "cwt_classify": (_I, [_P, _P, _P, _I, _I, _I, _P, _P]),
    "cwt_attention_infer": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _I64, _P, _P, _P, _P]),
    "cwt_classify_scaled": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P]),
    "cwt_episode_tail": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _P, _P, _P, _P,
                              _P]),
    "cwt_inner_adapt_tail": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _F, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _P,
                                  _P, _P, _P, _P, _P]),
    "cwt_seg_metrics": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "cwt_seg_metrics_pair": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "cwt_seg_ce_fwd_bwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "cwt_classify_bwd": (_I, [_P, _P, _P, _I, _I, _I, _P, _P]),
    "cwt_iou_preds": (_I, [_P, _P, _P, _I64, _I, _I, _P, _P]),
    "cwt_cos_classify": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P]),
    "cwt_cos_classify_bwd": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P]),
    "cwt_corr": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "cwt_mutual_matching": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "cwt_match_corr_forward": (_I, [_P, _P, _I, _I, _I, _I, _P, _I, _F, _P, _I, _P, _P, _P]),
    "cwt_match_corr_forward_cv4": (_I, [_P, _P, _I, _I, _I, _I, _P, _I, _F, _P, _I, _P, _P, _P]),
    "cwt_match_masks": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P]),
    "cwt_channel_sum": (_I, [_P, _P, _I, _I, _I64, _P, _P]),
    "cwt_sce_descriptor": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "cwt_match_readout": (_I, [_P, _P, _I, _I, _I, _F, _P, _I, _P, _P]),
    "cwt_match_masks_train": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _F, C.c_uint64, _P]),
    "cwt_match_readout_backward": (_I, [_P, _P, _I, _I, _I, _F, _P, _I, _P, _P, _P, _P, _P]),
    "cwt_weight_average": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cwt_mmn_blend": (_I, [_P, _P, _P, _I, _I64, _F, _P, _P, _P]),
    "cwt_match_corr_saved_floats": (_I, [_I, _I, _I, _I, _I, _I, C.POINTER(_I64)]),
    "cwt_match_corr_forward_train": (_I, [_P, _P, _I, _I, _I, _I, _P, _I, _F, _P, _I, _P, _P, _P, _P]),
    "cwt_match_corr_backward": (_I, [_P, _P, _I, _I, _I, _I, _P, _I, _F, _P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "cwt_corr_backward": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _P]),
    "cwt_weight_average_train": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cwt_weight_average_backward": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                         _P, _P, _P]),
    "cwt_mmn_blend_backward": (_I, [_P, _P, _P, _I, _I64, _F, _P, _P, _P]),
    "cwt_linear_backward": (_I, [_P, _P, _I64, _I, _P, _I, _P, _P, _P, _P, _I, _P, _P]),
    "cwt_deform_attn_backward": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "cwt_norm_blend_backward": (_I, [_P, _P, _P, _I64, _I, _F, _P, _P, _P, _P]),
    "cwt_linear": (_I, [_P, _P, _I64, _I, _P, _P, _I, _I, _I, _P, _P]),
    "cwt_sine_pos_add": (_I, [_P, _P, _I, _I, _I, _I, _F, _I, _F, _F, _P, _P]),
    "cwt_deform_attn": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "cwt_norm_blend": (_I, [_P, _P, _P, _I64, _I, _F, _P, _P]),
    "cwt_extract_features_mid": (_I, [_P, _P, _P, _I, _I, _P, _P, _P, _P, _P]),
    "cwt_sgd_step": (_I, [_P, _P, _P, _P, _I64, _F, _F, _F, _I, _I, _P]),
    "cwt_pretrain_create": (_I, [_P, _I, _I, _I, C.POINTER(C.c_char_p), C.POINTER(_P), C.POINTER(_I64), _F,
                                 C.POINTER(_P)]),
    "cwt_pretrain_destroy": (_I, [_P]),
    "cwt_pretrain_step": (_I, [_P, _P, _P, _P, _I, _I, _P, _P, _P]),
    "cwt_pretrain_forward": (_I, [_P, _P, _P, _I, _I, _I, _P, _P]),
    "cwt_pretrain_get": (_I, [_P, C.c_char_p, _I, _P, _I64]),
    "cwt_pretrain_evaluate": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "cwt_pretrain_set": (_I, [_P, C.c_char_p, _I, _P, _I64]),
    "cwt_pretrain_num_params": (_I, [_P, C.POINTER(_I64), C.POINTER(_I64)]),
    "cwt_cu_count": (_I, [_P, _P]),
    "cwt_adapt_workgroups": (_I, [_P, _I, _I, _I, _I, _I, _P]),
    "cwt_adapt_fuses_tail": (_I, [_P, _I, _I, _I, _I, _P]),
    "cwt_stream_create_masked": (_I, [_P, _P, _I, _P]),
    "cwt_stream_destroy": (_I, [_P]),
    "cwt_debug_conv": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I,
                            _I, _I, _I, _I, _P]),
    "cwt_debug_split_act": (_I, [_P, _P, _I64, _I, _I, _P, _P]),
    "cwt_debug_unsplit_act": (_I, [_P, _P, _I64, _I, _P, _I, _P]),
    "cwt_debug_pack_wsplit": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "cwt_debug_conv_s": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _I, _I,
                              _P, _I, _I, _I, _P]),
    "cwt_debug_conv_b16": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _I, _I,
                                _P, _I, _I, _I, _P]),
    "cwt_debug_cp4d_layer": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _I, _P]),
    "cwt_debug_conv_f32d": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _I,
                                 _I, _I, _P]),
    "cwt_debug_conv_x6": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _I,
                               _I, _I, _P]),
    "cwt_debug_conv_x6w": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P, _I, _I, _P, _I, _I, _I,
                                _I, _I, _P]),
    "cwt_debug_census": (_I, [_P, _I, _P, _P]),
    "cwt_debug_tail_stamps": (_I, [_P, _P, _I64, _P]),
    "cwt_debug_occupy": (_I, [_P, _I, _I, _P]),
    "cwt_debug_pretrain_op": (_I, [_P, _I, C.POINTER(_P), C.POINTER(_I64), C.POINTER(_F), _P]),
    "cwt_debug_adapt_stamps": (_I, [_P, _P, _I64, C.POINTER(_I64)]),
    "cwt_ctx_set_adapt_units": (_I, [_P, _I]),
    "cwt_ctx_status": (_I, [_P, C.POINTER(C.c_uint32), _I]),
    "cwt_ctx_set_conv_arith": (_I, [_P, _I]),
    "cwt_debug_adapt_spin_limit": (_I, [_P, _I64]),
    "cwt_debug_pretrain_capture": (_I, [_P, _I]),
    "cwt_debug_pretrain_tensor": (_I, [_P, C.c_char_p, _P, _I64]),
    "cwt_profile_enable": (_I, [_P, _I]),
    "cwt_profile_count": (_I, [_P]),
    "cwt_profile_record": (_I, [_P, _I, C.c_char_p, _I, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                C.POINTER(_F)]),
}

_lib = None
_lock = threading.RLock()
_ctx = {}


class CwtError(RuntimeError):
    pass


def check_provenance(version: str, path: str):
    """Refuse a library built from other sources than the tree's (build.py source_hash, compiled
    into cwt_version()).  CWT_LIB_PATH builds (A/B timing of another build) are exempt."""
    from . import build as _build
    if os.environ.get("CWT_LIB_PATH") or not os.path.isdir(_build.CSRC):
        return
    want = _build.source_hash()
    got = version.rsplit("src=", 1)[-1] if "src=" in version else None
    if got != want:
        raise CwtError(f"{path} is stale: built from sources {got}, the tree's are {want}; "
                       "run `python -m few_shot_seg_cwt_amd.build`")


def load_library(path: str = LIB_PATH):
    """Load libcwt.so and declare every prototype (works without a GPU)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise CwtError(f"{path} not built: run `python -m few_shot_seg_cwt_amd.build` "
                               "(the product path has no CPU fallback)")
            lib = C.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            check_provenance(lib.cwt_version().decode(), path)
            _lib = lib
    return _lib


def lib():
    return load_library()


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().cwt_last_error().decode(errors="replace")
        raise CwtError(f"{what} failed (code {rc}): {msg}")


_override = threading.local()
_extra_ctx = {}   # device -> [additional contexts] (workspace sets of concurrent streams)


def _create_ctx(device: int):
    p = C.c_void_p()
    rc = load_library().cwt_ctx_create(device, C.byref(p))
    if rc != 0:
        raise CwtError(f"cwt_ctx_create failed: {_lib.cwt_last_error().decode()}")
    return p


def ctx(device: int | None = None):
    """The calling thread's context for the device: the per-device default, or the one a
    ``using_ctx`` block selected (a context owns the workspaces; calls on one context are
    externally serialised, so concurrent streams each use a context of their own)."""
    if not torch.cuda.is_available():
        raise CwtError("libcwt needs a HIP device (torch.cuda.is_available() is False); no CPU fallback")
    if device is None:
        device = torch.cuda.current_device()
    sel = getattr(_override, "ctx", None)
    if sel is not None and sel[0] == device:
        return sel[1]
    with _lock:
        if device not in _ctx:
            _ctx[device] = _create_ctx(device)
        return _ctx[device]


def new_ctx(device: int | None = None):
    """An additional context on the device (its own workspace set), kept for the process."""
    if device is None:
        device = torch.cuda.current_device()
    ctx(device)
    with _lock:
        p = _create_ctx(device)
        _extra_ctx.setdefault(device, []).append(p)
        return p


def destroy_ctx(p, device: int | None = None) -> None:
    """Destroy an additional context made by :func:`new_ctx` (its workspaces are freed; the
    caller has synchronised every stream that used it)."""
    if device is None:
        device = torch.cuda.current_device()
    with _lock:
        lst = _extra_ctx.get(device, [])
        for i, q in enumerate(lst):
            if q is p or getattr(q, "value", None) == getattr(p, "value", p):
                del lst[i]
                check(load_library().cwt_ctx_destroy(p), "cwt_ctx_destroy")
                return
    raise CwtError("destroy_ctx: not an additional context of this device")


class using_ctx:
    """``with using_ctx(c): ...`` routes this thread's libcwt calls on c's device to context c."""

    def __init__(self, c, device: int | None = None):
        self.c, self.device = c, torch.cuda.current_device() if device is None else device

    def __enter__(self):
        self.prev = getattr(_override, "ctx", None)
        _override.ctx = (self.device, self.c)
        return self.c

    def __exit__(self, *exc):
        _override.ctx = self.prev
        return False


def all_ctx(device: int | None = None):
    if device is None:
        device = torch.cuda.current_device()
    return [ctx(device)] + list(_extra_ctx.get(device, []))


STATUS_ADAPT_BARRIER = 1   # CWT_STATUS_ADAPT_BARRIER (include/cwt.h)
STATUS_TAIL_BARRIER = 2    # CWT_STATUS_TAIL_BARRIER


def check_status(device: int | None = None, clear: bool = True) -> None:
    """Raise CwtError if a kernel enqueued on any of the device's contexts reported an
    asynchronous failure (cwt_ctx_status).  Call after a synchronising readback; no GPU call."""
    w = C.c_uint32()
    bad = 0
    for c in all_ctx(device):
        check(lib().cwt_ctx_status(c, C.byref(w), int(clear)), "cwt_ctx_status")
        bad |= w.value
    if bad & STATUS_TAIL_BARRIER:
        raise CwtError("the fused episode tail's grid barrier timed out (its workgroups were not all co-resident): "
                       "the CWT output, logits and IoU counts of an episode on this device are wrong")
    if bad & STATUS_ADAPT_BARRIER:
        raise CwtError("the persistent inner loop's grid barrier timed out (its workgroups were not all "
                       "co-resident): the adapted classifier W of an episode on this device is wrong")
    if bad:
        raise CwtError(f"asynchronous libcwt failure, status 0x{bad:x}")


def stream_ptr(device=None) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t: torch.Tensor | None) -> C.c_void_p | None:
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def require(t: torch.Tensor, name: str, dtype=torch.float32, device=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise CwtError(f"{name} must be a device tensor (no CPU fallback)")
    return t


def profile_enable(level: int, device=None):
    """0 off; 1 phases + bottleneck conv (cheap, for timed regions); 2 every launch.  Applies
    to every context of the device."""
    for c in all_ctx(device):
        check(lib().cwt_profile_enable(c, int(level)), "cwt_profile_enable")


def profile_records(device=None):
    """[(name, flops, bytes, ms)] of the launches recorded since profile_enable, over every
    context of the device (default context first)."""
    out = []
    buf = C.create_string_buffer(256)
    fl, by, ms = C.c_double(), C.c_double(), C.c_float()
    for c in all_ctx(device):
        for i in range(lib().cwt_profile_count(c)):
            check(lib().cwt_profile_record(c, i, buf, 256, C.byref(fl), C.byref(by), C.byref(ms)),
                  "cwt_profile_record")
            out.append((buf.value.decode(), fl.value, by.value, ms.value))
    return out


def cu_count(device: int | None = None) -> int:
    """Number of compute units of the device (cwt_cu_count)."""
    import ctypes
    n = ctypes.c_int(0)
    check(lib().cwt_cu_count(ctx(device), ctypes.byref(n)), "cwt_cu_count")
    return n.value


class MaskedStream:
    """A HIP stream restricted to a set of CUs (cwt_stream_create_masked), usable as a torch
    stream through ``.torch`` (torch.cuda.ExternalStream).  Destroyed with the object."""

    def __init__(self, cus, device: int | None = None):
        import ctypes
        import torch
        self.device = torch.cuda.current_device() if device is None else device
        ncu = cu_count(self.device)
        words = (ncu + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        self.cus = sorted(set(int(c) for c in cus))
        if not self.cus or self.cus[0] < 0 or self.cus[-1] >= ncu:
            raise ValueError(f"CU ids must lie in [0, {ncu})")
        for c in self.cus:
            mask[c // 32] |= 1 << (c % 32)
        ptr = ctypes.c_void_p()
        check(lib().cwt_stream_create_masked(ctx(self.device), mask, words, ctypes.byref(ptr)),
              "cwt_stream_create_masked")
        self.ptr = ptr.value
        self.torch = torch.cuda.ExternalStream(self.ptr, device=torch.device("cuda", self.device))

    def __del__(self):
        p = getattr(self, "ptr", None)
        if p:
            try:
                lib().cwt_stream_destroy(p)
            except Exception:
                pass
            self.ptr = None
