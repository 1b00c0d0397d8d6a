"""Drop-in for the reference's frozen feature extractor (src/model/pspnet.py).

``get_model(args)`` returns a :class:`PSPNet` whose ``extract_features(x)`` has the
reference signature (pspnet.py:172-181): ``x`` [N,3,S,S] fp32 -> ``(f [N,512,h,w], [])``.
The whole extractor (stem, 16/33 dilated bottlenecks, PPM, 3x3 bottleneck conv) runs as
HIP kernels in libcwt.so; ``f`` is returned as an [N,512,h,w] tensor in channels_last
memory format (NHWC), which is what every downstream kernel reads.

Weights are loaded with ``load_state_dict`` using the reference key names (the
reference's ``PSPNet.state_dict()``, `gamma` first, pspnet.py:141).  The backbone weights
are frozen in every CWT driver (train.py:77-91), but the module follows ``train()`` /
``eval()`` as the reference's does: after ``model.train()`` (train.py:184, the start of every
epoch) ``extract_features`` runs every BatchNorm on batch statistics, moves the running
statistics by momentum 0.1 (on the device; later eval extractions use them) and applies the
bottleneck's Dropout2d(p=args.dropout) -- cwt_extract_features_train_bn.  ``bn_train_mode:
False`` in args keeps eval semantics under ``train()`` (the golden fixture without the quirk).
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .util import dropout_seed
from .synthetic import BN_EPS, feature_side, pspnet_param_specs


def get_model(args) -> "PSPNet":
    """pspnet.py:15 get_model(args) -> PSPNet(args, zoom_factor=8, use_ppm=True)."""
    return PSPNet(args)


def _arg(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default)


class PSPNet:
    """Frozen ResNet-50/101 + PPM extractor on MI355X (pspnet.py:70-141)."""

    def __init__(self, args, device=None):
        self.layers = int(_arg(args, "layers", 50))
        if self.layers not in (50, 101):
            raise ValueError("layers must be 50 or 101")
        if _arg(args, "arch", "resnet") != "resnet":
            raise NotImplementedError("only arch=resnet is on the CWT path (vgg is out of scope)")
        if list(_arg(args, "bins", [1, 2, 3, 6])) != [1, 2, 3, 6]:
            raise NotImplementedError("PPM bins must be [1, 2, 3, 6] (pascal.yaml:48)")
        if int(_arg(args, "bottleneck_dim", 512)) != 512:
            raise NotImplementedError("bottleneck_dim must be 512")
        if _arg(args, "m_scale", False):
            raise NotImplementedError("m_scale is not on the CWT path")
        self.bottleneck_dim = 512
        self.device = torch.device("cuda", device if device is not None else torch.cuda.current_device()) \
            if torch.cuda.is_available() else None
        self._state = None
        self._handle = None
        self.training = False
        self.bn_train_mode = bool(_arg(args, "bn_train_mode", True))
        self.dropout_p = float(_arg(args, "dropout", 0.1))   # bottleneck Dropout2d (pspnet.py:128)
        self.bn_momentum = 0.1                                 # nn.BatchNorm2d default
        self._stats_moved = False
        # conv-stack arithmetic (BASELINE config #5): "fp32" (reference numerics, default) or
        # "bf16" (bf16 MFMA convs, bf16 activations between convs, fp32 feature map out)
        self.conv_dtype = str(_arg(args, "conv_dtype", "fp32"))
        if self.conv_dtype not in self._PRECISION:
            raise ValueError(f"conv_dtype must be one of {sorted(self._PRECISION)}")
        # per-layer features for the MMN / MatchNet variants (pspnet.py:172-181): returned when
        # rmid names layers ('l34', 'mid3', ...); get_feat_list keeps each layer's last block
        # (all_lr 'l'; every block of a named layer is not built)
        self.rmid = _arg(args, "rmid", None)
        self.all_lr = str(_arg(args, "all_lr", "l"))
        self.mid_features = self.rmid is not None and ("l" in str(self.rmid) or "mid" in str(self.rmid))
        if self.mid_features and any(ch.isdigit() for ch in self.all_lr):
            raise NotImplementedError("all_lr naming layers (every bottleneck's features) is not built")

    _PRECISION = {"fp32": 0, "bf16": 1}  # CWT_CONV_FP32 / CWT_CONV_BF16 (include/cwt.h)

    def set_conv_dtype(self, dtype: str):
        """Switch the conv-stack arithmetic of the loaded extractor ("fp32" or "bf16")."""
        if dtype not in self._PRECISION:
            raise ValueError(f"conv_dtype must be one of {sorted(self._PRECISION)}")
        self.conv_dtype = dtype
        if self._handle is not None:
            _lib.check(_lib.lib().cwt_backbone_set_precision(self._handle, self._PRECISION[dtype]),
                       "cwt_backbone_set_precision")
        return self

    def _release(self):
        if getattr(self, "_handle", None) is not None and _lib._lib is not None:
            _lib.lib().cwt_backbone_destroy(self._handle)
        self._handle = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    # -- nn.Module-like surface used by the drivers --------------------------------------
    def eval(self):
        self.training = False
        return self

    def train(self, mode: bool = True):
        # train-mode BN + Dropout2d in extract_features (module docstring)
        self.training = bool(mode) and self.bn_train_mode
        return self

    def cuda(self, *a, **k):
        return self

    def parameters(self):
        return iter(())

    def state_dict(self):
        if self._state is None:
            raise RuntimeError("no weights loaded")
        if self._stats_moved:   # running statistics moved on the device by train-mode extractions
            for k in list(self._state):
                if k.endswith(".running_mean"):
                    p = k[: -len(".running_mean")]
                    C_ = self._state[k].shape[0]
                    buf = np.empty((4, C_), np.float32)
                    _lib.check(_lib.lib().cwt_backbone_read_bn(self._handle, p.encode(), buf.ctypes.data, C_),
                               "cwt_backbone_read_bn")
                    self._state[k] = buf[2].copy()
                    self._state[p + ".running_var"] = buf[3].copy()
            self._stats_moved = False
        return OrderedDict((k, torch.from_numpy(np.array(v))) for k, v in self._state.items())

    def load_state_dict(self, state_dict, strict: bool = True):
        """Accepts the reference PSPNet.state_dict() (torch tensors or numpy arrays).
        Keys may carry the DDP 'module.' prefix (train.py:67-68, convert_pth.py:9-14)."""
        sd = OrderedDict()
        for k, v in state_dict.items():
            k = k[7:] if k.startswith("module.") else k
            sd[k] = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
        specs = pspnet_param_specs(self.layers, self.bottleneck_dim)
        if strict:
            want = {n for n, _, _ in specs}
            missing = [n for n in want if n not in sd]
            if missing:
                raise KeyError(f"missing keys in state_dict: {missing[:5]}{'...' if len(missing) > 5 else ''}")
        names, ptrs, numels, keep = [], [], [], []
        for n, shape, kind in specs:
            if n not in sd or kind in ("bn_nbt", "gamma", "cls"):
                continue
            a = np.ascontiguousarray(sd[n], dtype=np.float32)
            if tuple(a.shape) != tuple(shape):
                raise ValueError(f"{n}: shape {a.shape} != {shape}")
            keep.append(a)
            names.append(n.encode())
            ptrs.append(a.ctypes.data)
            numels.append(a.size)
        lib = _lib.lib()
        arr_n = (C.c_char_p * len(names))(*names)
        arr_p = (C.c_void_p * len(ptrs))(*ptrs)
        arr_e = (C.c_int64 * len(numels))(*numels)
        handle = C.c_void_p()
        _lib.check(lib.cwt_backbone_load(_lib.ctx(self.device.index), self.layers, len(names), arr_n, arr_p, arr_e,
                                         BN_EPS, C.byref(handle)), "cwt_backbone_load")
        self._release()
        self._handle = handle
        self._state = sd
        self._stats_moved = False
        self.set_conv_dtype(self.conv_dtype)
        return self

    def feature_res(self, S: int):
        h = feature_side(S)
        return (h, h)

    # -- hot path ------------------------------------------------------------------------
    def extract_features(self, x: torch.Tensor, out: torch.Tensor | None = None):
        """pspnet.py:172-181: returns (f [N,512,h,w] channels_last, []), or with an rmid naming
        layers (f, {2: [layer2], 3: [layer3], 4: [layer4]}) (channels_last, fp32)."""
        if self._state is None:
            raise RuntimeError("load_state_dict first")
        _lib.require(x, "x")
        if x.dim() != 4 or x.shape[1] != 3 or x.shape[2] != x.shape[3]:
            raise ValueError(f"x must be [N,3,S,S], got {tuple(x.shape)}")
        N, _, S, _ = x.shape
        assert (S - 1) % 8 == 0, "pspnet.py:150: (S-1) % 8 == 0"
        h = feature_side(S)
        x = x.contiguous()
        if out is None:
            out = torch.empty((N, 512, h, h), device=x.device, dtype=torch.float32,
                              memory_format=torch.channels_last)
        if x.device != self.device:
            raise ValueError(f"x is on {x.device}, the backbone on {self.device}")
        if self.training and self.mid_features:
            raise NotImplementedError("per-layer features (rmid) are built for the eval-mode extractor only")
        if self.training:
            seed = dropout_seed()   # Dropout2d masks; the host RNG stream stays the reference's
            _lib.check(_lib.lib().cwt_extract_features_train_bn(
                _lib.ctx(x.device.index), self._handle, _lib.ptr(x), N, S, _lib.ptr(out), self.bn_momentum,
                self.dropout_p, seed, _lib.stream_ptr(x.device)), "cwt_extract_features_train_bn")
            self._stats_moved = True
            return out, []
        if self.mid_features:
            mids = {lid: torch.empty((N, c, h, h), device=x.device, dtype=torch.float32,
                                     memory_format=torch.channels_last) for lid, c in ((2, 512), (3, 1024), (4, 2048))}
            _lib.check(_lib.lib().cwt_extract_features_mid(
                _lib.ctx(x.device.index), self._handle, _lib.ptr(x), N, S, _lib.ptr(out), _lib.ptr(mids[2]),
                _lib.ptr(mids[3]), _lib.ptr(mids[4]), _lib.stream_ptr(x.device)), "cwt_extract_features_mid")
            return out, {lid: [t] for lid, t in mids.items()}
        _lib.check(_lib.lib().cwt_extract_features(_lib.ctx(x.device.index), self._handle, _lib.ptr(x), N, S,
                                                   _lib.ptr(out),
                                                   _lib.stream_ptr(x.device)), "cwt_extract_features")
        return out, []

    __call__ = extract_features
