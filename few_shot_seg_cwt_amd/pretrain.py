"""Stage-1 pretraining of the PSPNet on HIP (reference src/pretrain.py).

The reference trains the whole PSPNet on the base classes before the CWT stage: per iteration
``model.train()``, ``loss = compute_loss(args, model, images, gt, num_classes_tr)`` (label-
smoothed CE of the upsampled logits, pretrain.py:163-219), ``optimizer.zero_grad()``,
``loss.backward()``, ``optimizer.step()`` (SGD with momentum / weight decay / nesterov over two
parameter groups: layer0-4 at ``lr``, ppm / bottleneck / classifier at ``lr * scale_lr``,
pretrain.py:60-72), and the cosine schedule per iteration (pretrain.py:118-119).

Here :class:`PretrainPSPNet` holds the model on the device (libcwt ``cwt_pretrain``) and
:meth:`PretrainPSPNet.train_step` is that whole iteration as one call: forward with training-mode
BN, loss, backward of every conv / BN / PPM / classifier parameter and both SGD groups, in exact
fp32 (f32 MFMA).  No torch op computes anything on this path; it raises without the library or a
GPU.
"""
from __future__ import annotations

import ctypes as C
import math
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .synthetic import BN_EPS, pspnet_param_specs


class PretrainHparams(C.Structure):
    """cwt_pretrain_hparams (include/cwt.h)."""
    _fields_ = [("lr", C.c_float), ("lr_head", C.c_float), ("momentum", C.c_float), ("weight_decay", C.c_float),
                ("nesterov", C.c_int), ("smoothing", C.c_int), ("bn_momentum", C.c_float), ("drop_p", C.c_float),
                ("seed", C.c_uint64), ("ignore_index", C.c_int)]


def _arg(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default)


def cosine_lr(base_lr: float, it: int, total: int, eta_min: float = 1e-6) -> float:
    """CosineAnnealingLR(optimizer, T_max=total, eta_min=1e-6) after ``it`` scheduler steps
    (optimizer.py:33; stepped every iteration, pretrain.py:118-119), closed form."""
    return eta_min + (base_lr - eta_min) * (1.0 + math.cos(math.pi * it / total)) / 2.0


class PretrainPSPNet:
    """``get_model(args)`` + ``get_optimizer(args, params_list)`` of pretrain.py:60-72 on HIP.

    ``state_dict``: a PSPNet state dict with the reference key names (tensors or arrays);
    ``classifier.weight`` is [num_classes_tr, 512, 1, 1].  ``state_dict()`` reads the trained
    model back in the same names and layouts.
    """

    def __init__(self, args, state_dict, device=None):
        self.layers = int(_arg(args, "layers", 50))
        self.num_classes = int(_arg(args, "num_classes_tr", 16))
        self.args = args
        if device is None:
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        names, arrs = self._index_state(state_dict)
        self._keep = arrs
        cn = (C.c_char_p * len(names))(*[n.encode() for n in names])
        cd = (C.c_void_p * len(names))(*[a.ctypes.data for a in arrs])
        ce = (C.c_int64 * len(names))(*[a.size for a in arrs])
        h = C.c_void_p()
        _lib.check(_lib.lib().cwt_pretrain_create(_lib.ctx(self.device.index), self.layers, self.num_classes,
                                                  len(names), cn, cd, ce, BN_EPS, C.byref(h)),
                   "cwt_pretrain_create")
        self._h = h
        self._keep = None
        self.loss = torch.zeros(1, device=self.device)
        self.iteration = 0
        self.training = True

    def _index_state(self, state_dict):
        """Host bookkeeping over a reference PSPNet state dict; returns the device tensors'
        (names, float32 arrays)."""
        self._shapes = {}
        # the full reference key sequence (pspnet.py:70-141 state_dict order): ``gamma`` is a
        # PSPNet parameter outside every optimizer group (pretrain.py:68-76), carried unchanged;
        # ``*.num_batches_tracked`` counts the training-mode forwards as nn.BatchNorm2d does
        self._order = []
        self._gamma = torch.tensor(0.2)
        self._nbt0 = {}
        self._train_forwards = 0
        names, arrs = [], []
        for k, v in state_dict.items():
            self._order.append(k)
            if k == "gamma":
                self._gamma = torch.as_tensor(np.asarray(v.detach().cpu() if isinstance(v, torch.Tensor) else v,
                                                         dtype=np.float32)).clone()
                continue
            if k.endswith("num_batches_tracked"):
                self._nbt0[k] = int(np.asarray(v.detach().cpu() if isinstance(v, torch.Tensor) else v))
                continue
            a = np.ascontiguousarray(v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v),
                                     dtype=np.float32)
            names.append(k)
            arrs.append(a)
            self._shapes[k] = a.shape
        return names, arrs

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                _lib.lib().cwt_pretrain_destroy(h)
            except Exception:
                pass
            self._h = None

    def train(self, mode: bool = True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    def hparams(self, lr: float | None = None, seed: int = 0, lr_head: float | None = None) -> PretrainHparams:
        """``lr`` is the backbone groups' current lr (layer0-4), ``lr_head`` the head groups'
        (ppm, bottleneck, classifier; default ``lr * scale_lr``, their base ratio).  Under the
        cosine schedule each group anneals from its OWN base lr to eta_min (optimizer.py:32), so
        :func:`train_epoch` passes both."""
        a = self.args
        lr = float(_arg(a, "lr", 0.0025)) if lr is None else float(lr)
        hp = PretrainHparams()
        hp.lr = lr
        hp.lr_head = lr * float(_arg(a, "scale_lr", 1.0)) if lr_head is None else float(lr_head)
        self._group_lr = (hp.lr, hp.lr_head)
        hp.momentum = float(_arg(a, "momentum", 0.9))
        hp.weight_decay = float(_arg(a, "weight_decay", 1e-4))
        hp.nesterov = int(bool(_arg(a, "nesterov", False)))
        hp.smoothing = int(bool(_arg(a, "smoothing", True)))
        hp.bn_momentum = 0.1
        hp.drop_p = float(_arg(a, "dropout", 0.1))
        hp.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        hp.ignore_index = 255
        return hp

    def train_step(self, images: torch.Tensor, targets: torch.Tensor, lr: float | None = None, seed: int | None = None,
                   hp: PretrainHparams | None = None, lr_head: float | None = None) -> torch.Tensor:
        """One iteration of pretrain.py:104-121: images [N, 3, S, S] fp32, targets [N, S, S]
        int64 (255 ignored), both on the device.  Returns the loss (device scalar, the value
        before the step)."""
        _lib.require(images, "images")
        _lib.require(targets, "targets", torch.int64)
        if images.dim() != 4 or images.shape[1] != 3 or targets.shape != (images.shape[0], *images.shape[2:]):
            raise ValueError("images must be [N,3,S,S] and targets [N,S,S]")
        images, targets = images.contiguous(), targets.contiguous()
        if hp is None:
            hp = self.hparams(lr, self.iteration if seed is None else seed, lr_head)
        else:
            self._group_lr = (float(hp.lr), float(hp.lr_head))
        _lib.check(_lib.lib().cwt_pretrain_step(_lib.ctx(self.device.index), self._h, _lib.ptr(images),
                                                _lib.ptr(targets), images.shape[0], images.shape[2],
                                                C.addressof(hp), _lib.ptr(self.loss), _lib.stream_ptr(self.device)),
                   "cwt_pretrain_step")
        self.iteration += 1
        self._train_forwards += 1
        return self.loss[0]

    def logits(self, images: torch.Tensor) -> torch.Tensor:
        """The classifier output before PSPNet.classify's upsample (pspnet.py:183-187) under the
        current mode: [N, num_classes, h, h] in channels_last memory format."""
        _lib.require(images, "images")
        images = images.contiguous()
        N, S = images.shape[0], images.shape[2]
        h = (S - 1) // 8 + 1
        out = torch.empty(N, h, h, self.num_classes, device=self.device)
        _lib.check(_lib.lib().cwt_pretrain_forward(_lib.ctx(self.device.index), self._h, _lib.ptr(images), N, S,
                                                   int(self.training), _lib.ptr(out), _lib.stream_ptr(self.device)),
                   "cwt_pretrain_forward")
        return out.permute(0, 3, 1, 2)

    def evaluate(self, images: torch.Tensor, targets: torch.Tensor):
        """One batch of standard_validate (pretrain.py:223-250) / the logging block (:123-131)
        under the current mode: returns (loss, n_valid, intersection, union, target) as device
        tensors -- nn.CrossEntropyLoss(ignore_index=255) of the upsampled logits and
        intersectionAndUnionGPU(logits.argmax(1), gt, num_classes_tr, 255)."""
        _lib.require(images, "images")
        _lib.require(targets, "targets", torch.int64)
        images, targets = images.contiguous(), targets.contiguous()
        lo = torch.empty(2, device=self.device)
        iu = torch.empty(3, self.num_classes, device=self.device)
        _lib.check(_lib.lib().cwt_pretrain_evaluate(_lib.ctx(self.device.index), self._h, _lib.ptr(images),
                                                    _lib.ptr(targets), images.shape[0], images.shape[2],
                                                    int(self.training), _lib.ptr(lo), _lib.ptr(iu),
                                                    _lib.stream_ptr(self.device)), "cwt_pretrain_evaluate")
        return lo[0], lo[1], iu[0], iu[1], iu[2]

    def _get(self, name: str, what: int, shape) -> torch.Tensor:
        out = np.empty(shape, np.float32)
        _lib.check(_lib.lib().cwt_pretrain_get(self._h, name.encode(), what, out.ctypes.data, out.size),
                   f"cwt_pretrain_get({name})")
        return torch.from_numpy(out)

    def parameter_names(self):
        return [n for n in self._shapes if not (n.endswith("running_mean") or n.endswith("running_var"))]

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        """Host copy of the reference ``PSPNet.state_dict()``: every key in the reference order
        (``gamma`` first, pspnet.py:141), parameters, BN running statistics and
        ``num_batches_tracked`` (int64, +1 per training step), so the position-wise loader of
        test.py:61-81 pairs every key with its own tensor."""
        sd = OrderedDict()
        for n in self._order:
            if n == "gamma":
                sd[n] = self._gamma.clone()
            elif n.endswith("num_batches_tracked"):
                sd[n] = torch.tensor(self._nbt0[n] + self._train_forwards, dtype=torch.int64)
            elif n.endswith("running_mean") or n.endswith("running_var"):
                sd[n] = self._get(n, 3, self._shapes[n])
            else:
                sd[n] = self._get(n, 0, self._shapes[n])
        return sd

    def param(self, name: str) -> torch.Tensor:
        """One parameter, host copy in PyTorch layout."""
        return self._get(name, 0, self._shapes[name])

    state_dict_entry = param

    def running(self, name: str) -> torch.Tensor:
        """``<bn>.running_mean`` / ``<bn>.running_var``."""
        return self._get(name, 3, self._shapes[name])

    def grad(self, name: str) -> torch.Tensor:
        """The gradient of the last step (after zero_grad + backward, before the SGD update)."""
        return self._get(name, 1, self._shapes[name])

    def momentum_buffer(self, name: str) -> torch.Tensor:
        return self._get(name, 2, self._shapes[name])

    def _set(self, name: str, what: int, value) -> None:
        a = np.ascontiguousarray(value.detach().cpu().numpy() if isinstance(value, torch.Tensor) else value,
                                 dtype=np.float32)
        if a.size != int(np.prod(self._shapes[name])):
            raise ValueError(f"{name}: {a.shape} does not match {self._shapes[name]}")
        _lib.check(_lib.lib().cwt_pretrain_set(self._h, name.encode(), what, a.ctypes.data, a.size),
                   f"cwt_pretrain_set({name})")

    def load_state_dict(self, sd) -> None:
        """model.load_state_dict (strict over the trainable tensors and BN running statistics;
        ``gamma`` and ``num_batches_tracked`` are taken when present)."""
        for n in self._shapes:
            if n not in sd:
                raise KeyError(f"missing key {n}")
            what = 3 if (n.endswith("running_mean") or n.endswith("running_var")) else 0
            self._set(n, what, sd[n])
        if "gamma" in sd:
            self._gamma = torch.as_tensor(np.asarray(sd["gamma"], dtype=np.float32)).clone()
        for n in self._nbt0:
            if n in sd:
                self._nbt0[n] = int(np.asarray(sd[n])) - self._train_forwards

    MODULES = ("layer0", "layer1", "layer2", "layer3", "layer4", "ppm", "bottleneck", "classifier")
    HEAD_MODULES = ("ppm", "bottleneck", "classifier")

    def param_groups(self):
        """The eight groups of pretrain.py:68-76, one per module in the reference order
        (layer0-4 at ``lr``; ppm, bottleneck, classifier at ``lr * scale_lr``), each the
        module's ``parameters()`` names in registration order (``gamma`` is in none)."""
        names = self.parameter_names()
        return [[n for n in names if n.split(".", 1)[0] == m] for m in self.MODULES]

    def optimizer_state_dict(self, lr: float | None = None, lr_head: float | None = None) -> dict:
        """torch.optim.SGD.state_dict() of the reference's optimizer (pretrain.py:68-76): eight
        param_groups, state keyed by the parameter's position over all groups, momentum buffers
        in PyTorch layout.  Each group carries its current lr (the last step's, or ``lr`` /
        ``lr_head`` when given) and the scheduler's ``initial_lr`` (its base lr)."""
        a = self.args
        base = float(_arg(a, "lr", 0.0025))
        scale = float(_arg(a, "scale_lr", 1.0))
        cur_b, cur_h = getattr(self, "_group_lr", (base, base * scale))
        if lr is not None:
            cur_b = float(lr)
            cur_h = cur_b * scale if lr_head is None else float(lr_head)
        elif lr_head is not None:
            cur_h = float(lr_head)
        groups, state, idx = [], {}, 0
        for m, names in zip(self.MODULES, self.param_groups()):
            head = m in self.HEAD_MODULES
            ids = []
            for n in names:
                if self.iteration > 0:
                    state[idx] = {"momentum_buffer": self.momentum_buffer(n)}
                ids.append(idx)
                idx += 1
            groups.append({"lr": cur_h if head else cur_b,
                           "momentum": float(_arg(a, "momentum", 0.9)), "dampening": 0,
                           "weight_decay": float(_arg(a, "weight_decay", 1e-4)),
                           "nesterov": bool(_arg(a, "nesterov", False)), "maximize": False, "foreach": None,
                           "differentiable": False, "fused": None,
                           "initial_lr": base * scale if head else base, "params": ids})
        return {"state": state, "param_groups": groups}

    def load_optimizer_state_dict(self, sd: dict) -> None:
        names = sum(self.param_groups(), [])
        for i, n in enumerate(names):
            st = sd.get("state", {}).get(i)
            if st is not None and st.get("momentum_buffer") is not None:
                self._set(n, 2, st["momentum_buffer"])
                self.iteration = max(self.iteration, 1)

    def save_checkpoint(self, path: str, epoch: int, lr: float | None = None, lr_head: float | None = None) -> None:
        """torch.save({'epoch', 'state_dict', 'optimizer'}) as pretrain.py:147-152 / 157-159."""
        torch.save({"epoch": epoch, "state_dict": self.state_dict(),
                    "optimizer": self.optimizer_state_dict(lr, lr_head)}, path)

    def load_checkpoint(self, path: str) -> dict:
        ck = torch.load(path, map_location="cpu", weights_only=True)
        self.load_state_dict(ck["state_dict"])
        if "optimizer" in ck:
            self.load_optimizer_state_dict(ck["optimizer"])
        return ck

    def num_params(self):
        t, b = C.c_int64(), C.c_int64()
        _lib.check(_lib.lib().cwt_pretrain_num_params(self._h, C.byref(t), C.byref(b)), "cwt_pretrain_num_params")
        return t.value, b.value


def synthetic_pretrain_state(layers: int = 50, num_classes: int = 16, seed: int = 2021):
    """PRNG PSPNet state with a num_classes classifier (synthetic.make_pspnet_state)."""
    from .synthetic import make_pspnet_state
    return make_pspnet_state(layers=layers, seed=seed, num_classes_tr=num_classes)


def train_epoch(model: PretrainPSPNet, batches, epoch: int, iters_per_epoch: int, epochs: int, base_lr: float):
    """The inner loop of pretrain.py:104-121 over ``batches`` (an iterable of (images, gt)
    device tensors) with the per-iteration cosine schedule; returns the running loss (the
    reference's loss_meter average over the logged iterations is host-side bookkeeping)."""
    losses = []
    scale = float(_arg(model.args, "scale_lr", 1.0))
    for i, (images, gt) in enumerate(batches):
        it = epoch * iters_per_epoch + i
        total = iters_per_epoch * epochs
        # CosineAnnealingLR anneals every group from its own base lr to eta_min (optimizer.py:32)
        losses.append(model.train_step(images, gt, lr=cosine_lr(base_lr, it, total),
                                       lr_head=cosine_lr(base_lr * scale, it, total)))
        # scheduler.step() follows every optimizer.step() (pretrain.py:118-121): the optimizer's
        # state then holds the NEXT iteration's lr, which is what a checkpoint saves
        model._group_lr = (cosine_lr(base_lr, it + 1, total), cosine_lr(base_lr * scale, it + 1, total))
    return torch.stack(losses).mean() if losses else torch.zeros(())


def standard_validate(args, val_loader, model: PretrainPSPNet):
    """pretrain.py:223-250: eval mode over the loader's (images, gt) batches (device tensors);
    per-class intersections and unions summed over batches, the loss averaged per batch as the
    reference's AverageMeter does.  Returns (mIoU, mean loss) as host floats."""
    model.eval()
    inter = uni = None
    losses = []
    for images, gt in val_loader:
        loss, _, i, u, _ = model.evaluate(images, gt)
        inter = i.clone() if inter is None else inter + i
        uni = u.clone() if uni is None else uni + u
        losses.append(loss)
    model.train()
    if inter is None:
        return 0.0, 0.0
    miou = float((inter / (uni + 1e-10)).mean())
    return miou, float(torch.stack(losses).mean())
