"""Checkpoint compatibility with the reference's files.

* CWT checkpoints: ``{'epoch', 'state_dict', 'optimizer'}`` written by train.py:147-152 /
  158-163 under ``get_model_dir_trans(args)`` (util.py:167-179) as ``best.pth`` / ``final.pth``
  and read back by test.py:83-89 (``checkpoint['state_dict']`` only).  ``state_dict`` holds
  the MultiHeadAttentionOne keys (w_qkvs.weight, layer_norm.{weight,bias}, fc.{weight,bias});
  ``optimizer`` is torch.optim.SGD's layout with one momentum buffer per parameter -- the flat
  device buffer of :class:`~few_shot_seg_cwt_amd.transformer.MultiHeadAttentionOne` and
  :class:`~few_shot_seg_cwt_amd.optimizer.HipSGD` is split into those views on save and
  concatenated on load, so either side reads the other's files.
* Backbone weights: by name with the DDP ``module.`` prefix, skipping ``classifier`` and
  ``gamma`` (train.py:57-75), or by position, skipping ``classifier`` (test.py:61-81); shape
  mismatches are reported and skipped as the reference does.

Files are read with ``torch.load(..., weights_only=True)``: tensors, dicts, lists and
numbers only, nothing executed from the file.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch

_SGD_GROUP_DEFAULTS = dict(dampening=0, maximize=False, foreach=None, differentiable=False, fused=None)


def _g(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default)


def get_model_dir(args) -> str:
    """util.py:150-164: <model_dir>/<train_name>/split=<s>/model/shot_<k>/pspnet_<arch><layers>."""
    return os.path.join(_g(args, "model_dir"), _g(args, "train_name"), f"split={_g(args, 'train_split')}", "model",
                        f"shot_{_g(args, 'shot')}", f"pspnet_{_g(args, 'arch')}{_g(args, 'layers')}")


def get_model_dir_trans(args) -> str:
    """util.py:167-179: <model_dir>/<train_name>/split=<s>/model/shot_<k>/transformer_<arch><layers>."""
    return os.path.join(_g(args, "model_dir"), _g(args, "train_name"), f"split={_g(args, 'train_split')}", "model",
                        f"shot_{_g(args, 'shot')}", f"transformer_{_g(args, 'arch')}{_g(args, 'layers')}")


# ---------------------------------------------------------------------------------------------
# optimizer state in torch.optim.SGD's per-parameter layout
# ---------------------------------------------------------------------------------------------

def optimizer_state_dict(optimizer, transformer) -> dict:
    """HipSGD state over the transformer's flat buffer -> torch.optim.SGD.state_dict() layout
    over the reference's parameters (transformer.parameters() order: w_qkvs.weight,
    layer_norm.weight, layer_norm.bias, fc.weight, fc.bias)."""
    layout = transformer._layout   # (name, shape, offset, numel) in parameter order
    sd = optimizer.state_dict()
    flat_buf = sd["state"].get(0, {}).get("momentum_buffer")
    state = {}
    if flat_buf is not None:
        fb = flat_buf.detach().reshape(-1).cpu()
        for i, (n, shp, off, k) in enumerate(layout):
            state[i] = {"momentum_buffer": fb[off:off + k].view(shp).clone()}
    group = dict(sd["param_groups"][0])
    group.update({k: group.get(k, d) for k, d in _SGD_GROUP_DEFAULTS.items()})
    group["params"] = list(range(len(layout)))
    return {"state": state, "param_groups": [group]}


def load_optimizer_state_dict(optimizer, transformer, sd: dict):
    """Inverse of :func:`optimizer_state_dict`; also accepts HipSGD's own flat layout."""
    views = transformer.named_views()
    group = sd["param_groups"][0]
    optimizer.lr = float(group["lr"])
    optimizer.momentum = float(group["momentum"])
    optimizer.weight_decay = float(group["weight_decay"])
    optimizer.nesterov = bool(group["nesterov"])
    st = sd.get("state", {})
    if not st:
        optimizer.bufs = [None]
        return optimizer
    flat = transformer.flat
    if len(st) == 1 and st[0]["momentum_buffer"].numel() == flat.numel():
        buf = st[0]["momentum_buffer"].reshape(-1)
    else:
        if sorted(st) != list(range(len(views))):
            raise ValueError(f"optimizer state has {len(st)} entries, the CWT has {len(views)} parameters")
        parts = []
        for i, (n, v) in enumerate(views):
            b = st[i]["momentum_buffer"]
            if tuple(b.shape) != tuple(v.shape):
                raise ValueError(f"momentum buffer {i} ({n}): {tuple(b.shape)} != {tuple(v.shape)}")
            parts.append(b.reshape(-1))
        buf = torch.cat(parts)
    optimizer.bufs = [buf.to(flat.device, torch.float32).clone()]
    return optimizer


# ---------------------------------------------------------------------------------------------
# CWT checkpoints
# ---------------------------------------------------------------------------------------------

def save_transformer_checkpoint(path: str, epoch: int, transformer, optimizer):
    """train.py:147-152 / 158-163 (``best.pth`` / ``final.pth``)."""
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    sd = OrderedDict((k, v.detach().cpu()) for k, v in transformer.state_dict().items())
    torch.save({"epoch": epoch, "state_dict": sd, "optimizer": optimizer_state_dict(optimizer, transformer)}, path)


def load_transformer_checkpoint(path: str, transformer, optimizer=None) -> dict:
    """test.py:83-89: ``transformer.load_state_dict(torch.load(path)['state_dict'])``; the
    optimizer state too when given (the reference never resumes it).  Returns the checkpoint."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    transformer.load_state_dict(ckpt["state_dict"])
    if optimizer is not None and "optimizer" in ckpt:
        load_optimizer_state_dict(optimizer, transformer, ckpt["optimizer"])
    return ckpt


# ---------------------------------------------------------------------------------------------
# backbone weights (frozen PSPNet)
# ---------------------------------------------------------------------------------------------

def map_backbone_by_name(model_sd: "OrderedDict[str, torch.Tensor]", pre_weight: dict, log=print) -> OrderedDict:
    """train.py:57-75: every key of the model except ``classifier``/``gamma`` takes
    ``pre_weight['module.' + key]`` when the shapes agree (a mismatch is printed and the
    model's value kept; a missing key raises KeyError, as the reference would)."""
    out = OrderedDict(model_sd)
    for key in model_sd:
        if "classifier" in key or "gamma" in key:
            continue
        src = pre_weight["module." + key]
        if tuple(model_sd[key].shape) == tuple(src.shape):
            out[key] = src
        else:
            log("Mismatched shape {}: {}, {}".format(key, tuple(src.shape), tuple(model_sd[key].shape)))
    return out


def map_backbone_by_position(model_sd: "OrderedDict[str, torch.Tensor]", pre_weight: dict, log=print) -> OrderedDict:
    """test.py:61-81: the i-th model key takes the i-th checkpoint entry (zip order), except
    keys containing ``classifier``; shape mismatches are printed and skipped."""
    out = OrderedDict(model_sd)
    for key1, key2 in zip(list(model_sd.keys()), list(pre_weight.keys())):
        if "classifier" in key1:
            continue
        if tuple(model_sd[key1].shape) == tuple(pre_weight[key2].shape):
            out[key1] = pre_weight[key2]
        else:
            log("Pre-trained {} shape and model {} shape: {}, {}".format(
                key2, key1, tuple(pre_weight[key2].shape), tuple(model_sd[key1].shape)))
    return out


def reference_model_state(model) -> OrderedDict:
    """The reference PSPNet.state_dict() key order and shapes for ``model`` (gamma first,
    classifier last; pspnet.py:70-141) -- the ``pre_dict`` the reference loaders walk.  The
    values are the model's loaded weights where it has them, zeros otherwise."""
    from .synthetic import pspnet_param_specs
    have = model._state or {}
    out = OrderedDict()
    for n, shape, kind in pspnet_param_specs(model.layers, model.bottleneck_dim):
        out[n] = torch.as_tensor(have[n]) if n in have else torch.zeros(shape, dtype=torch.int64 if kind == "bn_nbt"
                                                                          else torch.float32)
    return out


def load_backbone(model, path: str, by: str = "name", log=print):
    """Load a frozen-backbone checkpoint (``{'state_dict': ...}``) into ``model`` the way
    train.py (``by='name'``) or test.py (``by='position'``) does, then upload it."""
    pre_weight = torch.load(path, map_location="cpu", weights_only=True)["state_dict"]
    base = reference_model_state(model)
    mapped = (map_backbone_by_name if by == "name" else map_backbone_by_position)(base, pre_weight, log)
    model.load_state_dict(mapped, strict=True)
    return model
