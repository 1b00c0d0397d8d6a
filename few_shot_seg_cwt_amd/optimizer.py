"""Outer-loop optimiser (reference src/optimizer.py:8-17 get_optimizer) on the device.

``HipSGD`` mirrors ``torch.optim.SGD(params, lr, momentum, weight_decay, nesterov)`` for the
CWT's single flat parameter buffer: one cwt_sgd_step kernel per step.
"""
from __future__ import annotations

import torch

from . import _lib


class HipSGD:
    def __init__(self, params, lr: float, momentum: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False):
        self.params = [p for p in params]
        self.lr, self.momentum, self.weight_decay, self.nesterov = lr, momentum, weight_decay, nesterov
        self.bufs = [None for _ in self.params]

    def zero_grad(self, set_to_none: bool = False):
        for p in self.params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    @torch.no_grad()
    def step(self):
        for i, p in enumerate(self.params):
            if p.grad is None:
                continue
            first = self.bufs[i] is None
            if self.momentum != 0.0 and first:
                self.bufs[i] = torch.empty_like(p)
            buf = self.bufs[i]
            _lib.check(_lib.lib().cwt_sgd_step(_lib.ctx(p.device.index), _lib.ptr(p.data), _lib.ptr(p.grad),
                                               _lib.ptr(buf), p.numel(), self.lr, self.momentum, self.weight_decay,
                                               int(self.nesterov), int(first), _lib.stream_ptr(p.device)),
                       "cwt_sgd_step")
            torch.autograd.graph.increment_version(p)   # the kernel wrote p: caches keyed on its version

    def state_dict(self):
        return {"state": {i: {"momentum_buffer": b} for i, b in enumerate(self.bufs) if b is not None},
                "param_groups": [{"lr": self.lr, "momentum": self.momentum, "weight_decay": self.weight_decay,
                                  "nesterov": self.nesterov, "dampening": 0, "params": list(range(len(self.params)))}]}


def get_optimizer(args, parameters) -> HipSGD:
    """optimizer.py:8-17 (SGD branch); parameters as in the reference: a list of
    {'params': ..., 'lr': ...} groups or an iterable of tensors."""
    groups = list(parameters)
    if groups and isinstance(groups[0], dict):
        if len(groups) != 1:
            raise NotImplementedError("one parameter group (the CWT)")
        params, lr = list(groups[0]["params"]), groups[0]["lr"]
    else:
        params, lr = groups, getattr(args, "trans_lr", 0.001) if not isinstance(args, dict) else args["trans_lr"]
    main_optim = args["main_optim"] if isinstance(args, dict) else getattr(args, "main_optim", "SGD")
    if main_optim != "SGD":
        raise NotImplementedError("only main_optim=SGD is on the CWT path (train.sh)")
    g = (lambda k: args[k]) if isinstance(args, dict) else (lambda k: getattr(args, k))
    return HipSGD(params, lr=lr, momentum=g("momentum"), weight_decay=g("weight_decay"), nesterov=g("nesterov"))
