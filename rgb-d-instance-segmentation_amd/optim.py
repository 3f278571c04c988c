"""AdamW on the HIP kernel (csrc/adamw.hip, rgbd_adamw_multi): the optimizer the reference's HF
Trainer builds (finetuning.py:98; lr 1e-5 constant, config.json:12-13), with torch.optim.AdamW's
update (decoupled weight decay, no amsgrad, no maximize).  One launch per group of up to 48
tensors; the step count lives on the device, so the step can be captured into a HIP graph
(``capturable`` is always true).  fp32 parameters and gradients on the GPU only.

bench.py's optimizer (in-backward groups and the captured step); DESIGN.md §9."""
import ctypes

import torch

from . import _lib
from ._lib import check
from .ops import _stream

_MAXT = 48


class HipAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("HipAdamW: invalid hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, capturable=True))

    def _group_state(self, group):
        """The group's parameters with gradients; their moments, and ONE step count per group
        (every parameter of a training step gets a gradient every step, as here; a parameter
        that first receives one later joins the group's count instead of starting its own)."""
        params = [p for p in group["params"] if p.grad is not None]
        shared = None
        for p in group["params"]:
            if p in self.state and "step" in self.state[p]:
                shared = self.state[p]["step"]
                break
        for p in params:
            if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous():
                raise RuntimeError("HipAdamW: contiguous float32 CUDA parameters only (no CPU fallback)")
            g = p.grad
            if g.dtype != torch.float32 or not g.is_contiguous() or g.is_sparse:
                raise RuntimeError("HipAdamW: dense contiguous float32 gradients only")
            st = self.state[p]
            if not st:
                if shared is None:
                    shared = torch.zeros((), dtype=torch.float32, device=p.device)
                st["step"] = shared
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return params, shared

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = _lib.lib()
        for group in self.param_groups:
            params, step = self._group_state(group)
            if not params:
                continue
            step.add_(1.0)  # on the device: a captured graph replays the increment
            b1, b2 = group["betas"]
            for i in range(0, len(params), _MAXT):
                run = params[i:i + _MAXT]
                n = len(run)
                P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in run])
                G = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p in run])
                M = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg"].data_ptr() for p in run])
                V = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg_sq"].data_ptr() for p in run])
                N = (ctypes.c_longlong * n)(*[p.numel() for p in run])
                check(L.rgbd_adamw_multi(n, P, G, M, V, N, ctypes.c_void_p(step.data_ptr()), float(group["lr"]),
                                         float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                                         _stream(run[0].device)), "rgbd_adamw_multi")
        return loss
