"""AdamW on the HIP kernel (csrc/adamw.hip, rgbd_adamw_multi), with torch.optim.AdamW's update
(decoupled weight decay, no amsgrad, no maximize).  One launch per group of up to 48 tensors;
the step count lives on the device, so the step can be captured into a HIP graph
(``capturable`` is always true).  fp32 parameters and gradients on the GPU only.

The constructor defaults are torch's (weight_decay 1e-2).  The optimizer the reference's HF
Trainer builds (finetuning.py:98) is ``HipAdamW(params, **HF_TRAINER_ADAMW)``: lr 1e-5 constant
(mask2former/config.json:12-13) and TrainingArguments' defaults for the rest — weight_decay
0.0 (config.json does not set it), betas (0.9, 0.999), eps 1e-8.

A parameter that a HIP layer casts to bfloat16 (dense.cast_weight, under autocast) gets its bf16
copy rewritten by the same launch (rgbd_adamw_multi_shadow) and re-keyed, so the next forward
takes it without one cast launch per weight.

bench.py's optimizer (in-backward groups and the captured step); DESIGN.md §9."""
import ctypes

import torch

from . import _lib
from ._lib import check
from .ops import _stream

_MAXT = 48
# HF TrainingArguments' AdamW (adam_beta1/2, adam_epsilon, weight_decay defaults) at the
# reference's learning rate (mask2former/config.json:12)
HF_TRAINER_ADAMW = dict(lr=1e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0)


def _shadow(p):
    """The bfloat16 copy of ``p`` that dense.cast_weight holds (the bf16 GEMM operand of a HIP
    layer under autocast), re-used as the buffer the step writes the updated copy into; None when
    the parameter has none."""
    hit = getattr(p, "_rgbd_cast", None)
    if hit is None or hit[0][3] != torch.bfloat16:
        return None
    x = hit[1]
    if x.dtype != torch.bfloat16 or x.shape != p.shape or not x.is_contiguous() or x.device != p.device:
        return None
    return x


class HipAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("HipAdamW: invalid hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, capturable=True))

    def _group_state(self, group):
        """The group's parameters with gradients, their moments, and ONE step count per group
        (one device tensor, so a captured graph advances every parameter's step with one kernel).
        That is torch's per-parameter count only while every parameter of the group is stepped
        every time; a parameter that would join a group whose count already runs (its first
        gradient arriving after other parameters' first step) would inherit the group's count
        and a wrong bias correction, so it is refused."""
        params = [p for p in group["params"] if p.grad is not None]
        shared = None
        for p in group["params"]:
            if p in self.state and "step" in self.state[p]:
                shared = self.state[p]["step"]
                break
        if shared is not None and any(not self.state[p] for p in params):
            raise RuntimeError("HipAdamW: a parameter received its first gradient after the rest of its group "
                               "had stepped; its step count would not be its own (put it in its own group)")
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
            shadows = [_shadow(p) for p in params]
            for i in range(0, len(params), _MAXT):
                run = params[i:i + _MAXT]
                n = len(run)
                P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in run])
                G = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p in run])
                M = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg"].data_ptr() for p in run])
                V = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg_sq"].data_ptr() for p in run])
                N = (ctypes.c_longlong * n)(*[p.numel() for p in run])
                sh = shadows[i:i + _MAXT]
                args = (float(group["lr"]), float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                        _stream(run[0].device))
                if any(x is not None for x in sh):
                    S = (ctypes.c_void_p * n)(*[None if x is None else x.data_ptr() for x in sh])
                    check(L.rgbd_adamw_multi_shadow(n, P, G, M, V, S, N, ctypes.c_void_p(step.data_ptr()), *args),
                          "rgbd_adamw_multi_shadow")
                else:
                    check(L.rgbd_adamw_multi(n, P, G, M, V, N, ctypes.c_void_p(step.data_ptr()), *args),
                          "rgbd_adamw_multi")
            # the kernel wrote through raw pointers: bump the version counters (host only, safe
            # under capture) so autograd's saved-tensor checks and version-keyed caches see it
            torch.autograd.graph.increment_version(params)
            for p, x in zip(params, shadows):
                if x is not None:  # the bf16 copy the kernel wrote is current: dense.cast_weight's key
                    # after this step (the global post-step hook advances the epoch by one)
                    p._rgbd_cast = ((p.data_ptr(), p._version, getattr(p, "_rgbd_epoch", 0) + 1, torch.bfloat16), x)
        return loss

    def load_state_dict(self, state_dict):
        """torch's load, then the one-step-count-per-group invariant restored: torch moves each
        parameter's ``step`` separately, which would untie them (after which only the first
        parameter's count would advance).  Every parameter of a group gets the group's first
        stored count as its (shared) step tensor; the counts of a group must agree."""
        super().load_state_dict(state_dict)
        for group in self.param_groups:
            steps = [self.state[p]["step"] for p in group["params"] if p in self.state and "step" in self.state[p]]
            if not steps:
                continue
            vals = {float(s) for s in steps}
            if len(vals) != 1:
                raise ValueError(f"HipAdamW.load_state_dict: parameters of one group at different steps {sorted(vals)}")
            dev = group["params"][0].device
            shared = steps[0].detach().to(device=dev, dtype=torch.float32).clone()
            for p in group["params"]:
                if p in self.state and "step" in self.state[p]:
                    self.state[p]["step"] = shared
