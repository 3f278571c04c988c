"""Data-parallel gradient exchange of the hot-path parameters.

The reference trains under the HF Trainer's implicit DDP: every step all-reduces (mean) the
gradients of the 37.3 M grad-receiving parameters; for the hot path those are the DSAM and
DGGM parameters (17.4 M + 5.8 k).  The ratio predictor and the Swin encoder receive no
gradient (Q1/Q2), so nothing else is exchanged; the ratio predictor's BatchNorm uses per-rank
batch statistics (no SyncBN in the reference).  One flat float32 bucket per call: a single
RCCL ring all-reduce over xGMI (backend "nccl") or gloo on the CPU for tests.
"""
import torch
import torch.distributed as dist


class GradBucket:
    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(n, dtype=torch.float32, device=self.params[0].device)

    def allreduce_mean(self, group=None):
        world = dist.get_world_size(group)
        if world == 1:
            return
        off = 0
        for p in self.params:
            k = p.numel()
            if p.grad is None:
                self.flat[off:off + k].zero_()
            else:
                self.flat[off:off + k].copy_(p.grad.reshape(-1))
            off += k
        dist.all_reduce(self.flat, group=group)
        self.flat.div_(world)
        off = 0
        for p in self.params:
            k = p.numel()
            g = self.flat[off:off + k].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            off += k
