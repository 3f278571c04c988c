"""Data-parallel gradient exchange of the hot-path parameters.

The reference trains under the HF Trainer's implicit DDP: every step all-reduces (mean) the
gradients of the 37.3 M grad-receiving parameters; for the hot path those are the DSAM and
DGGM parameters (17.4 M + 5.8 k).  The ratio predictor and the Swin encoder receive no
gradient (Q1/Q2), so nothing else is exchanged; the ratio predictor's BatchNorm uses per-rank
batch statistics (no SyncBN in the reference).

Two forms:
* ``GradBucket`` — one flat float32 bucket, one blocking all-reduce after backward.
* ``OverlappedGradReducer`` — one bucket per DSAM module in the order the fused backward
  produces them (dsam2 13.3 M, dsam1 3.3 M, dsam0 + DGGM 0.8 M).  ``hot_path(...,
  grad_hook=reducer.ready)`` hands each module's gradients over the moment its weight-gradient
  kernels have been enqueued; the bucket is filled by one cat kernel and its all-reduce
  (RCCL over xGMI with backend "nccl") is issued asynchronously, so the 53 MB dsam2 exchange runs
  under the dX / dW kernels of dsam1 and dsam0.  ``finish()`` waits, divides by the world size
  and copies the means into ``p.grad`` with one foreach kernel.  Every rank issues the same
  collectives in the same order (the cascade order is fixed), which DDP requires.
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


def hot_path_grad_groups(dsam_modules, dggm_module):
    """Parameter groups in the order the fused backward (hot_path.HotPathFunction) emits them:
    dsam2, dsam1, then dsam0 together with the DGGM layers."""
    def dsam_params(m):
        ps = []
        for i in range(4):
            ps += [m.conv_layers[i].weight, m.conv_layers[i].bias]
        return ps + [m.rgb_projection.weight]
    dggm = []
    for i in range(4):
        conv = dggm_module.depth_enhancement_layers[i][0]
        dggm += [conv.weight, conv.bias]
    return [dsam_params(dsam_modules[2]), dsam_params(dsam_modules[1]), dsam_params(dsam_modules[0]) + dggm]


class OverlappedGradReducer:
    """Per-group asynchronous all-reduce(mean) of gradients issued during backward."""

    def __init__(self, groups, group=None):
        self.groups = [list(g) for g in groups]
        self.pg = group
        dev = self.groups[0][0].device
        self.flats = [torch.empty(sum(p.numel() for p in g), dtype=torch.float32, device=dev) for g in self.groups]
        self.works = [None] * len(self.groups)

    def ready(self, idx, grads):
        """Gradients of group ``idx`` (same order as its parameters; None counts as zero)."""
        g = self.groups[idx]
        if len(grads) != len(g):
            raise ValueError(f"group {idx}: {len(grads)} gradients for {len(g)} parameters")
        flat = self.flats[idx]
        parts = [(t if t is not None else torch.zeros_like(p)).reshape(-1).float() for t, p in zip(grads, g)]
        torch.cat(parts, out=flat)
        self.works[idx] = dist.all_reduce(flat, group=self.pg, async_op=True)

    def finish(self):
        """Wait for every bucket and write the mean gradients into ``p.grad``."""
        world = dist.get_world_size(self.pg)
        for idx, g in enumerate(self.groups):
            work = self.works[idx]
            if work is None:
                raise RuntimeError(f"gradient group {idx} was never handed to the reducer")
            work.wait()
            self.works[idx] = None
            flat = self.flats[idx]
            flat.div_(world)
            views, dsts = [], []
            off = 0
            for p in g:
                k = p.numel()
                v = flat[off:off + k].view_as(p)
                off += k
                if p.grad is None:
                    p.grad = v.clone()
                else:
                    views.append(v)
                    dsts.append(p.grad)
            if dsts:
                torch._foreach_copy_(dsts, views)
