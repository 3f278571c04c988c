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
        self.prev = [None] * len(self.groups)

    def ready(self, idx, grads):
        """Gradients of group ``idx`` (same order as its parameters; None counts as zero).

        Called from inside the backward, before autograd accumulates ``grads`` into ``p.grad``.
        A ``p.grad`` that already holds a value (gradient accumulation over several backwards)
        is snapshotted here, so ``finish()`` leaves ``previous + mean(this backward)`` in it, as
        DDP's reducer does; with ``p.grad`` None (``zero_grad(set_to_none=True)``) no copy is
        made.  Do not also wrap these parameters in torch DDP: they would be reduced twice."""
        g = self.groups[idx]
        if len(grads) != len(g):
            raise ValueError(f"group {idx}: {len(grads)} gradients for {len(g)} parameters")
        self.prev[idx] = [None if p.grad is None else p.grad.detach().clone() for p in g]
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
            for p, prev in zip(g, self.prev[idx]):
                k = p.numel()
                v = flat[off:off + k].view_as(p)
                off += k
                if prev is not None:
                    v = v + prev
                if p.grad is None:
                    p.grad = v.clone()
                else:
                    views.append(v)
                    dsts.append(p.grad)
            self.prev[idx] = None
            if dsts:
                torch._foreach_copy_(dsts, views)


    def take(self, idx):
        """For an optimizer step inside the backward: make the current stream wait for group
        ``idx``'s all-reduce and return its mean gradients (views of the bucket, valid until the
        group's next ``ready``).  Needs ``p.grad`` None before the backward (no accumulation)."""
        if any(p is not None for p in self.prev[idx]):
            raise RuntimeError("in-backward optimizer steps do not accumulate gradients: zero_grad(set_to_none=True)")
        work = self.works[idx]
        work.wait()
        self.works[idx] = None
        self.prev[idx] = None
        flat = self.flats[idx]
        flat.div_(dist.get_world_size(self.pg))
        out, off = [], 0
        for p in self.groups[idx]:
            out.append(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        return out


class SerialGradReducer:
    """The same exchange as ``OverlappedGradReducer`` in a form a HIP graph can hold: after the
    backward (every side stream joined), on the current stream, one flat float32 bucket per group
    (cascade order), its all-reduce (RCCL: captured as a kernel node on the process group's stream,
    joined back before the next kernel), the division by the world size and the copy of the means
    into ``p.grad``.  Nothing of the backward runs beside a collective, so the captured step keeps
    the hot path's two concurrent branches (graph_guard); the price is the exchange's exposed
    time.  Unlike ``GradBucket`` it also issues the collective at world size 1 (the RCCL path on a
    one-GPU box).  Every parameter must have received a gradient (the hot path's all do)."""

    def __init__(self, groups, group=None):
        self.groups = [list(g) for g in groups]
        self.pg = group
        dev = self.groups[0][0].device
        self.flats = [torch.empty(sum(p.numel() for p in g), dtype=torch.float32, device=dev) for g in self.groups]

    def finish(self):
        world = dist.get_world_size(self.pg)
        for g, flat in zip(self.groups, self.flats):
            if any(p.grad is None for p in g):
                raise RuntimeError("SerialGradReducer: a parameter received no gradient")
            torch.cat([p.grad.reshape(-1).float() for p in g], out=flat)
            dist.all_reduce(flat, group=self.pg)
            flat.div_(world)
            views, off = [], 0
            for p in g:
                views.append(flat[off:off + p.numel()].view_as(p))
                off += p.numel()
            torch._foreach_copy_([p.grad for p in g], views)


class InBackwardOptimizer:
    """Optimizer steps of the hot-path parameter groups issued from inside the backward, through
    ``hot_path(..., grad_hook=opt.hook)``.  ``steps`` partitions the groups (in the order the
    backward hands them over): one optimizer per part, stepped on the stream of the part's last
    group the moment that group's gradients are enqueued.  The default [[0], [1, 2]] steps the
    dsam2 parameters (13.3 M of the 17.4 M) under the dsam1 / dsam0 backward and the rest in one
    launch at the end (small groups alone make latency-bound optimizer launches).  AdamW updates
    every parameter from its own gradient and state only, so parameters and optimizer state are
    bitwise those of one ``optimizer.step()`` after the backward (this step has no gradient
    clipping; a global-norm clip would need every gradient first).  With a reducer (data
    parallel) a part's step first waits, on its stream, for its groups' all-reduces and uses the
    means: DDP + step.  After the backward ``p.grad`` holds this rank's local gradients
    (autograd's assignment, no kernel); clear them with ``zero_grad(set_to_none=True)``."""

    def __init__(self, groups, make_opt, reducer=None, steps=((0,), (1, 2))):
        self.groups = [list(g) for g in groups]
        self.steps = [tuple(s) for s in steps]
        if sorted(i for s in self.steps for i in s) != list(range(len(self.groups))):
            raise ValueError(f"steps {steps} must partition groups 0..{len(self.groups) - 1}")
        self.opts = [make_opt([p for i in s for p in self.groups[i]]) for s in self.steps]
        self.reducer = reducer
        self.held = {}

    def hook(self, idx, grads):
        g = self.groups[idx]
        if len(grads) != len(g):
            raise ValueError(f"group {idx}: {len(grads)} gradients for {len(g)} parameters")
        if self.reducer is not None:
            self.reducer.ready(idx, grads)
        self.held[idx] = grads
        for k, s in enumerate(self.steps):
            if s[-1] != idx:
                continue
            ps = []
            for i in s:
                gi = self.reducer.take(i) if self.reducer is not None else self.held[i]
                for p, t in zip(self.groups[i], gi):
                    p.grad = t
                ps += self.groups[i]
                del self.held[i]
            self.opts[k].step()
            for p in ps:  # autograd then hands p.grad this backward's tensors (assignment, no add)
                p.grad = None

    def zero_grad(self, set_to_none=True):
        for o in self.opts:
            o.zero_grad(set_to_none=set_to_none)


class BufferBroadcaster:
    """DDP's ``broadcast_buffers=True`` for the modules outside torch DDP: at the start of every
    forward, rank 0's buffers overwrite every other rank's (torch DDP ``_sync_buffers`` before
    each forward).  Under the reference's Trainer that applies to the ratio predictor's BatchNorm
    running statistics (SURVEY §2 "(2) DDP broadcast of buffers"): each rank updates them from
    its own batch statistics (no SyncBN), and the next forward starts from rank 0's.  Buffers
    are flattened per dtype (float32 statistics, int64 counters), so a step costs one broadcast
    per dtype."""

    def __init__(self, modules, group=None):
        self.pg = group
        bufs = [b for m in modules for b in m.buffers()]
        self.by_dtype = {}
        for b in bufs:
            self.by_dtype.setdefault(b.dtype, []).append(b)
        self.flats = {dt: torch.empty(sum(b.numel() for b in bs), dtype=dt, device=bs[0].device)
                      for dt, bs in self.by_dtype.items()}

    def sync(self, src=0):
        if dist.get_world_size(self.pg) == 1:
            return
        for dt, bs in self.by_dtype.items():
            flat = self.flats[dt]
            torch.cat([b.reshape(-1) for b in bs], out=flat)
            dist.broadcast(flat, src=src, group=self.pg)
            views, off = [], 0
            for b in bs:
                views.append(flat[off:off + b.numel()].view_as(b))
                off += b.numel()
            torch._foreach_copy_(bs, views)


def broadcast_parameters(modules, group=None, src=0):
    """DDP's construction-time broadcast of rank 0's parameters and buffers."""
    if dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for m in modules:
            for t in list(m.parameters()) + list(m.buffers()):
                dist.broadcast(t.data, src=src, group=group)
