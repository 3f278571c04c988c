"""One hot-path training step — forward, backward, optimizer — captured into a HIP graph.

The bf16 step at 640x480, B=8 issues about 80 kernels (K1 -> K4 train mode -> K3 -> K5 x3 -> K2,
the backward cascade, AdamW) from Python through ctypes and the autograd engine.  Where the host
falls behind the device (the step's first kernels, the hand-off from backward to the optimizer,
the small plan kernels between the DSAM GEMMs) the GPU idles; replaying the captured step costs
one graph launch.  Everything in the step is capture-safe by construction:
  * no host synchronisation (the ratio stays on the device, Q2; the decomposition status can be
    checked through ops.DeferredStatus outside the graph),
  * every kernel runs on the current stream, with workspaces kept per stream (ops._workspace),
  * the bf16 DSAM filters are re-packed on the device from the optimizer's updated weights
    inside the step, and only for the region codes present (a device bit mask),
  * the ratio predictor's dropout advances a device counter, so replays draw fresh masks,
  * the optimizer must be capturable (torch.optim.AdamW(..., capturable=True)).
Gradients are written, not accumulated: the graph is captured with every .grad None, so each
replay's backward produces fresh gradients in the graph's memory pool, as
``zero_grad(set_to_none=True)`` + backward does eagerly.

Single process only: with data parallelism the step's gradient all-reduce runs through
``OverlappedGradReducer``'s asynchronous RCCL calls, which stay eager.
"""
import torch

from .graph_guard import check_and_instantiate


class CapturedTrainStep:
    """``fb()`` runs forward + backward and leaves the gradients in ``p.grad``; ``opt`` is the
    optimizer stepping those parameters.  ``warmup`` eager steps (on the capture stream; they
    update the parameters like any training step) size the workspaces and pack caches, then
    the step is captured.  Calling the object replays it and returns ``fb``'s outputs, static
    tensors overwritten by the next replay."""

    def __init__(self, fb, opt, warmup=2, opts=None, clear=None):
        """``opt`` None: ``fb`` steps the optimizers itself (distributed.InBackwardOptimizer),
        ``opts`` lists them (checked for capturable) and ``clear()`` clears the gradients."""
        opts = [opt] if opt is not None else list(opts or ())
        if not opts:
            raise ValueError("CapturedTrainStep needs the optimizer(s) the step uses")
        for o in opts:
            for g in o.param_groups:
                if not g.get("capturable", False):
                    raise ValueError("CapturedTrainStep needs a capturable optimizer (capturable=True)")
        self.fb, self.opt = fb, opt
        # every parameter the step's optimizers own: a replay updates them on the device without
        # the host-side post-step hook, so __call__ advances their step epoch itself (the casts
        # cached under dense.cast_weight's key would otherwise go stale between replays)
        self.params = [p for o in opts for g in o.param_groups for p in g["params"]]
        clear = clear or (lambda: [o.zero_grad(set_to_none=True) for o in opts])
        self.stream = torch.cuda.Stream()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            for _ in range(max(warmup, 1)):
                self.fb()
                if opt is not None:
                    self.opt.step()
                clear()
        torch.cuda.current_stream().wait_stream(self.stream)
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(self.graph, stream=self.stream):
            self.outs = self.fb()
            if opt is not None:
                self.opt.step()
        # at most two concurrent branches, or the bundled runtime's first launch crashes (§5.1)
        self.width = check_and_instantiate(self.graph, "CapturedTrainStep")

    def __call__(self):
        self.graph.replay()
        for p in self.params:
            p._rgbd_epoch = getattr(p, "_rgbd_epoch", 0) + 1
        return self.outs
