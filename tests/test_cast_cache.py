"""dense.cast_weight's cache (rgbd_amd/dense.py): a parameter's low-precision copy is reused until
the parameter changes — through an in-place op (version counter), a new storage, or an optimizer
step that writes it without bumping the version (torch's fused AdamW; simulated here by an
optimizer that updates through ``.data``): the step epoch recorded by the global post-step hook.
Parameters no optimizer steps (the frozen Swin-T, Q1) keep their copy.  CPU only."""
import torch

from rgbd_amd.dense import cast_weight


class _SilentSGD(torch.optim.Optimizer):
    """Updates parameters without bumping their version counters, as the fused AdamW does."""

    def __init__(self, params):
        super().__init__(params, {})

    def step(self, closure=None):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    p.data.add_(p.grad, alpha=-1.0)


def test_cache_hits_and_invalidation():
    a = torch.nn.Parameter(torch.randn(8, 4))
    frozen = torch.nn.Parameter(torch.randn(8, 4))
    c1 = cast_weight(a, torch.bfloat16)
    assert cast_weight(a, torch.bfloat16) is c1          # hit
    f1 = cast_weight(frozen, torch.bfloat16)
    opt = _SilentSGD([a, frozen])
    a.grad = torch.ones_like(a)                            # frozen has no gradient: not stepped
    v = a._version
    opt.step()
    assert a._version == v                                 # the update did not bump the version
    c2 = cast_weight(a, torch.bfloat16)
    assert c2 is not c1 and torch.equal(c2, (a.detach() - 0).to(torch.bfloat16))
    assert cast_weight(frozen, torch.bfloat16) is f1       # never stepped: still cached
    with torch.no_grad():
        frozen.mul_(2.0)                                   # in place: version bump
    f2 = cast_weight(frozen, torch.bfloat16)
    assert f2 is not f1 and torch.equal(f2, frozen.detach().to(torch.bfloat16))
    assert cast_weight(a, torch.float32) is not None       # same dtype: no copy
    assert cast_weight(a, torch.float32).data_ptr() == a.data_ptr()


def test_target_rows_cache_is_identity_keyed():
    """point_loss's target-row cache matches label tensors by identity and
    keeps them alive, so a new batch's labels (same shape, possibly the same recycled address)
    never hit the previous batch's rows."""
    from rgbd_amd.point_loss import HipMask2FormerLoss
    loss = HipMask2FormerLoss.__new__(HipMask2FormerLoss)
    a = [torch.zeros(2, 4, 4), torch.ones(1, 4, 4)]
    r1, o1 = loss._target_rows(a, torch.float32)
    assert loss._target_rows(a, torch.float32)[0] is r1          # hit: same tensors
    assert o1 == [0, 2]
    del a
    b = [torch.ones(2, 4, 4), torch.zeros(1, 4, 4)]              # new labels, same shapes
    r2, _ = loss._target_rows(b, torch.float32)
    assert r2 is not r1 and torch.equal(r2, torch.cat(b))
    with torch.no_grad():
        b[0].zero_()                                             # in place: version bump
    r3, _ = loss._target_rows(b, torch.float32)
    assert torch.equal(r3, torch.cat(b))
