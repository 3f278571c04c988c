"""The hot-path training step replayed from a HIP graph (rgbd_amd/train_graph.py, bench.py's
N=1 timed step) computes exactly what the eager step computes: after the same number of steps
from the same weights, every trained parameter and every ratio-predictor BatchNorm buffer is
bitwise equal, and the dropout counter has advanced once per step in both."""
import sys
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import _rgbd_import  # noqa: E402,F401

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ctx(bench, args):
    ctx = bench.build(args, DEV)
    rp = ctx["rp"]
    rp._rgbd_dropout_ctr = torch.zeros((1,), dtype=torch.int64, device=DEV)
    rp._rgbd_dropout_seed = 0x5EED1234  # the same dropout stream in both arms
    return ctx


def _state(ctx):
    out = [p.detach().clone() for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()]
    out += [b.detach().clone() for b in ctx["rp"].buffers()]
    return out


def test_captured_step_equals_eager_steps():
    import bench
    from rgbd_amd.train_graph import CapturedTrainStep
    args = bench.parse(["--height", "96", "--width", "128", "--batch", "3"])
    a, b = _ctx(bench, args), _ctx(bench, args)
    fa, oa, _, _ = bench.make_parts(a, 1, capturable=True)
    for _ in range(4):
        fa()
        oa()
    fb, ob, _, _ = bench.make_parts(b, 1, capturable=True)
    step = CapturedTrainStep(fb, ob.opt, warmup=2)  # 2 eager steps, then capture
    for _ in range(2):
        outs = step()
    torch.cuda.synchronize()
    assert int(a["rp"]._rgbd_dropout_ctr.item()) == 4 == int(b["rp"]._rgbd_dropout_ctr.item())
    sa, sb = _state(a), _state(b)
    assert len(sa) == len(sb)
    for i, (x, y) in enumerate(zip(sa, sb)):
        assert torch.equal(x, y), f"state tensor {i} differs after 4 steps"
    assert len(outs) == 4 and all(torch.isfinite(o.float()).all() for o in outs)


def test_captured_in_backward_optimizer_equals_eager_steps():
    """bench.py's timed N=1 step: the AdamW steps issued inside the backward, one per parameter
    group (distributed.InBackwardOptimizer), replayed from a graph, against plain eager steps
    with one optimizer.step() after each backward: bitwise the same parameters and buffers."""
    import bench
    from rgbd_amd.train_graph import CapturedTrainStep
    args = bench.parse(["--height", "96", "--width", "128", "--batch", "3"])
    a, b = _ctx(bench, args), _ctx(bench, args)
    fa, oa, _, _ = bench.make_parts(a, 1, capturable=True)
    for _ in range(4):
        fa()
        oa()
    fb, ob, _, _ = bench.make_parts(b, 1, capturable=True, overlap_opt=True)
    assert ob.opt is None and len(ob.opts) >= 1
    step = CapturedTrainStep(fb, None, warmup=2, opts=ob.opts, clear=ob)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip(_state(a), _state(b))):
        assert torch.equal(x, y), f"state tensor {i} differs after 4 steps"


def test_captured_step_needs_capturable_optimizer():
    import bench
    from rgbd_amd.train_graph import CapturedTrainStep
    args = bench.parse(["--height", "64", "--width", "96", "--batch", "2"])
    ctx = _ctx(bench, args)
    fb, _, _, _ = bench.make_parts(ctx, 1)  # (bench's own optimizer, HipAdamW, is always capturable)
    params = [p for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()]
    with pytest.raises(ValueError, match="capturable"):
        CapturedTrainStep(fb, torch.optim.AdamW(params, lr=1e-5, fused=True))


def test_pipelined_captured_step_equals_sequential_steps():
    """bench.py's pipelined step (make_parts pipeline=True): the next batch's ratio predictor on
    a second stream beside this batch's hot path, captured; after 4 training steps every trained
    parameter is bitwise that of 4 sequential eager steps, and — the pipeline having run one
    ratio forward ahead — the BatchNorm buffers and dropout counter equal the sequential arm's
    after one more forward."""
    import bench
    from rgbd_amd.train_graph import CapturedTrainStep
    args = bench.parse(["--height", "96", "--width", "128", "--batch", "3"])
    a, b = _ctx(bench, args), _ctx(bench, args)
    fa, oa, _, _ = bench.make_parts(a, 1, capturable=True)
    for _ in range(4):
        fa()
        oa()
    from rgbd_amd import ops
    a["rp"](ops.assemble_pixel_values(a["depth_u8"], a["rgb_u8"])[:, 3:6])  # the pipeline's read-ahead
    fb, ob, _, _ = bench.make_parts(b, 1, capturable=True, overlap_opt=True, pipeline=True)
    step = CapturedTrainStep(fb, None, warmup=2, opts=ob.opts, clear=ob)
    assert step.width <= 2
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    assert int(a["rp"]._rgbd_dropout_ctr.item()) == 5 == int(b["rp"]._rgbd_dropout_ctr.item())
    for i, (x, y) in enumerate(zip(_state(a), _state(b))):
        assert torch.equal(x, y), f"state tensor {i} differs after 4 steps"


def test_replay_advances_cast_cache_epoch():
    """dense.cast_weight caches a parameter's bf16 copy under (address,
    version, step epoch). A graph replay updates the parameters on the device without the host
    post-step hook, so CapturedTrainStep advances the epoch itself: an eager forward after
    replay / eager / replay sees the updated weights, not the cast cached in between."""
    from rgbd_amd.dense import HipLinear, cast_weight
    from rgbd_amd.train_graph import CapturedTrainStep
    torch.manual_seed(0)
    lin = torch.nn.Linear(64, 32).to(DEV)
    lin.__class__ = HipLinear
    opt = torch.optim.AdamW(lin.parameters(), lr=1e-2, capturable=True)
    x = torch.randn(128, 64, device=DEV)

    def fb():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = lin(x)
        y.float().square().mean().backward()
        return (y,)

    step = CapturedTrainStep(fb, opt, warmup=2)
    for _ in range(2):
        step()
        torch.cuda.synchronize()
        c = cast_weight(lin.weight, torch.bfloat16)   # the eager forward's cast
        assert torch.equal(c, lin.weight.detach().to(torch.bfloat16)), "stale bf16 cast after replay"
