"""No kernel reads workspace bytes it has not written this call.

Every entry point takes a caller-provided scratch buffer (``ops._workspace``: one per entry point
and stream, allocated with ``torch.empty`` and reused across calls).  A kernel that reads a cell
no kernel of the same call wrote (round 5: three corner cells of the stem-moment border tables,
fixed in ab770b2) returns whatever the previous call or allocation left there — usually the same
bytes, so it passes every comparison by luck.  Here the hot-path training step (K1 assembly, the
ratio predictor in train mode with its batch-statistics BatchNorms and dropout, the decomposition,
the DSAM cascade and the DGGM, forward and backward) and the ratio predictor's eval forward run
three times from the same module state: once as they are, then with every non-zeroed workspace
filled with 0xFF bytes (NaN in float32 and bf16) and with 0x3C bytes (a finite float) before the
call.  Outputs, gradients, BatchNorm buffers and the ratio must be bitwise identical.
Workspaces whose contents calls rely on (counters each call leaves at zero, ``zeroed=True``) are
left alone."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _poison(byte):
    from rgbd_amd import ops
    n = 0
    for key, buf in ops._ws_cache.items():
        if key in ops._ws_zeroed or buf.device != DEV:
            continue
        buf.fill_(byte)
        n += 1
    torch.cuda.synchronize()
    return n


def _state(ctx):
    mods = [ctx["rp"], ctx["dg"]] + ctx["dsams"]
    return [copy.deepcopy(m.state_dict()) for m in mods]


def _load(ctx, state, seed):
    mods = [ctx["rp"], ctx["dg"]] + ctx["dsams"]
    for m, sd in zip(mods, state):
        m.load_state_dict(sd)
        for p in m.parameters():
            p.grad = None
    # the same dropout draws every run: a fixed base seed and the device counter at zero
    ctx["rp"]._rgbd_dropout_seed = seed
    ctx["rp"]._rgbd_dropout_ctr = torch.zeros((1,), dtype=torch.int64, device=DEV)


@pytest.mark.parametrize("H,W,B", [(90, 125, 2), (480, 640, 8)], ids=["ragged_90x125_b2", "C2_640x480_b8"])
def test_hot_path_train_step_ignores_workspace_contents(H, W, B):
    import bench
    args = bench.parse(["--height", str(H), "--width", str(W), "--batch", str(B)])
    ctx = bench.build(args, DEV)
    fb, _, _, _ = bench.make_parts(ctx, 1)
    state = _state(ctx)
    seed = 0x5EED
    _load(ctx, state, seed)
    fb()  # sizes every workspace and fills the pack caches
    torch.cuda.synchronize()

    def run(byte):
        _load(ctx, state, seed)
        poisoned = _poison(byte) if byte is not None else 0
        feats = fb()
        ctx["rp"].eval()
        with torch.no_grad():
            if byte is not None:
                _poison(byte)
            r_eval = ctx["rp"](bench_pv(ctx))
        ctx["rp"].train()
        torch.cuda.synchronize()
        out = [f.detach().clone() for f in feats] + [r_eval.clone()]
        out += [p.grad.detach().clone() for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()]
        out += [b.detach().clone() for b in ctx["rp"].buffers()]
        return out, poisoned

    def bench_pv(ctx_):
        from rgbd_amd import ops
        return ops.assemble_pixel_values(ctx_["depth_u8"], ctx_["rgb_u8"])[:, 3:6]

    ref, _ = run(None)
    for byte in (0xFF, 0x3C):
        got, n = run(byte)
        assert n > 0, "no workspace was poisoned"
        bad = [i for i, (a, b) in enumerate(zip(ref, got)) if not torch.equal(a, b)]
        assert not bad, f"poison 0x{byte:02X}: tensors {bad} of {len(ref)} differ from the unpoisoned run"
