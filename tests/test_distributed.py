"""world_size-2 and -8 (BASELINE C3 / C4 rank counts) tests of the data-parallel exchange: gloo on CPU tensors, and (gpu) two ranks on one
MI355X running the fused hot path with the overlapped reducer."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _rgbd_import  # noqa: F401
    from rgbd_amd.distributed import GradBucket
    from rgbd_amd.modules import DSAModule, DepthGradientInjectionResidual
    torch.manual_seed(0)
    mods = [DSAModule(8, 16), DepthGradientInjectionResidual([4, 8], 3)]
    params = [p for m in mods for p in m.parameters()]
    for i, p in enumerate(params):
        p.grad = torch.full_like(p, float(rank + 1) * (i + 1))  # rank-dependent gradients
    params[3].grad = None if rank == 0 else params[3].grad        # a missing grad counts as zero
    GradBucket(params).allreduce_mean()
    ok = True
    for i, p in enumerate(params):
        full, part = (world + 1) / 2, (world * (world + 1) / 2 - 1) / world  # mean of r + 1; rank 0 missing
        exp = full * (i + 1) if i != 3 else part * (i + 1)
        ok &= bool(torch.allclose(p.grad, torch.full_like(p, exp)))
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_grad_allreduce_world(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _worker_overlapped(rank, world, port, q):
    """OverlappedGradReducer on CPU tensors: groups handed over in cascade order, None = zero."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _rgbd_import  # noqa: F401
    from rgbd_amd.distributed import OverlappedGradReducer, hot_path_grad_groups
    from rgbd_amd.modules import DSAModule, DepthGradientInjectionResidual
    torch.manual_seed(0)
    dsams = [DSAModule(4, 8), DSAModule(8, 16), DSAModule(16, 32)]
    dg = DepthGradientInjectionResidual([4, 8, 16, 32], 3)
    groups = hot_path_grad_groups(dsams, dg)
    assert [len(g) for g in groups] == [9, 9, 17]
    red = OverlappedGradReducer(groups)
    ok = True
    for step in range(3):  # buffers are reused across steps
        # step 0: p.grad None (zero_grad(set_to_none=True)) -> overwritten with the mean;
        # step 1: p.grad holds step 0's mean (gradient accumulation) -> previous + mean;
        # step 2: p.grad reset to None again
        exp = []
        for gi, g in enumerate(groups):
            grads = []
            for i, p in enumerate(g):
                if step != 1:
                    p.grad = None
                prev = torch.zeros_like(p) if p.grad is None else p.grad.clone()
                t = torch.randn(p.shape, generator=torch.Generator().manual_seed(1000 * step + 100 * gi + i))
                grads.append(None if (rank == 0 and i == 1) else t * (rank + 1))
                full, part = (world + 1) / 2, (world * (world + 1) / 2 - 1) / world
                exp.append(prev + t * (part if i == 1 else full))  # mean over ranks of t*(r+1), rank 0 missing i==1
            red.ready(gi, grads)
        red.finish()
        got = [p.grad for g in groups for p in g]
        # float32 sums of `world` terms: a few ulps of the largest term
        tol = 4 * world * torch.finfo(torch.float32).eps
        errs = [float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(got, exp)]
        if max(errs) > tol:
            print(f"rank {rank} step {step}: rel err {max(errs):.3g} > {tol:.3g}", flush=True)
            ok = False
    try:
        red.finish()  # nothing handed over: must fail loudly
        ok = False
    except RuntimeError:
        pass
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_overlapped_reducer_world(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overlapped, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _worker_gpu_hot_path(rank, world, port, q):
    """Both ranks on cuda:0 over gloo: the overlapped reducer fed by the fused backward's hook
    yields exactly the mean of the two ranks' standalone gradients."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [root, os.path.join(root, "tests", "golden")]
        import _rgbd_import  # noqa: F401
        import golden_inputs as gi
        from rgbd_amd import init as winit
        from rgbd_amd.distributed import OverlappedGradReducer, hot_path_grad_groups
        from rgbd_amd.hot_path import hot_path
        from rgbd_amd.modules import DSAModule, DepthGradientInjectionResidual
        dev = torch.device("cuda:0")
        H, W, B = 64, 96, 2
        sizes = gi.swin_sizes(H, W)
        pre = "model.pixel_level_module."
        dsams = []
        for k, (ci, co) in enumerate([(96, 192), (192, 384), (384, 768)]):
            m = DSAModule(ci, co)
            winit.init_deterministic(m, prefix=f"{pre}dsam{k}.")
            dsams.append(m.to(dev))
        dg = DepthGradientInjectionResidual([96, 192, 384, 768], 3)
        winit.init_deterministic(dg, prefix=f"{pre}depth_gradient_injection.")
        dg = dg.to(dev)
        params = [p for m in dsams + [dg] for p in m.parameters()]

        def inputs(r):
            pv = torch.from_numpy(gi.pixel_values(40 + r, B, H, W)).to(dev)
            ratios = torch.tensor([[0.12 + 0.1 * r], [0.3]], device=dev)
            colors = [torch.from_numpy(gi.feature(f"ddp.c{k}.{r}", (B, c, *sizes[k]))).to(dev)
                      for k, c in enumerate([96, 192, 384, 768])]
            return pv, ratios, colors

        def grads(r, hook=None):
            for p in params:
                p.grad = None
            pv, ratios, colors = inputs(r)
            outs = hot_path(pv, ratios, colors, dsams, dg, grad_hook=hook)
            torch.autograd.backward(outs, [torch.full_like(o, 1e-2 * (k + 1)) * (1 + r) for k, o in enumerate(outs)])
            return [p.grad.clone() for p in params]

        ref = [(a + b) / 2 for a, b in zip(grads(0), grads(1))]
        red = OverlappedGradReducer(hot_path_grad_groups(dsams, dg))
        grads(rank, hook=red.ready)
        red.finish()
        torch.cuda.synchronize()
        err = max(float(((p.grad - e).abs().max() / (e.abs().max() + 1e-12))) for p, e in zip(params, ref))
        q.put((rank, err))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))


@pytest.mark.gpu
def test_gpu_hot_path_ddp_overlap_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_gpu_hot_path, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert isinstance(res[r], float), res[r]
        assert res[r] < 1e-6, res


def _worker_serial(rank, world, port, q):
    """SerialGradReducer (the captured N > 1 step's exchange) on CPU tensors: every group's
    gradients replaced by their mean over the ranks; a missing gradient fails loudly."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _rgbd_import  # noqa: F401
    from rgbd_amd.distributed import SerialGradReducer, hot_path_grad_groups
    from rgbd_amd.modules import DSAModule, DepthGradientInjectionResidual
    torch.manual_seed(0)
    dsams = [DSAModule(4, 8), DSAModule(8, 16), DSAModule(16, 32)]
    dg = DepthGradientInjectionResidual([4, 8, 16, 32], 3)
    groups = hot_path_grad_groups(dsams, dg)
    red = SerialGradReducer(groups)
    ok = True
    for step in range(2):  # the flat buckets are reused
        exp = []
        for gi, g in enumerate(groups):
            for i, p in enumerate(g):
                t = torch.randn(p.shape, generator=torch.Generator().manual_seed(1000 * step + 100 * gi + i))
                p.grad = t * (rank + 1)
                exp.append(t * (world + 1) / 2)
        red.finish()
        got = [p.grad for g in groups for p in g]
        tol = 4 * world * torch.finfo(torch.float32).eps
        errs = [float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(got, exp)]
        ok = ok and max(errs) <= tol
    groups[1][0].grad = None
    try:
        red.finish()
        ok = False
    except RuntimeError:
        pass
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_serial_reducer_world(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_serial, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}
