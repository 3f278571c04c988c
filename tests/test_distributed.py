"""world_size-2 gloo test of the data-parallel exchange (CPU, no GPU needed)."""
import os
import socket

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
        exp = (1.0 + 2.0) / 2 * (i + 1) if i != 3 else 2.0 * (i + 1) / 2
        ok &= bool(torch.allclose(p.grad, torch.full_like(p, exp)))
    q.put((rank, ok))
    dist.destroy_process_group()


def test_grad_allreduce_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
