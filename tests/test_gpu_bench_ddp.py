"""Row (e) on the GPU: bench.py's data-parallel step at world size 2 (BASELINE C3) and 8 (C4) — gloo
with every rank on the one MI355X of a one-GPU test box (RCCL refuses two ranks on one device), and
RCCL ("nccl", one rank per device) when the box shows enough GPUs (skipped otherwise), so the
driver's multi-GPU scaling run is not the first execution of the RCCL path.

* the launcher: ``bench.py --gpus 2`` spawns two ranks and reports n_gpus 2 / global batch 16;
* DDP semantics of the step (the reference's Trainer, finetuning.py:98-113): after the
  overlapped reducer, every rank holds the mean of the two ranks' standalone gradients, and
  every forward starts from rank 0's ratio-predictor BatchNorm buffers (broadcast_buffers);
* the timed step's AdamW steps inside the backward give bitwise the parameters of DDP + one
  optimizer step after the backward."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _need_devices(backend, world=2):
    if world == 1 and backend != "nccl":
        pytest.skip("world 1 exercises the RCCL path only")
    if backend == "nccl" and torch.cuda.device_count() < world:
        pytest.skip(f"RCCL needs one device per rank: this box shows fewer than {world} GPUs")


BACKENDS = ["gloo", "nccl"]


@pytest.mark.timeout(400)
@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("world,H,W", [(1, 480, 640), (2, 96, 128), (2, 480, 640), (8, 96, 128), (8, 480, 640)],
                         ids=["w1_640x480", "w2_96x128", "C3_w2_640x480", "w8_96x128", "C4_w8_640x480"])
def test_bench_launcher_json(world, H, W, backend):
    """bench.py --gpus N end to end (its own launcher, 8 images per rank) at BASELINE's C3 (2 ranks,
    global batch 16) and C4 (8 ranks, global batch 64); gloo with every rank on the test box's one
    GPU, or RCCL with one rank per GPU.  World 1 over RCCL (``--ddp 1``): the process group, the
    overlapped all-reduces and their stream waits and the buffer broadcasts on a one-GPU box."""
    _need_devices(backend, world)
    extra = ["--ddp", "1"] if world == 1 else []
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", str(world), *extra, "--backend", backend, "--steps", "2",
                        "--warmup", "1", "--cpu-baseline", "0", "--c5-stream", "0", "--inference", "0", "--parity", "0",
                        "--height", str(H), "--width", str(W)],
                       capture_output=True, text=True, timeout=380, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]  # stdout: the one JSON line only
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["global_batch"] == 8 * world
    assert out["distributed"]["world_size"] == world and out["config"]["parallelism"] == f"dp{world}"
    assert out["distributed"]["backend"] == backend
    assert out["value"] > 0
    if backend == "nccl":  # the captured step with its collectives replayed beside the eager one
        assert out["ddp_captured_img_s"] is not None, out["ddp_captured_note"]
        assert out["ddp_captured_overlap_img_s"] is not None, out["ddp_captured_note"]
        assert out["ddp_overlapped_eager_img_s"] is not None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, shape, backend):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        if backend == "nccl":  # RCCL: one device per rank
            dev = torch.device("cuda", rank)
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dev = torch.device("cuda:0")
            dist.init_process_group("gloo", rank=rank, world_size=world)
        sys.path.insert(0, str(REPO))
        import bench
        H, W, B = shape
        args = bench.parse(["--height", str(H), "--width", str(W), "--batch", str(B)])
        # standalone gradients of both shards (ratio predictor in eval: a deterministic ratio)
        ref = []
        for r in range(world):
            ctx = bench.build(args, dev, rank=r)
            ctx["rp"].eval()
            fb, _, _, _ = bench.make_parts(ctx, 1)
            fb()
            ref.append([p.grad.clone() for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()])
        mean = [torch.stack(gs).sum(0) / world for gs in zip(*ref)]
        # the DDP step of this rank
        ctx = bench.build(args, dev, rank=rank)
        ctx["rp"].eval()
        fb, _, _, _ = bench.make_parts(ctx, world, ddp=True)
        fb()
        got = [p.grad for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()]
        grad_err = max(float(((a - e).abs().max() / (e.abs().max() + 1e-12))) for a, e in zip(got, mean))
        # buffer broadcast in train mode: rank 1 starts from different BN statistics; the forward
        # must see rank 0's
        ctx = bench.build(args, dev, rank=rank)
        bns = [b for b in ctx["rp"].buffers()]
        with torch.no_grad():
            for b in bns:
                if b.is_floating_point():
                    b.add_(0.5 * rank)
        seen = {}
        ctx["rp"].register_forward_pre_hook(lambda m, a: seen.__setitem__("bufs", [b.clone() for b in m.buffers()]))
        fb, _, _, _ = bench.make_parts(ctx, world, ddp=True)
        fb()
        flat = torch.cat([b.double().reshape(-1) for b in seen["bufs"]])
        flat = flat.to(dev) if backend == "nccl" else flat.cpu()
        other = flat.clone()
        dist.broadcast(other, src=0)
        buf_err = float((flat - other).abs().max())
        # the AdamW steps inside the backward (bench.py's timed step): each group waits for its
        # all-reduce on its stream and steps on the mean -> the parameters of DDP + one step
        outs = []
        for overlap in (False, True):
            ctx = bench.build(args, dev, rank=rank)
            ctx["rp"].eval()
            fb, ostep, _, _ = bench.make_parts(ctx, world, overlap_opt=overlap, ddp=True)
            for _ in range(2):
                fb()
                ostep()
            outs.append([p.detach().clone() for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()])
        opt_err = max(float((a - e).abs().max()) for a, e in zip(outs[1], outs[0]))
        torch.cuda.synchronize()
        q.put((rank, (grad_err, buf_err, opt_err)))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("world,shape", [(1, (480, 640, 8)), (2, (96, 128, 3)), (2, (480, 640, 8)), (8, (96, 128, 3)),
                                         (8, (480, 640, 8))],
                         ids=["w1_640x480_b8", "w2_96x128_b3", "C3_w2_640x480_b8", "w8_96x128_b3", "C4_w8_640x480_b8"])
def test_ddp_step_gradients_and_buffers(world, shape, backend):
    """Small shape, and BASELINE configs[2] / [3] (C3 / C4) at their workload: 640x480, 8 images per
    rank, bf16, world size 2 / 8 (global batch 16 / 64) — gloo with every rank on the one GPU of the
    test box, or RCCL with one rank per GPU where the box has enough.  Every rank's reduced
    gradients equal the mean of all shards' standalone gradients (1e-5), the BatchNorm buffers the
    forward sees are rank 0's (bitwise), and the in-backward AdamW equals DDP + one step (bitwise)."""
    _need_devices(backend, world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, shape, backend)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=560) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(res[r], tuple), res[r]
        grad_err, buf_err, opt_err = res[r]
        assert grad_err < 1e-5, res
        assert buf_err == 0.0, res
        assert opt_err == 0.0, res


def _captured_worker(port, q, shape, steps):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        sys.path.insert(0, str(REPO))
        import bench
        H, W, B = shape
        args = bench.parse(["--height", str(H), "--width", str(W), "--batch", str(B)])

        def state(ctx):
            return ([p.detach().clone() for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()]
                    + [b.detach().clone() for b in ctx["rp"].buffers()])
        # CapturedTrainStep's two warmup steps + `steps` replays = 2 + steps training steps, against
        # the same schedule run eagerly (serial exchange, one AdamW after it) and the eager bench
        # step (all-reduces overlapped with the backward, AdamW inside it)
        def build():  # ratio predictor in eval: the same ratio in every run (its dropout draws
            ctx = bench.build(args, dev)  # come from a process-wide counter)
            ctx["rp"].eval()
            return ctx

        def eager(**kw):
            ctx = build()
            fb, ostep, _, _ = bench.make_parts(ctx, 1, ddp=True, **kw)
            for _ in range(2 + steps):
                fb()
                ostep()
            return state(ctx)
        ref_serial = eager(serial_ddp=True)
        ref_overlap = eager(overlap_opt=True)
        ref_ov1 = eager(serial_ddp="overlap")

        def captured(form):
            ctx = build()
            cs, why = bench.captured_ddp_step(ctx, 1, dev, serial_ddp=form)
            assert cs is not None, why
            for _ in range(steps):
                cs()
            torch.cuda.synchronize()
            return state(ctx), cs.width
        got, width = captured(True)
        got_ov, width_ov = captured("overlap")
        diff = [i for i, (a, e) in enumerate(zip(got, ref_serial)) if not torch.equal(a, e)]
        diff += [100 + i for i, (a, e) in enumerate(zip(got_ov, ref_ov1)) if not torch.equal(a, e)]
        rel = max(float((a.double() - e.double()).abs().max() / (e.double().abs().max() + 1e-30))
                  for a, e in zip(ref_serial, ref_overlap) if a.is_floating_point())
        print(f"captured vs eager serial: {len(diff)} tensors differ; eager serial vs overlapped: max rel {rel:.3g}")
        q.put((0, (diff, max(width, width_ov), rel)))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((0, traceback.format_exc() + repr(e)))


@pytest.mark.timeout(400)
def test_captured_rccl_step_bitwise_eager_world1():
    """The N > 1 captured step (bench.captured_ddp_step: BN-buffer broadcasts, forward, backward,
    one RCCL all-reduce per gradient bucket after the backward, AdamW — all inside one HIP graph)
    at world 1 over RCCL on the box's one GPU: the graph captures and instantiates (at most two
    concurrent branches), its replays run the collectives, and the parameters and ratio-predictor
    buffers after 2 warmup steps + 3 replays are bitwise those of the eager run of the same
    schedule, and against the eager bench step (all-reduces overlapped with the backward, AdamW
    inside it) within 1e-6 relative.  The same for the captured form with the backward on one
    stream and the all-reduces + in-backward AdamW overlapped beside it (finetuning.py:98-113)."""
    _need_devices("nccl", 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_captured_worker, args=(_free_port(), q, (96, 128, 3), 3))
    p.start()
    rank, res = q.get(timeout=380)
    p.join(timeout=60)
    assert isinstance(res, tuple), res
    diff, width, rel = res
    assert width <= 2
    assert diff == [], f"state tensors differ: {diff}"
    assert rel <= 1e-6, rel  # the two exchange schedules: the same means, the same AdamW
