"""Benchmark of the MI355X-native DGGM + E-DSAM hot path (BASELINE.json metric).

One step = one training pass of the v0.4.0 pixel-level hot path over
a batch of synthetic NYUv2-shaped frames (640x480, 8 images per GPU, bf16 MFMA):
  u8 RGB + u8 depth (resident in HBM)
  -> 10-channel pixel_values incl. DGGM Sobel planes         (K1, rgbd_assemble_pixel_values)
  -> (N > 1) rank 0's ratio-predictor BatchNorm buffers broadcast (DDP broadcast_buffers)
  -> ratio predictor, train-mode BatchNorm + dropout          (K4, rgbd_ratio_forward)
  -> depth decomposition once per image                       (K3, rgbd_edsam_decompose)
  -> DSAM x3 masked implicit GEMMs (cascade) + DGGM + sum     (K5, K2)
  -> backward from a fixed synthetic upstream gradient of the 4 backbone features:
     DSAM dW/db/dX cascade + DGGM dW/db                        (K5, K2)
  -> (N > 1) RCCL all-reduce (mean) of the hot-path parameter gradients, overlapped with the
     backward cascade (DDP semantics of the reference's Trainer, finetuning.py:98-113)
  -> AdamW step on the hot-path parameters (HF Trainer's optimizer; lr 1e-5 constant,
     mask2former/config.json), so every step re-packs the changed DSAM filters.
The Swin encoder / pixel decoder / transformer decoder are outside the hot path (SURVEY §8(f)
"next"); their colour-feature inputs are synthetic tensors of the Swin-T shapes.

Launch: ``python bench.py --gpus N`` spawns N rank processes itself (before any GPU call) when
no launcher set WORLD_SIZE; under ``torch.distributed.run`` each rank reads RANK / LOCAL_RANK /
WORLD_SIZE from the environment.  8 images per rank (scaling "weak").

Prints ONE JSON line (rank 0).  ``value`` = images processed by all ranks / max-over-ranks
time.  ``roofline`` is for the dominant kernel (the ratio predictor's 3x3 128->256 conv,
k_rp_conv5_v4), timed with HIP events on its launch stream over this run's eager timed steps;
``kernels`` carries the same for K5 and the whole step's t_ideal / t_measured.
``cpu_baseline`` = the oracle (PyTorch-CPU fp32 restatement of the reference, tests-only
code) on bounded samples of the same workloads on this host's cores (BASELINE.md plan).
``parity`` = the mask-logit max-abs-err of the full drop-in model at 640x480 against the
reference's committed fixture (tests/golden/g7_model640.npz), float32 (bound 1e-3) and, under
``parity.bf16``, with the hot path in bf16 as benched (stated relative bound), measured outside
the timed region.
"""
import argparse
import ctypes
import json
import re
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _rgbd_import  # noqa: E402,F401

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md, chip table)
HBM_PEAK_GBS = 8000.0
CONV5_FLOP_PER_PX = 2 * 128 * 9 * 256  # 3x3 128->256 (custom_model.py:1413)
CONV5_KERNEL = "k_rp_conv5_v4"
DSAM_CH = [(96, 192), (192, 384), (384, 768)]
# SURVEY §8(d), per input pixel of the batch (P = B*H*W): reference-algorithmic work
K4_FLOP_PER_PX = 703_616          # ratio predictor forward
K5_FWD_FLOP_PER_PX = 77_760       # 3 DSAMs x (4 masked 3x3 s2 convs + projection)
K5_BWD_FLOP_PER_PX = 129_600      # dX (dsam1, dsam2) + dW (all) of the same convs
K1_BYTES_PER_PX = 6.0
K2_BYTES_PER_PX = 71.5
K3_BYTES_PER_PX = 12.04
ADAMW_BYTES_PER_PARAM = 28        # fused AdamW: read p, g, m, v; write p, m, v (f32)


# The committed evidence of this tree's default bench step (rocprofv3 kernel trace + PMC passes,
# see its README): named explicitly, updated with each evidence commit, never picked by sort order.
EVIDENCE_DIR = "profiles/r06_v4"


def pmc_traffic(kernel, default_shape):
    """HBM bytes per launch of ``kernel`` from EVIDENCE_DIR/pmc_traffic.json (FETCH_SIZE doubled
    per the gfx950 correction, plus WRITE_SIZE, one pass each, over this bench's default step).
    rocprofv3 cannot run inside this process, so the counters come from their own passes; null
    for a non-default shape or when the evidence has no such row."""
    path = REPO / EVIDENCE_DIR / "pmc_traffic.json"
    if not default_shape or not path.exists():
        return None
    for key, row in json.loads(path.read_text()).items():
        name = key.split(" grid=")[0]  # a template argument list (e.g. "<false>") aside
        if (name == kernel or name.split("<")[0] == kernel) and "hbm_bytes" in row:
            return row["hbm_bytes"], str(path.relative_to(REPO))
    return None


def profile_avg_ns(kernel, default_shape):
    """(average ns per launch, source, calls) of ``kernel`` in EVIDENCE_DIR/kernel_stats.csv
    (``rocprofv3 --kernel-trace --stats`` of this bench's default step); None for a non-default
    shape or when the trace has no such kernel."""
    import csv
    path = REPO / EVIDENCE_DIR / "kernel_stats.csv"
    if not default_shape or not path.exists():
        return None
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row.get("Name", "").replace("(anonymous namespace)::", "")
            head = re.sub(r"<.*>", "", name.split("(")[0])  # template arguments may hold spaces
            base = head.split()[-1].split("::")[-1] if head.split() else ""
            if base == kernel:
                return float(row["AverageNs"]), str(path.relative_to(REPO)), int(row["Calls"])
    return None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse several ranks on one GPU)")
    ap.add_argument("--ddp", type=int, default=None,
                    help="run the data-parallel path (process group, overlapped all-reduce, buffer broadcast) "
                         "even at N=1 (default: only for N > 1); --ddp 1 --gpus 1 executes the RCCL code on one GPU")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on the host (rank 0, N=1)")
    ap.add_argument("--inference", type=int, default=1, help="also report forward-only img/s")
    ap.add_argument("--c5-stream", type=int, default=1,
                    help="also report the C5 RealSense 1280x720 B=1 streaming inference rate (rank 0, N=1)")
    ap.add_argument("--parity", type=int, default=1,
                    help="report the fp32 mask-logit max-abs-err vs the committed 640x480 fixture (rank 0)")
    ap.add_argument("--full-model", type=int, default=1,
                    help="also report the whole drop-in model's bf16 training step at 640x480 B=8 (rank 0, N=1)")
    ap.add_argument("--graph", type=int, default=1,
                    help="N=1: time the step replayed from a HIP graph (rgbd_amd/train_graph.py); the eager "
                         "rate and the per-kernel HIP-event timings come from an eager pass beside it")
    ap.add_argument("--pipeline-report", type=int, default=0,
                    help="N=1: also time the captured step software-pipelined across batches (pipelined_img_s)")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv):
    """One child process per rank, started before this process touches the GPU, with the
    environment torch.distributed.run would give it.  Returns the first non-zero exit code (the
    other ranks are then terminated) or 0."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + list(argv), env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc


def launcher_selftest():
    """CPU plumbing check of spawn_ranks (tests/test_bench_launcher.py): gloo on CPU tensors."""
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"world": dist.get_world_size(), "rank_sum": float(t.item()),
                          "local_rank": int(os.environ["LOCAL_RANK"])}), flush=True)
    dist.destroy_process_group()


# ------------------------------------------------------------------ workload
def build(args, dev, rank=0):
    from rgbd_amd import init as winit, synthetic
    from rgbd_amd.modules import DSAModule, DepthGradientInjectionResidual, EnhancedDepthImageRatioPredictor
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    pre = "model.pixel_level_module."
    rp = EnhancedDepthImageRatioPredictor(3)
    winit.init_deterministic(rp, prefix=pre + "ratio_predictor.")
    dsams = []
    for k, (ci, co) in enumerate(DSAM_CH):
        m = DSAModule(ci, co)
        winit.init_deterministic(m, prefix=f"{pre}dsam{k}.")
        dsams.append(m)
    dg = DepthGradientInjectionResidual([96, 192, 384, 768], 3)
    winit.init_deterministic(dg, prefix=pre + "depth_gradient_injection.")
    for m in [rp, dg] + dsams:
        m.compute_dtype = dtype
        m.to(dev).train()
    B, H, W = args.batch, args.height, args.width
    scenes = [synthetic.make_scene(synthetic.scene_seed(3, rank * B + i), H, W) for i in range(B)]
    depth_u8 = torch.from_numpy(np.stack([s["depth_u8"] for s in scenes])).to(dev)
    rgb_u8 = torch.from_numpy(np.stack([s["rgb_u8"] for s in scenes])).contiguous().to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    sizes = []
    h, w = -(-H // 4), -(-W // 4)
    for _ in range(4):
        sizes.append((h, w))
        h, w = -(-h // 2), -(-w // 2)
    colors = [torch.randn((B, c, *sizes[k]), generator=g, device=dev).to(dtype)
              for k, c in enumerate([96, 192, 384, 768])]
    gouts = [torch.randn((B, c, *sizes[k]), generator=g, device=dev).to(dtype) * 1e-2
             for k, c in enumerate([96, 192, 384, 768])]
    return dict(rp=rp, dsams=dsams, dg=dg, dtype=dtype, depth_u8=depth_u8, rgb_u8=rgb_u8, colors=colors,
                gouts=gouts, scenes=scenes, sizes=sizes)


def make_parts(ctx, world, capturable=False, overlap_opt=False, pipeline=False, ddp=None, serial_ddp=False):
    """(forward_backward, optimizer_step, reducer, broadcaster) of one training step.
    forward_backward() leaves the (all-reduced, for N > 1) gradients in p.grad;
    optimizer_step.opt is the AdamW instance (``capturable`` for graph capture).
    ``overlap_opt``: the AdamW steps run inside the backward instead, one per parameter group as
    its gradients are enqueued (distributed.InBackwardOptimizer; bitwise the same update);
    forward_backward() then trains and optimizer_step() only clears the gradients
    (optimizer_step.opt None, optimizer_step.opts the per-group optimizers).
    ``pipeline``: software-pipelined across batches — the ratio predictor (K1 assembly + K4) of
    the NEXT batch runs on a second stream beside this batch's decomposition / DSAM / DGGM
    forward, backward and AdamW, and this batch uses the ratio the previous step computed.  The
    predictor is forward-only and never trained (its output leaves autograd through .item(),
    custom_model.py:339-351, Q2) and nothing of batch k's backward feeds batch k+1's predictor,
    so every parameter, BatchNorm buffer and dropout draw is bitwise that of the sequential
    schedule (tests/test_gpu_train_graph.py).  The hot path then keeps all its own launches on the
    main stream (two concurrent branches when captured).
    ``serial_ddp`` (with ddp): the gradient exchange after the backward on the main stream
    (distributed.SerialGradReducer) and one AdamW step after it — the form a HIP graph can hold
    with the collectives inside (the N > 1 captured step); ``serial_ddp="overlap"``: the backward's
    launches all on the main stream and the overlapped reducer + in-backward AdamW beside them
    (the all-reduces are then the graph's second branch)."""
    from rgbd_amd import ops
    from rgbd_amd.distributed import (BufferBroadcaster, InBackwardOptimizer, OverlappedGradReducer,
                                      hot_path_grad_groups)
    from rgbd_amd.hot_path import hot_path, prepare
    from rgbd_amd.optim import HF_TRAINER_ADAMW, HipAdamW
    params = [p for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()]
    groups = hot_path_grad_groups(ctx["dsams"], ctx["dg"])
    # DDP: one bucket per DSAM module, all-reduced asynchronously while the backward cascade runs
    ddp = world > 1 if ddp is None else bool(ddp)
    serial = None
    bwd_side = not (ddp and serial_ddp == "overlap")
    if ddp and serial_ddp == "overlap":
        reducer, overlap_opt = OverlappedGradReducer(groups), True
    elif ddp and serial_ddp:
        from rgbd_amd.distributed import SerialGradReducer
        serial, reducer, overlap_opt = SerialGradReducer(groups), None, False
    else:
        reducer = OverlappedGradReducer(groups) if ddp else None
    bcast = BufferBroadcaster([ctx["rp"]]) if ddp else None
    hook = None if reducer is None else reducer.ready
    if overlap_opt:
        # dsam2's update as soon as its gradients are in (under the rest of the backward), the
        # rest in one launch at the end
        inb = InBackwardOptimizer(groups, lambda g: HipAdamW(g, **HF_TRAINER_ADAMW), reducer, steps=((0,), (1, 2)))
        hook, opt = inb.hook, None
    else:
        opt = HipAdamW(params, **HF_TRAINER_ADAMW)  # AdamW on HIP (rgbd_adamw_multi); always capturable

    if pipeline:
        from rgbd_amd.hot_path import side_stream
        dev = ctx["depth_u8"].device
        side = side_stream(dev)
        # static buffers (outside any captured graph): the next batch's ratio, and this batch's copy
        ratio_next = torch.empty((ctx["depth_u8"].shape[0], 1), dtype=torch.float32, device=dev)
        ratio_cur = torch.empty_like(ratio_next)

        def next_ratio():  # the next batch's K1 + K4 (the bench's synthetic stream repeats its batch)
            pvn = ops.assemble_pixel_values(ctx["depth_u8"], ctx["rgb_u8"])
            ratio_next.copy_(ctx["rp"](pvn[:, 3:6]))
        next_ratio()  # prime the pipeline with the first batch's ratio

    def forward_backward():
        if pipeline:
            main = torch.cuda.current_stream(dev)
            ratio_cur.copy_(ratio_next)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                next_ratio()
            pv = ops.assemble_pixel_values(ctx["depth_u8"], ctx["rgb_u8"])
            prep = prepare(pv, ctx["colors"], ctx["dtype"], overlap=False, dsam_modules=ctx["dsams"])
            feats = hot_path(pv, ratio_cur, ctx["colors"], ctx["dsams"], ctx["dg"], dtype=ctx["dtype"],
                             grad_hook=hook, prepared=prep, overlap=False)
            torch.autograd.backward(feats, ctx["gouts"])
            main.wait_stream(side)
            return feats
        pv = ops.assemble_pixel_values(ctx["depth_u8"], ctx["rgb_u8"])
        if bcast is not None:  # DDP broadcast_buffers: every forward starts from rank 0's BN stats
            bcast.sync()
        prep = prepare(pv, ctx["colors"], ctx["dtype"], dsam_modules=ctx["dsams"])  # beside the ratio predictor
        ratio = ctx["rp"](pv[:, 3:6])
        feats = hot_path(pv, ratio, ctx["colors"], ctx["dsams"], ctx["dg"], dtype=ctx["dtype"], grad_hook=hook,
                         prepared=prep, overlap_bwd=bwd_side)
        torch.autograd.backward(feats, ctx["gouts"])
        if reducer is not None and not overlap_opt:  # DDP gradient exchange (RCCL over xGMI)
            reducer.finish()
        if serial is not None:  # the same exchange after the backward, capturable
            serial.finish()
        return feats

    def optimizer_step():
        if overlap_opt:
            inb.zero_grad(set_to_none=True)
            return
        opt.step()
        opt.zero_grad(set_to_none=True)
    optimizer_step.opt = opt
    optimizer_step.opts = inb.opts if overlap_opt else [opt]

    return forward_backward, optimizer_step, reducer, bcast


def captured_ddp_step(ctx, world, dev, serial_ddp=True):
    """N > 1: the data-parallel step with its collectives inside one HIP graph (make_parts
    ``serial_ddp``: buffer broadcast, forward, backward, gradient all-reduce, AdamW), or None
    when any rank could not capture it (every rank agrees before any replay, so no rank waits in
    a collective the others never issue).  Returns (step, None) or (None, reason)."""
    from rgbd_amd.train_graph import CapturedTrainStep
    fb, ostep, _, _ = make_parts(ctx, world, capturable=True, ddp=True, serial_ddp=serial_ddp)
    cs, why = None, None
    try:
        if ostep.opt is None:  # in-backward AdamW: the step's optimizers, cleared by ostep()
            cs = CapturedTrainStep(fb, None, opts=ostep.opts, clear=ostep)
        else:
            cs = CapturedTrainStep(fb, ostep.opt, clear=lambda: ostep.opt.zero_grad(set_to_none=True))
    except Exception as e:  # noqa: BLE001 - reported in the line, the eager step stays the value
        why = f"{type(e).__name__}: {e}"[:300]
    ok = torch.tensor([0 if cs is None else 1], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        return None, why or "another rank could not capture the step"
    return cs, None


def make_step(ctx, world, inference=False, graph=False, pipeline=False, ddp=None):
    from rgbd_amd import ops
    from rgbd_amd.hot_path import hot_path, prepare
    if inference:
        def istep():
            pv = ops.assemble_pixel_values(ctx["depth_u8"], ctx["rgb_u8"])
            with torch.no_grad():
                prep = prepare(pv, ctx["colors"], ctx["dtype"], dsam_modules=ctx["dsams"])
                ratio = ctx["rp"](pv[:, 3:6])
                return hot_path(pv, ratio, ctx["colors"], ctx["dsams"], ctx["dg"], dtype=ctx["dtype"], prepared=prep)
        return istep
    if graph:  # single process: the whole step replayed from a HIP graph, captured on first use
        from rgbd_amd.train_graph import CapturedTrainStep
        fb, ostep, _, _ = make_parts(ctx, world, capturable=True, overlap_opt=True, pipeline=pipeline, ddp=ddp)
        held = {}

        def gstep():
            if "g" not in held:
                held["g"] = CapturedTrainStep(fb, ostep.opt, opts=ostep.opts, clear=ostep)
            return held["g"]()
        return gstep
    fb, ostep, _, _ = make_parts(ctx, world, overlap_opt=True, ddp=ddp)

    def step():
        feats = fb()
        ostep()
        return feats
    return step


def timed(step, steps, warmup, world, on_start=None, ddp=None):
    ddp = world > 1 if ddp is None else ddp
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if on_start is not None:
        on_start()
    if ddp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if ddp:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if ddp:
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


# ------------------------------------------------------------------ side measurements
def c5_stream(ctx, frames=100):
    """BASELINE configs[4]: RealSense 1280x720 RGB-D stream inference, one frame per step, the
    hot path in eval mode replayed from a HIP graph (rgbd_amd/stream.py).  Reports the graph
    rate with the frame resident, the graph rate including the pinned-host -> HBM copy of the
    raw u8 frame (RGB + depth, 3.7 MB), and the same path launched eagerly from Python."""
    from rgbd_amd import synthetic
    from rgbd_amd.stream import StreamingHotPath
    H, W = 720, 1280
    sp = StreamingHotPath(ctx["rp"], ctx["dsams"], ctx["dg"], H, W, B=1, dtype=ctx["dtype"])
    sc = synthetic.make_scene(synthetic.scene_seed(5, 0), H, W)
    d_host = torch.from_numpy(sc["depth_u8"][None]).pin_memory()
    c_host = torch.from_numpy(sc["rgb_u8"][None]).contiguous().pin_memory()
    g = torch.Generator(device="cuda").manual_seed(5)
    colors = [torch.randn(c.shape, generator=g, device="cuda").to(c.dtype) for c in sp.colors]
    sp(d_host, c_host, colors)  # captures

    def rate(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            fn()
        torch.cuda.synchronize()
        return round(frames / (time.perf_counter() - t0), 1)
    graph = rate(lambda: sp())
    graph_h2d = rate(lambda: sp(d_host, c_host))
    with torch.no_grad():
        eager = rate(lambda: sp._run())
    for m in [ctx["rp"], ctx["dg"]] + ctx["dsams"]:
        m.train()
    return {"shape": f"{W}x{H}", "batch": 1, "dtype": "bf16" if ctx["dtype"] == torch.bfloat16 else "f32",
            "graph_img_s": graph, "graph_with_h2d_img_s": graph_h2d, "eager_img_s": eager, "frames": frames}


def cpu_threads():
    """Threads for the CPU baseline: every core of this process's affinity set, capped by the
    host's per-job CPU share when the environment states one (OMP_NUM_THREADS; 16 per GPU on
    the GPU box) — both numbers are reported."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cap = os.environ.get("OMP_NUM_THREADS")
    return aff, (min(aff, int(cap)) if cap and cap.isdigit() and int(cap) > 0 else aff)


def cpu_baseline(ctx, args):
    """BASELINE.md's CPU plan on the oracle (PyTorch-CPU fp32 + numpy restatement of the
    reference, tests-only code): 1 warm-up + 3 timed iterations each of
      (value) the hot-path training step, fwd+bwd (ratio predictor train mode, decomposition,
              DSAM x3, DGGM), 640x480, B=2 — the GPU workload on a bounded sample;
      (hot_path_eval_b8) hot path only, eval, 640x480, B=8 (BASELINE run 1);
      (c5_eval_b1) hot path only, eval, 1280x720, B=1 (BASELINE run 2)."""
    from oracle import dggm_pre, hot_path as hot_o
    from rgbd_amd import synthetic
    aff, threads = cpu_threads()
    torch.set_num_threads(threads)

    sd = {}
    for k, m in enumerate(ctx["dsams"]):
        sd.update({f"dsam{k}.{kk}": v.detach().float().cpu().clone().requires_grad_(v.is_floating_point())
                   for kk, v in m.state_dict().items()})
    sd.update({f"depth_gradient_injection.{kk}": v.detach().float().cpu().clone().requires_grad_(True)
               for kk, v in ctx["dg"].state_dict().items()})
    rp_sd = {f"ratio_predictor.{kk}": v.detach().cpu().clone() for kk, v in ctx["rp"].state_dict().items()}
    sd.update(rp_sd)

    def inputs(scenes, H, W):
        pv = torch.from_numpy(np.stack([np.concatenate([synthetic.rgbd_planes(s), dggm_pre.dggm_planes(s["depth_u8"])])
                                        for s in scenes]))
        sizes, h, w = [], -(-H // 4), -(-W // 4)
        for _ in range(4):
            sizes.append((h, w))
            h, w = -(-h // 2), -(-w // 2)
        g = torch.Generator().manual_seed(7)
        colors = [torch.randn((len(scenes), c, *sizes[k]), generator=g) for k, c in enumerate([96, 192, 384, 768])]
        return pv, colors

    def run(fn, n_img):
        fn()  # warm-up
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        dt = (time.perf_counter() - t0) / 3
        return round(n_img / dt, 4), round(dt, 3)

    H, W = args.height, args.width
    pv2, col2 = inputs(ctx["scenes"][:2], H, W)
    gouts = [g[:2].float().cpu() for g in ctx["gouts"]]

    def train_step():
        for v in sd.values():
            v.grad = None
        feats, _, _ = hot_o.hot_path_forward(col2, pv2, sd, training=True)
        torch.autograd.backward(feats, gouts)
    train, train_s = run(train_step, 2)

    scenes8 = [synthetic.make_scene(synthetic.scene_seed(3, i), H, W) for i in range(8)]
    pv8, col8 = inputs(scenes8, H, W)

    def eval8():
        with torch.no_grad():
            hot_o.hot_path_forward(col8, pv8, sd, training=False)
    ev8, ev8_s = run(eval8, 8)

    c5 = synthetic.make_scene(synthetic.scene_seed(5, 0), 720, 1280)
    pv5, col5 = inputs([c5], 720, 1280)

    def eval_c5():
        with torch.no_grad():
            hot_o.hot_path_forward(col5, pv5, sd, training=False)
    c5r, c5_s = run(eval_c5, 1)
    return {"value": train, "unit": "img/s", "cores": threads, "affinity_cores": aff, "kind": "port",
            "sample": f"2 images {W}x{H}, hot-path train step fwd+bwd (ratio predictor train mode, decomposition, "
                      f"DSAM x3, DGGM), oracle fp32 on {threads} thread(s); 1 warm-up + 3 timed iterations "
                      f"({train_s} s each)",
            "runs": {"hot_path_eval_b8_640x480_img_s": ev8, "hot_path_eval_b8_s_per_iter": ev8_s,
                     "c5_eval_b1_1280x720_img_s": c5r, "c5_eval_s_per_iter": c5_s}}


BF16_LOGIT_REL_TOL = 2e-2  # bf16 hot path: max |mask logit - reference| / max |reference logit|


def _codes_flipped(pv, r_ref, r_got, H, W):
    """Fraction of region-code cells (the three DSAM input resolutions) whose code differs between
    the decomposition at the reference's float32 ratio and at ``r_got`` — the discrete decisions a
    bf16 ratio flips.  Both sides run the HIP decomposition, which is bit-exact to the oracle at a
    given ratio (tests/test_gpu_bf16_parity.py), so the first side is the reference's decisions."""
    from rgbd_amd import ops
    sizes, h, w = [], -(-H // 4), -(-W // 4)
    for _ in range(3):
        sizes.append((h, w))
        h, w = -(-h // 2), -(-w // 2)
    ca, _ = ops.edsam_decompose(pv, r_ref, sizes)
    cb, _ = ops.edsam_decompose(pv, r_got, sizes)
    return [round(float((a != b).float().mean()), 6) for a, b in zip(ca, cb)]


G9_ATTN = REPO / "tests" / "golden" / "g9_attn_masks.npz"
FLIP_EXPLAIN_FACTOR = 4.0  # a flipped attention bit is explained when |ref logit| <= 4 x the call's |delta logit|


class ReferenceMasks:
    """The reference's attention masks at every mask-predictor call of the masked-attention
    decoder (tests/golden/g9_attn_masks.npz, made by importing the reference: make_golden.py
    attn; tag "g6": the G6 training forward's, stored in g6_grads.npz), for the G5 (320x240),
    G7 (640x480) or G6 (320x240, batch 2) input.  ``attach(model, force)`` hooks the model's mask
    predictor (HF modeling_mask2former.py:1896-1933 feeds its second output to the next decoder
    layer) and records per call the model's own mask (head 0 of every image) and its
    interpolated logits at the fixture's near-threshold positions; with ``force`` the reference's
    mask replaces the model's, so every decoder layer sees the reference's attention pattern and
    the remaining logit error is arithmetic only."""

    def __init__(self, tag, path=None):
        path = path or (REPO / "tests" / "golden" / "g6_grads.npz" if tag == "g6" else G9_ATTN)
        z = np.load(path, allow_pickle=False)
        self.input_sha = str(z[f"{tag}_input_sha"]) if f"{tag}_input_sha" in z else str(z["input_sha"])
        self.calls = []
        for c in range(int(z[f"{tag}_ncalls"])):
            shape = tuple(int(v) for v in z[f"{tag}_c{c}_shape"])
            shape = shape if len(shape) == 3 else (1,) + shape  # [B][Q][L]
            bits = np.unpackbits(z[f"{tag}_c{c}_bits"], count=int(np.prod(shape))).astype(bool).reshape(shape)
            self.calls.append({"mask": bits, "size": tuple(int(v) for v in z[f"{tag}_c{c}_size"]),
                               "near_idx": z[f"{tag}_c{c}_near_idx"], "near_val": z[f"{tag}_c{c}_near_val"]})

    def attach(self, model, force, rec):
        import torch.nn.functional as F
        mp = model.model.transformer_module.decoder.mask_predictor

        def hook(mod, inp, out):
            c = len(rec)
            if c >= len(self.calls):
                raise RuntimeError("more mask-predictor calls than the fixture holds")
            ref = self.calls[c]
            logits, attn = out[0], out[1]
            B = logits.shape[0]
            if B != ref["mask"].shape[0]:
                raise ValueError(f"ReferenceMasks: batch {B}, fixture {ref['mask'].shape[0]}")
            val = F.interpolate(logits.detach().float(), size=ref["size"], mode="bilinear",
                                align_corners=False).flatten(2).reshape(-1)
            near = torch.from_numpy(ref["near_idx"]).to(val.device)
            nh = attn.shape[0] // B
            rec.append((attn.view(B, nh, *attn.shape[1:])[:, 0].cpu().numpy(), val[near].cpu().numpy()))
            if not force:
                return None
            m = torch.from_numpy(ref["mask"]).to(attn.device)
            return logits, m[:, None].expand(B, nh, *m.shape[1:]).reshape(B * nh, *m.shape[1:]).contiguous()
        return mp.register_forward_hook(hook)

    def flips(self, rec, deltas=None, upto_first=False):
        """Per call: flipped bits of the model's own masks against the reference's, and how many
        are unexplained — the reference logit not within FLIP_EXPLAIN_FACTOR x that call's
        |delta logit| (``deltas``: the forced run's per-call max |own - ref| over the fixture's
        near-threshold positions; default this run's).  ``upto_first``: only up to the first
        call with a flip (later calls of an unforced run inherit that flip's consequences)."""
        total, unexplained, first = 0, 0, None
        own_deltas = []
        for c, (own, own_near) in enumerate(rec):
            ref = self.calls[c]
            own_deltas.append(float(np.abs(own_near - ref["near_val"]).max()) if own_near.size else 0.0)
        deltas = own_deltas if deltas is None else deltas
        for c, (own, _) in enumerate(rec):
            ref = self.calls[c]
            idx = np.flatnonzero((own != ref["mask"]).ravel())
            if not idx.size:
                continue
            first = c if first is None else first
            pos = np.minimum(np.searchsorted(ref["near_idx"], idx), max(ref["near_idx"].size - 1, 0))
            vals = np.full(idx.size, np.inf)
            if ref["near_idx"].size:
                hit = ref["near_idx"][pos] == idx
                vals[hit] = np.abs(ref["near_val"][pos[hit]])
            total += int(idx.size)
            unexplained += int((vals > FLIP_EXPLAIN_FACTOR * deltas[c]).sum())
            if upto_first:
                break
        return {"flips": total, "unexplained": unexplained, "first_call": first,
                "max_delta_logit": max(own_deltas) if own_deltas else 0.0, "deltas": own_deltas}


def parity(dev, dtype=torch.float32, ratio_fp32=False, fixture="g7", colour_bf16=False, out_bf16=False):
    """BASELINE.json's second metric: the full drop-in model (HF Swin / pixel decoder /
    transformer decoder around the HIP hot path, f1/f2 kernels installed), B=1, eval,
    deterministic weights, against the reference CPU run committed as
    tests/golden/g7_model640.npz (640x480) or g5_model.npz (320x240, ``fixture`` "g5"), made by
    tests/golden/make_golden.py.  The 10-channel input is assembled on the GPU by K1 from the
    scene's u8 planes; its sha256 must equal the one the fixture was generated from.

    Two runs: the model as is, and the same with the reference's attention masks forced into
    every masked-attention decoder layer (``ReferenceMasks``, G9) — the forced run's error is
    arithmetic only; the unforced run additionally carries every attention bit the arithmetic
    flips across the sigmoid(logit) < 0.5 binarisation (counted: ``attention_flips``).

    ``dtype`` bfloat16: the hot path (ratio predictor, DSAM, DGGM) in bf16 as the bench runs it —
    the ratio, and so the window decisions, come from the bf16 ratio predictor; the HF modules
    around it stay float32.  ``ratio_fp32``: the ratio predictor alone in float32 (the
    reference's ratio, so the reference's window decisions): what remains is the error of the
    bf16 DSAM / DGGM arithmetic.  ``colour_bf16``: the float32 hot path fed with the Swin colour
    maps rounded to bfloat16 (what the bf16 hot path takes in): the share of the bf16 error that
    is the rounding of its inputs alone; ``out_bf16`` in addition rounds the hot path's four
    output features to bfloat16 (what the bf16 hot path hands the float32 pixel decoder)."""
    import hashlib
    from rgbd_amd import init as winit, ops, synthetic
    from rgbd_amd.config import standard_config
    from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
    cid, H, W, path = {"g7": (7, 480, 640, "g7_model640.npz"), "g5": (1, 240, 320, "g5_model.npz")}[fixture]
    gz = np.load(REPO / "tests" / "golden" / path, allow_pickle=False)
    sc = synthetic.make_scene(synthetic.scene_seed(cid, 0), H, W)
    pv = ops.assemble_pixel_values(torch.from_numpy(sc["depth_u8"][None]).to(dev),
                                   torch.from_numpy(sc["rgb_u8"][None]).contiguous().to(dev))
    sha_ok = hashlib.sha256(pv.cpu().numpy().tobytes()).hexdigest() == str(gz["input_sha"])
    torch.manual_seed(0)
    m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
    winit.init_deterministic(m)
    m = m.to(dev).eval().set_compute_dtype(dtype)
    rp = m.model.pixel_level_module.ratio_predictor
    if ratio_fp32:
        rp.compute_dtype = torch.float32
    if colour_bf16 or out_bf16:
        plm = m.model.pixel_level_module
        hpf = plm.hot_path_features
        rnd = (lambda ts: [t.to(torch.bfloat16).float() for t in ts])

        def patched(pv_, colors, **kw):
            feats = hpf(pv_, rnd(colors) if colour_bf16 else list(colors), **kw)
            return rnd(feats) if out_bf16 else feats
        plm.hot_path_features = patched
    refm = ReferenceMasks(fixture)
    runs = {}
    for force in (False, True):
        rec = []
        h = refm.attach(m, force, rec)
        try:
            with torch.no_grad():
                out = m(pixel_values=pv)
        finally:
            h.remove()
        runs[force] = (out, rec)
    with torch.no_grad():
        ratio = rp(pv[:, 3:6])
    if fixture == "g7":
        ref, pick = gz["mask_val"], gz["mask_idx"]
    else:
        ref, pick = gz["mask_logits"].ravel(), slice(None)

    def err_of(out):
        ml = out.masks_queries_logits.float().cpu().numpy().ravel()
        return (float(np.abs(ml[pick] - ref).max()),
                float(np.abs(out.class_queries_logits.float().cpu().numpy() - gz["class_logits"]).max()))
    err, cls = err_of(runs[False][0])
    ferr, fcls = err_of(runs[True][0])
    forced = refm.flips(runs[True][1])
    unforced = refm.flips(runs[False][1], deltas=forced["deltas"])
    first = refm.flips(runs[False][1], deltas=forced["deltas"], upto_first=True)
    rrel = float(np.abs(ratio.float().cpu().numpy() - gz["ratio"]).max() / np.abs(gz["ratio"]).max())
    flips = None
    if dtype != torch.float32:
        r_ref = torch.from_numpy(np.asarray(gz["ratio"], np.float32).reshape(-1, 1)).to(dev)
        flips = _codes_flipped(pv, r_ref, ratio.float().reshape(-1, 1), H, W)
    del m
    torch.cuda.empty_cache()
    res = {"mask_logit_max_abs_err": err, "class_logit_max_abs_err": cls, "ratio_rel_err": rrel,
           "mask_logit_max_abs_err_masks_forced": ferr, "class_logit_max_abs_err_masks_forced": fcls,
           "attention_flips": {"unforced_run": unforced["flips"], "forced_run_own_masks": forced["flips"],
                               "first_flipped_call": first["first_call"],
                               "first_call_unexplained": first["unexplained"],
                               "max_delta_logit_forced": forced["max_delta_logit"],
                               "explain_factor": FLIP_EXPLAIN_FACTOR},
           "input_sha_match": sha_ok, "dtype": "f32" if dtype == torch.float32 else "bf16", "shape": f"{W}x{H}",
           "fixture": f"tests/golden/{path}", "sampled_logits": int(np.asarray(ref).size),
           "note": ("masks_forced: the reference's attention masks (tests/golden/g9_attn_masks.npz) injected into "
                    "every masked-attention decoder layer, so the error is arithmetic only; attention_flips: bits "
                    "of the model's own masks that differ from the reference's (forced run: each call on the "
                    "reference's inputs; first_call_unexplained: flips of the unforced run's first flipped call "
                    "whose reference logit lies beyond explain_factor x the forced run's |delta logit|)")}
    if colour_bf16 or out_bf16:
        scale = float(np.abs(ref).max())
        res.update(mask_logit_max_rel_err=err / scale, mask_logit_max_rel_err_masks_forced=ferr / scale,
                   note_attrib=("float32 hot path" + (" on bf16-rounded colour maps" if colour_bf16 else "") +
                                (" with its outputs rounded to bf16" if out_bf16 else "") +
                                ": that share of the bf16 error"))
    elif dtype == torch.float32:
        res["tolerance"] = 1e-3
    else:
        scale = float(np.abs(ref).max())
        res.update(mask_logit_max_rel_err=err / scale, mask_logit_max_rel_err_masks_forced=ferr / scale,
                   tolerance_rel=BF16_LOGIT_REL_TOL, region_code_cells_flipped=flips,
                   ratio_predictor="float32 (reference ratio injected)" if ratio_fp32 else "bf16",
                   note_bf16="bf16 hot path (ratio predictor, DSAM, DGGM) in the float32 HF model; rel = max-abs-err / "
                             "max |reference logit|; region_code_cells_flipped = fraction of DSAM region-code cells "
                             "(3 input scales) whose code differs from the decomposition at the reference ratio")
    return res


def full_model(dev, B=8, H=480, W=640, steps=5, warmup=2, graph=True):
    """The whole drop-in model (CustomMask2FormerForUniversalSegmentation v0.4.0: Swin-T, the hot
    path, the MSDeformAttn pixel decoder, the masked-attention decoder, the Hungarian-matched
    loss with 9 auxiliary outputs; custom_model.py:37-53), one bf16-autocast training step
    (forward with labels, backward, the HF Trainer's AdamW) on synthetic NYUv2-shaped scenes with
    their instance masks, deterministic random-init weights (48 labels).  Timed eagerly and as
    one captured HIP graph (train_graph.CapturedTrainStep, at most two concurrent branches);
    ``img_s`` is the captured step when the capture succeeds.  ``kernel_ms`` = the five kernels
    with the most device time in one eager step (torch.profiler over the HIP runtime)."""
    from rgbd_amd import init as winit, ops, synthetic
    from rgbd_amd.config import standard_config
    from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
    from rgbd_amd.optim import HF_TRAINER_ADAMW, HipAdamW
    from rgbd_amd.train_graph import CapturedTrainStep
    scenes = [synthetic.make_scene(synthetic.scene_seed(4, i), H, W) for i in range(B)]
    depth = torch.from_numpy(np.stack([s["depth_u8"] for s in scenes])).to(dev)
    rgb = torch.from_numpy(np.stack([s["rgb_u8"] for s in scenes])).contiguous().to(dev)
    mask_labels = [torch.from_numpy(s["masks"].astype(np.float32)).to(dev) for s in scenes]
    class_labels = [torch.from_numpy(s["classes"]).to(dev) for s in scenes]
    torch.manual_seed(0)
    m = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
    winit.init_deterministic(m)
    m.set_compute_dtype(torch.bfloat16).to(dev).train()
    opt = HipAdamW([p for p in m.parameters() if p.requires_grad], **HF_TRAINER_ADAMW)

    def fb():
        pv = ops.assemble_pixel_values(depth, rgb)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m(pixel_values=pv, mask_labels=mask_labels, class_labels=class_labels)
        out.loss.backward()
        return out.loss.detach()

    def step():
        loss = fb()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    def timed(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            out = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n, out
    for _ in range(warmup):
        step()
    dt_eager, loss = timed(step, steps)
    res = {"workload": "whole drop-in model training step (Swin-T + hot path + pixel decoder + masked-attention "
                       "decoder + Hungarian-matched loss, 9 aux outputs, AdamW), bf16 autocast",
           "batch": B, "shape": f"{W}x{H}", "steps": steps, "eager_img_s": round(B / dt_eager, 2),
           "eager_ms_per_step": round(dt_eager * 1e3, 2), "loss": round(float(loss), 4)}
    dt, how = dt_eager, "eager"
    if graph:
        try:
            cs = CapturedTrainStep(fb, opt, warmup=1)
            for _ in range(warmup):
                cs()
            dt_graph, loss_g = timed(cs, steps)
            m.model.pixel_level_module.check_statuses()
            res.update({"graph_img_s": round(B / dt_graph, 2), "graph_ms_per_step": round(dt_graph * 1e3, 2),
                        "graph_branches": cs.width, "graph_loss": round(float(loss_g), 4)})
            dt, how = dt_graph, "captured graph"
            del cs
        except Exception as e:  # reported; the eager number stands
            res["graph_error"] = repr(e)[:300]
    res["img_s"], res["ms_per_step"] = round(B / dt, 2), round(dt * 1e3, 2)
    res["timed"] = how
    try:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            step()
            torch.cuda.synchronize()
        tot, cnt = {}, {}
        for ev in prof.events():
            if ev.device_type.name == "CUDA" or getattr(ev, "device_time", 0):
                t = getattr(ev, "device_time", None) or getattr(ev, "cuda_time", 0)
                if t:
                    tot[ev.name] = tot.get(ev.name, 0.0) + t
                    cnt[ev.name] = cnt.get(ev.name, 0) + 1
        top = sorted(tot.items(), key=lambda kv: -kv[1])[:5]
        res.update({"kernel_ms_top5": {k[:90]: round(v / 1e3, 3) for k, v in top},
                    "launches_top5": {k[:90]: cnt[k] for k, _ in top},
                    "kernel_ms_total": round(sum(tot.values()) / 1e3, 2), "launches": int(sum(cnt.values()))})
    except Exception as e:  # the profiler is a report, not the measurement
        res["profiler_error"] = repr(e)[:200]
    del m, opt
    torch.cuda.empty_cache()
    return res


def read_timings(L):
    """{scope: (total ms, launches)} of the HIP-event timers since rgbd_timing_enable(1)."""
    cnt = ctypes.c_int(0)
    ms = {}
    for name in ("rp_conv3x3", "rp_chain", "dsam_fwd", "dsam_dx", "dsam_wgrad", "decompose", "dggm_fwd",
                 "dggm_bwd", "assemble"):
        tot = L.rgbd_timing_read(name.encode(), ctypes.byref(cnt))
        ms[name] = (tot, cnt.value)
    return ms


def kernel_fractions(ms, ctx, B, H, W, step_ms, world, n_steps):
    """K5 achieved rates (reference-algorithmic and executed FLOPs) and the whole step's
    t_ideal / t_measured from the HIP-event timings of the ``n_steps`` timed eager
    steps (the timers run over exactly those steps)."""
    P = B * H * W
    ho = [(-(-H // 4) + 1) // 2, (-(-H // 8) + 1) // 2, (-(-H // 16) + 1) // 2]
    wo = [(-(-W // 4) + 1) // 2, (-(-W // 8) + 1) // 2, (-(-W // 16) + 1) // 2]
    conv = [2 * 9 * ci * co * B * ho[k] * wo[k] for k, (ci, co) in enumerate(DSAM_CH)]  # one 3x3 s2 conv
    k5_ms = (ms["dsam_fwd"][0] + ms["dsam_dx"][0] + ms["dsam_wgrad"][0]) / n_steps
    k5_exec = 3 * sum(conv) - conv[0]           # merged filter: fwd x3 + dX (dsam1, dsam2) + dW x3
    k5_alg = (K5_FWD_FLOP_PER_PX + K5_BWD_FLOP_PER_PX) * P
    per = {k: round(v[0] / max(v[1], 1), 4) for k, v in ms.items()}
    n_params = sum(p.numel() for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters())
    t_ideal = (K4_FLOP_PER_PX * P / (MFMA_BF16_PEAK_TFLOPS * 1e12)
               + (K5_FWD_FLOP_PER_PX + K5_BWD_FLOP_PER_PX) * P / (MFMA_BF16_PEAK_TFLOPS * 1e12)
               + (K1_BYTES_PER_PX + K2_BYTES_PER_PX + K3_BYTES_PER_PX) * P / (HBM_PEAK_GBS * 1e9)
               + ADAMW_BYTES_PER_PARAM * n_params / (HBM_PEAK_GBS * 1e9)) * 1e3
    return ms, per, {
        "k5_dsam": {"ms_per_step": round(k5_ms, 4),
                    "algorithmic_tflop_s": round(k5_alg / (k5_ms * 1e-3) / 1e12, 1),
                    "executed_tflop_s": round(k5_exec / (k5_ms * 1e-3) / 1e12, 1),
                    "frac_algorithmic": round(k5_alg / (k5_ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
                    "frac_executed": round(k5_exec / (k5_ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
                    "note": "algorithmic = reference FLOPs (4 masked convs + projection per DSAM); executed = one "
                            "code-merged filter per output pixel and tap"},
        "whole_step": {"t_ideal_ms": round(t_ideal, 4), "t_measured_ms": round(step_ms, 4),
                       "frac": round(t_ideal / step_ms, 4),
                       "note": "t_ideal = K4+K5 FLOPs at bf16 MFMA peak + K1/K2/K3/AdamW bytes at HBM peak "
                               "(SURVEY §8(d)); per rank" + ("" if world == 1 else ", collectives excluded")},
    }


# ------------------------------------------------------------------ main
def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.launcher_selftest:
        return launcher_selftest()
    # stdout carries exactly the one JSON line: everything else the process (and the libraries it
    # loads: RCCL prints its version banner on stdout at communicator init) writes to fd 1 goes
    # to stderr
    sys.stdout.flush()
    line_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ddp = world > 1 if args.ddp is None else bool(args.ddp)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if ddp:
        if world == 1:  # one rank without a launcher: a local rendezvous
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    from rgbd_amd import _lib
    from rgbd_amd.distributed import broadcast_parameters
    L = _lib.lib()
    ctx = build(args, dev, rank)
    if ddp:  # DDP construction: rank 0's parameters and buffers everywhere
        broadcast_parameters([ctx["rp"], ctx["dg"]] + ctx["dsams"])
    step = make_step(ctx, world, ddp=ddp)
    # eager pass: per-kernel HIP-event timing over its timed steps only
    dt_eager = timed(step, args.steps, args.warmup, world, on_start=lambda: L.rgbd_timing_enable(1), ddp=ddp)
    timings = read_timings(L)
    L.rgbd_timing_enable(0)
    use_graph = bool(args.graph) and not ddp
    # the line's number: the captured step at N = 1; at N > 1 the eager step timed again with the
    # per-kernel HIP events off (they cost ~0.3 ms of host time per step: 3.23 vs 2.92 ms,
    # profiles/r05_v2/prof_host.txt)
    dt = (timed(make_step(ctx, world, graph=True), args.steps, args.warmup, world) if use_graph
          else timed(step, args.steps, 1, world, ddp=ddp))
    # the same captured step software-pipelined across batches (make_parts ``pipeline``)
    dt_pipe = timed(make_step(ctx, world, graph=True, pipeline=True), args.steps, args.warmup, world) \
        if use_graph and args.pipeline_report else None
    # N > 1 (RCCL): the step with its collectives inside one HIP graph (serial exchange after the
    # backward), timed beside the eager overlapped step; the line takes the faster of the two
    dt_capt, capt_why, dt_capt_ov, capt_ov_why = None, None, None, None
    if ddp and args.graph and dist.get_backend() == "nccl":
        for form in (True, "overlap"):
            cstep, why = captured_ddp_step(ctx, world, dev, serial_ddp=form)
            dtc = None
            if cstep is not None:
                dtc = timed(cstep, args.steps, args.warmup, world, ddp=ddp)
                for p in cstep.params:  # the graph's gradient tensors: not the next eager step's
                    p.grad = None
                del cstep
            if form is True:
                dt_capt, capt_why = dtc, why
            else:
                dt_capt_ov, capt_ov_why = dtc, why
    dt_overlap_eager = dt if ddp else None
    ddp_form = "eager, all-reduces overlapped" if ddp else None
    for dtc, form in ((dt_capt, "captured, all-reduces after the backward"),
                      (dt_capt_ov, "captured, all-reduces overlapped")):
        if dtc is not None and dtc < dt:
            dt, use_graph, ddp_form = dtc, True, form
    # the same eager step with no collective on every rank at once: the line's own scaling reference
    dt_local = timed(make_step(ctx, 1), args.steps, args.warmup, world, ddp=ddp) if ddp else None
    B = args.batch
    step_ms = dt / args.steps * 1e3
    raw, per, fracs = kernel_fractions(timings, ctx, B, args.height, args.width, step_ms, world, args.steps)
    conv_ms, conv_launches = raw["rp_conv3x3"]
    value = B * world * args.steps / dt
    inf = None
    if args.inference:
        istep = make_step(ctx, world, inference=True)
        idt = timed(istep, args.steps, args.warmup, world, ddp=ddp)
        inf = round(B * world * args.steps / idt, 2)
        for m in [ctx["rp"], ctx["dg"]] + ctx["dsams"]:
            m.train()
    conv_avg_ms = conv_ms / max(conv_launches, 1)
    flop = CONV5_FLOP_PER_PX * B * args.height * args.width
    achieved = flop / (conv_avg_ms * 1e-3) / 1e12
    default_shape = (B, args.height, args.width, args.dtype) == (8, 480, 640, "bf16")
    traffic = pmc_traffic(CONV5_KERNEL, default_shape)
    prof = profile_avg_ns(CONV5_KERNEL, default_shape)
    achieved_prof = None if prof is None else flop / (prof[0] * 1e-9) / 1e12
    out = {
        "metric": "NYUv2 640x480 RGB-D img/s (fwd+bwd) of the DGGM+E-DSAM hot path",
        "value": round(value, 2),
        "unit": "img/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.dtype == "bf16" else "f32",
        "data": "synthetic (seeded NYUv2-shaped RGB-D scenes; deterministic random-init weights)",
        "config": {"workload": f"hot-path train step (ratio predictor train-mode + decomposition + DSAM x3 + "
                               f"DGGM, fwd+bwd + AdamW), {args.width}x{args.height}, batch {B}/GPU",
                   "global_batch": B * world, "height": args.height, "width": args.width,
                   "parallelism": f"dp{world}"},
        "distributed": {"world_size": dist.get_world_size() if ddp else 1,
                        "backend": (dist.get_backend() if ddp else None),
                        "collectives_per_step": ("3 all-reduce (grad buckets dsam2, dsam1, dsam0+DGGM; async under "
                                                 "the backward in the eager step, after it in the captured one) + "
                                                 "2 broadcasts (ratio-predictor BN buffers)") if ddp else None},
        "optimizer": ("AdamW (lr 1e-5, weight_decay 0.0, betas (0.9, 0.999), eps 1e-8: HF TrainingArguments defaults) on the hot-path parameters, stepped inside the backward; "
                      "no gradient-norm clip: the reference Trainer's max_grad_norm=1.0 clips the norm of the whole "
                      "model's gradients (37.3 M parameters, most of them outside this path)"),
        "graph": use_graph,
        "eager_img_s": round(B * world * args.steps / dt_eager, 2),
        "eager_note": ("eager_img_s: the eager pass with the per-kernel HIP events on (the kernel_ms figures); at "
                       "N > 1 the line's value is the eager step timed again with them off"),
        "pipelined_img_s": None if dt_pipe is None else round(B * world * args.steps / dt_pipe, 2),
        "pipelined_note": ("the captured step with the next batch's ratio predictor on a second stream beside this "
                           "batch's DSAM / DGGM forward, backward and AdamW (bitwise the sequential schedule's "
                           "parameters: the predictor is forward-only and frozen, Q2)"),
        "scaling_baseline_img_s": (None if dt_local is None else round(B * world * args.steps / dt_local, 2)),
        "scaling_baseline_note": ("N > 1: scaling_baseline_img_s = the eager step with no all-reduce / broadcast on "
                                  "every rank at once, so value / scaling_baseline_img_s is the cost of the "
                                  "data-parallel exchange; the N=1 line replays a HIP graph (its eager_img_s is the "
                                  "eager N=1 rate)"),
        "ddp_form": ddp_form,
        "ddp_captured_img_s": None if dt_capt is None else round(B * world * args.steps / dt_capt, 2),
        "ddp_captured_overlap_img_s": None if dt_capt_ov is None else round(B * world * args.steps / dt_capt_ov, 2),
        "ddp_overlapped_eager_img_s": (None if dt_overlap_eager is None
                                       else round(B * world * args.steps / dt_overlap_eager, 2)),
        "ddp_captured_note": ("N > 1 over RCCL, three forms of the same step, value the fastest (ddp_form): captured "
                              "with its collectives (BN-buffer broadcasts, one all-reduce per gradient bucket after "
                              "the backward, then AdamW; ddp_captured_img_s); captured with the backward on one "
                              "stream and the all-reduces + AdamW steps overlapped beside it "
                              "(ddp_captured_overlap_img_s); eager with the all-reduces overlapped with the "
                              "backward's two streams (ddp_overlapped_eager_img_s)"
                              + ("" if capt_why is None else f"; serial form not captured: {capt_why}")
                              + ("" if capt_ov_why is None else f"; overlapped form not captured: {capt_ov_why}")),
        "inference_img_s": inf,
        "kernel_ms": per,
        "roofline": {"bound": "mfma", "kernel": "k_rp_conv5_v4 (3x3 128->256, custom_model.py:1413)",
                     "achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4),
                     "events_avg_us": round(conv_avg_ms * 1e3, 2), "events_launches": conv_launches,
                     "frac_profile": None if achieved_prof is None else round(achieved_prof / MFMA_BF16_PEAK_TFLOPS, 4),
                     "profile_avg_us": None if prof is None else round(prof[0] / 1e3, 2),
                     "profile_source": None if prof is None else prof[1],
                     "profile_vs_events": None if prof is None else round(prof[0] / 1e6 / conv_avg_ms, 4),
                     "traffic": None if traffic is None else round(traffic[0]),
                     "traffic_unit": "bytes/launch", "traffic_source": None if traffic is None else traffic[1],
                     "algorithmic_bytes": (128 + 256) * 2 * B * args.height * args.width,
                     "timing": ("achieved / frac: conv5's algorithmic FLOP per launch over its average duration "
                                "measured in THIS run by HIP events around each conv5 launch on its stream over the "
                                "eager timed steps (events_launches launches, no profiler attached); frac_profile: "
                                "the same FLOP over the average in the committed rocprofv3 trace of this tree's "
                                "bench step (profile_source, bench.EVIDENCE_DIR; the profiler costs the kernel a "
                                "few per cent, DESIGN.md §5.8.1); profile_vs_events = the two averages' ratio")},
        "kernels": fracs,
    }
    if rank == 0 and args.parity:
        out["parity"] = parity(dev)
        out["parity"]["bf16"] = parity(dev, torch.bfloat16)
        # the same with the reference's float32 ratio: the bf16 error with no flipped decision
        out["parity"]["bf16_ratio_fp32"] = parity(dev, torch.bfloat16, ratio_fp32=True)
        # G5 (C1's 320x240) beside G7, fp32
        out["parity"]["g5_320x240"] = parity(dev, fixture="g5")
        # bf16 error attribution: the float32 hot path on bf16-rounded colour maps
        out["parity"]["bf16_attrib_colour_rounding"] = parity(dev, fixture="g7", colour_bf16=True)
        out["parity"]["bf16_attrib_colour_and_output_rounding"] = parity(dev, fixture="g7", colour_bf16=True,
                                                                        out_bf16=True)
    if rank == 0 and world == 1 and args.c5_stream:
        out["c5_stream"] = c5_stream(ctx)
    if rank == 0 and world == 1 and args.full_model:
        out["full_model"] = full_model(dev)
    if rank == 0 and world == 1 and args.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(ctx, args)
    if rank == 0:
        print(json.dumps(out), file=line_out, flush=True)
    if ddp:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
