"""Benchmark of the MI355X-native DGGM + E-DSAM hot path (BASELINE.json metric).

One step = one training pass of the v0.4.0 pixel-level hot path over
a batch of synthetic NYUv2-shaped frames (640x480, 8 images per GPU, bf16 MFMA):
  u8 RGB + u8 depth (resident in HBM)
  -> 10-channel pixel_values incl. DGGM Sobel planes         (K1, rgbd_assemble_pixel_values)
  -> ratio predictor, train-mode BatchNorm + dropout          (K4, rgbd_ratio_forward)
  -> depth decomposition once per image                       (K3, rgbd_edsam_decompose)
  -> DSAM x3 masked implicit GEMMs (cascade) + DGGM + sum     (K5, K2)
  -> backward from a fixed synthetic upstream gradient of the 4 backbone features:
     DSAM dW/db/dX cascade + DGGM dW/db                        (K5, K2)
  -> (N > 1) RCCL all-reduce of the hot-path parameter gradients (DDP semantics)
  -> AdamW step on the hot-path parameters (HF Trainer's optimizer; lr 1e-5 constant,
     mask2former/config.json), so every step re-packs the changed DSAM filters.
The Swin encoder / pixel decoder / transformer decoder are outside the hot path (SURVEY §8(f)
"next"); their colour-feature inputs are synthetic tensors of the Swin-T shapes.

Prints ONE JSON line (rank 0).  ``value`` = images processed by all ranks / max-over-ranks
time.  ``roofline`` is for the dominant kernel (the ratio predictor's 3x3 128->256 conv,
k_rp_conv3x3), timed with HIP events on its launch stream inside the timed region.
``cpu_baseline`` = the oracle (PyTorch-CPU fp32 restatement of the reference, tests-only
code) on a bounded sample of the same workload on this host's cores.
"""
import argparse
import ctypes
import json
import os
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
CONV5_KERNEL = "k_rp_conv3x3_v3"


def pmc_traffic(kernel, default_shape):
    """HBM bytes per launch of ``kernel`` from the newest committed PMC table
    (profiles/*/pmc_traffic.json, written by tools/gpu_traffic.sh + tools/traffic_table.py over
    this bench's default step: FETCH_SIZE doubled per the gfx950 correction, plus WRITE_SIZE).
    rocprofv3 cannot run inside this process, so the counters come from their own passes; the
    value is null for a non-default shape or when no table holds this kernel."""
    if not default_shape:
        return None
    best = None
    for path in sorted((REPO / "profiles").glob("*/pmc_traffic.json")):
        for key, row in json.loads(path.read_text()).items():
            if key.split(" grid=")[0] == kernel and "hbm_bytes" in row:
                best = (row["hbm_bytes"], str(path.relative_to(REPO)))
    return best


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on the host (rank 0, N=1)")
    ap.add_argument("--cpu-sample", type=int, default=1, help="images in the bounded CPU sample")
    ap.add_argument("--inference", type=int, default=1, help="also report forward-only img/s")
    ap.add_argument("--c5-stream", type=int, default=1,
                    help="also report the C5 RealSense 1280x720 B=1 streaming inference rate (rank 0, N=1)")
    return ap.parse_args(argv)


def build(args, dev):
    from rgbd_amd import init as winit, synthetic
    from rgbd_amd.modules import DSAModule, DepthGradientInjectionResidual, EnhancedDepthImageRatioPredictor
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    pre = "model.pixel_level_module."
    rp = EnhancedDepthImageRatioPredictor(3)
    winit.init_deterministic(rp, prefix=pre + "ratio_predictor.")
    dsams = []
    for k, (ci, co) in enumerate([(96, 192), (192, 384), (384, 768)]):
        m = DSAModule(ci, co)
        winit.init_deterministic(m, prefix=f"{pre}dsam{k}.")
        dsams.append(m)
    dg = DepthGradientInjectionResidual([96, 192, 384, 768], 3)
    winit.init_deterministic(dg, prefix=pre + "depth_gradient_injection.")
    for m in [rp, dg] + dsams:
        m.compute_dtype = dtype
        m.to(dev).train()
    B, H, W = args.batch, args.height, args.width
    rank = int(os.environ.get("RANK", "0"))
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


def make_step(ctx, world, inference=False):
    from rgbd_amd import ops
    from rgbd_amd.hot_path import hot_path
    from rgbd_amd.distributed import OverlappedGradReducer, hot_path_grad_groups
    params = [p for m in ctx["dsams"] + [ctx["dg"]] for p in m.parameters()]
    # DDP: one bucket per DSAM module, all-reduced asynchronously while the backward cascade runs
    reducer = OverlappedGradReducer(hot_path_grad_groups(ctx["dsams"], ctx["dg"])) if world > 1 else None
    hook = None if reducer is None else reducer.ready
    opt = None if inference else torch.optim.AdamW(params, lr=1e-5, fused=True)

    def step():
        pv = ops.assemble_pixel_values(ctx["depth_u8"], ctx["rgb_u8"])
        if inference:
            with torch.no_grad():
                ratio = ctx["rp"](pv[:, 3:6])
                return hot_path(pv, ratio, ctx["colors"], ctx["dsams"], ctx["dg"], dtype=ctx["dtype"])
        ratio = ctx["rp"](pv[:, 3:6])
        feats = hot_path(pv, ratio, ctx["colors"], ctx["dsams"], ctx["dg"], dtype=ctx["dtype"], grad_hook=hook)
        torch.autograd.backward(feats, ctx["gouts"])
        if reducer is not None:  # DDP gradient exchange of the hot-path parameters (RCCL over xGMI)
            reducer.finish()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return feats
    return step


def timed(step, steps, warmup, world):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


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
    return {"shape": f"{W}x{H}", "batch": 1, "dtype": "bf16" if ctx["dtype"] == torch.bfloat16 else "f32",
            "graph_img_s": graph, "graph_with_h2d_img_s": graph_h2d, "eager_img_s": eager, "frames": frames}


def cpu_baseline(ctx, args):
    """Oracle (PyTorch-CPU fp32 restatement, tests-only code) on a bounded sample: the same
    training hot path (ratio predictor train mode + decomposition + DSAM x3 + DGGM, forward and
    backward) for ``--cpu-sample`` images at the same resolution."""
    from oracle import dggm_pre, hot_path as hot_o
    from rgbd_amd import synthetic
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = max(1, min(threads, 16))
    torch.set_num_threads(threads)
    n = args.cpu_sample
    H, W = args.height, args.width
    pv = []
    for s in ctx["scenes"][:n]:
        pv.append(np.concatenate([synthetic.rgbd_planes(s), dggm_pre.dggm_planes(s["depth_u8"])]))
    sd = {}
    pre = ""
    for k, m in enumerate(ctx["dsams"]):
        sd.update({f"dsam{k}.{kk}": v.detach().float().cpu().clone().requires_grad_(v.is_floating_point())
                   for kk, v in m.state_dict().items()})
    sd.update({f"depth_gradient_injection.{kk}": v.detach().float().cpu().clone().requires_grad_(True)
               for kk, v in ctx["dg"].state_dict().items()})
    sd.update({f"ratio_predictor.{kk}": v.detach().cpu().clone() for kk, v in ctx["rp"].state_dict().items()})
    colors = [c[:n].float().cpu() for c in ctx["colors"]]
    gouts = [g[:n].float().cpu() for g in ctx["gouts"]]
    pvt = torch.from_numpy(np.stack(pv))
    t0 = time.perf_counter()
    feats, _, _ = hot_o.hot_path_forward(colors, pvt, sd, prefix=pre, training=True)
    torch.autograd.backward(feats, gouts)
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 4), "unit": "img/s", "cores": threads, "kind": "port",
            "sample": f"{n} image(s) {W}x{H}, full hot-path train step (fwd+bwd), oracle fp32 on {threads} thread(s)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from rgbd_amd import _lib
    L = _lib.lib()
    ctx = build(args, dev)
    step = make_step(ctx, world)
    # timed region, kernel timing on for the dominant kernel
    L.rgbd_timing_enable(1)
    dt = timed(step, args.steps, args.warmup, world)
    cnt = ctypes.c_int(0)
    conv_ms = L.rgbd_timing_read(b"rp_conv3x3", ctypes.byref(cnt))
    conv_launches = cnt.value
    others = {}
    for name in ("rp_chain", "dsam_fwd", "dsam_dx", "dsam_wgrad", "decompose", "dggm_fwd", "dggm_bwd", "assemble"):
        ms = L.rgbd_timing_read(name.encode(), ctypes.byref(cnt))
        others[name] = round(ms / max(cnt.value, 1), 4)
    L.rgbd_timing_enable(0)
    B = args.batch
    imgs = B * world * args.steps
    value = imgs / dt
    inf = None
    if args.inference:
        istep = make_step(ctx, world, inference=True)
        idt = timed(istep, args.steps, args.warmup, world)
        inf = round(B * world * args.steps / idt, 2)
    conv_avg_ms = conv_ms / max(conv_launches, 1)
    flop = CONV5_FLOP_PER_PX * B * args.height * args.width
    achieved = flop / (conv_avg_ms * 1e-3) / 1e12
    traffic = pmc_traffic(CONV5_KERNEL, (B, args.height, args.width, args.dtype) == (8, 480, 640, "bf16"))
    out = {
        "metric": "NYUv2 640x480 RGB-D img/s (fwd+bwd) of the DGGM+E-DSAM hot path",
        "value": round(value, 2),
        "unit": "img/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.dtype == "bf16" else "f32",
        "data": "synthetic (seeded NYUv2-shaped RGB-D scenes; deterministic random-init weights)",
        "config": {"workload": f"hot-path train step (ratio predictor train-mode + decomposition + DSAM x3 + "
                               f"DGGM, fwd+bwd + AdamW), {args.width}x{args.height}, batch {B}/GPU",
                   "global_batch": B * world, "height": args.height, "width": args.width,
                   "parallelism": f"dp{world}"},
        "inference_img_s": inf,
        "kernel_ms": dict(rp_conv3x3=round(conv_avg_ms, 4), **others),
        "roofline": {"bound": "mfma", "kernel": "k_rp_conv3x3 (3x3 128->256, custom_model.py:1413)",
                     "achieved": round(achieved, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4),
                     "traffic": None if traffic is None else round(traffic[0]),
                     "traffic_unit": "bytes/launch", "traffic_source": None if traffic is None else traffic[1],
                     "algorithmic_bytes": (128 + 256) * 2 * B * args.height * args.width},
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(ctx, args)
    if rank == 0 and world == 1 and args.c5_stream:
        out["c5_stream"] = c5_stream(ctx)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
