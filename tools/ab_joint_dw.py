"""A/B of the bf16 backward's dW schedule (hot_path.JOINT_DW): dsam1's and dsam0's dW GEMMs in one
persistent launch vs two launches (dW1 on the side stream), on the bench's training step (640x480,
B=8, the captured HIP graph), interleaved in one process so both arms see the same device and
clock state.  Prints the median ms per step of each arm over --rounds rounds of --iters replays.
"""
import argparse
import json
import os
import statistics
import sys
import time

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
import torch  # noqa: E402

import bench  # noqa: E402


def micro(dev, iters):
    """dsam1 + dsam0 dW at the bench's shapes on one stream: the joint launch vs the two planned
    launches back to back (plans made outside the timed region, one per run)."""
    from rgbd_amd import ops, synthetic
    B, H, W = 8, 480, 640
    planes, _, _ = synthetic.make_batch(7, B, H, W)
    d3 = torch.from_numpy(planes[:, 3:6]).to(dev)
    sizes = [(120, 160), (60, 80), (30, 40)]
    codes, info = ops.edsam_decompose(d3, torch.linspace(0.05, 0.45, B, device=dev), sizes)
    ch = [(96, 192), (192, 384)]
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    xs = [torch.randn((B, *sizes[k], ch[k][0]), generator=g, device=dev).bfloat16() for k in (0, 1)]
    gys = [torch.randn((B, sizes[k][0] // 2, sizes[k][1] // 2, ch[k][1]), generator=g, device=dev).bfloat16()
           for k in (0, 1)]
    n = iters
    plans = [ops.dsam_plan([(ops.LEG_DW, codes[k], *ch[k]) for k in (1, 0)]) for _ in range(3 * n)]

    def joint(p):
        ops.dsam_bwd_weight_multi([(gys[1], xs[1], codes[1], p[0]), (gys[0], xs[0], codes[0], p[1])], info)

    def two(p):
        ops.dsam_bwd_weight(None, xs[1], codes[1], info, gout_nhwc=gys[1], plan=p[0])
        ops.dsam_bwd_weight(None, xs[0], codes[0], info, gout_nhwc=gys[0], plan=p[1])
    out = {}
    for rnd in range(3):
        for name, fn in (("joint", joint), ("two_launch", two)):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(n // 2):
                fn(plans[rnd * n + (0 if name == "joint" else n // 2) + i])
            e1.record()
            torch.cuda.synchronize()
            out.setdefault(name, []).append(round(e0.elapsed_time(e1) / (n // 2) * 1e3, 1))
    print(json.dumps({"micro_us": out}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--micro", type=int, default=1, help="also time the dW launches alone")
    a = ap.parse_args()
    dev = torch.device("cuda")
    if a.micro:
        micro(dev, a.iters)
    ctx = bench.build(bench.parse([]), dev)
    from rgbd_amd import hot_path as hp
    steps = {}
    for joint in (True, False):
        hp.JOINT_DW = joint
        st = bench.make_step(ctx, 1, graph=bool(a.graph))
        for _ in range(3):  # capture (graph) and warm up under this arm's schedule
            st()
        torch.cuda.synchronize()
        steps["joint" if joint else "two_launch"] = (joint, st)
    res = {k: [] for k in steps}
    for rnd in range(a.rounds):
        for name, (joint, st) in steps.items():
            hp.JOINT_DW = joint  # eager arms read it per step; graphs replay what they captured
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                st()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / a.iters * 1e3)
        print(rnd, {k: round(v[-1], 3) for k, v in res.items()}, flush=True)
    out = {k: {"median_ms": round(statistics.median(v), 3), "min_ms": round(min(v), 3)} for k, v in res.items()}
    out["graph"] = bool(a.graph)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
