"""Probe: how much of the ratio predictor of batch k+1 can run beside the rest of
batch k's training step.  The ratio predictor is forward-only and its weights never train (Q2),
so its work for the next batch depends on nothing in this batch's backward; its BatchNorm
running statistics still update in batch order (one stream).  Eager steps, the bench's workload
(640x480, B=8, bf16), the same input every step; the hot path's own side stream is off in both
arms so that the pipelined arm has exactly two concurrent branches.  Prints img/s of the
sequential and the pipelined loop and the ratio-predictor time alone."""
import json
import os
import sys
import time

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda")
    args = bench.parse([])
    ctx = bench.build(args, dev)
    from rgbd_amd import ops
    from rgbd_amd.distributed import InBackwardOptimizer, hot_path_grad_groups
    from rgbd_amd.hot_path import hot_path, prepare
    groups = hot_path_grad_groups(ctx["dsams"], ctx["dg"])
    inb = InBackwardOptimizer(groups, lambda g: torch.optim.AdamW(g, lr=1e-5, fused=True), None, steps=((0,), (1, 2)))
    B = ctx["depth_u8"].shape[0]

    def ratio_of():
        pv = ops.assemble_pixel_values(ctx["depth_u8"], ctx["rgb_u8"])
        return pv, ctx["rp"](pv[:, 3:6])

    def rest(pv, ratio):
        prep = prepare(pv, ctx["colors"], ctx["dtype"])
        feats = hot_path(pv, ratio, ctx["colors"], ctx["dsams"], ctx["dg"], dtype=ctx["dtype"], grad_hook=inb.hook,
                         prepared=prep)
        torch.autograd.backward(feats, ctx["gouts"])
        inb.zero_grad(set_to_none=True)

    def sequential(n):
        for _ in range(n):
            rest(*ratio_of())

    s2 = torch.cuda.Stream()

    def pipelined(n):
        main = torch.cuda.current_stream()
        s2.wait_stream(main)
        with torch.cuda.stream(s2):
            cur = ratio_of()
        for i in range(n):
            main.wait_stream(s2)  # batch i's ratio is ready
            for t in cur:
                t.record_stream(main)
            if i + 1 < n:
                with torch.cuda.stream(s2):  # batch i+1's ratio predictor beside batch i's step
                    nxt = ratio_of()
            rest(*cur)
            if i + 1 < n:
                cur = nxt

    def ratio_only(n):
        for _ in range(n):
            ratio_of()

    res = {}
    for name, fn in (("sequential", sequential), ("pipelined", pipelined), ("ratio_only", ratio_only),
                     ("sequential_2", sequential), ("pipelined_2", pipelined)):
        fn(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(20)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        res[name] = {"ms_per_step": round(dt * 1e3, 3), "img_s": round(B / dt, 1)}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
