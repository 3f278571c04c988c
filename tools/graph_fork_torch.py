"""torch-level counterpart of tools/graph_fork_repro.cpp: the hot path's fork/join structure
(torch.cuda.Stream.wait_stream, record_stream, torch.cuda.graph with its private memory pool)
captured after other graphs were captured, replayed and released, with plain torch kernels
instead of the hot path's.  usage: graph_fork_torch.py <mode> <n_prior_graphs>; modes as the
C++ program (0 one side stream, 1 two side streams from one point, 2 one side stream forked
twice from one point).  Also writes the instantiated graph's DOT dump."""
import sys

import torch


def main():
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    prior = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda")
    x = torch.randn(1 << 20, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    keep = []
    for g in range(prior):
        cs = torch.cuda.Stream()
        gr = torch.cuda.CUDAGraph()
        y = torch.zeros_like(x)
        with torch.cuda.graph(gr, stream=cs):
            y.add_(x)
            if g & 1:
                s1.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s1):
                    z = x * 2
                torch.cuda.current_stream().wait_stream(s1)
                y.add_(z)
        for _ in range(2):
            gr.replay()
        torch.cuda.synchronize()
        if g % 3 == 0:
            keep.append(gr)  # some graphs stay alive, as in a test session
        del gr
    print(f"prior graphs: {prior} done", flush=True)
    cs = torch.cuda.Stream()
    gr = torch.cuda.CUDAGraph()
    gr.enable_debug_mode()
    y = torch.zeros_like(x)
    with torch.cuda.graph(gr, stream=cs):
        main = torch.cuda.current_stream()
        y.add_(x)
        outs = []
        if mode == 0:
            s1.wait_stream(main)
            x.record_stream(s1)
            with torch.cuda.stream(s1):
                outs.append(x * 3)
            y.add_(x)
            main.wait_stream(s1)
        elif mode == 1:
            s1.wait_stream(main)
            s2.wait_stream(main)
            with torch.cuda.stream(s1):
                outs.append(x * 3)
            with torch.cuda.stream(s2):
                outs.append(x * 4)
            y.add_(x)
            main.wait_stream(s1)
            y.add_(outs[0])
            main.wait_stream(s2)
        else:
            s1.wait_stream(main)
            with torch.cuda.stream(s1):
                outs.append(x * 3)
            s1.wait_stream(main)
            with torch.cuda.stream(s1):
                outs.append(x * 4)
            y.add_(x)
            main.wait_stream(s1)
        for o in outs:
            o.record_stream(main)
            y.add_(o)
    gr.debug_dump(f"gpurun_out/graph_fork_torch_mode{mode}.dot")
    print(f"mode {mode}: captured", flush=True)
    for r in range(3):
        gr.replay()
        torch.cuda.synchronize()
        print(f"replay {r} ok", flush=True)
    print(f"mode {mode}: no fault")


if __name__ == "__main__":
    main()
