"""The concurrency guard on captured graphs (rgbd_amd/graph_guard.py).

CPU: the DAG width (maximum antichain = minimum chain cover) on hand-made graphs.
GPU: every graph the product captures — the bench's training step (CapturedTrainStep) and the
C5 streaming path (StreamingHotPath) — has at most two concurrent branches; a capture with
three concurrent branches is refused before it is instantiated (it is never launched: the
bundled runtime's first launch of such a graph is the crash the guard exists for)."""
import pytest
import torch

from rgbd_amd.graph_guard import MAX_BRANCHES, dag_width


def test_width_chain_and_forks():
    assert dag_width(0, []) == 0
    assert dag_width(1, []) == 1
    assert dag_width(4, [(0, 1), (1, 2), (2, 3)]) == 1
    # fork/join with one side branch: 0 -> {1, 2} -> 3
    assert dag_width(4, [(0, 1), (0, 2), (1, 3), (2, 3)]) == 2
    # three concurrent branches
    assert dag_width(5, [(0, 1), (0, 2), (0, 3), (1, 4), (2, 4), (3, 4)]) == 3
    # two streams with cross edges (what one side stream beside the capture stream gives)
    main = [(0, 1), (1, 2), (2, 3), (3, 4)]
    side = [(5, 6), (6, 7)]
    cross = [(0, 5), (7, 3), (1, 6)]
    assert dag_width(8, main + side + cross) == 2
    # a transitive edge does not add width
    assert dag_width(3, [(0, 1), (1, 2), (0, 2)]) == 1
    # width counts nodes ordered only through a path (no direct edge)
    assert dag_width(6, [(0, 1), (1, 2), (3, 4), (4, 5), (2, 3)]) == 1


def test_width_cycle_refused():
    with pytest.raises(ValueError):
        dag_width(2, [(0, 1), (1, 0)])


@pytest.mark.gpu
def test_captured_train_step_and_stream_within_two_branches():
    import bench
    from rgbd_amd.stream import StreamingHotPath
    from rgbd_amd.train_graph import CapturedTrainStep
    dev = torch.device("cuda")
    args = bench.parse(["--height", "96", "--width", "128", "--batch", "2"])
    ctx = bench.build(args, dev)
    fb, ob, _, _ = bench.make_parts(ctx, 1, capturable=True, overlap_opt=True)
    step = CapturedTrainStep(fb, None, warmup=1, opts=ob.opts, clear=ob)
    assert 1 <= step.width <= MAX_BRANCHES
    step()
    sp = StreamingHotPath(ctx["rp"], ctx["dsams"], ctx["dg"], 96, 128, B=1, dtype=ctx["dtype"]).capture()
    assert 1 <= sp.width <= MAX_BRANCHES
    sp()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_three_branch_capture_refused_unlaunched():
    from rgbd_amd.graph_guard import check_and_instantiate, graph_width
    x = torch.ones(1 << 16, device="cuda")
    s0 = torch.cuda.Stream()
    sides = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    outs = []
    with torch.cuda.graph(g, stream=s0):
        y = x * 2
        for s in sides:
            s.wait_stream(s0)
            with torch.cuda.stream(s):
                outs.append(y + 1)
        outs.append(y - 1)
        for s in sides:
            s0.wait_stream(s)
        z = outs[0] + outs[1] + outs[2]
    width, nodes = graph_width(g.raw_cuda_graph())
    assert width == 3 and nodes >= 5
    with pytest.raises(RuntimeError, match="concurrent branches"):
        check_and_instantiate(g, "test")
    del z
