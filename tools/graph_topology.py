"""Topology of the captured bench training step under three fork structures:

  current  one side stream, one fork per branch point (what hot_path._Side does)
  dupfork  every fork issued twice from the same point of the main stream
  twoside  forks alternate between the side stream and a second side stream

The step is captured with keep_graph=True and the raw hipGraph_t is read through the HIP runtime
(hipGraphGetNodes / GetEdges / NodeGetType / NodeGetDependencies): node counts by type, edges,
duplicate edges, nodes listing one dependency twice, and the DOT (hipGraphDebugDotPrint) written
to gpurun_out/graph_<mode>.dot.  The graph is instantiated (--instantiate) but replayed only with
--replay, so the structures that crashed hipGraphLaunch in round 2 can be inspected without a launch.

    python tools/graph_topology.py current dupfork twoside
"""
import argparse
import collections
import ctypes
import json
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
import torch  # noqa: E402

import bench  # noqa: E402
import _rgbd_import  # noqa: E402,F401
from rgbd_amd import hot_path  # noqa: E402

NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty", 6: "wait_event",
              7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait", 10: "mem_alloc", 11: "mem_free"}

_orig_run, _orig_join, _orig_init = hot_path._Side.run, hot_path._Side.join, hot_path._Side.__init__


def set_mode(mode):
    hot_path._Side.run, hot_path._Side.join, hot_path._Side.__init__ = _orig_run, _orig_join, _orig_init
    if mode == "dupfork":
        def run(self, fn, *inputs):
            if self.on:
                self.side.wait_stream(self.main)  # the extra fork from the same point
            return _orig_run(self, fn, *inputs)
        hot_path._Side.run = run
    elif mode == "twoside":
        second = {}

        def init(self, dev, enabled):
            _orig_init(self, dev, enabled)
            if enabled:
                if dev.index not in second:
                    second[dev.index] = hot_path._hip_stream(dev)
                self.pair = [self.side, second[dev.index]]
                self.turn = 0
                self.used = set()

        def run(self, fn, *inputs):
            if self.on:
                self.side = self.pair[self.turn]
                self.used.add(self.turn)
                self.turn ^= 1
            return _orig_run(self, fn, *inputs)

        def join(self):
            if not self.on or not self.forked:
                return
            for i in sorted(self.used):
                self.main.wait_stream(self.pair[i])
            self.used = set()
            self.side = self.pair[0]
            _orig_join(self)
        hot_path._Side.__init__, hot_path._Side.run, hot_path._Side.join = init, run, join


def analyse(graph_handle, dot_path):
    hip = ctypes.CDLL("libamdhip64.so")
    g = ctypes.c_void_p(graph_handle)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(g, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) == 0
    idx = {nodes[i]: i for i in range(n.value)}
    types = collections.Counter()
    node_type = []
    for i in range(n.value):
        t = ctypes.c_int(-1)
        assert hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t)) == 0
        node_type.append(NODE_TYPES.get(t.value, str(t.value)))
        types[node_type[-1]] += 1
    ne = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(g, None, None, ctypes.byref(ne)) == 0
    fr, to = (ctypes.c_void_p * max(ne.value, 1))(), (ctypes.c_void_p * max(ne.value, 1))()
    assert hip.hipGraphGetEdges(g, fr, to, ctypes.byref(ne)) == 0
    edges = [(idx.get(fr[i], -1), idx.get(to[i], -1)) for i in range(ne.value)]
    dup_edges = [e for e, c in collections.Counter(edges).items() if c > 1]
    dup_deps = []
    indeg = []
    for i in range(n.value):
        nd = ctypes.c_size_t(0)
        assert hip.hipGraphNodeGetDependencies(ctypes.c_void_p(nodes[i]), None, ctypes.byref(nd)) == 0
        deps = (ctypes.c_void_p * max(nd.value, 1))()
        assert hip.hipGraphNodeGetDependencies(ctypes.c_void_p(nodes[i]), deps, ctypes.byref(nd)) == 0
        d = [idx.get(deps[k], -1) for k in range(nd.value)]
        indeg.append(len(d))
        if len(set(d)) != len(d):
            dup_deps.append((i, node_type[i], d))
    # dependencies implied by others (a -> c while a -> b -> ... -> c): harmless, but counted
    succ = collections.defaultdict(set)
    for a, b in edges:
        succ[a].add(b)
    hip.hipGraphDebugDotPrint(g, dot_path.encode(), ctypes.c_uint(0xFFFF))
    return {"nodes": n.value, "types": dict(types), "edges": ne.value, "duplicate_edges": len(dup_edges),
            "duplicate_edge_examples": dup_edges[:5], "nodes_with_duplicate_deps": len(dup_deps),
            "duplicate_dep_examples": [(i, t, d) for i, t, d in dup_deps[:5]],
            "max_in_degree": max(indeg) if indeg else 0, "roots": sum(1 for d in indeg if d == 0),
            "dot": os.path.relpath(dot_path, _R)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("modes", nargs="+", choices=["current", "dupfork", "twoside"])
    ap.add_argument("--instantiate", type=int, default=1)
    ap.add_argument("--replay", type=int, default=0)
    a = ap.parse_args()
    os.makedirs(os.path.join(_R, "gpurun_out"), exist_ok=True)
    dev = torch.device("cuda")
    args = bench.parse([])
    ctx = bench.build(args, dev)
    keep = []
    for mode in a.modes:
        set_mode(mode)
        fb, ostep, _, _ = bench.make_parts(ctx, 1, capturable=True, overlap_opt=True)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                fb()
                ostep()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, stream=s):
            fb()
        info = analyse(g.raw_cuda_graph(), os.path.join(_R, "gpurun_out", f"graph_{mode}.dot"))
        if a.instantiate:
            g.instantiate()
        for _ in range(a.replay):
            g.replay()
        torch.cuda.synchronize()
        info["mode"] = mode
        info["replays"] = a.replay
        print(json.dumps(info), flush=True)
        keep.append(g)
    set_mode("current")


if __name__ == "__main__":
    main()
