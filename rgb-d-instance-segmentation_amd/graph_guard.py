"""Guard on the concurrency of captured HIP graphs.

The HIP runtime torch ships (ROCm 7.0) reads past the end of its parallel-stream vector in
``hip::Graph::UpdateStreams`` on the first launch of a graph with more than two concurrent
branches (segfault in hipGraphLaunch, located in round 3).  The hot path keeps one side stream
beside the capture stream, so every graph it captures has at most two concurrent branches; this
module checks that property on the raw ``hipGraph_t`` before the graph is instantiated, so a
future fork cannot bring the crash back silently.

The number of concurrent branches is the graph's width: the largest set of nodes no two of
which are ordered by a dependency path (a maximum antichain).  By Dilworth's theorem it equals
the smallest number of chains covering the nodes, computed here as ``nodes - maximum matching``
in the bipartite graph of the transitive closure.
"""
import ctypes

MAX_BRANCHES = 2
_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")  # the runtime torch already loaded
    return _HIP


def dag_width(n, edges):
    """Width (maximum antichain size) of a DAG with nodes 0..n-1 and ``edges`` (a, b): a before b.

    n - (maximum matching in the bipartite graph of the transitive closure).  A captured training
    step has thousands of nodes, so the matching starts from a greedy chain cover (nodes in
    topological order, each appended to the first chain whose tail reaches it) and is completed
    with iterative augmenting-path searches over reachability bitsets (no recursion)."""
    adj = [[] for _ in range(n)]
    indeg = [0] * n
    for a, b in edges:
        adj[a].append(b)
        indeg[b] += 1
    order, ready = [], [i for i in range(n) if indeg[i] == 0]
    while ready:
        v = ready.pop()
        order.append(v)
        for w in adj[v]:
            indeg[w] -= 1
            if indeg[w] == 0:
                ready.append(w)
    if len(order) != n:
        raise ValueError("graph has a cycle")
    reach = [0] * n  # descendants of v as a bitset
    for v in reversed(order):
        r = 0
        for w in adj[v]:
            r |= reach[w] | (1 << w)
        reach[v] = r
    match_l, match_r = [-1] * n, [-1] * n  # left v -> right w (v before w on one chain)
    tails = []
    for v in order:
        for i, t in enumerate(tails):
            if (reach[t] >> v) & 1:
                match_l[t], match_r[v] = v, t
                tails[i] = v
                break
        else:
            tails.append(v)

    def augment(u):
        seen, parent = 0, {}
        stack = [[u, reach[u]]]
        while stack:
            top = stack[-1]
            r = top[1] & ~seen
            if not r:
                stack.pop()
                continue
            low = r & -r
            w = low.bit_length() - 1
            top[1] = r ^ low
            seen |= low
            parent[w] = top[0]
            if match_r[w] < 0:
                while True:  # flip the alternating path back to u
                    v = parent[w]
                    prev = match_l[v]
                    match_l[v], match_r[w] = w, v
                    if v == u:
                        return True
                    w = prev
            stack.append([match_r[w], reach[match_r[w]]])
        return False
    for u in range(n):
        if match_l[u] < 0:
            augment(u)
    return n - sum(1 for v in range(n) if match_l[v] >= 0)


def graph_width(graph_handle):
    """Width of a raw hipGraph_t (``torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()``)."""
    hip = _hip()
    g = ctypes.c_void_p(graph_handle)
    n = ctypes.c_size_t(0)
    if hip.hipGraphGetNodes(g, None, ctypes.byref(n)) != 0:
        raise RuntimeError("hipGraphGetNodes failed")
    nodes = (ctypes.c_void_p * max(n.value, 1))()
    if hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)) != 0:
        raise RuntimeError("hipGraphGetNodes failed")
    idx = {nodes[i]: i for i in range(n.value)}
    ne = ctypes.c_size_t(0)
    if hip.hipGraphGetEdges(g, None, None, ctypes.byref(ne)) != 0:
        raise RuntimeError("hipGraphGetEdges failed")
    fr, to = (ctypes.c_void_p * max(ne.value, 1))(), (ctypes.c_void_p * max(ne.value, 1))()
    if hip.hipGraphGetEdges(g, fr, to, ctypes.byref(ne)) != 0:
        raise RuntimeError("hipGraphGetEdges failed")
    edges = [(idx[fr[i]], idx[to[i]]) for i in range(ne.value)]
    return dag_width(n.value, edges), n.value


def check_and_instantiate(graph, what):
    """For a graph captured with ``keep_graph=True``: refuse more than MAX_BRANCHES concurrent
    branches, then instantiate.  Returns the width."""
    width, nodes = graph_width(graph.raw_cuda_graph())
    if width > MAX_BRANCHES:
        raise RuntimeError(f"{what}: the captured graph has {width} concurrent branches ({nodes} nodes); the "
                           f"bundled HIP runtime crashes in hipGraphLaunch above {MAX_BRANCHES} (DESIGN.md §5.1)")
    graph.instantiate()
    return width
