"""The optimizer step on HIP (csrc/adamw.hip, rgbd_amd.optim.HipAdamW) against torch.optim.AdamW
(fused): parameters of the hot path's shapes plus ragged sizes (numel not a multiple of 4, a
single element, more tensors than one launch holds), several steps with weight decay, the
reference's lr 1e-5 (config.json:12-13) and a larger one; then captured into a CUDA graph and
replayed.  Tolerance: 2 ulp-scale (rtol 1e-6) of the parameters — both compute the same float32
formula, the instruction order (fused multiply-adds) may differ."""
import pytest
import torch

import _rgbd_import  # noqa: F401

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
SHAPES = [(768, 384, 3, 3), (4, 768), (192, 96, 3, 3), (4097,), (1,), (3, 5, 7)] + [(33,)] * 50


def _pair(seed, lr, wd):
    from rgbd_amd.optim import HipAdamW
    g = torch.Generator(device="cpu").manual_seed(seed)
    a = [torch.randn(s, generator=g).to(DEV).requires_grad_() for s in SHAPES]
    b = [p.detach().clone().requires_grad_() for p in a]
    return a, b, HipAdamW(a, lr=lr, weight_decay=wd), torch.optim.AdamW(b, lr=lr, weight_decay=wd, fused=True), g


@pytest.mark.parametrize("lr,wd", [(1e-5, 0.0), (1e-3, 0.05)])
def test_adamw_matches_torch_fused(lr, wd):
    a, b, oa, ob, g = _pair(1, lr, wd)
    for _ in range(4):
        for pa, pb in zip(a, b):
            gr = torch.randn(pa.shape, generator=g).to(DEV)
            pa.grad, pb.grad = gr.clone(), gr.clone()
        oa.step()
        ob.step()
    for pa, pb in zip(a, b):
        torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(oa.state[pa]["exp_avg_sq"], ob.state[pb]["exp_avg_sq"], rtol=1e-6, atol=1e-12)
    assert float(oa.state[a[0]]["step"]) == 4.0


def test_adamw_graph_replay():
    a, b, oa, ob, g = _pair(2, 1e-3, 0.01)
    grads = [torch.randn(p.shape, generator=g).to(DEV) for p in a]
    for pa, pb, gr in zip(a, b, grads):
        pa.grad, pb.grad = gr.clone(), gr.clone()
    oa.step()  # state allocated outside the capture
    ob.step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            oa.step()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        graph.replay()
        ob.step()
    torch.cuda.synchronize()
    for pa, pb in zip(a, b):
        torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-7)
    assert float(oa.state[a[0]]["step"]) == 4.0


def test_adamw_rejects_cpu_and_bf16():
    from rgbd_amd.optim import HipAdamW
    p = torch.zeros(4, requires_grad=True)
    p.grad = torch.zeros(4)
    with pytest.raises(RuntimeError):
        HipAdamW([p]).step()
    q = torch.zeros(4, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    q.grad = torch.zeros_like(q)
    with pytest.raises(RuntimeError):
        HipAdamW([q]).step()


def test_bf16_shadow_written_by_the_step():
    """A parameter with a cached bf16 cast (dense.cast_weight) gets that copy rewritten by the
    AdamW launch (rgbd_adamw_multi_shadow) and re-keyed: the next cast_weight returns the same
    tensor, bitwise p.to(bfloat16) of the updated parameter, with no cast launch."""
    from rgbd_amd.dense import cast_weight
    from rgbd_amd.optim import HipAdamW
    torch.manual_seed(0)
    a = torch.nn.Parameter(torch.randn(1000, 37, device="cuda"))
    b = torch.nn.Parameter(torch.randn(4099, device="cuda"))  # no cast: no shadow
    opt = HipAdamW([a, b], lr=1e-2)
    c0 = cast_weight(a, torch.bfloat16)
    for _ in range(3):
        a.grad = torch.randn_like(a)
        b.grad = torch.randn_like(b)
        opt.step()
        c = cast_weight(a, torch.bfloat16)
        assert c is c0
        assert torch.equal(c, a.detach().to(torch.bfloat16))
    assert getattr(b, "_rgbd_cast", None) is None
