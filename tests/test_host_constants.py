"""ops.device_const / ops.host_constants: the per-step host numbers (level shapes, per-image
offsets, instance counts) are copied to the device once per distinct value and shared."""
import pytest
import torch

from rgbd_amd import ops


def test_device_const_is_shared_per_value_and_dtype():
    a = ops.device_const([[80, 60], [40, 30]], torch.long, "cpu")
    b = ops.device_const([[80, 60], [40, 30]], torch.long, "cpu")
    c = ops.device_const([[80, 60], [40, 30]], torch.int32, "cpu")
    d = ops.device_const(((80, 60), (40, 31)), torch.long, "cpu")
    assert a is b and a is not c and a is not d
    assert a.tolist() == [[80, 60], [40, 30]] and c.dtype == torch.int32


def test_device_const_rejects_non_numbers():
    with pytest.raises(TypeError):
        ops.device_const(["a"], torch.long, "cpu")


def test_host_constants_patch_is_scoped():
    orig = torch.as_tensor
    with ops.host_constants():
        assert torch.as_tensor is not orig
        # not a device constant: CPU targets and tensors go to torch unchanged
        assert torch.as_tensor([1, 2], device="cpu").tolist() == [1, 2]
        t = torch.ones(2)
        assert torch.as_tensor(t) is t
    assert torch.as_tensor is orig
    with pytest.raises(ValueError):
        with ops.host_constants():
            raise ValueError("restored on error too")
    assert torch.as_tensor is orig


def test_host_constants_only_in_the_entering_thread(monkeypatch):
    """the patch serves device constants only to the thread inside the block; other
    threads (data loaders, pin-memory workers) get torch's own as_tensor."""
    import threading
    seen = []
    monkeypatch.setattr(ops, "device_const", lambda v, dt, dev: seen.append(v) or "const")
    other = {}

    def worker():
        try:
            other["r"] = torch.as_tensor([3, 4], device="cuda")
        except Exception as e:  # no GPU here: torch's own path raises, which is the point
            other["r"] = type(e).__name__

    with ops.host_constants():
        assert torch.as_tensor([1, 2], device="cuda") == "const"
        t = threading.Thread(target=worker)
        t.start()
        t.join()
    assert seen == [(1, 2)]
    assert other["r"] != "const"


def test_device_const_table_is_bounded_and_keeps_pinned_entries():
    """Per-batch values (the matcher's target counts) must not grow the table without bound: it
    is least-recently-used with a cap, and entries a captured graph read are never evicted."""
    ops._consts.clear()
    ops._pinned.clear()
    keep = ops.device_const([12345, 1], torch.long, "cpu")
    key = next(iter(ops._consts))
    ops._pinned.add(key)  # as if read during a capture
    hot = ops.device_const([7, 7, 7], torch.int32, "cpu")
    for i in range(ops._CONST_CAP + 100):
        ops.device_const([i, i + 1], torch.long, "cpu")
        if i % 50 == 0:
            assert ops.device_const([7, 7, 7], torch.int32, "cpu") is hot  # recently used: kept
    assert len(ops._consts) <= ops._CONST_CAP
    assert ops.device_const([12345, 1], torch.long, "cpu") is keep
    assert ops.device_const([0, 1], torch.long, "cpu").tolist() == [0, 1]  # evicted, rebuilt
    ops._consts.clear()
    ops._pinned.clear()
