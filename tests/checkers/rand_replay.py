"""Test-only: replay the reference run's ``torch.rand`` draws on the GPU.

The reference's loss draws its sample points with ``torch.rand`` (transformers 5.15
modeling_mask2former.py:455 in the matcher, :705 and :721 in sample_points_using_uncertainty)
from the CPU generator seeded with ``torch.manual_seed(1234)`` (tests/golden/make_golden.py
g6_fixture).  On the GPU the same calls would draw from the device generator, so a GPU run's
points differ.  ``CpuRandReplay`` serves every ``torch.rand`` call made while it is active from a
private CPU generator with the reference's seed, in call order, and moves the values to the
requested device: as long as the call sequence (shapes, order) is the reference's — the fixture
holds each call's shape and the sha256 of its values, checked by ``check`` — the values are
bitwise the reference's."""
import hashlib

import numpy as np
import torch


class CpuRandReplay(torch.overrides.TorchFunctionMode):
    def __init__(self, seed):
        super().__init__()
        self.gen = torch.Generator().manual_seed(int(seed))
        self.calls = []

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = dict(kwargs or {})
        if func is not torch.rand:
            return func(*args, **kwargs)
        device = kwargs.pop("device", None)
        dtype = kwargs.pop("dtype", None) or torch.get_default_dtype()
        kwargs.pop("generator", None)
        cpu = torch.rand(*args, generator=self.gen, dtype=dtype, **kwargs)  # the mode is off in here
        self.calls.append((tuple(cpu.shape), hashlib.sha256(np.ascontiguousarray(cpu.numpy()).tobytes()).hexdigest()))
        return cpu.to(device) if device is not None else cpu

    def check(self, fixture):
        """The replayed draws are the reference's: same number of calls, same shapes, same bytes."""
        shapes = [str(list(s)) for s, _ in self.calls]
        want_shapes = [str(s) for s in fixture["rand_shapes"]]
        assert shapes == want_shapes, f"torch.rand call sequence differs: {shapes[:4]}... vs {want_shapes[:4]}..."
        assert [h for _, h in self.calls] == [str(h) for h in fixture["rand_sha"]], "replayed draws differ"
