"""f4 oracle: the restatement of the reference's instance post-processing (oracle/postprocess.py)
pinned on the CPU against what the reference actually runs — torch.topk(sorted=False) for the
discrete top-k order, and the HF image processor's post_process_instance_segmentation for the
whole result."""
import sys
import types
from pathlib import Path

import numpy as np
import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from oracle.postprocess import nth_element_topk, post_process_instance_segmentation  # noqa: E402


def _cases():
    rng = np.random.default_rng(0)
    for t in range(160):
        Q, C = int(rng.integers(1, 120)), int(rng.integers(1, 60))
        if Q * 64 <= Q * C:
            continue
        kind = t % 4
        n = Q * C
        if kind == 0:
            v = rng.random(n).astype(np.float32)
        elif kind == 1:  # many exact ties
            v = (rng.integers(0, 5, n) / 5).astype(np.float32)
        elif kind == 2:  # NaN ranks first
            v = rng.random(n).astype(np.float32)
            v[rng.integers(0, n, max(1, n // 40))] = np.nan
        else:  # class probabilities as the processor makes them
            x = torch.from_numpy(rng.standard_normal((Q, C + 1)).astype(np.float32) * 3)
            v = torch.softmax(x, -1)[:, :-1].flatten().numpy()
        yield Q, v


def test_nth_element_order_equals_torch_cpu_topk():
    n = 0
    for Q, v in _cases():
        _, ti = torch.topk(torch.from_numpy(v), Q, sorted=False)
        _, oi = nth_element_topk(v, Q)
        assert np.array_equal(ti.numpy(), oi), (Q, v.size)
        n += 1
    assert n > 100


@pytest.mark.parametrize("target", [None, [(480, 640), (240, 320)]])
def test_oracle_equals_hf_processor(target):
    from transformers.models.mask2former.image_processing_pil_mask2former import Mask2FormerImageProcessorPil
    rng = np.random.default_rng(3)
    B, Q, C, h, w = 2, 100, 48, 60, 80
    cl = rng.standard_normal((B, Q, C + 1)).astype(np.float32) * 4
    cl[:, :, 5] += 6.0  # confident queries, so segments survive the default threshold
    ml = rng.standard_normal((B, Q, h, w)).astype(np.float32) * 3
    outs = types.SimpleNamespace(class_queries_logits=torch.from_numpy(cl), masks_queries_logits=torch.from_numpy(ml))
    ref = Mask2FormerImageProcessorPil().post_process_instance_segmentation(outs, target_sizes=target)
    got = post_process_instance_segmentation(cl, ml, target_sizes=target)
    for r, g in zip(ref, got):
        assert torch.equal(r["segmentation"], g["segmentation"])
        assert r["segments_info"] == g["segments_info"]
        assert len(r["segments_info"]) > 0
