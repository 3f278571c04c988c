"""f4 on the GPU: rgbd_pp_instance (csrc/postprocess.hip) against the HF image processor the
reference calls (predictor.py:697-700) on the CPU: identical top-k order (hence segment ids,
labels and overwrite order), identical painted maps, pred scores to float32 summation order."""
import sys
import types
from pathlib import Path

import numpy as np
import pytest
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import _rgbd_import  # noqa: E402,F401

pytestmark = pytest.mark.gpu


def _ref(cl, ml, **kw):
    from transformers.models.mask2former.image_processing_pil_mask2former import Mask2FormerImageProcessorPil
    outs = types.SimpleNamespace(class_queries_logits=torch.from_numpy(cl), masks_queries_logits=torch.from_numpy(ml))
    return Mask2FormerImageProcessorPil().post_process_instance_segmentation(outs, **kw)


def _compare(ref, got):
    for r, g in zip(ref, got):
        assert g["segmentation"].dtype == torch.float32 and g["segmentation"].device.type == "cpu"
        assert torch.equal(r["segmentation"], g["segmentation"]), \
            int((r["segmentation"] != g["segmentation"]).sum())
        assert len(r["segments_info"]) == len(g["segments_info"])
        for a, b in zip(r["segments_info"], g["segments_info"]):
            assert (a["id"], a["label_id"], a["was_fused"]) == (b["id"], b["label_id"], b["was_fused"])
            assert abs(a["score"] - b["score"]) <= 2e-6 + 1e-5 * abs(a["score"]), (a, b)


@pytest.mark.parametrize("target", [None, [(480, 640), (240, 320), (97, 131)], [(768, 1024)] * 3])
@pytest.mark.parametrize("kind", ["random", "ties"])
def test_instance_post_processing_matches_hf(target, kind):
    from rgbd_amd.postprocess import post_process_instance_segmentation
    rng = np.random.default_rng(11)
    B, Q, C, h, w = 3, 100, 48, 120, 160
    if kind == "random":
        cl = rng.standard_normal((B, Q, C + 1)).astype(np.float32) * 4
        cl[:, ::3, 7] += 7.0
    else:  # integer logits: exactly tied class probabilities everywhere (the nth_element order decides)
        cl = rng.integers(-3, 4, (B, Q, C + 1)).astype(np.float32)
        cl[:, ::2, 2] = 9.0
    ml = rng.standard_normal((B, Q, h, w)).astype(np.float32) * 3
    ref = _ref(cl, ml, target_sizes=target, threshold=0.3)
    outs = types.SimpleNamespace(class_queries_logits=torch.from_numpy(cl), masks_queries_logits=torch.from_numpy(ml))
    got = post_process_instance_segmentation(outs, target_sizes=target, threshold=0.3)
    assert sum(len(r["segments_info"]) for r in ref) > 0
    _compare(ref, got)


def test_install_on_image_processor_and_rle():
    from transformers.models.mask2former.image_processing_pil_mask2former import Mask2FormerImageProcessorPil
    from rgbd_amd.postprocess import install
    rng = np.random.default_rng(5)
    cl = rng.standard_normal((2, 100, 49)).astype(np.float32) * 4
    cl[:, ::4, 3] += 8.0
    ml = rng.standard_normal((2, 100, 60, 80)).astype(np.float32) * 3
    outs = types.SimpleNamespace(class_queries_logits=torch.from_numpy(cl), masks_queries_logits=torch.from_numpy(ml))
    ref = Mask2FormerImageProcessorPil().post_process_instance_segmentation(outs, target_sizes=[(240, 320)] * 2,
                                                                            return_coco_annotation=True)
    proc = install(Mask2FormerImageProcessorPil())
    got = proc.post_process_instance_segmentation(outs, target_sizes=[(240, 320)] * 2, return_coco_annotation=True)
    for r, g in zip(ref, got):
        assert r["segmentation"] == g["segmentation"]  # RLE lists
        assert [s["id"] for s in r["segments_info"]] == [s["id"] for s in g["segments_info"]]


def test_rejects_bad_arguments():
    from rgbd_amd.postprocess import post_process_instance_segmentation
    outs = types.SimpleNamespace(class_queries_logits=torch.zeros((1, 4, 3)), masks_queries_logits=torch.zeros((1, 4, 8, 8)))
    with pytest.raises(ValueError):
        post_process_instance_segmentation(outs, return_coco_annotation=True, return_binary_maps=True)


@pytest.mark.parametrize("target", [None, [(480, 640), (97, 131)]])
@pytest.mark.parametrize("threshold", [0.3, 1.1])
def test_binary_maps_match_hf(target, threshold):
    """return_binary_maps=True, as the reference's Evaluator calls it (model_essential_part.py:87-92):
    the kept masks stacked in segment order, bit-identical; the -1 map when nothing is kept."""
    from rgbd_amd.postprocess import post_process_instance_segmentation
    rng = np.random.default_rng(17)
    B, Q, C, h, w = 2, 100, 48, 120, 160
    cl = rng.standard_normal((B, Q, C + 1)).astype(np.float32) * 4
    cl[:, ::3, 5] += 7.0
    ml = rng.standard_normal((B, Q, h, w)).astype(np.float32) * 3
    ref = _ref(cl, ml, target_sizes=target, threshold=threshold, return_binary_maps=True)
    outs = types.SimpleNamespace(class_queries_logits=torch.from_numpy(cl), masks_queries_logits=torch.from_numpy(ml))
    got = post_process_instance_segmentation(outs, target_sizes=target, threshold=threshold, return_binary_maps=True)
    if threshold > 1.0:
        assert all(len(r["segments_info"]) == 0 for r in ref)
    else:
        assert all(r["segmentation"].dim() == 3 for r in ref)
    _compare(ref, got)


def test_install_falls_back_to_hf_outside_the_device_path():
    """A class table too large for the LDS top-k takes the processor's own method."""
    from transformers.models.mask2former.image_processing_pil_mask2former import Mask2FormerImageProcessorPil
    from rgbd_amd.postprocess import install
    rng = np.random.default_rng(3)
    cl = rng.standard_normal((1, 100, 301)).astype(np.float32) * 4  # 100 x 300 x 8 B > 160 KiB
    ml = rng.standard_normal((1, 100, 30, 40)).astype(np.float32) * 3
    outs = types.SimpleNamespace(class_queries_logits=torch.from_numpy(cl), masks_queries_logits=torch.from_numpy(ml))
    ref = Mask2FormerImageProcessorPil().post_process_instance_segmentation(outs, threshold=0.0, return_binary_maps=True)
    proc = install(Mask2FormerImageProcessorPil())
    got = proc.post_process_instance_segmentation(outs, threshold=0.0, return_binary_maps=True)
    _compare(ref, got)
