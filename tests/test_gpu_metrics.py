"""f4 on the GPU: the mask-IoU kernels (csrc/mask_iou.hip) against numpy, the whole segm mAP
(rgbd_amd/metrics.py) against the pycocotools restatement (oracle/cocoeval.py), and the
reference's Evaluator protocol (rgbd_amd/evaluator.py) end to end on model-shaped predictions,
with the HF image processor's post-processing and with the device one installed — identical
numbers.  Parity unpinned against torchmetrics itself (not installed)."""
import types

import numpy as np
import pytest
import torch

from oracle import cocoeval
from rgbd_amd import metrics

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape", [(48, 64), (37, 53), (480, 640)])
def test_pack_and_intersections_match_numpy(shape):
    from rgbd_amd import _lib
    from rgbd_amd.ops import _p, _stream
    rng = np.random.default_rng(shape[0])
    a = rng.random((5, *shape)) > 0.6
    b = rng.random((3, *shape)) > 0.3
    pa = metrics._Packed(torch.from_numpy(a), torch.device(DEV))
    pb = metrics._Packed(torch.from_numpy(b), torch.device(DEV))
    inter = metrics._intersections(pa, pb, torch.device(DEV)).cpu().numpy()
    af, bf = a.reshape(5, -1).astype(np.int64), b.reshape(3, -1).astype(np.int64)
    np.testing.assert_array_equal(inter, af @ bf.T)
    np.testing.assert_array_equal(pa.area.cpu().numpy(), af.sum(1))
    np.testing.assert_array_equal(pb.area.cpu().numpy(), bf.sum(1))
    # the bitmap layout the header states: bit j of word w = pixel 64 w + j
    words = pa.bits.cpu().numpy().view(np.uint64)[0]
    flat = a[0].reshape(-1)
    for w in (0, len(words) - 1):
        px = flat[64 * w:64 * w + 64]
        assert int(words[w]) == sum(1 << j for j, v in enumerate(px) if v)
    assert _lib.lib().rgbd_mask_intersections(_p(pa.bits), 0, _p(pb.bits), 3, shape[0] * shape[1], None,
                                              _stream(torch.device(DEV))) == 0  # empty side: nothing to do


def _scene(rng, H, W, n_gt, n_det, n_cls=4):
    def rect():
        m = np.zeros((H, W), bool)
        y, x = rng.integers(0, H - 8), rng.integers(0, W - 8)
        m[y:y + rng.integers(4, H // 2), x:x + rng.integers(4, W // 2)] = True
        return m
    gts = [rect() for _ in range(n_gt)]
    dets = [np.roll(gts[rng.integers(0, n_gt)], (rng.integers(-4, 5), rng.integers(-4, 5)), (0, 1))
            if n_gt and rng.random() < 0.6 else rect() for _ in range(n_det)]
    return ({"masks": torch.from_numpy(np.stack(dets) if dets else np.zeros((0, H, W), bool)),
             "scores": torch.from_numpy(np.round(rng.random(n_det), 2).astype(np.float32)),
             "labels": torch.from_numpy(rng.integers(0, n_cls, n_det))},
            {"masks": torch.from_numpy(np.stack(gts) if gts else np.zeros((0, H, W), bool)),
             "labels": torch.from_numpy(rng.integers(0, n_cls, n_gt))})


def test_mean_average_precision_matches_cocoeval_restatement():
    rng = np.random.default_rng(1)
    m = metrics.MeanAveragePrecision(iou_type="segm", class_metrics=True)
    preds, targets = [], []
    for batch in range(3):
        pairs = [_scene(rng, 96, 128, int(rng.integers(0, 8)), int(rng.integers(0, 20))) for _ in range(4)]
        m.update([p for p, _ in pairs], [t for _, t in pairs])
        preds += [p for p, _ in pairs]
        targets += [t for _, t in pairs]
    got = m.compute()
    want = cocoeval.mean_average_precision([{k: v.numpy() for k, v in p.items()} for p in preds],
                                           [{k: v.numpy() for k, v in t.items()} for t in targets], class_metrics=True)
    for k, v in want.items():
        np.testing.assert_allclose(np.asarray(got[k], np.float64), np.asarray(v, np.float64), rtol=1e-6, atol=1e-7,
                                   err_msg=k)
    assert 0.0 < float(got["map"]) < 1.0


def test_evaluator_protocol_device_vs_hf_postprocessing():
    """The reference's compute_metrics protocol (batch_eval_metrics): two update batches, then
    compute_result; the predictions are model-shaped logits, the targets binary masks."""
    from transformers.models.mask2former.image_processing_pil_mask2former import Mask2FormerImageProcessorPil
    from rgbd_amd.evaluator import Evaluator
    from rgbd_amd.postprocess import install
    rng = np.random.default_rng(7)
    B, Q, C, h, w, H, W = 2, 100, 6, 60, 80, 240, 320
    batches = []
    for _ in range(2):
        cl = rng.standard_normal((B, Q, C + 1)).astype(np.float32) * 3
        cl[:, ::5, 2] += 6.0
        ml = rng.standard_normal((B, Q, h, w)).astype(np.float32) * 3
        tm = [torch.from_numpy(rng.random((4, H, W)) > 0.7).float() for _ in range(B)]
        tl = [torch.from_numpy(rng.integers(0, C, 4)) for _ in range(B)]
        batches.append(types.SimpleNamespace(predictions=(torch.from_numpy(cl), torch.from_numpy(ml)),
                                             label_ids=(tm, tl)))
    id2label = {i: f"c{i}" for i in range(C)}
    results = []
    for proc in (Mask2FormerImageProcessorPil(), install(Mask2FormerImageProcessorPil())):
        ev = Evaluator(proc, id2label, threshold=0.0)
        assert ev(batches[0]) is None
        results.append(ev(batches[1], compute_result=True))
    assert results[0] == results[1]
    assert "map" in results[0] and any(k.startswith("map_c") for k in results[0])
