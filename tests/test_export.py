"""f4 JSON export (rgbd_amd/export.py) against the pycocotools restatement (oracle/rle.py) and the
reference's per-image conversion loops (mask2former/predictor.py:376-457, 528-625) restated on it.
CPU: the encoder runs on whatever device holds the maps; the GPU path is the same torch code."""
import json

import numpy as np
import pytest
import torch

from oracle import rle as rle_o
from rgbd_amd import export


def _masks(seed):
    rng = np.random.default_rng(seed)
    out = [np.zeros((5, 7), np.uint8), np.ones((5, 7), np.uint8), np.eye(6, 9, dtype=np.uint8)]
    m = np.zeros((4, 4), np.uint8)
    m[0, 0] = 1  # first pixel set: counts start with 0
    out.append(m)
    out.append((rng.random((48, 64)) > 0.5).astype(np.uint8))       # many short runs (deltas < 0)
    big = np.zeros((480, 640), np.uint8)
    big[100:300, 50:600] = 1
    big[310:470, 20:30] = 1
    out.append(big)                                                   # long runs (multi-group counts)
    return out


@pytest.mark.parametrize("seed", [0, 1])
def test_rle_matches_pycocotools_restatement(seed):
    masks = _masks(seed)
    for m in masks:
        (got, bbox), = export.encode_masks(torch.from_numpy(m)[None])
        want = rle_o.encode(m)
        assert got == want
        h, w, counts = rle_o.rle_encode(m)
        assert rle_o.rle_from_string(got["counts"]) == counts
        np.testing.assert_array_equal(rle_o.rle_decode(h, w, rle_o.rle_from_string(got["counts"])), m)
        assert bbox == rle_o.bbox_from_mask(m)


def _ref_prediction_json(pred, original_size):
    """_convert_single_prediction_to_json restated on the oracle encoder."""
    seg = pred["segmentation"].numpy()
    h, w = original_size if original_size is not None else seg.shape[:2]
    out = {"labels": [], "scores": [], "bboxes": [], "masks": []}
    for s in pred["segments_info"]:
        m = (seg == s["id"]).astype(np.uint8)
        if m.sum() == 0:
            continue
        out["labels"].append(int(s["label_id"]))
        out["scores"].append(float(s.get("score", 1.0)))
        out["bboxes"].append(rle_o.bbox_from_mask(m))
        out["masks"].append({"size": [int(h), int(w)], "counts": rle_o.encode(m)["counts"]})
    return out


def test_prediction_json_matches_reference_loop(tmp_path):
    rng = np.random.default_rng(3)
    seg = torch.full((60, 80), -1.0)
    for k in range(5):
        y, x = rng.integers(0, 50), rng.integers(0, 70)
        seg[y:y + rng.integers(3, 10), x:x + rng.integers(3, 10)] = float(k)
    info = [{"id": k, "label_id": int(rng.integers(0, 48)), "was_fused": False, "score": float(rng.random())}
            for k in range(5)] + [{"id": 7, "label_id": 1, "was_fused": False, "score": 0.5}]  # 7: empty, skipped
    pred = {"segmentation": seg, "segments_info": info}
    got = export.prediction_to_json(pred, (60, 80))
    assert got == _ref_prediction_json(pred, (60, 80))
    assert len(got["labels"]) == 5
    files = export.convert_predictions_to_json([pred, pred], ["a", "b"], tmp_path, [(60, 80), (60, 80)])
    assert [f.name for f in files] == ["a.json", "b.json"]
    assert json.loads(files[0].read_text()) == got


def test_gt_json_both_label_forms():
    rng = np.random.default_rng(4)
    masks = (rng.random((4, 30, 40)) > 0.7).astype(np.float32)
    masks[2] = 0.0                      # empty: skipped
    ids = np.array([3, 0, 5, 9])        # id 0: background, skipped
    got = export.gt_label_to_json([masks, ids], (30, 40))
    assert got["labels"] == [3, 9] and got["scores"] == [1.0, 1.0]
    assert got["masks"][1]["counts"] == rle_o.encode((masks[3] > 0).astype(np.uint8))["counts"]
    idmap = np.zeros((30, 40), np.int64)
    idmap[2:9, 3:20] = 4
    idmap[15:25, 5:8] = 2
    got2 = export.gt_label_to_json([idmap, None])
    assert got2["labels"] == [2, 4]
    assert got2["bboxes"] == [rle_o.bbox_from_mask(idmap == 2), rle_o.bbox_from_mask(idmap == 4)]
