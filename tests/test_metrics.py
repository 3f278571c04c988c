"""f4 segm mAP: the product's COCOeval restatement (rgbd_amd/metrics.py, host part) against the
loop-for-loop pycocotools restatement (oracle/cocoeval.py) on random and hand-built cases.  The
intersections the GPU computes are formed here with numpy (CPU test); tests/test_gpu_metrics.py
runs the whole metric with the HIP kernels.  Parity unpinned against torchmetrics itself (absent)."""
import numpy as np
import pytest

from oracle import cocoeval
from rgbd_amd import metrics


def _records(preds, targets):
    recs = []
    for p, t in zip(preds, targets):
        d = np.asarray(p["masks"], bool)
        g = np.asarray(t["masks"], bool)
        d = d.reshape(d.shape[0], d.shape[1] * d.shape[2])
        g = g.reshape(g.shape[0], g.shape[1] * g.shape[2])
        recs.append({"inter": d.astype(np.int64) @ g.astype(np.int64).T, "det_area": d.sum(1), "gt_area": g.sum(1),
                     "scores": np.asarray(p["scores"], np.float64), "det_labels": np.asarray(p["labels"]),
                     "gt_labels": np.asarray(t["labels"])})
    return recs


def _compare(preds, targets):
    got = metrics.coco_segm_summary(_records(preds, targets), class_metrics=True)
    want = cocoeval.mean_average_precision(preds, targets, class_metrics=True)
    for k, v in want.items():
        np.testing.assert_allclose(np.asarray(got[k], np.float64), np.asarray(v, np.float64), rtol=1e-6, atol=1e-7,
                                   err_msg=k)
    return got


def _rect(H, W, y0, x0, h, w):
    m = np.zeros((H, W), bool)
    m[y0:y0 + h, x0:x0 + w] = True
    return m


def _scene(rng, H=64, W=80, n_gt=6, n_det=12, n_cls=3):
    gts = [_rect(H, W, rng.integers(0, H - 8), rng.integers(0, W - 8), rng.integers(3, 40), rng.integers(3, 40))
           for _ in range(n_gt)]
    dets = []
    for _ in range(n_det):
        if gts and rng.random() < 0.6:  # a jittered copy of a ground truth
            g = gts[rng.integers(0, len(gts))]
            dets.append(np.roll(g, (rng.integers(-3, 4), rng.integers(-3, 4)), axis=(0, 1)))
        else:
            dets.append(_rect(H, W, rng.integers(0, H - 4), rng.integers(0, W - 4), rng.integers(2, 30),
                              rng.integers(2, 30)))
    scores = np.round(rng.random(n_det), 2)  # ties on purpose (stable-sort order decides)
    return ({"masks": np.stack(dets) if dets else np.zeros((0, H, W), bool), "scores": scores,
             "labels": rng.integers(0, n_cls, n_det)},
            {"masks": np.stack(gts) if gts else np.zeros((0, H, W), bool), "labels": rng.integers(0, n_cls, n_gt)})


@pytest.mark.parametrize("seed", range(4))
def test_random_scenes_match_cocoeval_restatement(seed):
    rng = np.random.default_rng(seed)
    pairs = [_scene(rng, n_gt=int(rng.integers(0, 7)), n_det=int(rng.integers(0, 14))) for _ in range(5)]
    _compare([p for p, _ in pairs], [t for _, t in pairs])


def test_more_than_100_detections_and_area_ranges():
    rng = np.random.default_rng(9)
    H, W = 200, 200
    gts = [_rect(H, W, 0, 0, 5, 5), _rect(H, W, 20, 20, 50, 50), _rect(H, W, 80, 80, 110, 110)]  # small/medium/large
    dets = [g.copy() for g in gts] + [_rect(H, W, rng.integers(0, 190), rng.integers(0, 190), 6, 6) for _ in range(120)]
    scores = np.concatenate([[0.5, 0.4, 0.3], rng.random(120)])
    p = {"masks": np.stack(dets), "scores": scores, "labels": np.zeros(123, int)}
    t = {"masks": np.stack(gts), "labels": np.zeros(3, int)}
    _compare([p], [t])


def test_hand_cases():
    H, W = 40, 40
    g = [_rect(H, W, 0, 0, 20, 20), _rect(H, W, 20, 20, 20, 20)]
    # perfect detections: every defined number is 1
    got = _compare([{"masks": np.stack(g), "scores": np.array([0.9, 0.8]), "labels": np.array([1, 2])}],
                   [{"masks": np.stack(g), "labels": np.array([1, 2])}])
    assert float(got["map"]) == pytest.approx(1.0) and float(got["mar_100"]) == pytest.approx(1.0)
    # no detections: precision 0, recall 0
    got = _compare([{"masks": np.zeros((0, H, W), bool), "scores": np.zeros(0), "labels": np.zeros(0, int)}],
                   [{"masks": np.stack(g), "labels": np.array([1, 1])}])
    assert float(got["map"]) == 0.0 and float(got["mar_100"]) == 0.0
    # a false positive scored above the true positive: AP = 0.5 at every threshold
    fp = _rect(H, W, 0, 25, 10, 10)
    got = _compare([{"masks": np.stack([fp, g[0]]), "scores": np.array([0.9, 0.8]), "labels": np.array([3, 3])}],
                   [{"masks": g[0][None], "labels": np.array([3])}])
    assert float(got["map"]) == pytest.approx(0.5)
