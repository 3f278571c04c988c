"""f4: the segm mean average precision of the reference's Evaluator, with the mask IoU on the GPU.

Reference: ``Evaluator`` (mask2former/utils/model_essential_part.py:31-157) accumulates
``torchmetrics.detection.MeanAveragePrecision(iou_type="segm", class_metrics=True)`` over the
evaluation batches; torchmetrics hands the masks to pycocotools (RLE, ``maskApi.rleIou``) and
runs ``COCOeval`` (``evaluate`` / ``accumulate`` / ``summarize``).  Neither library is installed
here, so this module restates that evaluation:

  * update(): every image's detection and ground-truth masks are packed into bitmaps on the GPU
    with their areas (csrc/mask_iou.hip ``rgbd_pack_mask_bits``), the intersections of every
    (detection, ground truth) pair follow in one launch per image (``rgbd_mask_intersections``),
    and one device-to-host copy per update keeps only those small arrays (the bitmaps are
    freed; torchmetrics likewise keeps compact RLEs, not masks);
  * compute(): per image IoU = inter / union (0 when inter == 0, as rleIou), then COCOeval's per (image, category) greedy matching at the 10 IoU thresholds
    0.50:0.05:0.95 and the area ranges all / small (< 32^2) / medium / large (> 96^2), detections
    ordered by score (stable) and capped at 100, the 101-point interpolated precision and the
    recall per category, and the 12 summary numbers; with ``class_metrics`` the per-category
    mAP and mAR@100 (torchmetrics' per-class COCOeval runs equal the per-category slices).

The output dict has torchmetrics' keys (map, map_50, map_75, map_small, map_medium, map_large,
mar_1, mar_10, mar_100, mar_small, mar_medium, mar_large, map_per_class, mar_100_per_class,
classes) as float32 / int32 tensors.  Parity: unpinned against torchmetrics / pycocotools
(absent); checked against a loop-for-loop restatement of COCOeval (oracle/cocoeval.py) and
hand-computed cases (tests/test_metrics.py, tests/test_gpu_metrics.py).
"""
import numpy as np
import torch

from . import _lib
from ._lib import check
from .ops import _need_cuda, _p, _stream

IOU_THRS = np.linspace(0.5, 0.95, int(np.round((0.95 - 0.5) / 0.05)) + 1, endpoint=True)
REC_THRS = np.linspace(0.0, 1.00, int(np.round((1.00 - 0.0) / 0.01)) + 1, endpoint=True)
MAX_DETS = [1, 10, 100]
AREA_RNG = [[0 ** 2, 1e5 ** 2], [0 ** 2, 32 ** 2], [32 ** 2, 96 ** 2], [96 ** 2, 1e5 ** 2]]


class _Packed:
    """Masks of one image side (detections or ground truth), packed on the device."""

    def __init__(self, masks, dev):
        n = int(masks.shape[0])
        self.n = n
        self.shape = tuple(int(x) for x in masks.shape[-2:])
        npx = self.shape[0] * self.shape[1]
        self.npx = npx
        words = (npx + 63) // 64
        self.bits = torch.empty((max(n, 1), words), dtype=torch.int64, device=dev)
        area = torch.empty((max(n, 1),), dtype=torch.int32, device=dev)
        if n:
            m = masks.to(device=dev).reshape(n, npx)
            m = (m != 0).to(torch.uint8).contiguous()
            _need_cuda(m)
            check(_lib.lib().rgbd_pack_mask_bits(_p(m), n, npx, _p(self.bits), _p(area), _stream(dev)),
                  "rgbd_pack_mask_bits")
        self.area = area[:n]


def _intersections(a: _Packed, b: _Packed, dev):
    if a.shape != b.shape:
        raise ValueError(f"detection masks {a.shape} and ground-truth masks {b.shape} differ in size")
    inter = torch.zeros((max(a.n, 1), max(b.n, 1)), dtype=torch.int32, device=dev)
    if a.n and b.n:
        check(_lib.lib().rgbd_mask_intersections(_p(a.bits), a.n, _p(b.bits), b.n, a.npx, _p(inter), _stream(dev)),
              "rgbd_mask_intersections")
    return inter[:a.n, :b.n]


def mask_ious(inter: np.ndarray, area_d: np.ndarray, area_g: np.ndarray) -> np.ndarray:
    """maskApi rleIou (iscrowd 0): i / (ad + ag - i), 0 where i == 0."""
    inter = inter.astype(np.float64)
    union = area_d[:, None].astype(np.float64) + area_g[None, :].astype(np.float64) - inter
    out = np.zeros_like(inter)
    nz = inter > 0
    out[nz] = inter[nz] / union[nz]
    return out


def evaluate_img(ious, dt_scores, dt_areas, gt_areas, a_rng, max_det):
    """COCOeval.evaluateImg for one (image, category, area range); detections already in score
    order (stable) and capped at 100, ``ious`` [D, G] in that order.  None when neither side has
    anything (pycocotools' convention)."""
    G, D = len(gt_areas), len(dt_scores)
    if G == 0 and D == 0:
        return None
    gt_ig = np.array([1 if (a < a_rng[0] or a > a_rng[1]) else 0 for a in gt_areas], dtype=np.int64)
    gtind = np.argsort(gt_ig, kind="mergesort")
    gt_ig = gt_ig[gtind]
    dtind = np.argsort(-np.asarray(dt_scores, dtype=np.float64), kind="mergesort")[:max_det]
    scores = np.asarray(dt_scores, dtype=np.float64)[dtind]
    d_area = np.asarray(dt_areas, dtype=np.float64)[dtind]
    iou = ious[dtind][:, gtind] if ious.size else np.zeros((len(dtind), G))
    T = len(IOU_THRS)
    gtm = np.zeros((T, G), dtype=np.int64)
    dtm = np.zeros((T, len(dtind)), dtype=np.int64)
    dt_ig = np.zeros((T, len(dtind)), dtype=bool)
    if G:
        for ti, t in enumerate(IOU_THRS):
            for di in range(len(dtind)):
                best = min(t, 1 - 1e-10)
                m = -1
                for gi in range(G):
                    if gtm[ti, gi] > 0:  # iscrowd 0: a matched ground truth stays taken
                        continue
                    if m > -1 and gt_ig[m] == 0 and gt_ig[gi] == 1:
                        break
                    if iou[di, gi] < best:
                        continue
                    best = iou[di, gi]
                    m = gi
                if m == -1:
                    continue
                dt_ig[ti, di] = bool(gt_ig[m])
                dtm[ti, di] = gtind[m] + 1       # ground-truth ids 1.. (COCO annotation ids)
                gtm[ti, m] = di + 1
    out_of_range = np.array([(a < a_rng[0] or a > a_rng[1]) for a in d_area], dtype=bool).reshape(1, -1)
    dt_ig = np.logical_or(dt_ig, np.logical_and(dtm == 0, np.repeat(out_of_range, T, 0)))
    return {"dtScores": scores, "dtMatches": dtm, "dtIgnore": dt_ig, "gtIgnore": gt_ig}


def accumulate(evals, n_cats):
    """COCOeval.accumulate -> precision [T, R, K, A, M], recall [T, K, A, M] (-1 = no data).
    ``evals[k][a]``: the list over images of evaluate_img results for category k, area a."""
    T, R, A, M = len(IOU_THRS), len(REC_THRS), len(AREA_RNG), len(MAX_DETS)
    precision = -np.ones((T, R, n_cats, A, M))
    recall = -np.ones((T, n_cats, A, M))
    for k in range(n_cats):
        for a in range(A):
            E = [e for e in evals[k][a] if e is not None]
            if not E:
                continue
            for m, max_det in enumerate(MAX_DETS):
                dt_scores = np.concatenate([e["dtScores"][0:max_det] for e in E])
                inds = np.argsort(-dt_scores, kind="mergesort")
                dtm = np.concatenate([e["dtMatches"][:, 0:max_det] for e in E], axis=1)[:, inds]
                dt_ig = np.concatenate([e["dtIgnore"][:, 0:max_det] for e in E], axis=1)[:, inds]
                gt_ig = np.concatenate([e["gtIgnore"] for e in E])
                npig = np.count_nonzero(gt_ig == 0)
                if npig == 0:
                    continue
                tps = np.logical_and(dtm, np.logical_not(dt_ig))
                fps = np.logical_and(np.logical_not(dtm), np.logical_not(dt_ig))
                tp_sum = np.cumsum(tps, axis=1).astype(dtype=float)
                fp_sum = np.cumsum(fps, axis=1).astype(dtype=float)
                for t, (tp, fp) in enumerate(zip(tp_sum, fp_sum)):
                    nd = len(tp)
                    rc = tp / npig
                    pr = tp / (fp + tp + np.spacing(1))
                    q = np.zeros((R,))
                    recall[t, k, a, m] = rc[-1] if nd else 0
                    pr = pr.tolist()
                    for i in range(nd - 1, 0, -1):
                        if pr[i] > pr[i - 1]:
                            pr[i - 1] = pr[i]
                    ri_idx = np.searchsorted(rc, REC_THRS, side="left")
                    for ri, pi in enumerate(ri_idx):
                        if pi >= nd:
                            break
                        q[ri] = pr[pi]
                    precision[t, :, k, a, m] = q
    return precision, recall


def _mean_valid(s):
    v = s[s > -1]
    return -1.0 if v.size == 0 else float(np.mean(v))


def summarize(precision, recall, k_sel=None):
    """COCOeval.summarize's 12 numbers (torchmetrics' names); ``k_sel`` restricts categories."""
    ks = slice(None) if k_sel is None else [k_sel]
    m_idx = {d: i for i, d in enumerate(MAX_DETS)}

    def ap(iou=None, area=0, md=100):
        s = precision[:, :, ks, area, m_idx[md]]
        if iou is not None:
            s = s[np.where(IOU_THRS == iou)[0]]
        return _mean_valid(s)

    def ar(area=0, md=100):
        return _mean_valid(recall[:, ks, area, m_idx[md]])
    return {"map": ap(), "map_50": ap(0.5), "map_75": ap(0.75), "map_small": ap(area=1),
            "map_medium": ap(area=2), "map_large": ap(area=3), "mar_1": ar(md=1), "mar_10": ar(md=10),
            "mar_100": ar(), "mar_small": ar(area=1), "mar_medium": ar(area=2), "mar_large": ar(area=3)}


class MeanAveragePrecision:
    """torchmetrics.detection.MeanAveragePrecision(iou_type="segm", class_metrics=...) as the
    reference's Evaluator uses it: update(preds, target) with per-image dicts (preds: masks
    [N, H, W] bool, scores [N], labels [N]; target: masks, labels), compute(), reset()."""

    def __init__(self, iou_type="segm", class_metrics=False, device=None):
        if iou_type != "segm":
            raise NotImplementedError("only iou_type='segm' (the reference's Evaluator)")
        self.class_metrics = class_metrics
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.reset()

    def reset(self):
        self._images = []

    def update(self, preds, target):
        if len(preds) != len(target):
            raise ValueError("preds and target must have the same number of images")
        parts, shapes = [], []
        for p, t in zip(preds, target):
            det = _Packed(p["masks"], self.device)
            gt = _Packed(t["masks"], self.device)
            inter = _intersections(det, gt, self.device)
            parts += [inter.reshape(-1), det.area, gt.area]
            shapes.append((det.n, gt.n))
            self._images.append({
                "scores": np.asarray(torch.as_tensor(p["scores"]).float().cpu().numpy(), dtype=np.float64).reshape(-1),
                "det_labels": np.asarray(torch.as_tensor(p["labels"]).cpu().numpy()).astype(np.int64).reshape(-1),
                "gt_labels": np.asarray(torch.as_tensor(t["labels"]).cpu().numpy()).astype(np.int64).reshape(-1)})
        if not shapes:
            return
        flat = torch.cat(parts).cpu().numpy()  # the update's one copy back; bitmaps die with det / gt
        off = 0
        for im, (nd, ng) in zip(self._images[len(self._images) - len(shapes):], shapes):
            im["inter"] = flat[off:off + nd * ng].reshape(nd, ng)
            off += nd * ng
            im["det_area"] = flat[off:off + nd]
            off += nd
            im["gt_area"] = flat[off:off + ng]
            off += ng

    def compute(self):
        return coco_segm_summary(self._images, self.class_metrics)


def coco_segm_summary(records, class_metrics=False):
    """COCOeval over per-image records {inter [D, G], det_area [D], gt_area [G], scores [D],
    det_labels [D], gt_labels [G]} -> torchmetrics' result dict (host numpy; the device part is
    the intersections)."""
    labs = [r["det_labels"] for r in records] + [r["gt_labels"] for r in records]
    classes = sorted(set(int(x) for a in labs for x in np.asarray(a).tolist()))
    K, A = len(classes), len(AREA_RNG)
    cidx = {c: i for i, c in enumerate(classes)}
    evals = [[[] for _ in range(A)] for _ in range(K)]
    for r in records:
        inter, ad, ag = r["inter"], np.asarray(r["det_area"]), np.asarray(r["gt_area"])
        scores = np.asarray(r["scores"], dtype=np.float64)
        dlab, glab = np.asarray(r["det_labels"]), np.asarray(r["gt_labels"])
        for c in classes:
            di = np.flatnonzero(dlab == c)
            gi = np.flatnonzero(glab == c)
            # computeIoU: detections by score (stable), the first 100
            order = di[np.argsort(-scores[di], kind="mergesort")][:MAX_DETS[-1]]
            ious = mask_ious(inter[np.ix_(order, gi)], ad[order], ag[gi]) if len(order) and len(gi) else \
                np.zeros((len(order), len(gi)))
            for a in range(A):
                evals[cidx[c]][a].append(evaluate_img(ious, scores[order], ad[order], ag[gi], AREA_RNG[a],
                                                      MAX_DETS[-1]))
    precision, recall = accumulate(evals, K)
    out = {k: torch.tensor(v, dtype=torch.float32) for k, v in summarize(precision, recall).items()}
    if class_metrics and K:
        per = [summarize(precision, recall, k) for k in range(K)]
        out["map_per_class"] = torch.tensor([p["map"] for p in per], dtype=torch.float32)
        out["mar_100_per_class"] = torch.tensor([p["mar_100"] for p in per], dtype=torch.float32)
    else:
        out["map_per_class"] = torch.tensor([-1.0])
        out["mar_100_per_class"] = torch.tensor([-1.0])
    out["classes"] = torch.tensor(classes, dtype=torch.int32)
    return out
