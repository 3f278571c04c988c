"""Oracle (test infrastructure only): torchmetrics MeanAveragePrecision(iou_type="segm") as the
reference's Evaluator uses it (mask2former/utils/model_essential_part.py:56-157), restated from
the published pycocotools 2.0 ``COCOeval`` (evaluate / evaluateImg / accumulate / summarize,
pycocotools/cocoeval.py) and ``maskApi.c`` (area, rleIou), loop for loop on plain Python lists
and numpy boolean masks.  torchmetrics and pycocotools are not installed here: parity of the
product metric (rgbd_amd/metrics.py) against this restatement is all that can be checked
("parity unpinned" against the libraries themselves).

Inputs as torchmetrics takes them: per image, preds {masks [N, H, W] bool, scores [N], labels
[N]} and target {masks [M, H, W] bool, labels [M]}; iscrowd 0 everywhere; categories = the
sorted union of all labels; annotation ids from 1 in image order.
"""
import numpy as np

IOU_THRS = np.linspace(.5, 0.95, int(np.round((0.95 - .5) / .05)) + 1, endpoint=True)
REC_THRS = np.linspace(.0, 1.00, int(np.round((1.00 - .0) / .01)) + 1, endpoint=True)
MAX_DETS = [1, 10, 100]
AREA_RNG = [[0 ** 2, 1e5 ** 2], [0 ** 2, 32 ** 2], [32 ** 2, 96 ** 2], [96 ** 2, 1e5 ** 2]]
AREA_LBL = ["all", "small", "medium", "large"]


def _iou(d, g):
    """maskApi rleIou, iscrowd 0: |d & g| / |d | g|; 0 when the boxes (hence masks) do not meet."""
    i = int(np.logical_and(d, g).sum())
    if i == 0:
        return 0.0
    u = int(np.logical_or(d, g).sum())
    return i / u


class COCOevalSegm:
    def __init__(self, preds, targets):
        self.gts, self.dts = {}, {}
        cats = set()
        aid = 1
        for img, (p, t) in enumerate(zip(preds, targets)):
            for m, lab in zip(t["masks"], t["labels"]):
                cats.add(int(lab))
                self.gts.setdefault((img, int(lab)), []).append(
                    {"id": aid, "area": float(np.asarray(m).sum()), "mask": np.asarray(m, bool), "ignore": 0})
                aid += 1
            for m, s, lab in zip(p["masks"], p["scores"], p["labels"]):
                cats.add(int(lab))
                self.dts.setdefault((img, int(lab)), []).append(
                    {"id": aid, "area": float(np.asarray(m).sum()), "mask": np.asarray(m, bool), "score": float(s)})
                aid += 1
        self.img_ids = list(range(len(preds)))
        self.cat_ids = sorted(cats)

    def compute_iou(self, img, cat):
        gt = self.gts.get((img, cat), [])
        dt = self.dts.get((img, cat), [])
        if len(gt) == 0 and len(dt) == 0:
            return []
        inds = np.argsort([-d["score"] for d in dt], kind="mergesort")
        dt = [dt[i] for i in inds]
        if len(dt) > MAX_DETS[-1]:
            dt = dt[0:MAX_DETS[-1]]
        return np.array([[_iou(d["mask"], g["mask"]) for g in gt] for d in dt]).reshape(len(dt), len(gt))

    def evaluate_img(self, img, cat, a_rng, max_det):
        gt = self.gts.get((img, cat), [])
        dt = self.dts.get((img, cat), [])
        if len(gt) == 0 and len(dt) == 0:
            return None
        for g in gt:
            g["_ignore"] = 1 if (g["ignore"] or (g["area"] < a_rng[0] or g["area"] > a_rng[1])) else 0
        gtind = np.argsort([g["_ignore"] for g in gt], kind="mergesort")
        gt = [gt[i] for i in gtind]
        dtind = np.argsort([-d["score"] for d in dt], kind="mergesort")
        dt = [dt[i] for i in dtind[0:max_det]]
        ious = self.ious[img, cat][:, gtind] if len(self.ious[img, cat]) > 0 else self.ious[img, cat]
        T, G, D = len(IOU_THRS), len(gt), len(dt)
        gtm = np.zeros((T, G))
        dtm = np.zeros((T, D))
        gt_ig = np.array([g["_ignore"] for g in gt])
        dt_ig = np.zeros((T, D))
        if not len(ious) == 0:
            for tind, t in enumerate(IOU_THRS):
                for dind, d in enumerate(dt):
                    iou = min([t, 1 - 1e-10])
                    m = -1
                    for gind, g in enumerate(gt):
                        if gtm[tind, gind] > 0:
                            continue
                        if m > -1 and gt_ig[m] == 0 and gt_ig[gind] == 1:
                            break
                        if ious[dind, gind] < iou:
                            continue
                        iou = ious[dind, gind]
                        m = gind
                    if m == -1:
                        continue
                    dt_ig[tind, dind] = gt_ig[m]
                    dtm[tind, dind] = gt[m]["id"]
                    gtm[tind, m] = d["id"]
        a = np.array([d["area"] < a_rng[0] or d["area"] > a_rng[1] for d in dt]).reshape((1, len(dt)))
        dt_ig = np.logical_or(dt_ig, np.logical_and(dtm == 0, np.repeat(a, T, 0)))
        return {"dtScores": [d["score"] for d in dt], "dtMatches": dtm, "dtIgnore": dt_ig, "gtIgnore": gt_ig}

    def evaluate(self):
        self.ious = {(i, c): self.compute_iou(i, c) for i in self.img_ids for c in self.cat_ids}
        self.eval_imgs = [self.evaluate_img(i, c, a, MAX_DETS[-1])
                          for c in self.cat_ids for a in AREA_RNG for i in self.img_ids]

    def accumulate(self):
        T, R, K, A, M = len(IOU_THRS), len(REC_THRS), len(self.cat_ids), len(AREA_RNG), len(MAX_DETS)
        precision = -np.ones((T, R, K, A, M))
        recall = -np.ones((T, K, A, M))
        I0, A0 = len(self.img_ids), len(AREA_RNG)
        for k in range(K):
            Nk = k * A0 * I0
            for a in range(A):
                Na = a * I0
                for m, max_det in enumerate(MAX_DETS):
                    E = [self.eval_imgs[Nk + Na + i] for i in range(I0)]
                    E = [e for e in E if e is not None]
                    if len(E) == 0:
                        continue
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
                        tp, fp = np.array(tp), np.array(fp)
                        nd = len(tp)
                        rc = tp / npig
                        pr = tp / (fp + tp + np.spacing(1))
                        q = np.zeros((R,))
                        recall[t, k, a, m] = rc[-1] if nd else 0
                        pr, q = pr.tolist(), q.tolist()
                        for i in range(nd - 1, 0, -1):
                            if pr[i] > pr[i - 1]:
                                pr[i - 1] = pr[i]
                        inds = np.searchsorted(rc, REC_THRS, side="left")
                        try:
                            for ri, pi in enumerate(inds):
                                q[ri] = pr[pi]
                        except IndexError:
                            pass
                        precision[t, :, k, a, m] = np.array(q)
        self.precision, self.recall = precision, recall

    def _summarize(self, ap=1, iou_thr=None, area="all", max_dets=100, k=None):
        aind = [i for i, lbl in enumerate(AREA_LBL) if lbl == area]
        mind = [i for i, d in enumerate(MAX_DETS) if d == max_dets]
        ks = slice(None) if k is None else [k]
        if ap == 1:
            s = self.precision
            if iou_thr is not None:
                s = s[np.where(iou_thr == IOU_THRS)[0]]
            s = s[:, :, ks, aind, mind]
        else:
            s = self.recall
            if iou_thr is not None:
                s = s[np.where(iou_thr == IOU_THRS)[0]]
            s = s[:, ks, aind, mind]
        return -1.0 if len(s[s > -1]) == 0 else float(np.mean(s[s > -1]))

    def summarize(self, k=None):
        S = self._summarize
        return {"map": S(1, k=k), "map_50": S(1, .5, k=k), "map_75": S(1, .75, k=k),
                "map_small": S(1, area="small", k=k), "map_medium": S(1, area="medium", k=k),
                "map_large": S(1, area="large", k=k), "mar_1": S(0, max_dets=1, k=k), "mar_10": S(0, max_dets=10, k=k),
                "mar_100": S(0, k=k), "mar_small": S(0, area="small", k=k), "mar_medium": S(0, area="medium", k=k),
                "mar_large": S(0, area="large", k=k)}


def mean_average_precision(preds, targets, class_metrics=False):
    ev = COCOevalSegm(preds, targets)
    ev.evaluate()
    ev.accumulate()
    out = ev.summarize()
    if class_metrics:
        per = [ev.summarize(k) for k in range(len(ev.cat_ids))]
        out["map_per_class"] = [p["map"] for p in per]
        out["mar_100_per_class"] = [p["mar_100"] for p in per]
    out["classes"] = list(ev.cat_ids)
    return out
