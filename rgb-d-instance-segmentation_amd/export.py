"""f4: COCO-RLE JSON export of instance predictions and ground-truth labels.

Reference: mask2former/predictor.py — ``convert_model_a_to_json_format`` (:335-372) over
``_convert_single_prediction_to_json`` (:376-457) for the post-processed predictions, and
``convert_gt_labels_to_json_format`` (:491-525) over ``_convert_single_gt_label_to_json``
(:528-625) for the labels; one ``<image name>.json`` per image:

    {"labels": [int], "scores": [float], "bboxes": [[x, y, w, h]], "masks": [{"size": [h, w],
     "counts": <pycocotools compressed RLE string>}]}

The reference builds every instance's binary mask on the host (``segmentation == id``), its
bounding box, and ``pycocotools.mask.encode`` of it.  Here the per-instance run boundaries and
boxes come from one pass over the map on whatever device holds it (the device post-processing
leaves the maps on the GPU with ``keep_on_device``): the map is read column-major once per
instance as a boolean vector, run boundaries are the positions where it changes; the compressed
string (maskApi.c ``rleToString``) is formed on the host from the counts.  pycocotools is not
installed here: the encoding is pinned against a step-for-step restatement of maskApi.c
(oracle/rle.py) and its decode round trip (tests/test_export.py).
"""
import json
import logging
from pathlib import Path

import numpy as np
import torch

log = logging.getLogger(__name__)


def _to_string(counts) -> str:
    """maskApi.c rleToString (counts i > 2 delta-coded against count i - 2, 5-bit groups)."""
    out = []
    prev2 = prev1 = 0
    for i, cnt in enumerate(counts):
        x = cnt - prev2 if i > 2 else cnt
        prev2, prev1 = prev1, cnt
        while True:
            c = x & 0x1F
            x >>= 5
            more = (x != -1) if (c & 0x10) else (x != 0)
            out.append(chr((c | 0x20 if more else c) + 48))
            if not more:
                break
    return "".join(out)


def _runs(colmajor: torch.Tensor):
    """Counts of a column-major boolean vector: zeros first (0 when it starts set)."""
    n = colmajor.numel()
    change = torch.nonzero(colmajor[1:] != colmajor[:-1]).reshape(-1) + 1
    bounds = torch.cat([change.new_zeros(1), change, change.new_full((1,), n)]).cpu().numpy()
    counts = np.diff(bounds).tolist()
    if bool(colmajor[0]):
        counts = [0] + counts
    return counts


def encode_masks(masks: torch.Tensor):
    """masks bool/0-1 [N, h, w] (any device) -> list of (rle dict, bbox [x, y, w, h] or None), the
    pycocotools.mask.encode + _calculate_bbox_from_mask pair of the reference per mask."""
    N, h, w = masks.shape
    out = []
    cm = masks.bool().transpose(1, 2).reshape(N, -1)  # column-major per mask
    rows = masks.bool().any(dim=2)
    cols = masks.bool().any(dim=1)
    for i in range(N):
        counts = _runs(cm[i])
        r = torch.nonzero(rows[i]).reshape(-1)
        c = torch.nonzero(cols[i]).reshape(-1)
        bbox = None
        if r.numel():
            y0, y1, x0, x1 = int(r[0]), int(r[-1]), int(c[0]), int(c[-1])
            bbox = [float(x0), float(y0), float(x1 - x0 + 1), float(y1 - y0 + 1)]
        out.append(({"size": [int(h), int(w)], "counts": _to_string(counts)}, bbox))
    return out


def prediction_to_json(prediction: dict, original_size=None) -> dict:
    """_convert_single_prediction_to_json (predictor.py:376-457): every segment of the
    post-processed map whose mask is non-empty, in segments_info order."""
    seg = prediction["segmentation"]
    seg = seg if isinstance(seg, torch.Tensor) else torch.as_tensor(np.asarray(seg))
    info = prediction["segments_info"]
    h, w = (int(original_size[0]), int(original_size[1])) if original_size is not None else tuple(seg.shape[:2])
    labels, scores, bboxes, masks = [], [], [], []
    if info:
        ids = torch.tensor([s["id"] for s in info], dtype=seg.dtype, device=seg.device)
        enc = encode_masks(seg[None] == ids[:, None, None])
        for s, (rle, bbox) in zip(info, enc):
            if bbox is None:
                log.warning("instance id %s has an empty mask: skipped", s["id"])
                continue
            labels.append(int(s["label_id"]))
            scores.append(float(s.get("score", 1.0)))
            bboxes.append(bbox)
            masks.append({"size": [h, w], "counts": rle["counts"]})
    return {"labels": labels, "scores": scores, "bboxes": bboxes, "masks": masks}


def gt_label_to_json(label_info, original_size=None) -> dict:
    """_convert_single_gt_label_to_json (predictor.py:528-625): label_info = [masks, ids] with
    masks [N, h, w] (one per instance, > 0 = set) or an [h, w] instance-id map; ids <= 0 and
    empty masks are skipped; scores 1.0."""
    masks, ids = label_info
    masks = masks if isinstance(masks, torch.Tensor) else torch.as_tensor(np.asarray(masks))
    if masks.dim() not in (2, 3):
        raise ValueError(f"unsupported masks shape {tuple(masks.shape)}")
    h, w = (int(original_size[0]), int(original_size[1])) if original_size is not None else tuple(masks.shape[-2:])
    if masks.dim() == 3:
        ids_l = [int(i) for i in (np.asarray(ids).reshape(-1) if hasattr(ids, "__len__") else [ids] * masks.shape[0])]
        keep = [i for i in range(masks.shape[0]) if ids_l[i] > 0]
        sel = masks[keep] > 0 if keep else masks.new_zeros((0, *masks.shape[-2:]), dtype=torch.bool)
        lab = [ids_l[i] for i in keep]
    else:
        u = torch.unique(masks)
        u = u[u > 0]
        sel = masks[None] == u[:, None, None]
        lab = [int(x) for x in u.tolist()]
    labels, scores, bboxes, rles = [], [], [], []
    for lid, (rle, bbox) in zip(lab, encode_masks(sel) if len(lab) else []):
        if bbox is None:
            continue
        labels.append(lid)
        scores.append(1.0)
        bboxes.append(bbox)
        rles.append({"size": [h, w], "counts": rle["counts"]})
    return {"labels": labels, "scores": scores, "bboxes": bboxes, "masks": rles}


def _write_all(items, names, save_dir, convert, sizes):
    path = Path(save_dir)
    path.mkdir(parents=True, exist_ok=True)
    written = []
    for i, (item, name) in enumerate(zip(items, names)):
        data = convert(item, sizes[i] if sizes else None)
        f = path / f"{name}.json"
        with open(f, "w") as fh:
            json.dump(data, fh, indent=2)
        written.append(f)
    return written


def convert_predictions_to_json(predicted_instance_maps, image_names, save_dir, original_sizes=None):
    """convert_model_a_to_json_format (predictor.py:335-372): one JSON file per image."""
    return _write_all(predicted_instance_maps, image_names, save_dir, prediction_to_json, original_sizes)


def convert_gt_labels_to_json(label_data, image_names, save_dir, original_sizes=None):
    """convert_gt_labels_to_json_format (predictor.py:491-525)."""
    return _write_all(label_data, image_names, save_dir, gt_label_to_json, original_sizes)
