"""f4: COCO-RLE JSON export of instance predictions and ground-truth labels.

Reference: mask2former/predictor.py — ``convert_model_a_to_json_format`` (:335-372) over
``_convert_single_prediction_to_json`` (:376-457) for the post-processed predictions, and
``convert_gt_labels_to_json_format`` (:491-525) over ``_convert_single_gt_label_to_json``
(:528-625) for the labels; one ``<image name>.json`` per image:

    {"labels": [int], "scores": [float], "bboxes": [[x, y, w, h]], "masks": [{"size": [h, w],
     "counts": <pycocotools compressed RLE string>}]}

The reference builds every instance's binary mask on the host (``segmentation == id``), its
bounding box, and ``pycocotools.mask.encode`` of it.  Here the run boundaries and boxes of all
of an image's instances come from one pass on whatever device holds the map (the device
post-processing leaves the maps on the GPU with ``keep_on_device``): the stacked masks are read
column-major, run boundaries are the positions where a mask changes (one nonzero over all of
them), and one copy brings boundaries and boxes to the host, where the compressed string
(maskApi.c ``rleToString``) is formed from the counts.  pycocotools is not
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


def encode_masks(masks: torch.Tensor):
    """masks bool/0-1 [N, h, w] (any device) -> list of (rle dict, bbox [x, y, w, h] or None), the
    pycocotools.mask.encode + _calculate_bbox_from_mask pair of the reference per mask.

    All N masks at once on their device: the column-major change positions of every mask come
    from one nonzero over the [N, h*w - 1] change map, the boxes from the row / column
    occupancy, and the whole result reaches the host in one copy (no per-mask sync)."""
    N, h, w = masks.shape
    if N == 0:
        return []
    L = h * w
    mb = masks.bool()
    cm = mb.transpose(1, 2).reshape(N, L)                      # column-major per mask
    pos = torch.nonzero(cm[:, 1:] != cm[:, :-1])              # [M, 2]: (mask, change index - 1)
    rows, cols = mb.any(dim=2), mb.any(dim=1)                 # [N, h], [N, w]
    ar_h = torch.arange(h, device=mb.device)
    ar_w = torch.arange(w, device=mb.device)
    big = max(h, w) + 1
    y0 = torch.where(rows, ar_h, big).amin(1)
    y1 = torch.where(rows, ar_h, -1).amax(1)
    x0 = torch.where(cols, ar_w, big).amin(1)
    x1 = torch.where(cols, ar_w, -1).amax(1)
    meta = torch.stack([cm[:, 0].long(), y0, y1, x0, x1], 1)  # [N, 5]
    flat = torch.cat([meta.reshape(-1), pos.reshape(-1).long()]).cpu().numpy()
    meta_h = flat[:5 * N].reshape(N, 5)
    pos_h = flat[5 * N:].reshape(-1, 2)
    starts = np.searchsorted(pos_h[:, 0], np.arange(N + 1), side="left")
    out = []
    for i in range(N):
        change = pos_h[starts[i]:starts[i + 1], 1] + 1
        bounds = np.concatenate([[0], change, [L]])
        counts = np.diff(bounds).tolist()
        if meta_h[i, 0]:
            counts = [0] + counts
        bbox = None
        if meta_h[i, 2] >= 0:
            yy0, yy1, xx0, xx1 = (int(v) for v in meta_h[i, 1:])
            bbox = [float(xx0), float(yy0), float(xx1 - xx0 + 1), float(yy1 - yy0 + 1)]
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
