"""f4: the Trainer's ``compute_metrics`` for instance segmentation, kept on the device.

Drop-in for the reference's ``Evaluator`` (mask2former/utils/model_essential_part.py:31-157):
same constructor ``(image_processor, id2label, threshold)``, same call protocol under
``batch_eval_metrics=True`` (finetuning.py:52-53: ``__call__(evaluation_results,
compute_result)`` once per evaluation batch, ``None`` until the last), same result dict
(torchmetrics segm-mAP keys, the per-class lists split into ``map_<class>`` / ``mar_100_<class>``,
values rounded to 4 digits).

What happens to a batch here (the reference copies everything to the host first and
post-processes with the HF image processor on the CPU):

  1. the predictions (class logits [B, Q, L+1], mask logits [B, Q, h, w]) and the target masks
     stay on / move to the GPU — the Trainer hands the batch's device tensors to
     ``compute_metrics`` under ``batch_eval_metrics``;
  2. the instance post-processing of the whole batch is one ``rgbd_pp_instance`` launch
     (postprocess.py: the HF method's top-k, 384x384 upsampling, scores, nearest resize and
     paint, identical results); one device-to-host copy of the B x Q (label, score, segment id)
     tables gives every image's kept segments; their binary maps at the target size come from
     ``rgbd_pp_binary_maps`` without leaving the device;
  3. ``metrics.MeanAveragePrecision.update`` packs detections and ground truths into bitmaps,
     computes every image's [D, G] mask intersections and areas on the GPU and keeps only those
     small host arrays (one copy per batch);
  4. at ``compute_result`` COCOeval's matching and accumulation run on the host over those
     records (metrics.coco_segm_summary).

A class table too large for the device top-k (``postprocess._device_covers``) is
post-processed by the image processor's own method instead (the HF code path the reference
uses), then evaluated the same way.
"""
from dataclasses import dataclass
from typing import Mapping

import numpy as np
import torch

from . import postprocess
from .metrics import MeanAveragePrecision


@dataclass
class ModelOutput:  # what the image processor's post-processing reads
    class_queries_logits: torch.Tensor
    masks_queries_logits: torch.Tensor


def _to(t, dev, dtype=None):
    t = torch.as_tensor(t)
    return t.to(device=dev, dtype=dtype if dtype is not None else t.dtype)


class Evaluator:
    """segm mean average precision over the evaluation batches (model_essential_part.py:31)."""

    def __init__(self, image_processor, id2label: Mapping[int, str], threshold: float = 0.0, device=None):
        self.image_processor = image_processor
        self.id2label = id2label
        self.threshold = threshold
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.metric = MeanAveragePrecision(iou_type="segm", class_metrics=True, device=self.device)

    # -- one evaluation batch -------------------------------------------------------------
    def _targets(self, label_ids):
        masks, labels = label_ids[0], label_ids[1]
        return [{"masks": _to(m, self.device) != 0, "labels": _to(lab, self.device)} for m, lab in zip(masks, labels)]

    def _predictions(self, predictions, sizes):
        """Kept instances of every image as {masks [N, H, W] (device), labels [N], scores [N]};
        the HF method's segment order, labels and (6-digit rounded) scores."""
        cls_all, masks_all = predictions[0], predictions[1]
        outputs = ModelOutput(torch.as_tensor(cls_all), torch.as_tensor(masks_all))
        if not postprocess._device_covers(outputs):
            res = self.image_processor.post_process_instance_segmentation(
                outputs, threshold=self.threshold, target_sizes=sizes, return_binary_maps=True)
            return [self._from_segments(r["segmentation"], r["segments_info"], size) for r, size in zip(res, sizes)]
        out = []
        B = cls_all.shape[0]
        for b0 in range(0, B, postprocess.CHUNK):
            b1 = min(B, b0 + postprocess.CHUNK)
            cls = _to(cls_all[b0:b1], self.device, torch.float32).contiguous()
            masks = _to(masks_all[b0:b1], self.device, torch.float32).contiguous()
            chunk_sizes = sizes[b0:b1]
            segs, topk, ps, sid, ws = postprocess._run(cls, masks, chunk_sizes, float(self.threshold))
            C = cls.shape[-1] - 1
            # the batch's one host copy: (query index, score, segment id) per top-k entry
            tab = torch.stack([topk.double(), ps.double(), sid.double()]).cpu().numpy()
            for i, size in enumerate(chunk_sizes):
                keep = np.flatnonzero(tab[2, i] >= 0).tolist()
                if not keep:  # nothing kept: empty tensors, as the reference's void branch
                    out.append({"masks": torch.zeros((0, *size), dtype=torch.bool, device=self.device),
                                "labels": torch.zeros((0,), dtype=torch.int64),
                                "scores": torch.zeros((0,), dtype=torch.float32)})
                    continue
                maps = postprocess._binary_maps(ws, b1 - b0, cls.shape[1], i, size, sid, len(keep), self.device)
                labels = torch.tensor([int(tab[0, i, j]) % C for j in keep], dtype=torch.int64)
                # the HF method reports round(score, 6) as a Python float; the reference's tensor of them
                scores = torch.tensor([round(float(tab[1, i, j]), 6) for j in keep], dtype=torch.float32)
                out.append({"masks": maps != 0, "labels": labels, "scores": scores})
        return out

    def _from_segments(self, seg, info, size):
        if not info:
            return {"masks": torch.zeros((0, *size), dtype=torch.bool, device=self.device),
                    "labels": torch.zeros((0,), dtype=torch.int64), "scores": torch.zeros((0,), dtype=torch.float32)}
        return {"masks": _to(seg, self.device) != 0, "labels": torch.tensor([x["label_id"] for x in info]),
                "scores": torch.tensor([x["score"] for x in info])}

    @torch.no_grad()
    def __call__(self, evaluation_results, compute_result: bool = False):
        targets = self._targets(evaluation_results.label_ids)
        sizes = [tuple(int(s) for s in t["masks"].shape[-2:]) for t in targets]
        preds = self._predictions(evaluation_results.predictions, sizes)
        self.metric.update(preds, targets)  # intersections now; the bitmaps are freed here
        if not compute_result:
            return None
        res = self.metric.compute()
        self.metric.reset()
        classes = res.pop("classes").tolist()
        per_map = res.pop("map_per_class").tolist()
        per_mar = res.pop("mar_100_per_class").tolist()
        out = {k: round(float(v), 4) for k, v in res.items()}
        for c, m, r in zip(classes, per_map, per_mar):
            name = self.id2label[c] if self.id2label is not None else c
            out[f"map_{name}"] = round(float(m), 4)
            out[f"mar_100_{name}"] = round(float(r), 4)
        return out
