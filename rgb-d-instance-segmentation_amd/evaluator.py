"""f4: the reference's Evaluator (mask2former/utils/model_essential_part.py:31-157) on the device
path: the Trainer's ``compute_metrics`` for instance segmentation.

Same constructor (image_processor, id2label, threshold), same ``__call__(evaluation_results,
compute_result)`` protocol under ``batch_eval_metrics=True`` (finetuning.py:52-53), same target /
prediction post-processing (``post_process_instance_segmentation(..., threshold, target_sizes,
return_binary_maps=True)``) and the same returned dict (torchmetrics' keys with the per-class
lists split into ``map_<class>`` / ``mar_100_<class>``, every value rounded to 4 digits).  The
metric is metrics.MeanAveragePrecision(iou_type="segm", class_metrics=True): the mask IoU on
the GPU kernels, COCOeval's matching and accumulation on the host.  With an image processor that
went through ``postprocess.install`` the post-processing runs on the GPU as well.
"""
from dataclasses import dataclass
from typing import Dict, List, Mapping

import torch

from .metrics import MeanAveragePrecision


@dataclass
class ModelOutput:
    class_queries_logits: torch.Tensor
    masks_queries_logits: torch.Tensor


def nested_cpu(tensors):
    if isinstance(tensors, (list, tuple)):
        return type(tensors)(nested_cpu(t) for t in tensors)
    if isinstance(tensors, Mapping):
        return type(tensors)({k: nested_cpu(t) for k, t in tensors.items()})
    if isinstance(tensors, torch.Tensor):
        return tensors.cpu().detach()
    return tensors


class Evaluator:
    """Compute metrics for the instance segmentation task (model_essential_part.py:31)."""

    def __init__(self, image_processor, id2label: Mapping[int, str], threshold: float = 0.0, device=None):
        self.image_processor = image_processor
        self.id2label = id2label
        self.threshold = threshold
        self.device = device
        self.metric = self.get_metric()

    def get_metric(self):
        return MeanAveragePrecision(iou_type="segm", class_metrics=True, device=self.device)

    def reset_metric(self):
        self.metric.reset()

    def postprocess_target_batch(self, target_batch) -> List[Dict[str, torch.Tensor]]:
        batch_masks, batch_labels = target_batch[0], target_batch[1]
        return [{"masks": masks.to(dtype=torch.bool), "labels": labels} for masks, labels in zip(batch_masks, batch_labels)]

    def get_target_sizes(self, post_processed_targets) -> List[List[int]]:
        return [target["masks"].shape[-2:] for target in post_processed_targets]

    def postprocess_prediction_batch(self, prediction_batch, target_sizes) -> List[Dict[str, torch.Tensor]]:
        model_output = ModelOutput(class_queries_logits=prediction_batch[0], masks_queries_logits=prediction_batch[1])
        post_processed_output = self.image_processor.post_process_instance_segmentation(
            model_output, threshold=self.threshold, target_sizes=target_sizes, return_binary_maps=True)
        out = []
        for image_predictions, target_size in zip(post_processed_output, target_sizes):
            if image_predictions["segments_info"]:
                out.append({"masks": image_predictions["segmentation"].to(dtype=torch.bool),
                            "labels": torch.tensor([x["label_id"] for x in image_predictions["segments_info"]]),
                            "scores": torch.tensor([x["score"] for x in image_predictions["segments_info"]])})
            else:  # void predictions: empty tensors, as the reference
                out.append({"masks": torch.zeros([0, *target_size], dtype=torch.bool),
                            "labels": torch.tensor([]), "scores": torch.tensor([])})
        return out

    @torch.no_grad()
    def __call__(self, evaluation_results, compute_result: bool = False) -> Mapping[str, float]:
        prediction_batch = nested_cpu(evaluation_results.predictions)
        target_batch = nested_cpu(evaluation_results.label_ids)
        post_processed_targets = self.postprocess_target_batch(target_batch)
        target_sizes = self.get_target_sizes(post_processed_targets)
        post_processed_predictions = self.postprocess_prediction_batch(prediction_batch, target_sizes)
        self.metric.update(post_processed_predictions, post_processed_targets)
        if not compute_result:
            return None
        metrics = self.metric.compute()
        classes = metrics.pop("classes")
        map_per_class = metrics.pop("map_per_class")
        mar_100_per_class = metrics.pop("mar_100_per_class")
        for class_id, class_map, class_mar in zip(classes, map_per_class, mar_100_per_class):
            class_name = self.id2label[class_id.item()] if self.id2label is not None else class_id.item()
            metrics[f"map_{class_name}"] = class_map
            metrics[f"mar_100_{class_name}"] = class_mar
        metrics = {k: round(v.item(), 4) for k, v in metrics.items()}
        self.reset_metric()
        return metrics
