"""Test-only checker: the reference's per-image matcher cost in torch (transformers 5.15
modeling_mask2former.py:445-470, the library the reference trains through), restated op for op;
tests/test_gpu_point_loss.py compares the HIP batched costs against it."""
import torch
from transformers.models.mask2former.modeling_mask2former import (pair_wise_dice_loss,
                                                                  pair_wise_sigmoid_cross_entropy_loss,
                                                                  sample_point)


def matching_cost(matcher, masks_queries_logits, class_queries_logits, mask_labels, class_labels, i):
    """Cost matrix of image i, as the reference builds it (modeling_mask2former.py:445-470)."""
    probs = class_queries_logits[i].softmax(-1)
    pred = masks_queries_logits[i]
    c_class = -probs[:, class_labels[i]]
    tgt = mask_labels[i].to(pred)[:, None]
    pred = pred[:, None]
    pts = torch.rand(1, matcher.num_points, 2, device=pred.device)
    tgt = sample_point(tgt, pts.repeat(tgt.shape[0], 1, 1), align_corners=False).squeeze(1)
    pred = sample_point(pred, pts.repeat(pred.shape[0], 1, 1), align_corners=False).squeeze(1)
    c_mask = pair_wise_sigmoid_cross_entropy_loss(pred, tgt)
    c_dice = pair_wise_dice_loss(pred, tgt)
    cost = matcher.cost_mask * c_mask + matcher.cost_class * c_class + matcher.cost_dice * c_dice
    cost = torch.minimum(cost, torch.tensor(1e10))
    cost = torch.maximum(cost, torch.tensor(-1e10))
    return torch.nan_to_num(cost, 0)
