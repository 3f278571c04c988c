"""f3: the Mask2Former Hungarian matcher without the host round trip.

Reference: ``Mask2FormerHungarianMatcher.forward`` (transformers 5.15 modeling_mask2former.py:
412-483), used by ``Mask2FormerLoss`` (:762) for the final and every auxiliary decoder output.
Per image it builds the (queries x targets) cost — class probability, point-sampled sigmoid-CE and
dice — and calls ``scipy.optimize.linear_sum_assignment(cost_matrix.cpu())``: one device->host
sync and one CPU solve per image per output.

``HipHungarianMatcher`` draws the same ``torch.rand`` points in the same order, builds every
image's cost on the GPU kernels of point_loss.py (sampling, pair-wise CE / dice, clamping in one
launch for all images; tests/checkers/matching_cost.py keeps the reference's torch form as the
checker) and
solves all images' matrices in one ``rgbd_lsa_batch`` launch (csrc/lsap.hip: scipy's algorithm in float64, same
optimum including ties).  The matched indices stay on the GPU as int64 tensors, which the loss
indexes with directly.  ``install(model)`` swaps the class of every HF matcher in place.
"""
import torch
from torch import nn
from transformers.models.mask2former.modeling_mask2former import Mask2FormerHungarianMatcher

from . import ops


class HipHungarianMatcher(Mask2FormerHungarianMatcher):
    @torch.no_grad()
    def forward(self, masks_queries_logits, class_queries_logits, mask_labels, class_labels):
        # point sampling + pair-wise CE / dice of all images on the GPU kernels (point_loss.py),
        # the same torch.rand draws as the reference (the torch form: tests/checkers/matching_cost.py)
        from .point_loss import match_costs
        costs = match_costs(self, masks_queries_logits, class_queries_logits, mask_labels, class_labels)
        return ops.linear_sum_assignment_batch(costs)


def install(model: nn.Module) -> int:
    n = 0
    for m in model.modules():
        if type(m) is Mask2FormerHungarianMatcher:
            m.__class__ = HipHungarianMatcher
            n += 1
    return n


def uninstall(model: nn.Module) -> int:
    n = 0
    for m in model.modules():
        if type(m) is HipHungarianMatcher:
            m.__class__ = Mask2FormerHungarianMatcher
            n += 1
    return n
