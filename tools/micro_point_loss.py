"""Time the point-sampled mask terms at the C2 training shape (B=8, 100 queries, 120x160 mask
logits, 20 targets per image at 480x640, 12 544 points): the matcher's cost construction
(HF torch ops vs point_loss.match_costs) and loss_masks forward + backward over 160 matched pairs
(HF Mask2FormerLoss vs HipMask2FormerLoss).  x10 per training step (final + 9 auxiliary outputs)."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import matcher, point_loss  # noqa: E402
from transformers import Mask2FormerConfig  # noqa: E402
from transformers.models.mask2former.modeling_mask2former import (Mask2FormerHungarianMatcher,  # noqa: E402
                                                                  Mask2FormerLoss)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e3, 3)


def main():
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
    from checkers.matching_cost import matching_cost
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    B, Q, L, H, W, N = 8, 100, 49, 120, 160, 20
    masks = torch.randn((B, Q, H, W), generator=g, device=dev)
    classes = torch.randn((B, Q, L), generator=g, device=dev)
    mask_labels = [(torch.rand((N, H * 4, W * 4), generator=g, device=dev) > 0.7).float() for _ in range(B)]
    class_labels = [torch.randint(0, L - 1, (N,), generator=g, device=dev) for _ in range(B)]
    m = Mask2FormerHungarianMatcher(cost_class=2.0, cost_mask=5.0, cost_dice=5.0, num_points=12544)
    res = {"cost_hf_ms": timeit(lambda: [matching_cost(m, masks, classes, mask_labels, class_labels, i)
                                          for i in range(B)]),
           "cost_hip_ms": timeit(lambda: point_loss.match_costs(m, masks, classes, mask_labels, class_labels))}
    cfg = Mask2FormerConfig(num_labels=48)
    wd = {"loss_cross_entropy": 2.0, "loss_mask": 5.0, "loss_dice": 5.0}
    idx = [(torch.arange(N, device=dev) * 5, torch.arange(N, device=dev)) for _ in range(B)]
    for name, loss in (("hf", Mask2FormerLoss(cfg, wd)), ("hip", Mask2FormerLoss(cfg, wd))):
        if name == "hip":
            loss.__class__ = point_loss.HipMask2FormerLoss
        x = masks.clone().requires_grad_(True)

        def step():
            out = loss.loss_masks(x, mask_labels, idx, num_masks=float(B * N))
            (out["loss_mask"] + out["loss_dice"]).backward()
        res[f"loss_masks_fwd_bwd_{name}_ms"] = timeit(step)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
