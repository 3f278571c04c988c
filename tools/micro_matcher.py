"""Time the Hungarian matcher (transformers 5.15 Mask2FormerHungarianMatcher, scipy on the host)
against HipHungarianMatcher (one rgbd_lsa_batch launch, no host sync) at the C2 training shape:
B=8 images, 100 queries, 49 classes, 120x160 mask logits, 20 targets per image, 12544 points.
The loss calls the matcher for the final and 9 auxiliary outputs, so x10 per training step."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import matcher, ops  # noqa: E402
from transformers.models.mask2former.modeling_mask2former import Mask2FormerHungarianMatcher  # noqa: E402


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    B, Q, L, H, W, N = 8, 100, 49, 120, 160, 20
    masks = torch.randn((B, Q, H, W), generator=g, device=dev)
    classes = torch.randn((B, Q, L), generator=g, device=dev)
    mask_labels = [(torch.rand((N, H * 4, W * 4), generator=g, device=dev) > 0.7).float() for _ in range(B)]
    class_labels = [torch.randint(0, L - 1, (N,), generator=g, device=dev) for _ in range(B)]
    ref = Mask2FormerHungarianMatcher(cost_class=2.0, cost_mask=5.0, cost_dice=5.0, num_points=12544)
    hip = Mask2FormerHungarianMatcher(cost_class=2.0, cost_mask=5.0, cost_dice=5.0, num_points=12544)
    matcher.install(hip)
    res = {}
    for name, m in (("hf_scipy", ref), ("hip", hip)):
        for _ in range(3):
            m(masks, classes, mask_labels, class_labels)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            out = m(masks, classes, mask_labels, class_labels)
        torch.cuda.synchronize()
        res[name + "_ms_per_call"] = round((time.perf_counter() - t0) / 20 * 1e3, 3)
    # the assignment alone: 8 cost matrices of 100 x 20
    costs = [torch.randn((Q, N), generator=g, device=dev) for _ in range(B)]
    for _ in range(3):
        ops.linear_sum_assignment_batch(costs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        ops.linear_sum_assignment_batch(costs)
    torch.cuda.synchronize()
    res["lsa_batch8_100x20_ms"] = round((time.perf_counter() - t0) / 50 * 1e3, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
