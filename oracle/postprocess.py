"""CPU restatement of Mask2FormerImageProcessor.post_process_instance_segmentation (transformers
5.15 image_processing_mask2former.py:627-744) as the reference calls it from process_prediction
(mask2former/predictor.py:697-700, CPU tensors from Trainer.predict) — TEST INFRASTRUCTURE ONLY
(the checker of the HIP post-processing kernels, never the product path).

The discrete part is the top-k: ``scores.flatten(0, 1).topk(num_queries, sorted=False)`` on a
CPU tensor of Q*C class probabilities.  ATen's CPU top-k (ATen/native/TopKImpl.h,
topk_impl_loop) takes ``std::nth_element(queue, queue + k - 1, end, greater-with-NaN-first)``
over (value, index) pairs whenever k * 64 > Q * C — always for Mask2Former (k = Q) — and
returns the first k pairs in the order nth_element leaves them.  That order decides the
segment ids and which mask wins an overlapping pixel, so libstdc++'s introselect (GCC
bits/stl_algo.h: __introselect, __unguarded_partition_pivot, __move_median_to_first,
__heap_select, __insertion_sort; bits/stl_heap.h: __adjust_heap, __push_heap) is restated
step for step.  Pinned against torch.topk(sorted=False) itself on random, tie-heavy and
NaN-bearing inputs (tests/test_oracle_postprocess.py).
"""
import numpy as np
import torch


def _lg(n):
    return int(n).bit_length() - 1


def nth_element_topk(values, k):
    """Order of the first k (value, index) pairs after libstdc++ std::nth_element with
    comp(x, y) = (isnan(x) and not isnan(y)) or x > y, on pairs initialised (values[j], j).
    Returns (vals float32 [k], idx int64 [k])."""
    v = [float(x) for x in np.asarray(values, dtype=np.float32)]
    ix = list(range(len(v)))
    n = len(v)

    def comp(a, b):  # positions
        x, y = v[a], v[b]
        return (x != x and y == y) or x > y

    def comp_val(a, val):  # position vs a held value
        x = v[a]
        return (x != x and val == val) or x > val

    def comp_val2(val, b):
        y = v[b]
        return (val != val and y == y) or val > y

    def swap(a, b):
        v[a], v[b] = v[b], v[a]
        ix[a], ix[b] = ix[b], ix[a]

    def move_median_to_first(result, a, b, c):
        if comp(a, b):
            if comp(b, c):
                swap(result, b)
            elif comp(a, c):
                swap(result, c)
            else:
                swap(result, a)
        elif comp(a, c):
            swap(result, a)
        elif comp(b, c):
            swap(result, c)
        else:
            swap(result, b)

    def unguarded_partition(first, last, pivot):
        while True:
            while comp(first, pivot):
                first += 1
            last -= 1
            while comp(pivot, last):
                last -= 1
            if not first < last:
                return first
            swap(first, last)
            first += 1

    def push_heap(first, hole, top, val, vix):
        parent = (hole - 1) // 2
        while hole > top and comp_val(first + parent, val):
            v[first + hole], ix[first + hole] = v[first + parent], ix[first + parent]
            hole = parent
            parent = (hole - 1) // 2
        v[first + hole], ix[first + hole] = val, vix

    def adjust_heap(first, hole, length, val, vix):
        top = hole
        second = hole
        while second < (length - 1) // 2:
            second = 2 * (second + 1)
            if comp(first + second, first + second - 1):
                second -= 1
            v[first + hole], ix[first + hole] = v[first + second], ix[first + second]
            hole = second
        if (length & 1) == 0 and second == (length - 2) // 2:
            second = 2 * (second + 1)
            v[first + hole], ix[first + hole] = v[first + second - 1], ix[first + second - 1]
            hole = second - 1
        push_heap(first, hole, top, val, vix)

    def make_heap(first, last):
        length = last - first
        if length < 2:
            return
        parent = (length - 2) // 2
        while True:
            val, vix = v[first + parent], ix[first + parent]
            adjust_heap(first, parent, length, val, vix)
            if parent == 0:
                return
            parent -= 1

    def heap_select(first, middle, last):
        make_heap(first, middle)
        for i in range(middle, last):
            if comp(i, first):
                val, vix = v[i], ix[i]  # __pop_heap(first, middle, i)
                v[i], ix[i] = v[first], ix[first]
                adjust_heap(first, 0, middle - first, val, vix)

    def insertion_sort(first, last):
        if first == last:
            return
        for i in range(first + 1, last):
            if comp(i, first):
                val, vix = v[i], ix[i]
                for j in range(i, first, -1):
                    v[j], ix[j] = v[j - 1], ix[j - 1]
                v[first], ix[first] = val, vix
            else:  # __unguarded_linear_insert
                val, vix = v[i], ix[i]
                last_ = i
                nxt = i - 1
                while comp_val2(val, nxt):
                    v[last_], ix[last_] = v[nxt], ix[nxt]
                    last_ = nxt
                    nxt -= 1
                v[last_], ix[last_] = val, vix

    def introselect(first, nth, last, depth):
        while last - first > 3:
            if depth == 0:
                heap_select(first, nth + 1, last)
                swap(first, nth)
                return
            depth -= 1
            mid = first + (last - first) // 2
            move_median_to_first(first, first + 1, mid, last - 1)
            cut = unguarded_partition(first + 1, last, first)
            if cut <= nth:
                first = cut
            else:
                last = cut
        insertion_sort(first, last)

    if k > 0 and n > 0 and k - 1 != n:
        introselect(0, k - 1, n, _lg(n) * 2)
    return np.array(v[:k], dtype=np.float32), np.array(ix[:k], dtype=np.int64)


def topk_unsorted(values, k):
    """torch.topk(values, k, sorted=False) on the CPU for k * 64 > len(values) (ATen
    topk_impl_loop's nth_element branch; Mask2Former's k = num_queries always takes it)."""
    if k * 64 <= len(values):
        raise ValueError("partial_sort branch of ATen's CPU top-k: not restated")
    return nth_element_topk(values, k)


def post_process_instance_segmentation(class_logits, mask_logits, threshold=0.5, target_sizes=None, scores=None):
    """transformers 5.15 image_processing_mask2former.py:627-744 (return_coco_annotation and
    return_binary_maps False), float32 CPU torch.  ``scores`` optionally replaces the class
    softmax (so the discrete path can be checked on exactly the GPU's probabilities).
    Returns [{"segmentation": float32 [h, w], "segments_info": [...]}] per image."""
    class_logits = torch.as_tensor(class_logits, dtype=torch.float32)
    mask_logits = torch.as_tensor(mask_logits, dtype=torch.float32)
    masks = torch.nn.functional.interpolate(mask_logits, size=(384, 384), mode="bilinear", align_corners=False)
    B, Q, C1 = class_logits.shape
    C = C1 - 1
    out = []
    for i in range(B):
        sc = torch.nn.functional.softmax(class_logits[i], dim=-1)[:, :-1] if scores is None else torch.as_tensor(scores[i])
        vals, idx = nth_element_topk(sc.flatten().numpy(), Q)
        vals = torch.from_numpy(vals)
        idx = torch.from_numpy(idx)
        labels = idx % C
        q = torch.div(idx, C, rounding_mode="floor")
        mp = masks[i][q]
        pm = (mp > 0).float()
        mscore = (mp.sigmoid().flatten(1) * pm.flatten(1)).sum(1) / (pm.flatten(1).sum(1) + 1e-6)
        pscore = vals * mscore
        seg = torch.zeros((384, 384)) - 1
        if target_sizes is not None:
            seg = torch.zeros(target_sizes[i]) - 1
            pm = torch.nn.functional.interpolate(pm.unsqueeze(0), size=target_sizes[i], mode="nearest")[0]
        segments = []
        cur = 0
        for j in range(Q):
            s = pscore[j].item()
            if not torch.all(pm[j] == 0) and s >= threshold:
                seg[pm[j] == 1] = cur
                segments.append({"id": cur, "label_id": int(labels[j]), "was_fused": False, "score": round(s, 6)})
                cur += 1
        out.append({"segmentation": seg, "segments_info": segments, "topk_idx": idx.numpy(),
                    "pred_scores": pscore.numpy()})
    return out
