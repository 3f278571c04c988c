"""f3: the point-sampled mask terms of the Mask2Former matcher and loss on the GPU.

Reference (the library the reference trains through, transformers 5.15 modeling_mask2former.py):
``Mask2FormerHungarianMatcher.forward`` (:412-483) builds, per image, a point-sampled sigmoid-CE
and dice cost against every target (:445-470); ``Mask2FormerLoss.loss_masks`` (:580-630) samples
12 544 points per matched pair by uncertainty (:671-724) and averages sigmoid-CE and dice over
them.  Here the sampling (``rgbd_point_sample`` / ``_bwd``), the cost reduction
(``rgbd_match_cost``, all images in one launch) and the loss reductions with their backward
(``rgbd_point_losses`` / ``_bwd``) are HIP kernels (csrc/point_loss.hip).  The random point
coordinates (``torch.rand``), the uncertainty ``torch.topk`` and the index gathers stay torch
calls in the reference's order, so the RNG stream and the selected point set are the reference's
(the set: the top-k is taken unsorted, the loss sums do not depend on the points' order).

``install(model)`` swaps the HF loss (and its matcher) for ``HipMask2FormerLoss`` /
``matcher.HipHungarianMatcher`` in place; ``uninstall`` restores them.
"""
import os

import torch
from torch import nn
from transformers.models.mask2former.modeling_mask2former import Mask2FormerHungarianMatcher, Mask2FormerLoss

from . import _lib
from ._lib import RGBD_BF16, RGBD_F32, check
from .ops import LsaResult, _need_cuda, _p, _stream, device_const, device_vec

# loss_masks' uncertainty top-k: unsorted by default (the loss terms are sums over the point set,
# so only the float summation order changes; the segmented sort cost ~2.4 ms per whole-model
# step); True — or RGBD_SORTED_TOPK=1 — takes the reference's sorted selection (parity runs)
SORTED_TOPK = os.environ.get("RGBD_SORTED_TOPK", "0") == "1"


# one entry each, shared by the loss and its matcher (the final and the nine auxiliary outputs of a
# step see the same label tensors): the cache holds the label tensors themselves and matches them
# by identity (+ version counters), so their storage cannot be recycled under a stale entry
_ROWS_CACHE = []
_LABELS_CACHE = []


def target_rows(mask_labels, dtype):
    """Every image's target masks cast like the reference (``.to(pred_masks)``), as float32 rows
    [sum T, H, W] and their image offsets — built once per set of labels, None when the images
    differ in size (then the reference's zero-padded batch is used)."""
    versions = tuple(m._version for m in mask_labels)
    if _ROWS_CACHE:
        c_dtype, c_labels, c_versions, rows, offs = _ROWS_CACHE[0]
        if (c_dtype == dtype and len(c_labels) == len(mask_labels)
                and all(a is b for a, b in zip(c_labels, mask_labels)) and c_versions == versions):
            return rows, offs
    rows = offs = None
    if mask_labels and len({tuple(m.shape[-2:]) for m in mask_labels}) == 1:
        rows = torch.cat([m.reshape(-1, *m.shape[-2:]) for m in mask_labels]).to(dtype).float()
        offs, o = [], 0
        for m in mask_labels:
            offs.append(o)
            o += m.shape[0]
    _ROWS_CACHE[:] = [(dtype, tuple(mask_labels), versions, rows, offs)]
    return rows, offs


def labels_all(class_labels, device):
    """Every image's class labels concatenated (int64, on device), built once per set of labels."""
    versions = tuple(c._version for c in class_labels)
    if _LABELS_CACHE:
        c_labels, c_versions, t = _LABELS_CACHE[0]
        if (len(c_labels) == len(class_labels) and all(a is b for a, b in zip(c_labels, class_labels))
                and c_versions == versions):
            return t
    t = (torch.cat([c.reshape(-1) for c in class_labels]).to(device=device, dtype=torch.long) if class_labels
         else torch.zeros((0,), dtype=torch.long, device=device))
    _LABELS_CACHE[:] = [(tuple(class_labels), versions, t)]
    return t


def topk_indices(unc, k):
    """``torch.topk(unc, k, dim=1, sorted=False)[1]`` as a set: rgbd_topk_rows (one LDS radix
    select per row, every element above the k-th largest and then the lowest-index ties, in
    increasing index order).  SORTED_TOPK, or rows longer than the kernel's LDS holds, take
    torch.topk itself."""
    N, n = unc.shape
    L = _lib.lib()
    if SORTED_TOPK or n > L.rgbd_topk_rows_max_n() or k > n or k <= 0:
        return torch.topk(unc, k=k, dim=1, sorted=SORTED_TOPK)[1]
    u = unc.float().contiguous()
    idx = torch.empty((N, k), dtype=torch.long, device=unc.device)
    check(L.rgbd_topk_rows(_p(u), N, n, k, _p(idx), _stream(unc.device)), "rgbd_topk_rows")
    return idx


def point_sample(maps: torch.Tensor, coords: torch.Tensor) -> torch.Tensor:
    """maps float32 [N, h, w]; coords [G, P, 2] in [0, 1] (x, y), one point set per N / G
    consecutive maps -> [N, P]: ``sample_point(maps[:, None], coords, align_corners=False)``
    (modeling_mask2former.py:245-275).  Differentiable in ``maps``."""
    return _PointSample.apply(maps, coords)


def _sample(maps, coords):
    """float32 samples of float32 or bfloat16 maps (bf16 sampled in place: no float32 copy)."""
    maps = maps.detach()
    if maps.dtype not in (torch.float32, torch.bfloat16):
        maps = maps.float()
    maps = maps.contiguous()
    coords = coords.detach().float().contiguous()
    _need_cuda(maps, coords)
    N, h, w = maps.shape
    G, P, _ = coords.shape
    if N % max(G, 1) or (N and G == 0):
        raise ValueError(f"point_sample: {N} maps for {G} point sets")
    out = torch.empty((N, P), dtype=torch.float32, device=maps.device)
    if N:
        code = RGBD_BF16 if maps.dtype == torch.bfloat16 else RGBD_F32
        check(_lib.lib().rgbd_point_sample_t(code, _p(maps), N, h, w, _p(coords), N // G, P, _p(out),
                                             _stream(maps.device)), "rgbd_point_sample_t")
    return out


class _PointSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, maps, coords):
        ctx.save_for_backward(coords)
        ctx.shape = tuple(maps.shape)
        return _sample(maps, coords)

    @staticmethod
    def backward(ctx, gout):
        (coords,) = ctx.saved_tensors
        N, h, w = ctx.shape
        g = gout.float().contiguous()
        gmaps = torch.zeros((N, h, w), dtype=torch.float32, device=g.device)
        if N:
            c = coords.float().contiguous()
            check(_lib.lib().rgbd_point_sample_bwd(_p(g), N, h, w, _p(c), N // c.shape[0], c.shape[1], _p(gmaps),
                                                   _stream(g.device)), "rgbd_point_sample_bwd")
        return gmaps, None


class _PointLosses(torch.autograd.Function):
    """(logits [N, P], labels [N, P]) -> per-row (mean BCEWithLogits, dice)
    (sigmoid_cross_entropy_loss / dice_loss before their sums, :278-325)."""

    @staticmethod
    def forward(ctx, logits, labels):
        x = logits.detach().float().contiguous()
        y = labels.detach().float().contiguous()
        _need_cuda(x, y)
        N, P = x.shape
        ce = torch.empty((N,), dtype=torch.float32, device=x.device)
        dice = torch.empty_like(ce)
        sums = torch.empty((N, 3), dtype=torch.float32, device=x.device)
        check(_lib.lib().rgbd_point_losses(_p(x), _p(y), N, P, _p(ce), _p(dice), _p(sums), _stream(x.device)),
              "rgbd_point_losses")
        ctx.save_for_backward(x, y, sums)
        return ce, dice

    @staticmethod
    def backward(ctx, g_ce, g_dice):
        x, y, sums = ctx.saved_tensors
        N, P = x.shape
        g_ce = torch.zeros((N,), device=x.device) if g_ce is None else g_ce.float().contiguous()
        g_dice = torch.zeros((N,), device=x.device) if g_dice is None else g_dice.float().contiguous()
        gx = torch.empty_like(x)
        check(_lib.lib().rgbd_point_losses_bwd(_p(x), _p(y), N, P, _p(sums), _p(g_ce), _p(g_dice), _p(gx),
                                               _stream(x.device)), "rgbd_point_losses_bwd")
        return gx, None


def match_costs(matcher, masks_queries_logits, class_queries_logits, mask_labels, class_labels):
    """The matcher's cost matrices of every image ([Q, T_b] each), as
    Mask2FormerHungarianMatcher.forward builds them (:445-470): one ``torch.rand(1, P, 2)`` per
    image in image order, then the point sampling and the pair-wise CE / dice reduction on the
    GPU.  Batched: one softmax over all images (row-wise, the same rows), every image's targets
    sampled against its own points in one launch (the cached target rows: the labels rounded to
    the logits' dtype, as ``.to(pred)``), and the class cost read from the softmax inside the
    cost kernel — a handful of launches per output instead of several per image."""
    B, Q, h, w = masks_queries_logits.shape
    P = matcher.num_points
    dev = masks_queries_logits.device
    rows, _ = target_rows(mask_labels, masks_queries_logits.dtype)
    if rows is None:
        return _match_costs_per_image(matcher, masks_queries_logits, class_queries_logits, mask_labels, class_labels)
    probs = class_queries_logits.softmax(-1).float().contiguous()
    pts = torch.cat([torch.rand(1, P, 2, device=dev) for _ in range(B)])
    toff, coff, set_of_map = [0], [0], []
    for i in range(B):
        T = mask_labels[i].shape[0]
        toff.append(toff[-1] + T)
        coff.append(coff[-1] + Q * T)
        set_of_map += [i] * T
    pred = _sample(masks_queries_logits.reshape(B * Q, h, w), pts)
    if toff[-1]:
        tgt = torch.empty((toff[-1], P), dtype=torch.float32, device=dev)
        th, tw = rows.shape[-2:]
        som = device_vec(set_of_map, torch.int32, dev)  # held until the launch is enqueued
        check(_lib.lib().rgbd_point_sample_sets(RGBD_F32, _p(rows), toff[-1], th, tw, _p(pts.contiguous()),
                                                _p(som), P, _p(tgt), _stream(dev)), "rgbd_point_sample_sets")
    else:
        tgt = torch.zeros((1, P), device=dev)
    labels = labels_all(class_labels, dev)
    if labels.numel() == 0:
        labels = torch.zeros((1,), dtype=torch.long, device=dev)
    cost = torch.empty((max(coff[-1], 1),), dtype=torch.float32, device=dev)
    toff_t = device_vec(toff, torch.int32, dev)
    coff_t = device_vec(coff[:-1], torch.int64, dev)
    check(_lib.lib().rgbd_match_cost_probs(_p(pred), B, Q, P, _p(tgt), _p(toff_t), _p(probs), probs.shape[-1],
                                           _p(labels), _p(coff_t), float(matcher.cost_mask), float(matcher.cost_class),
                                           float(matcher.cost_dice), _p(cost), _stream(dev)), "rgbd_match_cost_probs")
    return [cost[coff[i]:coff[i + 1]].view(Q, toff[i + 1] - toff[i]) for i in range(B)]


def _match_costs_per_image(matcher, masks_queries_logits, class_queries_logits, mask_labels, class_labels):
    """match_costs with the targets cast and sampled image by image (images of different sizes)."""
    B, Q, h, w = masks_queries_logits.shape
    P = matcher.num_points
    dev = masks_queries_logits.device
    pts, tgts, ccls, toff, coff = [], [], [], [0], [0]
    for i in range(B):
        probs = class_queries_logits[i].softmax(-1)
        ccls.append((-probs[:, class_labels[i]]).float().reshape(-1))
        pts.append(torch.rand(1, P, 2, device=dev))
        tm = mask_labels[i].to(masks_queries_logits)
        tgts.append(_sample(tm.reshape(-1, *tm.shape[-2:]), pts[-1]) if tm.shape[0] else
                    torch.empty((0, P), device=dev))
        toff.append(toff[-1] + tm.shape[0])
        coff.append(coff[-1] + Q * tm.shape[0])
    pred = _sample(masks_queries_logits.reshape(B * Q, h, w), torch.cat(pts))
    tgt = torch.cat(tgts) if toff[-1] else torch.zeros((1, P), device=dev)
    cls = torch.cat(ccls) if coff[-1] else torch.zeros((1,), device=dev)
    cost = torch.empty((max(coff[-1], 1),), dtype=torch.float32, device=dev)
    toff_t = device_vec(toff, torch.int32, dev)
    coff_t = device_vec(coff[:-1], torch.int64, dev)
    check(_lib.lib().rgbd_match_cost(_p(pred), B, Q, P, _p(tgt), _p(toff_t), _p(cls), _p(coff_t),
                                     float(matcher.cost_mask), float(matcher.cost_class), float(matcher.cost_dice),
                                     _p(cost), _stream(dev)), "rgbd_match_cost")
    return [cost[coff[i]:coff[i + 1]].view(Q, toff[i + 1] - toff[i]) for i in range(B)]


class _MatchedRows(torch.autograd.Function):
    """``x[batch_idx, query_idx]`` for the matcher's indices (modeling_mask2former.py:601) as one
    row gather of x viewed [B*Q, ...]; backward scatters the rows into zeros with index_copy_.
    The matched (image, query) pairs are distinct (a one-to-one assignment), so that is the
    gradient advanced indexing gives, without its accumulate path's index sort."""

    @staticmethod
    def forward(ctx, x, flat):
        ctx.shape = x.shape
        ctx.save_for_backward(flat)
        return x.reshape(-1, *x.shape[2:]).index_select(0, flat)

    @staticmethod
    def backward(ctx, g):
        (flat,) = ctx.saved_tensors
        shape = ctx.shape
        gx = g.new_zeros((shape[0] * shape[1], *shape[2:]))
        gx.index_copy_(0, flat, g)
        return gx.view(shape), None


class HipMask2FormerLoss(Mask2FormerLoss):
    """Mask2FormerLoss with loss_masks' sampling and reductions on the GPU kernels."""

    def get_num_masks(self, class_labels, device):
        """modeling_mask2former.py:782-795 with the count as a shared device constant (no blocking
        copy per step); the accelerate all-reduce branch stays the library's."""
        try:
            from accelerate import PartialState
            distributed = PartialState._shared_state != {}
        except ImportError:
            distributed = False
        if distributed:
            return super().get_num_masks(class_labels, device)
        num_masks = device_vec(float(sum(len(c) for c in class_labels)), torch.float32, device)
        return torch.clamp(num_masks, min=1)

    def _target_rows(self, mask_labels, dtype):
        return target_rows(mask_labels, dtype)

    def _get_predictions_permutation_indices(self, indices):
        """(:642-646) from the batched assignment's concatenated indices: the image index of
        every match is a cached constant of the per-image counts, the query indices a view."""
        if isinstance(indices, LsaResult) and indices.rows_all is not None:
            dev = indices.rows_all.device
            batch = device_vec([i for i, n in enumerate(indices.counts) for _ in range(n)] or [0], torch.long, dev)
            return batch[:len(indices.rows_all)], indices.rows_all
        return super()._get_predictions_permutation_indices(indices)

    def _target_flat(self, indices, offs, dev):
        """Row index of every match's target among all images' targets (image offset + column)."""
        if isinstance(indices, LsaResult) and indices.cols_all is not None:
            shift = device_vec([offs[i] for i, n in enumerate(indices.counts) for _ in range(n)] or [0], torch.long, dev)
            return indices.cols_all + shift[:len(indices.cols_all)]
        return (torch.cat([j.to(dev) + offs[i] for i, (_, j) in enumerate(indices)]) if indices else
                torch.zeros((0,), dtype=torch.long, device=dev))

    def loss_labels(self, class_queries_logits, class_labels, indices):
        """Mask2FormerLoss.loss_labels (:548-578) with the matched targets' classes gathered from
        the concatenated labels in one index (the reference: one gather per image + cat) and
        scattered into the no-object fill by flat index (the matches are distinct)."""
        if not (isinstance(indices, LsaResult) and indices.rows_all is not None):
            return super().loss_labels(class_queries_logits, class_labels, indices)
        pred_logits = class_queries_logits
        batch_size, num_queries, _ = pred_logits.shape
        criterion = nn.CrossEntropyLoss(weight=self.empty_weight)
        dev = pred_logits.device
        offs, o = [], 0
        for c in class_labels:
            offs.append(o)
            o += c.shape[0]
        target_classes_o = labels_all(class_labels, dev).index_select(0, self._target_flat(indices, offs, dev))
        target_classes = torch.full((batch_size, num_queries), fill_value=self.num_labels, dtype=torch.int64,
                                    device=dev)
        b_idx, q_idx = self._get_predictions_permutation_indices(indices)
        target_classes.view(-1).index_copy_(0, b_idx * num_queries + q_idx, target_classes_o)
        loss_ce = criterion(pred_logits.transpose(1, 2), target_classes)
        return {"loss_cross_entropy": loss_ce}

    def loss_masks(self, masks_queries_logits, mask_labels, indices, num_masks):
        src_idx = self._get_predictions_permutation_indices(indices)
        B, Q = masks_queries_logits.shape[:2]
        pred_masks = _MatchedRows.apply(masks_queries_logits, src_idx[0] * Q + src_idx[1])  # [N, h, w]
        rows, offs = self._target_rows(mask_labels, masks_queries_logits.dtype)
        if rows is not None:
            dev = masks_queries_logits.device
            tflat = self._target_flat(indices, offs, dev)
            target_masks = rows.index_select(0, tflat)  # float32, already rounded to the logits' dtype
        else:
            tgt_idx = self._get_targets_permutation_indices(indices)
            target_masks, _ = self._pad_images_to_max_in_batch(mask_labels)
            target_masks = target_masks[tgt_idx].to(masks_queries_logits.dtype)
        N = pred_masks.shape[0]
        P = self.num_points
        if N == 0:
            # no target instance in the whole batch: HF's sums over zero rows give 0 for both
            # terms (and zero gradients); keep them attached to the graph like the reference's
            zero = masks_queries_logits.sum() * 0.0
            return {"loss_mask": zero, "loss_dice": zero.clone()}
        with torch.no_grad():
            # sample_points_using_uncertainty (:671-724), same torch.rand / topk calls and order
            n_over = int(P * self.oversample_ratio)
            coords = torch.rand(N, n_over, 2, device=pred_masks.device)
            unc = -(torch.abs(_sample(pred_masks, coords)))
            k = int(self.importance_sample_ratio * P)
            # the k most uncertain points as a set: the loss terms are sums over the points, so
            # their order is immaterial (up to float summation order) and topk's segmented sort
            # of the selection (~2.4 ms per whole-model step, rocprim merge sort) is skipped
            # deliberate deviation: unsorted; SORTED_TOPK restores the reference's
            # sorted selection for parity runs (the same set up to ties, the reference's order)
            idx = topk_indices(unc, k)
            shift = n_over * torch.arange(N, dtype=torch.long, device=pred_masks.device)
            idx += shift[:, None]
            coords = coords.view(-1, 2)[idx.view(-1), :].view(N, k, 2)
            if P - k > 0:
                coords = torch.cat([coords, torch.rand(N, P - k, 2, device=pred_masks.device)], dim=1)
            labels = _sample(target_masks.reshape(N, *target_masks.shape[-2:]), coords)
        logits = point_sample(pred_masks, coords)
        ce, dice = _PointLosses.apply(logits, labels)
        return {"loss_mask": ce.sum() / num_masks, "loss_dice": dice.sum() / num_masks}


def install(model: nn.Module) -> int:
    """Swap every HF Mask2FormerLoss (and its matcher) in ``model`` for the HIP versions."""
    from .matcher import HipHungarianMatcher
    n = 0
    for m in model.modules():
        if type(m) is Mask2FormerLoss:
            m.__class__ = HipMask2FormerLoss
            n += 1
        if type(m) is Mask2FormerHungarianMatcher:
            m.__class__ = HipHungarianMatcher
    return n


def uninstall(model: nn.Module) -> int:
    from .matcher import HipHungarianMatcher
    n = 0
    for m in model.modules():
        if type(m) is HipMask2FormerLoss:
            m.__class__ = Mask2FormerLoss
            n += 1
        if type(m) is HipHungarianMatcher:
            m.__class__ = Mask2FormerHungarianMatcher
    return n
