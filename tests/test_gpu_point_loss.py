"""f3: the point-sampled mask terms on the GPU kernels (csrc/point_loss.hip, rgbd_amd/point_loss.py)
against the library code the reference trains through (transformers 5.15
modeling_mask2former.py): sample_point (:245-275) and its autograd, the matcher's cost matrices
(:445-470, restated op for op in tests/checkers/matching_cost.py) and Mask2FormerLoss.loss_masks
(:580-630) with its gradient.  Same torch RNG state on both sides, so the same random points.
Tolerances: float32 reductions in a different order — 1e-5 relative on sampled values, 1e-5 relative on
costs and losses, 1e-4 relative on gradients."""
import pytest
import torch
import torch.nn.functional as F

from rgbd_amd import matcher, point_loss

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, e):
    return float((a - e).abs().max() / (e.abs().max() + 1e-12))


@pytest.mark.parametrize("N,G,h,w,P", [(6, 1, 30, 40, 1000), (5, 5, 17, 23, 777), (8, 2, 120, 160, 12544)])
def test_point_sample_matches_grid_sample(N, G, h, w, P):
    g = torch.Generator(device=DEV).manual_seed(N * 7 + P)
    maps = torch.randn((N, h, w), generator=g, device=DEV)
    coords = torch.rand((G, P, 2), generator=g, device=DEV)
    coords[0, :4] = torch.tensor([[0.0, 0.0], [1.0, 1.0], [0.0, 1.0], [0.999999, 0.5]], device=DEV)  # edges
    ref_c = coords.repeat_interleave(N // G, dim=0)
    mref = maps.clone().requires_grad_(True)
    ref = F.grid_sample(mref[:, None], 2.0 * ref_c[:, :, None] - 1.0, align_corners=False)[:, 0, :, 0]
    mh = maps.clone().requires_grad_(True)
    got = point_loss.point_sample(mh, coords)
    assert float((got - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))
    go = torch.randn(ref.shape, generator=g, device=DEV)
    ref.backward(go)
    got.backward(go)
    assert _rel(mh.grad, mref.grad) <= 1e-5


def _case(seed, B=3, Q=100, L=49, H=60, W=80, counts=(5, 0, 23)):
    g = torch.Generator(device=DEV).manual_seed(seed)
    masks = torch.randn((B, Q, H, W), generator=g, device=DEV)
    classes = torch.randn((B, Q, L), generator=g, device=DEV)
    mask_labels, class_labels = [], []
    for n in counts:
        mask_labels.append((torch.rand((n, H * 4, W * 4), generator=g, device=DEV) > 0.7).float())
        class_labels.append(torch.randint(0, L - 1, (n,), generator=g, device=DEV))
    return masks, classes, mask_labels, class_labels


def test_point_sample_bf16_maps_equal_widened_float32():
    """rgbd_point_sample_t on bf16 maps (the logits under autocast, no float32 copy) gives the
    bits of the float32 kernel on the same maps widened."""
    g = torch.Generator(device=DEV).manual_seed(3)
    maps = torch.randn((12, 120, 160), generator=g, device=DEV).to(torch.bfloat16)
    coords = torch.rand((3, 5000, 2), generator=g, device=DEV) * 1.2 - 0.1
    assert torch.equal(point_loss._sample(maps, coords), point_loss._sample(maps.float(), coords))


@pytest.mark.parametrize("seed", [0, 1])
def test_match_costs_match_reference(seed):
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerHungarianMatcher
    m = Mask2FormerHungarianMatcher(cost_class=2.0, cost_mask=5.0, cost_dice=5.0, num_points=12544)
    masks, classes, ml, cl = _case(seed)
    torch.manual_seed(21 + seed)
    from checkers.matching_cost import matching_cost
    ref = [matching_cost(m, masks, classes, ml, cl, i) for i in range(masks.shape[0])]
    torch.manual_seed(21 + seed)
    got = point_loss.match_costs(m, masks, classes, ml, cl)
    for r, h in zip(ref, got):
        assert r.shape == h.shape
        if r.numel():
            assert _rel(h, r) <= 1e-5, _rel(h, r)


def test_loss_masks_and_grad_match_reference():
    from transformers import Mask2FormerConfig
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerLoss
    cfg = Mask2FormerConfig(num_labels=48)
    ref_loss = Mask2FormerLoss(cfg, weight_dict={"loss_cross_entropy": 2.0, "loss_mask": 5.0, "loss_dice": 5.0})
    hip_loss = Mask2FormerLoss(cfg, weight_dict={"loss_cross_entropy": 2.0, "loss_mask": 5.0, "loss_dice": 5.0})
    hip_loss.__class__ = point_loss.HipMask2FormerLoss
    masks, classes, ml, cl = _case(3, B=2, counts=(7, 12))
    indices = [(torch.arange(n, device=DEV) * 3, torch.arange(n, device=DEV).flip(0)) for n in (7, 12)]
    mr = masks.clone().requires_grad_(True)
    mh = masks.clone().requires_grad_(True)
    torch.manual_seed(5)
    r = ref_loss.loss_masks(mr, ml, indices, num_masks=19.0)
    torch.manual_seed(5)
    h = hip_loss.loss_masks(mh, ml, indices, num_masks=19.0)
    for k in ("loss_mask", "loss_dice"):
        assert abs(float(h[k]) - float(r[k])) <= 1e-5 * abs(float(r[k])) + 1e-7, (k, float(h[k]), float(r[k]))
    (r["loss_mask"] * 5 + r["loss_dice"] * 5).backward()
    (h["loss_mask"] * 5 + h["loss_dice"] * 5).backward()
    assert _rel(mh.grad, mr.grad) <= 1e-4, _rel(mh.grad, mr.grad)


@pytest.mark.parametrize("ragged", [False, True], ids=["same_size", "ragged"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_loss_masks_repeated_outputs_match_reference(ragged, dt):
    """The final and auxiliary outputs call loss_masks with the same labels and different
    matches: the cached target rows (same-size images) or the reference's padded batch (ragged
    sizes), the sort-free matched-row gather and its gradient, each call against HF's."""
    from transformers import Mask2FormerConfig
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerLoss
    cfg = Mask2FormerConfig(num_labels=48)
    wd = {"loss_cross_entropy": 2.0, "loss_mask": 5.0, "loss_dice": 5.0}
    ref_loss, hip_loss = Mask2FormerLoss(cfg, weight_dict=wd), Mask2FormerLoss(cfg, weight_dict=wd)
    hip_loss.__class__ = point_loss.HipMask2FormerLoss
    masks, classes, ml, cl = _case(4, B=2, counts=(6, 9))
    if ragged:
        ml[1] = ml[1][:, :200, :300].contiguous()
    masks = masks.to(dt)
    for call in range(3):
        g = torch.Generator(device=DEV).manual_seed(30 + call)
        indices = [(torch.randperm(100, generator=g, device=DEV)[:n], torch.randperm(n, generator=g, device=DEV))
                   for n in (6, 9)]
        mr = masks.clone().requires_grad_(True)
        mh = masks.clone().requires_grad_(True)
        # bf16 logits as the model produces them: under autocast (grid_sample runs in float32)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dt == torch.bfloat16):
            torch.manual_seed(40 + call)
            r = ref_loss.loss_masks(mr, ml, indices, num_masks=15.0)
            torch.manual_seed(40 + call)
            h = hip_loss.loss_masks(mh, ml, indices, num_masks=15.0)
        for k in ("loss_mask", "loss_dice"):
            assert abs(float(h[k]) - float(r[k])) <= 1e-5 * abs(float(r[k])) + 1e-7, (call, k, float(h[k]), float(r[k]))
        (r["loss_mask"] * 5 + r["loss_dice"] * 5).backward()
        (h["loss_mask"] * 5 + h["loss_dice"] * 5).backward()
        assert mh.grad.dtype == dt
        assert _rel(mh.grad.float(), mr.grad.float()) <= (1e-4 if dt == torch.float32 else 1e-2), call


def test_install_swaps_loss_and_matcher():
    from transformers import Mask2FormerConfig
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerLoss
    cfg = Mask2FormerConfig(num_labels=48)
    holder = torch.nn.Module()
    holder.criterion = Mask2FormerLoss(cfg, weight_dict={"loss_cross_entropy": 2.0, "loss_mask": 5.0, "loss_dice": 5.0})
    assert point_loss.install(holder) == 1
    assert isinstance(holder.criterion, point_loss.HipMask2FormerLoss)
    assert isinstance(holder.criterion.matcher, matcher.HipHungarianMatcher)
    assert point_loss.uninstall(holder) == 1 and type(holder.criterion) is Mask2FormerLoss


def test_loss_all_images_empty_matches_reference():
    """A batch without any target instance: the whole Mask2FormerLoss (matcher, mask
    terms, classification term) equals HF's, mask and dice terms 0, and the backward runs."""
    from transformers import Mask2FormerConfig
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerLoss
    cfg = Mask2FormerConfig(num_labels=48)
    wd = {"loss_cross_entropy": 2.0, "loss_mask": 5.0, "loss_dice": 5.0}
    ref_loss, hip_loss = Mask2FormerLoss(cfg, weight_dict=wd).to(DEV), Mask2FormerLoss(cfg, weight_dict=wd).to(DEV)
    holder = torch.nn.Module()
    holder.criterion = hip_loss
    assert point_loss.install(holder) == 1
    masks, classes, ml, cl = _case(9, B=2, L=49, counts=(0, 0))
    mr = masks.clone().requires_grad_(True)
    mh = masks.clone().requires_grad_(True)
    torch.manual_seed(11)
    r = ref_loss(mr, classes, ml, cl)
    torch.manual_seed(11)
    h = holder.criterion(mh, classes, ml, cl)
    assert set(r) == set(h)
    for k in r:
        assert abs(float(h[k]) - float(r[k])) <= 1e-5 * abs(float(r[k])) + 1e-7, (k, float(h[k]), float(r[k]))
    assert float(h["loss_mask"]) == 0.0 and float(h["loss_dice"]) == 0.0
    sum(h.values()).backward()
    sum(r.values()).backward()
    assert torch.equal(mh.grad, mr.grad)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_match_costs_batched_equals_per_image(dt):
    """The batched cost construction (one softmax, every image's targets against its own points
    in one launch from the cached target rows, the class cost read from the softmax in the cost
    kernel) gives the bits of the image-by-image construction, with an image without targets."""
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerHungarianMatcher
    m = Mask2FormerHungarianMatcher(cost_class=2.0, cost_mask=5.0, cost_dice=5.0, num_points=12544)
    masks, classes, ml, cl = _case(7, B=4, counts=(5, 0, 23, 1))
    masks = masks.to(dt)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dt == torch.bfloat16):
        torch.manual_seed(3)
        ref = point_loss._match_costs_per_image(m, masks, classes, ml, cl)
        torch.manual_seed(3)
        got = point_loss.match_costs(m, masks, classes, ml, cl)
    assert len(ref) == len(got)
    for r, h in zip(ref, got):
        assert r.shape == h.shape and torch.equal(r, h)


def test_whole_loss_matches_reference():
    """Mask2FormerLoss.forward end to end (matcher, batched permutation indices, loss_labels from
    the concatenated labels, loss_masks) vs HF's, every term and the gradients."""
    from transformers import Mask2FormerConfig
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerLoss
    cfg = Mask2FormerConfig(num_labels=48)
    wd = {"loss_cross_entropy": 2.0, "loss_mask": 5.0, "loss_dice": 5.0}
    ref_loss, hip_loss = Mask2FormerLoss(cfg, weight_dict=wd).to(DEV), Mask2FormerLoss(cfg, weight_dict=wd).to(DEV)
    holder = torch.nn.Module()
    holder.criterion = hip_loss
    assert point_loss.install(holder) == 1
    masks, classes, ml, cl = _case(12, B=3, L=49, counts=(4, 0, 9))
    mr, mh = masks.clone().requires_grad_(True), masks.clone().requires_grad_(True)
    cr, ch = classes.clone().requires_grad_(True), classes.clone().requires_grad_(True)
    torch.manual_seed(13)
    r = ref_loss(mr, cr, ml, cl)
    torch.manual_seed(13)
    h = holder.criterion(mh, ch, ml, cl)
    assert set(r) == set(h)
    for k in r:
        assert abs(float(h[k]) - float(r[k])) <= 1e-5 * abs(float(r[k])) + 1e-7, (k, float(h[k]), float(r[k]))
    sum(r.values()).backward()
    sum(h.values()).backward()
    assert _rel(mh.grad, mr.grad) <= 1e-4
    assert _rel(ch.grad, cr.grad) <= 1e-5


@pytest.mark.parametrize("N,n,k", [(41, 37632, 9408), (3, 1000, 1), (5, 777, 777), (2, 37632, 30000), (0, 100, 5)])
@pytest.mark.parametrize("kind", ["distinct", "ties", "nan"])
def test_topk_rows_matches_torch_set(N, n, k, kind):
    """rgbd_topk_rows (loss_masks' uncertainty selection) gives torch.topk's index set when the
    values are distinct, and with ties at the k-th value the same multiset of values, taking the
    lowest indices among the tied (NaN ranks largest, as in torch)."""
    g = torch.Generator(device=DEV).manual_seed(n + k)
    x = -torch.rand((N, n), generator=g, device=DEV).abs()
    if kind == "ties":
        x = torch.round(x * 8) / 8
    if kind == "nan" and N:
        x[:, ::97] = float("nan")
    got = point_loss.topk_indices(x, k)
    assert got.shape == (N, k) and got.dtype == torch.long
    if N == 0:
        return
    ref_v, ref_i = torch.topk(x, k, dim=1, sorted=True)
    gs = torch.sort(got, dim=1).values
    assert torch.equal(gs, got)                                        # increasing index order
    assert (gs[:, 1:] != gs[:, :-1]).all()                             # distinct
    gv = torch.gather(x, 1, got)
    assert torch.equal(torch.sort(gv, dim=1, descending=True).values.nan_to_num(9.0),
                       ref_v.nan_to_num(9.0))                          # the same values
    if kind == "distinct":
        assert torch.equal(gs, torch.sort(ref_i, dim=1).values)
    else:  # the tied k-th value: the lowest indices
        kth = ref_v[:, -1:]
        for r in range(N):
            if torch.isnan(kth[r]).item():
                continue
            tied = torch.nonzero(x[r] == kth[r]).flatten()
            taken = got[r][x[r][got[r]] == kth[r]]
            assert torch.equal(taken, tied[:len(taken)])
