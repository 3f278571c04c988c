"""Deterministic inputs shared by make_golden.py (reference side) and the tests (oracle /
HIP side).  Everything is a pure function of names and seeds, so fixtures store only
outputs plus the sha256 of the inputs they were made from."""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))
import _rgbd_import  # noqa: E402,F401
from rgbd_amd import init as winit, synthetic  # noqa: E402

F32 = np.float32


def feature(name, shape):
    """Unit-variance uniform feature map (float32) from the counter hash."""
    n = int(np.prod(shape))
    return (winit.unit_uniform(name, n) * np.sqrt(3.0)).astype(F32).reshape(shape)


def sample_index(name, n, k):
    u = winit.unit_uniform(name, k)
    return np.clip(((u + 1.0) * 0.5 * n).astype(np.int64), 0, n - 1)


def swin_sizes(H, W):
    """Swin-T feature-map sizes at strides 4/8/16/32 (patch embed pads to /4, merging pads to /2)."""
    h, w = -(-H // 4), -(-W // 4)
    out = [(h, w)]
    for _ in range(3):
        h, w = -(-h // 2), -(-w // 2)
        out.append((h, w))
    return out


def pool_sizes(H, W):
    return swin_sizes(H, W)[:3]


def pixel_values(config_id, B, H, W):
    from oracle import dggm_pre
    planes, depth, _ = synthetic.make_batch(config_id, B, H, W)
    dg = np.stack([dggm_pre.dggm_planes(d) for d in depth])
    return np.ascontiguousarray(np.concatenate([planes, dg], axis=1).astype(F32))


def labels(config_id, B, H, W):
    scenes = [synthetic.make_scene(synthetic.scene_seed(config_id, i), H, W) for i in range(B)]
    return ([s["masks"].astype(F32) for s in scenes], [s["classes"] for s in scenes])


def instance_map(scene):
    """The instance channel of the reference's annotation PNG for a synthetic scene
    (dataloader.py:391-403): uint8 [H,W], 0 = background, rectangle i -> id 7*i + 3, plus the
    instance -> semantic id table built from the (instance, semantic) pairs."""
    inst = np.zeros(scene["masks"].shape[1:], np.uint8)
    table = {0: 0}
    for i, m in enumerate(scene["masks"]):
        inst[m > 0] = 7 * i + 3
        table[7 * i + 3] = int(scene["classes"][i])
    return inst, table


def label_kwargs():
    id2label = {i: f"label_{i}" for i in range(48)}
    return dict(id2label=id2label, label2id={v: k for k, v in id2label.items()})


def _designed(H, W, bins_counts, lo=0.0, hi=1.0, fill_lo=True):
    """Grey-level image whose histogram has the given {bin: count} (values at bin centres
    of the [lo, hi] 512-bin grid), the rest of the pixels at lo (bin 0) and one at hi."""
    step = (hi - lo) / 512.0
    vals = []
    for b, c in bins_counts.items():
        vals += [lo + (b + 0.5) * step] * c
    n = H * W
    assert len(vals) + 1 <= n
    v = np.full(n, lo if fill_lo else hi, dtype=np.float64)
    v[:len(vals)] = vals
    v[-1] = hi
    rng = np.random.default_rng(len(vals))
    v = rng.permutation(v).astype(F32).reshape(H, W)
    return np.stack([v, v, v])


def _scene_depth3(seed, H, W):
    s = synthetic.make_scene(seed, H, W)
    return synthetic.rgbd_planes(s)[3:6].astype(F32)


def decomposition_cases():
    """[(name, depth3 float32 [3,H,W], ratio)] covering SURVEY §8(c) G1's edge cases."""
    cases = []
    ratios = [0.01, 0.1, 0.25, 0.5, 0.37, 0.05]
    for s in range(6):
        cases.append((f"scene{s}", _scene_depth3(100 + s, 240, 320), ratios[s]))
    for s in range(10):
        cases.append((f"small{s}", _scene_depth3(200 + s, 64, 96), 0.05 + 0.045 * s))
    H, W = 64, 96
    u8 = lambda a: synthetic.normalize_u8(np.stack([a, a, a]).astype(np.uint8)).astype(F32)  # noqa: E731
    cases.append(("const", u8(np.full((H, W), 150)), 0.2))
    two = np.full((H, W), 80); two[:, W // 2:] = 200
    cases.append(("two_level", u8(two), 0.3))
    rng = np.random.default_rng(7)
    cases.append(("all_negative", u8(rng.integers(20, 61, size=(H, W))), 0.4))
    nop = np.full((H, W), 10); nop[H // 2:] = 240
    cases.append(("no_peak", u8(nop), 0.1))
    cases.append(("plateau", _designed(H, W, {100: 800, 101: 800, 102: 800, 300: 1000, 301: 1000, 400: 500}), 0.25))
    cases.append(("tied", _designed(H, W, {100: 1000, 200: 1000, 350: 1000, 450: 999}), 0.15))
    cases.append(("many_peaks", _designed(H, W, {50: 400, 120: 900, 180: 200, 260: 700, 330: 550, 420: 850}), 0.5))
    cases.append(("low_prominence", _designed(H, W, {100: 1500, 101: 1000, 102: 1005, 103: 995, 400: 600}), 0.3))
    nan = _scene_depth3(300, H, W)
    nan[:, rng.random((H, W)) < 0.02] = np.nan
    cases.append(("nan", nan, 0.2))
    cases.append(("odd_size", _scene_depth3(301, 90, 125), 0.33))
    cases.append(("all_nan", np.full((3, 8, 8), np.nan, F32), 0.1))
    tiny = np.full((3, H, W), 1.0, F32); tiny[:, 0, 0] = np.nextafter(F32(1.0), F32(2.0))
    cases.append(("tiny_range", tiny, 0.1))
    return cases


# decomposition cases used for the DSAM forward fixture: small0, const, no_peak, plateau, tied
G2_CASES = [6, 16, 19, 20, 21]
