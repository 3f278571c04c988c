"""a11 (10-channel assembly, dataloader.py:386-425) pinned to the reference's image processor:
g0_processor.npz holds Mask2FormerImageProcessor's own outputs (tests/golden/make_golden.py,
``processor_fixture``).  Channels 0:6 of pixel_values and the label tensors must be bit-exact."""
import hashlib

import numpy as np

import golden_inputs as gi
from oracle import labels as labels_o
from rgbd_amd import synthetic


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_normalisation_exhaustive_u8(golden):
    """Every u8 value in each of the three channels: rescale (float64) + normalise (float32,
    the config's mean/std) — the restatement K1 implements — equals the processor bit for bit."""
    g0 = golden("g0_processor")
    img = g0["lut_rgb_u8"]
    got = synthetic.normalize_u8(np.ascontiguousarray(img.transpose(2, 0, 1)))
    assert got.dtype == np.float32
    assert np.array_equal(got.view(np.uint32), g0["lut_out"].view(np.uint32))
    for c in range(3):
        assert len(np.unique(img[..., c])) == 256


def test_pixel_values_and_labels_match_processor(golden):
    g0 = golden("g0_processor")
    for tag, (H, W) in {"small": (64, 96), "c2": (480, 640)}.items():
        sc = synthetic.make_scene(synthetic.scene_seed(70, 0), H, W)
        pv6 = synthetic.rgbd_planes(sc)
        assert _sha(pv6) == str(g0[f"{tag}_pv6_sha"]), tag
        inst, table = gi.instance_map(sc)
        masks, classes = labels_o.instance_labels(inst, table, ignore_index=0)
        assert tuple(masks.shape) == tuple(g0[f"{tag}_masks_shape"])
        assert _sha(masks) == str(g0[f"{tag}_masks_sha"]), tag
        assert np.array_equal(classes, g0[f"{tag}_classes"])
    small = synthetic.rgbd_planes(synthetic.make_scene(synthetic.scene_seed(70, 0), 64, 96))
    assert np.array_equal(small.view(np.uint32), g0["small_pv6"].view(np.uint32))


def test_old_float32_rescale_would_differ(golden):
    """Documents the round-1 deviation this pins away: float32 x * f32(1/255) with std 0.224f
    differs from the processor by one ulp on most values."""
    g0 = golden("g0_processor")
    img = np.ascontiguousarray(g0["lut_rgb_u8"].transpose(2, 0, 1))
    mean = np.array([0.485, 0.456, 0.406], np.float32)[:, None, None]
    std = np.array([0.229, 0.224, 0.225], np.float32)[:, None, None]
    old = (img.astype(np.float32) * np.float32(1.0 / 255.0) - mean) / std
    assert (old != g0["lut_out"]).sum() > 1000
