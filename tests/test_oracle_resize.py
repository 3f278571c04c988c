"""a11 for frames not at model resolution: the resize restatements (oracle/resize.py) pinned.

* PIL BILINEAR / NEAREST restatements vs Pillow itself (installed here and on the GPU box) on
  up- and down-scales, odd sizes, colour and single-channel images: bit-exact.
* The processor's whole output at a resized size — the reference's Mask2FormerImageProcessor
  (g8_resize.npz, made by tests/golden/make_golden.py ``resize_fixture``): channels 0:6 of
  pixel_values and the label tensors from the restated resize + normalisation + binary masks,
  bit-exact.
* cv2 INTER_LINEAR (OpenCV absent: parity unpinned): the identities the restatement must keep
  (same size copies, constant images stay constant, integer-ratio upscale of a ramp is monotone).
"""
import hashlib

import numpy as np
import pytest
from PIL import Image

import golden_inputs as gi
from oracle import labels as labels_o, resize as R
from rgbd_amd import synthetic

SIZES = [(480, 640, 640, 640), (480, 640, 320, 320), (37, 53, 64, 96), (64, 96, 37, 53), (100, 100, 33, 77),
         (5, 7, 17, 3), (480, 640, 481, 641), (120, 160, 480, 640), (720, 1280, 480, 640), (64, 64, 16, 16)]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("H,W,oh,ow", SIZES)
@pytest.mark.parametrize("ch", [3, 0], ids=["rgb", "L"])
def test_pil_restatement_matches_pillow(H, W, oh, ow, ch):
    img = np.random.default_rng(H * W + oh).integers(0, 256, (H, W, ch) if ch else (H, W), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
    assert np.array_equal(R.pil_bilinear(img, oh, ow), ref)
    ref = np.asarray(Image.fromarray(img).resize((ow, oh), Image.NEAREST))
    assert np.array_equal(R.pil_nearest(img, oh, ow), ref)


def test_pil_nearest_index_walk_matches_pillow_on_many_sizes():
    """The NEAREST source index is Pillow's incremental double walk (not floor((x + 0.5) s)):
    300 random (in, out) pairs."""
    rng = np.random.default_rng(1)
    for a, b in rng.integers(1, 1500, (300, 2)):
        img = np.tile(np.arange(a, dtype=np.int32)[None, :], (2, 1))
        ref = np.asarray(Image.fromarray(img, mode="I").resize((int(b), 2), Image.NEAREST))[0]
        assert np.array_equal(R.pil_nearest_index(int(a), int(b)), ref), (a, b)


def test_processor_resize_output_matches_reference(golden):
    g8 = golden("g8_resize")
    for tag in ("small", "c2"):
        H, W, S = (int(v) for v in g8[f"{tag}_size"])
        sc = synthetic.make_scene(synthetic.scene_seed(71, 0), H, W)
        rgb = R.pil_bilinear(sc["rgb_u8"], S, S)
        d = R.pil_bilinear(sc["depth_u8"], S, S)
        pv6 = np.concatenate([synthetic.normalize_u8(np.ascontiguousarray(rgb.transpose(2, 0, 1))),
                              synthetic.normalize_u8(np.stack([d, d, d]))], axis=0)
        assert _sha(pv6) == str(g8[f"{tag}_pv6_sha"]), tag
        inst, table = gi.instance_map(sc)
        masks, classes = labels_o.instance_labels(R.pil_nearest(inst, S, S), table, ignore_index=0)
        assert tuple(masks.shape) == tuple(g8[f"{tag}_masks_shape"])
        assert _sha(masks) == str(g8[f"{tag}_masks_sha"]), tag
        assert np.array_equal(classes, g8[f"{tag}_classes"])
        if tag == "small":
            assert np.array_equal(pv6.view(np.uint32), g8["small_pv6"].view(np.uint32))


def test_cv2_linear_restatement_identities():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    assert np.array_equal(R.cv2_linear(img, (53, 37)), img)                    # same size: copy
    assert (R.cv2_linear(np.full((30, 40), 77, np.uint8), (64, 64)) == 77).all()  # constant stays
    ramp = np.tile(np.arange(0, 256, 4, dtype=np.uint8)[None, :], (8, 1))
    up = R.cv2_linear(ramp, (ramp.shape[1] * 2, 8))
    assert (np.diff(up[0].astype(int)) >= 0).all() and up[0, 0] == 0 and up[0, -1] == 252
    assert R.cv2_linear(img, (20, 30)).shape == (30, 20)                       # dsize = (width, height)
