"""a11 on the device for frames not at model resolution (csrc/resize.hip, rgbd_amd/data.py):
the PIL BILINEAR / NEAREST kernels bit-exact against Pillow and the restatement, the cv2 linear
kernel bit-exact against its restatement (parity unpinned vs OpenCV, absent), and
map_10channel(size=...) reproducing the reference processor's resized output (g8_resize.npz)."""
import hashlib

import numpy as np
import pytest
import torch
from PIL import Image

import golden_inputs as gi
from oracle import dggm_pre, resize as R
from rgbd_amd import data, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"
SIZES = [(480, 640, 640, 640), (480, 640, 320, 320), (37, 53, 64, 96), (64, 96, 37, 53), (5, 7, 17, 3),
         (720, 1280, 480, 640), (64, 64, 16, 16)]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("H,W,oh,ow", SIZES)
def test_pil_kernels_match_pillow(H, W, oh, ow):
    rng = np.random.default_rng(H + W + oh)
    rgb = rng.integers(0, 256, (2, H, W, 3), dtype=np.uint8)
    gray = rng.integers(0, 256, (2, H, W), dtype=np.uint8)
    out_rgb = data.pil_resize(torch.from_numpy(rgb).to(DEV), (oh, ow)).cpu().numpy()
    out_gray = data.pil_resize(torch.from_numpy(gray).to(DEV), (oh, ow)).cpu().numpy()
    out_near = data.pil_resize(torch.from_numpy(gray).to(DEV), (oh, ow), "nearest").cpu().numpy()
    for b in range(2):
        assert np.array_equal(out_rgb[b], np.asarray(Image.fromarray(rgb[b]).resize((ow, oh), Image.BILINEAR)))
        assert np.array_equal(out_gray[b], np.asarray(Image.fromarray(gray[b]).resize((ow, oh), Image.BILINEAR)))
        assert np.array_equal(out_near[b], np.asarray(Image.fromarray(gray[b]).resize((ow, oh), Image.NEAREST)))


@pytest.mark.parametrize("H,W,oh,ow", SIZES)
def test_cv2_linear_kernel_matches_restatement(H, W, oh, ow):
    d = np.random.default_rng(H * 3 + ow).integers(0, 256, (2, H, W), dtype=np.uint8)
    got = data.cv2_resize_linear(torch.from_numpy(d).to(DEV), (ow, oh)).cpu().numpy()
    for b in range(2):
        assert np.array_equal(got[b], R.cv2_linear(d[b], (ow, oh)))


def test_map_10channel_resized_matches_reference_processor(golden):
    g8 = golden("g8_resize")
    for tag in ("small", "c2"):
        H, W, S = (int(v) for v in g8[f"{tag}_size"])
        sc = synthetic.make_scene(synthetic.scene_seed(71, 0), H, W)
        inst, table = gi.instance_map(sc)
        ex = data.map_10channel(torch.from_numpy(sc["rgb_u8"][None]).to(DEV),
                                torch.from_numpy(sc["depth_u8"][None]).to(DEV),
                                torch.from_numpy(inst[None].astype(np.uint8)).to(DEV), [table], size=(S, S))
        pv = ex["pixel_values"][0].cpu().numpy()
        assert pv.shape == (10, S, S)
        assert _sha(pv[:6]) == str(g8[f"{tag}_pv6_sha"]), tag
        masks = ex["mask_labels"][0].cpu().numpy()
        assert tuple(masks.shape) == tuple(g8[f"{tag}_masks_shape"])
        assert _sha(masks) == str(g8[f"{tag}_masks_sha"]), tag
        assert np.array_equal(ex["class_labels"][0].cpu().numpy(), g8[f"{tag}_classes"])
        # channels 6:10: the DGGM Sobel planes of cv2.resize(depth, (S, S)) (restatement)
        planes = dggm_pre.dggm_planes(R.cv2_linear(sc["depth_u8"], (S, S)))
        assert np.array_equal(pv[6:10].view(np.uint32), planes.view(np.uint32))


def test_non_square_resize_is_refused():
    """The reference's cv2.resize(depth, (h, w)) transposes non-square sizes."""
    rgb = torch.zeros((1, 48, 64, 3), dtype=torch.uint8, device=DEV)
    d = torch.zeros((1, 48, 64), dtype=torch.uint8, device=DEV)
    with pytest.raises(ValueError, match="Q18"):
        data.map_10channel(rgb, d, size=(32, 64))
