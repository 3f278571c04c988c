"""Seeded synthetic RGB-D scenes of the NYUv2 shape ("Synthetic inputs").

There is no NYUv2 data (and no network) here, so every benchmark and parity input is a
pure function of ``seed``:
  * depth_u8 [H,W]: background plane a + b*x + c*y (a in [60,200]) + 4-6 axis-aligned
    rectangles at constant levels U{40..250} + N(0, 2^2) noise, rounded, clipped to
    [0,255]; 3 % of the pixels set to 0 (invalid holes).
  * rgb_u8 [H,W,3]: smooth random field (bilinearly upsampled coarse noise) in [0,255].
  * labels: one binary mask per rectangle + class ids U{0..47}.
The 10-channel ``pixel_values`` layout is the one ``map_10channel_case2`` builds
(reference mask2former/utils/dataloader.py:386-425): 0:3 ImageNet-normalised RGB,
3:6 ImageNet-normalised depth-as-RGB, 6:9 DGGM normalised gradient magnitude x3,
9 DGGM valid-gradient mask.  Channels 6:10 are produced by the DGGM-pre operator
(on device in the product, by the oracle in tests).
"""
import numpy as np

# image_mean / image_std / rescale_factor of the reference's processor config
# (mask2former/checkpoints/standard/preprocessor_config.json), float32 as transformers'
# normalize casts them; the config's std[1] is one float32 ulp below float32(0.224).
IMAGENET_MEAN = np.array([0.48500001430511475, 0.4560000002384186, 0.4059999883174896], dtype=np.float32)
IMAGENET_STD = np.array([0.2290000021457672, 0.2239999920129776, 0.22499999403953552], dtype=np.float32)
RESCALE_FACTOR = 0.00392156862745098


def scene_seed(config_id: int, index: int) -> int:
    return 1000 * config_id + index


def _smooth_field(rng, h, w, ch, cell=32):
    gh, gw = h // cell + 2, w // cell + 2
    g = rng.uniform(0.0, 255.0, size=(gh, gw, ch))
    ys = np.linspace(0, gh - 1.001, h)
    xs = np.linspace(0, gw - 1.001, w)
    y0 = np.floor(ys).astype(int); x0 = np.floor(xs).astype(int)
    fy = (ys - y0)[:, None, None]; fx = (xs - x0)[None, :, None]
    a = g[y0][:, x0]; b = g[y0][:, x0 + 1]; c = g[y0 + 1][:, x0]; d = g[y0 + 1][:, x0 + 1]
    return (a * (1 - fy) * (1 - fx) + b * (1 - fy) * fx + c * fy * (1 - fx) + d * fy * fx)


def make_scene(seed: int, h: int, w: int, hole_frac: float = 0.03):
    """Returns dict(depth_u8 [H,W] u8, rgb_u8 [H,W,3] u8, masks [N,H,W] u8, classes [N] i64)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    a = rng.uniform(60, 200)
    b = rng.uniform(-40, 40) / w
    c = rng.uniform(-40, 40) / h
    depth = a + b * xx + c * yy
    n_rect = int(rng.integers(4, 7))
    masks = np.zeros((n_rect, h, w), dtype=np.uint8)
    for i in range(n_rect):
        rh = int(rng.integers(max(2, h // 10), max(3, h // 2)))
        rw = int(rng.integers(max(2, w // 10), max(3, w // 2)))
        y0 = int(rng.integers(0, h - rh + 1)); x0 = int(rng.integers(0, w - rw + 1))
        depth[y0:y0 + rh, x0:x0 + rw] = float(rng.integers(40, 251))
        masks[i] = 0
        masks[i, y0:y0 + rh, x0:x0 + rw] = 1
        for j in range(i):  # later rectangles occlude earlier ones
            masks[j, y0:y0 + rh, x0:x0 + rw] = 0
    depth = depth + rng.normal(0.0, 2.0, size=(h, w))
    depth = np.clip(np.rint(depth), 0, 255).astype(np.uint8)
    holes = rng.random((h, w)) < hole_frac
    depth[holes] = 0
    rgb = np.clip(np.rint(_smooth_field(rng, h, w, 3)), 0, 255).astype(np.uint8)
    classes = rng.integers(0, 48, size=n_rect).astype(np.int64)
    return dict(depth_u8=depth, rgb_u8=rgb, masks=masks, classes=classes)


def normalize_u8(x_u8_chw: np.ndarray) -> np.ndarray:
    """Channels as Mask2FormerImageProcessor leaves them (reference dataloader.py:405-410):
    transformers image_transforms.rescale (float64 multiply, one rounding to float32), then
    normalize ((x - mean_c) / std_c in float32), per channel (C=3, CHW)."""
    x = (x_u8_chw.astype(np.float64) * RESCALE_FACTOR).astype(np.float32)
    return (x - IMAGENET_MEAN[:, None, None]) / IMAGENET_STD[:, None, None]


def rgbd_planes(scene):
    """Channels 0:6 of pixel_values (float32 [6,H,W]) for one scene."""
    rgb = normalize_u8(np.ascontiguousarray(scene["rgb_u8"].transpose(2, 0, 1)))
    d = scene["depth_u8"]
    dep = normalize_u8(np.stack([d, d, d], axis=0))
    return np.concatenate([rgb, dep], axis=0)


def make_batch(config_id: int, b: int, h: int, w: int, start: int = 0):
    """Returns (planes [B,6,H,W] f32, depth_u8 [B,H,W] u8, scenes list)."""
    scenes = [make_scene(scene_seed(config_id, start + i), h, w) for i in range(b)]
    planes = np.stack([rgbd_planes(s) for s in scenes])
    depth = np.stack([s["depth_u8"] for s in scenes])
    return planes, depth, scenes
