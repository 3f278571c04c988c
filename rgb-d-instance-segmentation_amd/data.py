"""a11 on the device: the v0.4.0 dataset map and collate function of the reference
(mask2former/utils/dataloader.py:386-425 ``map_10channel_case2``, :772-781 ``collate_fn_v2``).

The reference builds every example on the host inside ``datasets.map`` (PIL conversions,
Mask2FormerImageProcessor, cv2 Sobel) and stores float64 lists in Arrow.  Here the raw u8
planes go to HBM once and the kernels produce what the model consumes:

  pixel_values [B,10,H,W] f32  K1 (rgbd_assemble_pixel_values): channels 0:6 bit-exact to the
                               processor's rescale + normalise (preprocessor_config.json),
                               6:10 the DGGM Sobel planes (data_process.py:1247-1305)
  mask_labels  list of [N_b,H,W] f32, class_labels list of [N_b] int64
                               rgbd_instance_presence + rgbd_instance_masks: the processor's
                               convert_segmentation_map_to_binary_masks (ignore_index 0,
                               mask2former/config.json)

Frames at another resolution are resized on the device first (``resize_frames``), as the
reference resizes them (dataloader.py:405-414): the processor's PIL BILINEAR for the colour and
the depth-as-RGB images (channels 0:6; bit-exact to Pillow), PIL NEAREST for the instance map,
and ``cv2.resize(depth, (h, w), INTER_LINEAR)`` for the depth the DGGM Sobel planes come from
(channels 6:10; OpenCV is absent here, that restatement is parity unpinned).  The reference passes
(h, w) as cv2's dsize = (width, height), so its Sobel planes come out transposed for non-square
model sizes and the example cannot be assembled: a resize to a non-square size
raises ValueError here instead of transposing.
"""
import ctypes

import numpy as np
import torch

from . import _lib, ops
from ._lib import check


def instance_labels(instance_map: torch.Tensor, inst2sem, ignore_index: int = 0):
    """instance_map: uint8 [B,H,W] (the annotation's instance channel) on the GPU; inst2sem:
    one {instance id: semantic id} dict per image (or one for all).  -> (mask_labels list of
    float32 [N_b,H,W], class_labels list of int64 [N_b]), both on the GPU.  An instance id
    missing from its table raises KeyError, as the processor does."""
    ops._need_cuda(instance_map)
    if instance_map.dtype != torch.uint8 or instance_map.dim() != 3:
        raise ValueError("instance_map must be uint8 [B,H,W]")
    B, H, W = instance_map.shape
    tables = list(inst2sem) if isinstance(inst2sem, (list, tuple)) else [inst2sem] * B
    if len(tables) != B:
        raise ValueError("one instance -> semantic table per image expected")
    dev = instance_map.device
    L = _lib.lib()
    st = ops._stream(dev)
    pres = torch.empty((B, 8), dtype=torch.int32, device=dev)
    check(L.rgbd_instance_presence(ops._p(instance_map), B, H, W, ops._p(pres), st), "rgbd_instance_presence")
    bits = pres.cpu().numpy().view(np.uint32)  # 32 bytes per image: sizes the ragged outputs
    ids, img, classes = [], [], []
    for b in range(B):
        present = [k * 32 + i for k in range(8) for i in range(32) if (bits[b, k] >> i) & 1]
        lab = [i for i in present if ignore_index is None or i != ignore_index]
        ids += lab
        img += [b] * len(lab)
        classes.append(np.array([tables[b][int(i)] for i in lab], dtype=np.int64))
    n = len(ids)
    masks = torch.empty((max(n, 1), H, W), dtype=torch.float32, device=dev)
    if n:
        meta = torch.tensor([ids, img], dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
        check(L.rgbd_instance_masks(ops._p(instance_map), H, W, ctypes.c_void_p(meta[0].data_ptr()),
                                    ctypes.c_void_p(meta[1].data_ptr()), n, ops._p(masks), st),
              "rgbd_instance_masks")
    mask_labels, o = [], 0
    for b in range(B):
        k = len(classes[b])
        mask_labels.append(masks[o:o + k])
        o += k
    return mask_labels, [torch.from_numpy(c).to(dev) for c in classes]


def _resize(kind, src, out_h, out_w):
    src = src.contiguous()  # frames may arrive as strided views (e.g. a channel-reversed decode)
    ops._need_cuda(src)
    if src.dtype != torch.uint8:
        raise ValueError("resize: uint8 frames expected")
    B, H, W = src.shape[:3]
    C = src.shape[3] if src.dim() == 4 else 1
    L = _lib.lib()
    dst = torch.empty((B, out_h, out_w) + tuple(src.shape[3:]), dtype=torch.uint8, device=src.device)
    ws = ops._workspace(src.device, L.rgbd_resize_workspace_size(B, H, W, C, out_h, out_w), "resize")
    st = ops._stream(src.device)
    if kind == "bilinear":
        rc = L.rgbd_resize_pil_bilinear(ops._p(src), B, H, W, C, out_h, out_w, ops._p(dst), ops._p(ws), st)
    elif kind == "nearest":
        rc = L.rgbd_resize_pil_nearest(ops._p(src), B, H, W, C, out_h, out_w, ops._p(dst), ops._p(ws), st)
    else:
        rc = L.rgbd_resize_cv2_linear(ops._p(src), B, H, W, out_h, out_w, ops._p(dst), ops._p(ws), st)
    check(rc, f"rgbd_resize ({kind})")
    return dst


def pil_resize(img_u8: torch.Tensor, size, resample="bilinear"):
    """PIL.Image.resize((w, h), BILINEAR | NEAREST) of uint8 [B,H,W] or [B,H,W,C] frames."""
    return _resize(resample, img_u8, int(size[0]), int(size[1]))


def cv2_resize_linear(depth_u8: torch.Tensor, dsize):
    """cv2.resize(depth, dsize=(width, height), interpolation=cv2.INTER_LINEAR), uint8 [B,H,W]."""
    return _resize("cv2", depth_u8, int(dsize[1]), int(dsize[0]))


def resize_frames(rgb_u8, depth_u8, instance_map=None, size=None):
    """The resizes of map_10channel_case2 to the processor's size (h, w) (dataloader.py:405-414):
    -> (rgb [B,h,w,3] and depth [B,h,w] as the processor resizes them (PIL BILINEAR), the depth
    the Sobel planes use (cv2.resize(depth, (h, w)) INTER_LINEAR), the instance map (PIL
    NEAREST) or None)."""
    h, w = int(size[0]), int(size[1])
    B, H, W = depth_u8.shape
    if (h, w) == (H, W):
        return rgb_u8, depth_u8, depth_u8, instance_map
    if h != w:
        raise ValueError(f"resize to {h}x{w}: the reference's cv2.resize(depth, (h, w)) takes (h, w) as "
                         "(width, height) and transposes the gradient planes of non-square sizes (SURVEY Q18); "
                         "resize frames to a square model size, or pass frames at model resolution")
    rgb_r = pil_resize(rgb_u8, (h, w)) if rgb_u8 is not None else None
    # the processor's depth-as-RGB image has three equal channels: resizing the 'L' plane once
    # gives each of them (Pillow's 8bpc resample is per channel)
    depth_proc = pil_resize(depth_u8, (h, w))
    depth_cv2 = cv2_resize_linear(depth_u8, (h, w))
    inst = pil_resize(instance_map, (h, w), "nearest") if instance_map is not None else None
    return rgb_r, depth_proc, depth_cv2, inst


def map_10channel(rgb_u8: torch.Tensor, depth_u8: torch.Tensor, instance_map: torch.Tensor = None,
                  inst2sem=None, ignore_index: int = 0, size=None):
    """Batched map_10channel_case2: rgb_u8 [B,H,W,3], depth_u8 [B,H,W] (the 'L' depth), optional
    instance_map [B,H,W] + inst2sem, optional processor size (h, w) -> dict(pixel_values,
    mask_labels, class_labels)."""
    depth_sobel = depth_u8
    if size is not None:
        rgb_u8, depth_u8, depth_sobel, instance_map = resize_frames(rgb_u8, depth_u8, instance_map, size)
    pv = ops.assemble_pixel_values(depth_u8, rgb_u8)
    if depth_sobel is not depth_u8:  # channels 6:10 from the cv2-resized depth (:414-421)
        pv[:, 6:10] = ops.assemble_pixel_values(depth_sobel)[:, 6:10]
    out = {"pixel_values": pv}
    if instance_map is not None:
        out["mask_labels"], out["class_labels"] = instance_labels(instance_map, inst2sem, ignore_index)
    return out


def collate_fn_v2(examples):
    """dataloader.py:772-781: stack pixel_values (and pixel_mask), keep the ragged labels as lists."""
    batch = {"pixel_values": torch.stack([e["pixel_values"] for e in examples]),
             "class_labels": [e["class_labels"] for e in examples],
             "mask_labels": [e["mask_labels"] for e in examples]}
    if "pixel_mask" in examples[0]:
        batch["pixel_mask"] = torch.stack([e["pixel_mask"] for e in examples])
    return batch
