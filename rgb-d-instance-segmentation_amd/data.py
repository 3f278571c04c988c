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

Frames are taken at model resolution (the processor's resize is then the identity; the
reference's own cv2.resize swaps width and height for non-square frames).
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


def map_10channel(rgb_u8: torch.Tensor, depth_u8: torch.Tensor, instance_map: torch.Tensor = None,
                  inst2sem=None, ignore_index: int = 0):
    """Batched map_10channel_case2: rgb_u8 [B,H,W,3], depth_u8 [B,H,W] (the 'L' depth), optional
    instance_map [B,H,W] + inst2sem -> dict(pixel_values, mask_labels, class_labels)."""
    out = {"pixel_values": ops.assemble_pixel_values(depth_u8, rgb_u8)}
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
