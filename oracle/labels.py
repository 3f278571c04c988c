"""ORACLE (test infrastructure only) — the label half of map_10channel_case2
(reference mask2former/utils/dataloader.py:391-423): the annotation's instance channel goes
through Mask2FormerImageProcessor, whose convert_segmentation_map_to_binary_masks
(transformers image_processing_pil_mask2former.py:81-115, the numpy processor of transformers
4.47 that the reference's checkpoints were written with) produces

    labels       = sorted unique instance ids, minus ignore_index (0 in mask2former/config.json)
    mask_labels  = float32 [N, H, W], mask_labels[i] = (instance_map == labels[i])
    class_labels = int64 [N], instance_id_to_semantic_id[labels[i]]

Pinned bit-exact against the processor itself by tests/golden/g0_processor.npz."""
import numpy as np


def instance_labels(instance_map: np.ndarray, inst2sem: dict, ignore_index: int = 0):
    ids = np.unique(instance_map)
    if ignore_index is not None:
        ids = ids[ids != ignore_index]
    masks = np.stack([instance_map == i for i in ids]) if ids.size else np.zeros((0,) + instance_map.shape, bool)
    classes = np.array([inst2sem[int(i)] for i in ids], dtype=np.int64)
    return masks.astype(np.float32), classes
