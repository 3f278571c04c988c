"""The reference's entry point (mask2former/finetuning.py:86-92, :98-113, :127, predictor.py:697-700)
driven with the drop-in: ``from_pretrained(..., version="0.4.0")`` with relabelled classes and
``ignore_mismatched_sizes``, an HF Trainer over examples made by the on-device data path
(data.map_10channel + collate_fn_v2, the dataloader's map / collate), one training step,
``trainer.predict``, and the device post-processing installed into the image processor — the
plumbing a user of finetuning.py goes through, at a small input size."""
import sys
import types
from pathlib import Path

import numpy as np
import pytest
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import _rgbd_import  # noqa: E402,F401

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _examples(n, H, W):
    from rgbd_amd import data, synthetic
    out = []
    for i in range(n):
        sc = synthetic.make_scene(synthetic.scene_seed(91, i), H, W)
        inst = torch.zeros((1, H, W), dtype=torch.uint8)
        inst[0, H // 4:H // 2, W // 4:W // 2] = 1
        inst[0, H // 2:, W // 2:] = 2
        ex = data.map_10channel(torch.from_numpy(sc["rgb_u8"][None]).contiguous().to(DEV),
                                torch.from_numpy(sc["depth_u8"][None]).to(DEV), inst.to(DEV), {1: 3, 2: 7})
        out.append({"pixel_values": ex["pixel_values"][0].cpu(), "mask_labels": ex["mask_labels"][0].cpu(),
                    "class_labels": ex["class_labels"][0].cpu()})
    return out


def test_from_pretrained_trainer_train_predict(tmp_path):
    from transformers import Trainer, TrainingArguments
    from transformers.models.mask2former.image_processing_pil_mask2former import Mask2FormerImageProcessorPil
    from rgbd_amd import init as winit
    from rgbd_amd.config import standard_config
    from rgbd_amd.custom_model import CustomMask2FormerForUniversalSegmentation
    from rgbd_amd.data import collate_fn_v2
    from rgbd_amd.postprocess import install

    torch.manual_seed(0)
    base = CustomMask2FormerForUniversalSegmentation(standard_config(48), version="0.4.0")
    winit.init_deterministic(base)
    base.save_pretrained(tmp_path / "ckpt")
    id2label = {i: f"class_{i}" for i in range(10)}  # relabelled head: ignore_mismatched_sizes
    model = CustomMask2FormerForUniversalSegmentation.from_pretrained(
        tmp_path / "ckpt", label2id={v: k for k, v in id2label.items()}, id2label=id2label,
        ignore_mismatched_sizes=True, version="0.4.0")
    assert model.model.pixel_level_module.version == "0.4.0"
    assert model.class_predictor.out_features == 11
    sd0 = base.state_dict()
    for k, v in model.state_dict().items():  # everything but the resized class head is loaded
        if k in sd0 and sd0[k].shape == v.shape and not k.startswith("class_predictor"):
            assert torch.equal(v, sd0[k]), k

    H, W = 96, 128
    train, val = _examples(4, H, W), _examples(3, H, W)
    args = TrainingArguments(output_dir=str(tmp_path / "out"), per_device_train_batch_size=2,
                             per_device_eval_batch_size=2, max_steps=1, learning_rate=1e-5, report_to=[],
                             save_strategy="no", remove_unused_columns=False, dataloader_num_workers=0,
                             logging_strategy="no")
    proc = Mask2FormerImageProcessorPil()
    trainer = Trainer(model=model, args=args, train_dataset=train, eval_dataset=val, data_collator=collate_fn_v2,
                      processing_class=proc)
    before = {k: v.detach().clone() for k, v in model.named_parameters() if "dsam" in k and v.requires_grad}
    out = trainer.train()
    assert np.isfinite(out.training_loss)
    changed = [k for k, v in model.named_parameters() if k in before and not torch.equal(v.detach(), before[k])]
    assert changed, "no DSAM parameter was updated by the training step"

    result = trainer.predict(test_dataset=val)
    preds = result.predictions
    cls, masks = preds[0], preds[1]
    assert cls.shape[0] == 3 and cls.shape[-1] == 11 and masks.shape[0] == 3
    outs = types.SimpleNamespace(class_queries_logits=torch.from_numpy(cls), masks_queries_logits=torch.from_numpy(masks))
    ref = proc.post_process_instance_segmentation(outs, target_sizes=[(H, W)] * 3, threshold=0.0)
    got = install(Mask2FormerImageProcessorPil()).post_process_instance_segmentation(
        outs, target_sizes=[(H, W)] * 3, threshold=0.0)
    for r, g in zip(ref, got):
        assert torch.equal(r["segmentation"], g["segmentation"])
        assert [(s["id"], s["label_id"]) for s in r["segments_info"]] == [(s["id"], s["label_id"])
                                                                          for s in g["segments_info"]]
