"""Model hyper-parameters of the reference's ``checkpoints/standard/config.json``,
restated: Hugging Face Mask2FormerConfig defaults (100 queries, hidden 256, 6 pixel-decoder
encoder layers, 10 decoder layers, 12 544 training points) on a Swin-T backbone (depths
[2,2,6,2], embed 96, window 7) with drop_path_rate 0.3 and all four stages exported."""
from transformers import Mask2FormerConfig, SwinConfig


def standard_config(num_labels: int = 48, **kw):
    from .custom_model import CustomConfig
    swin = SwinConfig(image_size=224, patch_size=4, num_channels=3, embed_dim=96, depths=[2, 2, 6, 2],
                      num_heads=[3, 6, 12, 24], window_size=7, drop_path_rate=0.3,
                      out_features=["stage1", "stage2", "stage3", "stage4"])
    id2label = {i: f"label_{i}" for i in range(num_labels)}
    return CustomConfig(backbone_config=swin, id2label=id2label, label2id={v: k for k, v in id2label.items()}, **kw)
