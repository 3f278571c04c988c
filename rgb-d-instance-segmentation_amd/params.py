"""State-dict layout of the v0.4.0 hot path (SURVEY.md §8(b) "State-dict keys").

Keys are relative to ``model.pixel_level_module.`` and identical to the reference
(custom_model.py:127-134, 636-640, 1183-1191, 1378-1437) so checkpoints interchange.
"""
PLM_PREFIX = "model.pixel_level_module."

DSAM_CHANNELS = [(96, 192), (192, 384), (384, 768)]
COLOR_CHANNELS = [96, 192, 384, 768]


def _cbn(pre, cout, cin, k):
    return {f"{pre}.0.weight": (cout, cin, k, k), f"{pre}.0.bias": (cout,),
            f"{pre}.1.weight": (cout,), f"{pre}.1.bias": (cout,),
            f"{pre}.1.running_mean": (cout,), f"{pre}.1.running_var": (cout,)}


RATIO_SHAPES = {}
RATIO_SHAPES.update(_cbn("scale1_conv", 64, 3, 3))
RATIO_SHAPES.update(_cbn("scale2_conv", 64, 3, 5))
RATIO_SHAPES.update(_cbn("scale3_conv", 64, 3, 7))
RATIO_SHAPES.update(_cbn("feature_fusion", 128, 192, 1))
RATIO_SHAPES.update({"attention.0.weight": (64, 128, 1, 1), "attention.0.bias": (64,),
                     "attention.2.weight": (128, 64, 1, 1), "attention.2.bias": (128,)})
for _a, _b in (("0", "1"), ("4", "5")):
    _cin, _cout = (128, 256) if _a == "0" else (256, 512)
    RATIO_SHAPES.update({f"feature_extractor.{_a}.weight": (_cout, _cin, 3, 3),
                         f"feature_extractor.{_a}.bias": (_cout,),
                         f"feature_extractor.{_b}.weight": (_cout,), f"feature_extractor.{_b}.bias": (_cout,),
                         f"feature_extractor.{_b}.running_mean": (_cout,),
                         f"feature_extractor.{_b}.running_var": (_cout,)})
for _i, (_o, _n) in zip((0, 3, 6, 8), ((128, 512), (64, 128), (32, 64), (1, 32))):
    RATIO_SHAPES[f"fc_layers.{_i}.weight"] = (_o, _n)
    RATIO_SHAPES[f"fc_layers.{_i}.bias"] = (_o,)


def dsam_shapes(k):
    cin, cout = DSAM_CHANNELS[k]
    d = {}
    for i in range(4):
        d[f"conv_layers.{i}.weight"] = (cout, cin, 3, 3)
        d[f"conv_layers.{i}.bias"] = (cout,)
    d["rgb_projection.weight"] = (cout, cin, 3, 3)
    return d


DGGM_SHAPES = {}
for _i, _c in enumerate(COLOR_CHANNELS):
    DGGM_SHAPES[f"depth_enhancement_layers.{_i}.0.weight"] = (_c, 3, 1, 1)
    DGGM_SHAPES[f"depth_enhancement_layers.{_i}.0.bias"] = (_c,)


def hot_path_shapes():
    """{key relative to model.pixel_level_module.: shape} for every hot-path tensor."""
    out = {f"ratio_predictor.{k}": v for k, v in RATIO_SHAPES.items()}
    for k in range(3):
        out.update({f"dsam{k}.{kk}": v for kk, v in dsam_shapes(k).items()})
    out.update({f"depth_gradient_injection.{k}": v for k, v in DGGM_SHAPES.items()})
    return out
