"""C-ABI boundary checks that run without a GPU: the library loads, exports every symbol
include/rgbd_hip.h declares, and the host-side argument validation rejects bad calls
before anything is launched."""
import ctypes

import pytest

from rgbd_amd import _lib


def test_library_loads_and_exports_header_symbols():
    L = _lib.lib()
    declared = _lib.header_symbols()
    assert len(declared) >= 14
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, f"declared but not exported: {missing}"
    assert set(declared) == set(_lib.SIGNATURES), "ctypes table out of sync with the header"
    assert L.rgbd_version().startswith(b"rgbd_hip")


def test_decomp_info_layout_matches_header():
    assert _lib.DECOMP_INFO_DTYPE.itemsize == 4 * (3 + 3 + 2 + 3 + 3 + 3) + 4 * 512


def test_argument_validation_without_device():
    L = _lib.lib()
    null = ctypes.c_void_p(0)
    # null pointers / bad sizes are rejected on the host with RGBD_E_ARG, nothing launched
    assert L.rgbd_assemble_pixel_values(null, null, 1, 4, 4, null, null, null) == -1
    assert L.rgbd_dsam_fwd(0, null, null, null, 1, 32, 8, 8, 64, null, null, null, null, null, null, null) == -1
    fake = ctypes.c_void_p(0x1000)
    # Cin not a multiple of 8 -> unsupported shape
    assert L.rgbd_dsam_fwd(0, fake, fake, fake, 1, 12, 8, 8, 64, fake, fake, null, fake, null, null, null) == -2
    # unknown dtype
    assert L.rgbd_nchw_to_nhwc(7, fake, fake, 1, 1, 1, 1, null) == -3


def test_ops_refuse_cpu_tensors():
    import torch
    from rgbd_amd import ops
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.nchw_to_nhwc(torch.zeros(1, 8, 4, 4))


def test_mask_predictor_install_keeps_state_dict():
    """f1 drop-in: the decoder's Mask2FormerMaskPredictor becomes HipMaskPredictor by a class
    swap — same parameters, same state_dict keys (no GPU needed)."""
    from transformers.models.mask2former.modeling_mask2former import Mask2FormerMaskPredictor
    from rgbd_amd import mask_predictor
    m = Mask2FormerMaskPredictor(hidden_size=32, num_heads=4, mask_feature_size=32)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    assert mask_predictor.install(m) == 1
    assert type(m) is mask_predictor.HipMaskPredictor
    after = m.state_dict()
    assert list(after) == list(before) and all(bool((after[k] == before[k]).all()) for k in before)
    assert mask_predictor.install(m) == 0
