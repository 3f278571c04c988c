"""rgbd_amd — MI355X-native DGGM + E-DSAM hot path of the RGB-D Mask2Former (v0.4.0).

Drop-in for the reference's ``CustomMask2FormerPixelLevelModule`` v0.4.0 body
(mask2former/utils/custom_model.py:324-355) and its sub-modules.  All compute runs in
hand-written HIP kernels for gfx950 behind the C-ABI library ``librgbd_hip.so``
(declared in include/rgbd_hip.h); importing ``rgbd_amd.ops`` loads it and fails loudly
when it is missing.  Sub-modules are imported lazily so the pure-host pieces
(``init``, ``synthetic``) work without a GPU.
"""
__version__ = "0.1.0"
