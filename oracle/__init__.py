"""ORACLE — test infrastructure only.

CPU restatement of the reference's v0.4.0 DGGM + E-DSAM hot path
(TheoBald200814/RGB-D-Instance-Segmentation @ 2025-07-18), used ONLY as the checker by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg.  The
product package (``rgb-d-instance-segmentation_amd``) never imports anything here and
has no CPU fallback.

Integer / index / byte work (histogram, peak picking, windows, region masks, pooled
masks, DGGM valid mask) is restated in numpy with the exact float32 rounding sequence of
the reference's numpy 2.2 / scipy 1.15 calls; floating-point convolution work is
restated with PyTorch-CPU fp32 ops (the "torch fp32 reference" for float kernels).

Pinning:
  * edsam.py / dggm.py / ratio.py / hot_path.py are pinned by golden vectors generated
    by importing the reference itself in the build container (tests/golden/make_golden.py).
  * dggm_pre.py restates ``calculate_gradient_features``, which calls OpenCV's Sobel;
    OpenCV is not installed, so that function is **parity unpinned** against the
    reference and is cross-checked against scipy.ndimage instead (exact on u8 input).
"""
