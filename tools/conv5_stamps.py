"""Per-step s_memtime stamps of conv5 (k_rp_conv5_v4; workgroup 0, its first two items) from the
diagnostic build (make -C rgb-d-instance-segmentation_amd/csrc diag) or an experiment build made
with -DC4_STAMPS (tools/build_variant.sh NAME -DC4_STAMPS [...]):

    python tools/conv5_stamps.py rgb-d-instance-segmentation_amd/librgbd_hip_diag.so

Prints, per step, the cycles of each segment averaged over the loader waves (0-3) and the
compute waves (4-7): top -> weights issued -> first kx group (+ input issue) -> last MFMAs ->
wait + barrier, and the step period."""
import ctypes
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import _lib, init as winit, synthetic  # noqa: E402
from rgbd_amd.modules import EnhancedDepthImageRatioPredictor  # noqa: E402

h = ctypes.CDLL(os.path.join(_R, sys.argv[1]))
for name, (res, args) in _lib.SIGNATURES.items():
    if hasattr(h, name):
        fn = getattr(h, name)
        fn.restype, fn.argtypes = res, args
h.rgbd_debug_conv5_stamps.argtypes = [ctypes.c_void_p]
_lib._lib = h
m = EnhancedDepthImageRatioPredictor(3)
winit.init_deterministic(m, prefix="model.pixel_level_module.ratio_predictor.")
m.compute_dtype = torch.bfloat16
m = m.cuda().train()
planes, _, _ = synthetic.make_batch(3, 8, 480, 640)
d = torch.from_numpy(planes[:, 3:6].copy()).cuda()
for _ in range(5):
    m(d)
torch.cuda.synchronize()
buf = torch.zeros(2 * 12 * 8 * 5, dtype=torch.int64, device="cuda")
assert h.rgbd_debug_conv5_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
m(d)
torch.cuda.synchronize()
h.rgbd_debug_conv5_stamps(None)
s = buf.cpu().numpy().reshape(2, 12, 8, 5).astype(np.int64)
names = ["B issue", "kx0(+A)", "kx1-2", "wait+bar"]
for it in range(2):
    print(f"item {it}")
    for st in range(12):
        seg = np.diff(s[it, st], axis=1)  # [8 waves][4]
        per = (s[it, st + 1, :, 0] - s[it, st, :, 0]).mean() if st < 11 else float("nan")
        lo, hi = seg[:4].mean(0), seg[4:].mean(0)
        print(f"  st {st:2d} period {per:7.0f} | w0-3 " + " ".join(f"{n} {v:6.0f}" for n, v in zip(names, lo))
              + " | w4-7 " + " ".join(f"{v:6.0f}" for v in hi))
