"""conv5's DMA cost isolated (diagnostic build): the bench-shape ratio predictor (train mode, bf16,
B = 8, 640x480) with rgbd_debug_conv5_mode 0 (the kernel), 3 (no in-loop copies), 7 (and no
per-step barrier: the waves run free), 15 (and constant MFMA operands instead of LDS fragment
reads) — modes other than 0 compute garbage and are for timing only — alternated over rounds; prints the median conv5 time per mode (HIP events of the library's
timing scope) and, per mode, the mean per-step cycles of workgroup 0's waves (stamps)."""
import ctypes
import os
import statistics
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
os.environ.setdefault("RGBD_HIP_LIB", os.path.join(_R, "rgb-d-instance-segmentation_amd", "librgbd_hip_diag.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import _lib, init as winit, synthetic  # noqa: E402
from rgbd_amd.modules import EnhancedDepthImageRatioPredictor  # noqa: E402

m = EnhancedDepthImageRatioPredictor(3)
winit.init_deterministic(m, prefix="model.pixel_level_module.ratio_predictor.")
m.compute_dtype = torch.bfloat16
m = m.cuda().train()
planes, _, _ = synthetic.make_batch(3, 8, 480, 640)
d = torch.from_numpy(planes[:, 3:6].copy()).cuda()
L = _lib.lib()
ROUNDS, ITERS = 6, 8
MODES = tuple(int(m) for m in sys.argv[1].split(",")) if len(sys.argv) > 1 else (0, 3, 7, 15)
res = {md: [] for md in MODES}
for rnd in range(ROUNDS + 1):
    for md in MODES:
        assert L.rgbd_debug_conv5_mode(md) == 0
        m(d)
        torch.cuda.synchronize()
        L.rgbd_timing_enable(1)
        for _ in range(ITERS):
            m(d)
        torch.cuda.synchronize()
        cnt = ctypes.c_int(0)
        ms = L.rgbd_timing_read(b"rp_conv3x3", ctypes.byref(cnt))
        L.rgbd_timing_enable(0)
        if rnd:
            res[md].append(ms / max(cnt.value, 1))
STEPS, WAVES = 18, 8
names = {0: "kernel", 1: "no B copies", 2: "no A copies", 3: "no copies", 7: "+ no barrier", 15: "+ no LDS reads"}
for md in MODES:
    assert L.rgbd_debug_conv5_mode(md) == 0
    buf = torch.zeros(2 * STEPS * WAVES * 5, dtype=torch.int64, device="cuda")
    assert L.rgbd_debug_conv5_stamps(buf.data_ptr()) == 0
    m(d)
    torch.cuda.synchronize()
    assert L.rgbd_debug_conv5_stamps(None) == 0
    s = buf.cpu().numpy().reshape(2, STEPS, WAVES, 5).astype(np.int64)
    per = (s[1, STEPS - 1, :, 4] - s[1, 0, :, 0]).mean() / (STEPS - 1)
    seg = np.diff(s[1], axis=2).mean(0)  # [wave][4]: dma, ks0, ks1, wait
    print(f"mode {md} ({names[md]:12s}): conv5 {statistics.median(res[md]):.4f} ms (min {min(res[md]):.4f}); "
          f"{per:7.1f} cycles/step; loaders dma/ks0/ks1/wait {np.round(seg[:4].mean(0)).astype(int).tolist()}, "
          f"compute {np.round(seg[4:].mean(0)).astype(int).tolist()}")
assert L.rgbd_debug_conv5_mode(0) == 0
