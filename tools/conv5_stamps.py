"""Where conv5's cycles go per K step (diagnostic): runs the bench-shape ratio predictor (train
mode, B = 8, 640x480) with rgbd_debug_conv5_stamps set, so workgroup 0 of the conv5 launch records
s_memtime per wave and step of its first two tiles (the stamped instantiation of
k_rp_conv3x3_v3), and prints the mean cycles of each segment:
  dma    step top (after the barrier) -> DMA pieces issued
  ks0    -> k-step 0's 32 MFMAs issued (includes waiting for its fragments)
  ks1    -> k-step 1's 32 MFMAs issued
  wait   -> the closing s_waitcnt (own DMA landed, own LDS reads done)
  bar    -> the next step's top (the barrier)
for waves 0-3 (channel half 0, priority 0) and 4-7 (channel half 1, priority 1)."""
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
# the stamped kernels live in the diagnostic build only (make -C rgb-d-instance-segmentation_amd/csrc diag)
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
for _ in range(3):
    m(d)
torch.cuda.synchronize()
STEPS, WAVES = 18, 8
buf = torch.zeros(2 * STEPS * WAVES * 5, dtype=torch.int64, device="cuda")
L = _lib.lib()
assert L.rgbd_debug_conv5_stamps(buf.data_ptr()) == 0
m(d)
torch.cuda.synchronize()
assert L.rgbd_debug_conv5_stamps(None) == 0
s = buf.cpu().numpy().reshape(2, STEPS, WAVES, 5).astype(np.int64)
names = ["dma", "ks0", "ks1", "wait", "bar"]
for half, waves in (("waves 0-3", slice(0, 4)), ("waves 4-7", slice(4, 8))):
    seg = np.zeros((2, STEPS - 1, 4, 5))
    for t in range(2):
        for st in range(STEPS - 1):
            for wi, w in enumerate(range(WAVES)[waves]):
                v = s[t, st, w]
                nxt = s[t, st + 1, w, 0]
                seg[t, st, wi] = [v[1] - v[0], v[2] - v[1], v[3] - v[2], v[4] - v[3], nxt - v[4]]
    mean = seg.reshape(-1, 5).mean(0)
    print(f"{half}: " + "  ".join(f"{n} {x:7.1f}" for n, x in zip(names, mean)) + f"  | step {mean.sum():7.1f} cycles")
tot = (s[1, STEPS - 1, :, 4] - s[1, 0, :, 0]).mean() / (STEPS - 1)
print(f"tile 1, steps 0-17: {tot:.1f} cycles per step (mean over waves); MFMA floor per SIMD 2048")
per_step = np.diff(s[1, :, 0, 0])
print("wave 0 step-top deltas, tile 1:", per_step.tolist())
