"""Where the stem statistics' lag kernel spends its time (diagnostic): runs the bench-shape ratio
predictor (train mode, bf16, B = 8, 640x480) with rgbd_debug_stem_lag_stamps set, so every
workgroup and wave of k_stem_lag records s_memtime at entry, window staged, lag loop done, waves
joined, correlations written and plane sums written, and prints the mean / max cycles of each
segment, the kernel's span and how the workgroups' entry times spread over it."""
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
# the stamped kernel lives in the diagnostic build only (make -C rgb-d-instance-segmentation_amd/csrc diag)
os.environ.setdefault("RGBD_HIP_LIB", os.path.join(_R, "rgb-d-instance-segmentation_amd", "librgbd_hip_diag.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import _lib, init as winit, synthetic  # noqa: E402
from rgbd_amd.modules import EnhancedDepthImageRatioPredictor  # noqa: E402

B, H, W = 8, 480, 640
NWG = B * ((H + 31) // 32) * ((W + 255) // 256)
m = EnhancedDepthImageRatioPredictor(3)
winit.init_deterministic(m, prefix="model.pixel_level_module.ratio_predictor.")
m.compute_dtype = torch.bfloat16
m = m.cuda().train()
planes, _, _ = synthetic.make_batch(3, B, H, W)
d = torch.from_numpy(planes[:, 3:6].copy()).cuda()
for _ in range(3):
    m(d)
torch.cuda.synchronize()
buf = torch.zeros(NWG * 8 * 6, dtype=torch.int64, device="cuda")
L = _lib.lib()
for rep in range(2):
    buf.zero_()
    assert L.rgbd_debug_stem_lag_stamps(buf.data_ptr()) == 0
    m(d)
    torch.cuda.synchronize()
    assert L.rgbd_debug_stem_lag_stamps(None) == 0
    s = buf.cpu().numpy().reshape(NWG, 8, 6).astype(np.int64)
    assert (s > 0).all(), "some stamps were not written"
    seg = np.diff(s, axis=2)  # [wg][wave][5]
    names = ["stage", "lag loop", "join", "corr out", "plane sums"]
    print(f"rep {rep}: {NWG} workgroups x 8 waves, cycles per segment (s_memtime)")
    for i, n in enumerate(names):
        v = seg[:, :, i]
        print(f"  {n:11s} mean {v.mean():9.1f}  median {np.median(v):9.1f}  max {v.max():9.0f}")
    t0 = s[:, :, 0].min()
    ent = s[:, :, 0].min(1) - t0
    end = s[:, :, 5].max(1) - t0
    print(f"  span {end.max()} cycles; per-workgroup duration mean {np.mean(end - ent):.1f} max {np.max(end - ent)}")
    q = np.percentile(ent, [0, 25, 50, 75, 90, 100])
    print("  workgroup entry percentiles (0/25/50/75/90/100):", q.astype(int).tolist())
