"""Where the bf16 chain kernels' cycles go per tile (diagnostic): runs the bench-shape ratio
predictor (train mode, B = 8, 640x480) with rgbd_debug_chain_stamps set; workgroup 0 of phase 0
(stem statistics) and phase 1 (stem + fusion, statistics, raw fusion store) records s_memtime per
wave for its first four tiles.  Prints the mean cycles per segment:
  bar1+stage  tile top -> patch staged in LDS (two barriers)
  fetch       -> next tile's patch loads issued
  stem        -> stem MFMAs issued (phase 0: statistics done)
  pack        -> ReLU + bf16 fragments of the stem output
  fusion      -> fusion MFMAs issued
  tail        -> statistics + raw fusion store (tile end)
and the tile-to-tile period against the MFMA floor."""
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
buf = torch.zeros(2 * 4 * 8 * 7, dtype=torch.int64, device="cuda")
L = _lib.lib()
assert L.rgbd_debug_chain_stamps(buf.data_ptr()) == 0
m(d)
torch.cuda.synchronize()
assert L.rgbd_debug_chain_stamps(None) == 0
s = buf.cpu().numpy().reshape(2, 4, 8, 7).astype(np.int64)
for ph, names in ((0, ["bar1+stage", "fetch", "stem+stats"]),
                  (1, ["bar1+stage", "fetch", "stem", "pack", "fusion", "tail"])):
    segs = []
    for t in range(4):
        for w in range(8):
            v = s[ph, t, w]
            segs.append([v[i + 1] - v[i] for i in range(len(names))])
    mean = np.mean(segs, 0)
    period = np.mean([s[ph, t + 1, w, 0] - s[ph, t, w, 0] for t in range(3) for w in range(8)])
    mf = 120 * 16 * 2 if ph == 0 else 156 * 16 * 2
    print(f"phase {ph}: " + "  ".join(f"{n} {x:7.1f}" for n, x in zip(names, mean))
          + f"  | tile period {period:7.1f} cycles (MFMA floor per SIMD, 2 waves: {mf})")
