"""The ratio predictor's train-mode forward at the bench shape, --iters times (for a kernel trace:
run it under rocprofv3 --kernel-trace --stats, once per library build via RGBD_HIP_LIB).

    RGBD_HIP_LIB=$PWD/rgb-d-instance-segmentation_amd/gpurun_ab_old.so \\
        rocprofv3 --kernel-trace --stats -d gpurun_out/p_old -- python tools/prof_ratio.py
"""
import argparse
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
import torch  # noqa: E402

import _rgbd_import  # noqa: E402,F401
from rgbd_amd import init as winit, synthetic  # noqa: E402
from rgbd_amd.modules import EnhancedDepthImageRatioPredictor  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=30)
a = ap.parse_args()

m = EnhancedDepthImageRatioPredictor(3)
winit.init_deterministic(m, prefix="model.pixel_level_module.ratio_predictor.")
m.compute_dtype = torch.bfloat16
m = m.cuda().train()
planes, _, _ = synthetic.make_batch(3, 8, 480, 640)
d = torch.from_numpy(planes[:, 3:6].copy()).cuda()
for _ in range(a.iters):
    m(d)
torch.cuda.synchronize()
print("done", a.iters, os.environ.get("RGBD_HIP_LIB", "in-tree"))
