"""f4 timing: the reference's post-processing (HF processor on the CPU, as predictor.py runs it)
vs rgbd_pp_instance on the GPU, B images of Q=100 queries, 48 classes, 120x160 mask logits,
target 480x640.  The GPU figure includes the host->device copy of the logits and the
device->host copy of the maps (the reference's inputs and outputs live on the host)."""
import argparse, os, sys, time, types
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R]
import numpy as np, torch
import _rgbd_import  # noqa: F401
from rgbd_amd.postprocess import post_process_instance_segmentation
from transformers.models.mask2former.image_processing_pil_mask2former import Mask2FormerImageProcessorPil
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
rng = np.random.default_rng(0)
B = a.batch
cl = torch.from_numpy(rng.standard_normal((B, 100, 49)).astype(np.float32) * 4)
ml = torch.from_numpy(rng.standard_normal((B, 100, 120, 160)).astype(np.float32) * 3)
outs = types.SimpleNamespace(class_queries_logits=cl, masks_queries_logits=ml)
ts = [(480, 640)] * B
proc = Mask2FormerImageProcessorPil()
post_process_instance_segmentation(outs, target_sizes=ts)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.iters):
    post_process_instance_segmentation(outs, target_sizes=ts)
torch.cuda.synchronize()
gpu = (time.perf_counter() - t) / a.iters
t = time.perf_counter()
proc.post_process_instance_segmentation(outs, target_sizes=ts)
cpu = time.perf_counter() - t
print(f"post_process_instance_segmentation B={B}: gpu {gpu * 1e3:.1f} ms ({B / gpu:.1f} img/s), "
      f"hf cpu {cpu * 1e3:.1f} ms ({B / cpu:.1f} img/s, {torch.get_num_threads()} threads)")
