"""Where k_dsam_lds's cycles go (diagnostic): runs the bench's eager train step (B = 8, 640x480,
bf16) with rgbd_debug_dsam_stamps set for one step, so every workgroup of the five DSAM conv
launches (forward dsam0 / dsam1 / dsam2, dX of dsam2 / dsam1) records s_memtime per work item
(the stamped instantiation of k_dsam_lds).  Per launch it prints the items and steps, the mean
cycles of each item segment:
  tables  item taken -> row table / step table / bias sums built (global code loads, one barrier)
  dma0    -> first ring stage landed
  step    -> K loop done, per step
  hand    -> multi-chunk hand-off (partials stored, ticket; the last chunk loads and sums)
  epi     -> epilogue done (LDS image, residual loads, bf16 stores)
and the workgroups' busy spans (first item taken -> last item done, per workgroup: the launch
is as long as the longest), against the MFMA floor of a step (KC * 12 MFMAs per wave, two waves
per SIMD, 16 cycles each)."""
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
# the stamped kernels live in the diagnostic build only (make -C rgb-d-instance-segmentation_amd/csrc diag)
os.environ.setdefault("RGBD_HIP_LIB", os.path.join(_R, "rgb-d-instance-segmentation_amd", "librgbd_hip_diag.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from rgbd_amd import _lib  # noqa: E402

args = bench.parse([])
ctx = bench.build(args, torch.device("cuda"))
step = bench.make_step(ctx, 1)
for _ in range(3):
    step()
torch.cuda.synchronize()
NL, NWG, NIT = 8, 256, 4
buf = torch.zeros(NL * NWG * NIT * 8, dtype=torch.int64, device="cuda")
L = _lib.lib()
assert L.rgbd_debug_dsam_stamps(buf.data_ptr(), NL) == 0
step()
torch.cuda.synchronize()
assert L.rgbd_debug_dsam_stamps(None, 0) == 0
s = buf.cpu().numpy().reshape(NL, NWG, NIT, 8).astype(np.int64)
names = ["fwd dsam0", "fwd dsam1", "fwd dsam2", "dX dsam2", "dX dsam1", "?", "?", "?"]
for li in range(NL):
    S = s[li]
    used = S[:, :, 0] != 0
    if not used.any():
        continue
    nst = S[:, :, 6] & 0xFFFF
    nch = (S[:, :, 6] >> 16) & 0xFF
    items = used.sum()
    seg = {"tables": S[:, :, 1] - S[:, :, 0], "dma0": S[:, :, 2] - S[:, :, 1], "loop": S[:, :, 3] - S[:, :, 2],
           "hand": S[:, :, 4] - S[:, :, 3]}
    has_epi = used & (S[:, :, 5] != 0)
    epi = np.where(S[:, :, 4] != 0, S[:, :, 5] - S[:, :, 4], S[:, :, 5] - S[:, :, 3])
    multi = used & (nch > 1)
    per_step = seg["loop"][used] / np.maximum(nst[used], 1)
    wg_items = used.sum(1)
    first = np.where(used[:, 0], S[:, 0, 0], 0)
    last = np.zeros(NWG, np.int64)
    for w in range(NWG):
        k = wg_items[w]
        if k:
            r = S[w, k - 1]
            last[w] = max(r[5], r[4], r[3])
    span = (last - first)[wg_items > 0]
    print(f"== launch {li} ({names[li]}): {items} items stamped on {(wg_items > 0).sum()} workgroups "
          f"(items per wg: {np.bincount(wg_items).tolist()}), steps per item mean {nst[used].mean():.1f} "
          f"min {nst[used].min()} max {nst[used].max()}, multi-chunk items {multi.sum()}")
    print(f"   tables {seg['tables'][used].mean():7.0f}  dma0 {seg['dma0'][used].mean():7.0f}  "
          f"step {per_step.mean():7.0f} (median {np.median(per_step):.0f})  "
          f"hand {seg['hand'][multi].mean() if multi.any() else 0:7.0f}  "
          f"epi {epi[has_epi].mean() if has_epi.any() else 0:7.0f}  cycles")
    print(f"   workgroup busy span: mean {span.mean():.0f} max {span.max():.0f} min {span.min():.0f} cycles; "
          f"items with epilogue {has_epi.sum()}")
    # the workgroups that set the launch's length: their items
    for w in np.argsort(-(last - first))[:3]:
        desc = []
        for k in range(wg_items[w]):
            r = S[w, k]
            v = int(r[7])
            desc.append(f"[cls {v & 3} tile {v >> 5} chunk {(v >> 2) & 7}/{(r[6] >> 16) & 0xFF} steps {r[6] & 0xFFFF}: "
                        f"t {r[1] - r[0]} d {r[2] - r[1]} loop {r[3] - r[2]} h {(r[4] - r[3]) if r[4] else 0} "
                        f"e {(r[5] - max(r[4], r[3])) if r[5] else 0} gap-before {r[0] - (max(S[w, k - 1][3:6]) if k else first[w])}]")
        print(f"   wg {w} span {last[w] - first[w]}: " + " ".join(desc))
