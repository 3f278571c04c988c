"""k_dsam_lds's step cost decomposed (diagnostic build): the bench's eager train step (B = 8,
640x480, bf16) with the five DSAM conv launches (forward dsam0 / dsam1 / dsam2, dX of dsam2 /
dsam1) run as the stamped kernel under rgbd_debug_dsam_mode 0 (the kernel), 1 (no in-loop weight
copies), 2 (no in-loop input copies), 3 (no copies), 7 (and no per-step barrier), 8 (no fragment
reads, copies kept), 15 (none of them: the MFMA stream and the loop's bookkeeping), 32 / 64 / 96
(the weight / input / both copies kept but sourced from one L2-resident block) — modes other
than 0 compute garbage and are for timing only (their ring starts zeroed, so values stay finite).
Modes alternate over rounds; per mode and launch it prints the median over rounds of the mean
cycles per K step and of the longest workgroup span (the launch's length)."""
import os
import statistics
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests/golden")]
os.environ.setdefault("RGBD_HIP_LIB", os.path.join(_R, "rgb-d-instance-segmentation_amd", "librgbd_hip_diag.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from rgbd_amd import _lib  # noqa: E402

MODES = tuple(int(m) for m in sys.argv[1].split(",")) if len(sys.argv) > 1 else (0, 1, 2, 3, 7, 8, 15)
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
args = bench.parse([])
ctx = bench.build(args, torch.device("cuda"))
step = bench.make_step(ctx, 1)
for _ in range(3):
    step()
torch.cuda.synchronize()
NL, NWG, NIT = 5, 256, 4
L = _lib.lib()
names = ["fwd dsam0", "fwd dsam1", "fwd dsam2", "dX dsam2", "dX dsam1"]
per = {m: [[] for _ in range(NL)] for m in MODES}
span = {m: [[] for _ in range(NL)] for m in MODES}
for rnd in range(ROUNDS):
    for md in MODES:
        buf = torch.zeros(NL * NWG * NIT * 8, dtype=torch.int64, device="cuda")
        assert L.rgbd_debug_dsam_mode(md) == 0
        assert L.rgbd_debug_dsam_stamps(buf.data_ptr(), NL) == 0
        step()
        torch.cuda.synchronize()
        assert L.rgbd_debug_dsam_stamps(None, 0) == 0
        assert L.rgbd_debug_dsam_mode(0) == 0
        s = buf.cpu().numpy().reshape(NL, NWG, NIT, 8).astype(np.int64)
        for li in range(NL):
            S = s[li]
            used = S[:, :, 0] != 0
            if not used.any():
                continue
            nst = S[:, :, 6] & 0xFFFF
            loop = S[:, :, 3] - S[:, :, 2]
            per[md][li].append(float((loop[used] / np.maximum(nst[used], 1)).mean()))
            wg_items = used.sum(1)
            lens = []
            for w in range(NWG):
                k = wg_items[w]
                if k:
                    r = S[w, k - 1]
                    lens.append(max(r[5], r[4], r[3]) - S[w, 0, 0])
            span[md][li].append(float(max(lens)))
mname = {0: "kernel", 1: "no B copies", 2: "no A copies", 3: "no copies", 7: "+ no barrier", 8: "no frag reads",
         15: "MFMAs only", 32: "B L2-resident", 64: "A L2-resident", 96: "A, B L2-resident"}
print("cycles per K step (mean over items) / longest workgroup span (K cycles); median of", ROUNDS, "rounds")
print(f"{'mode':22s}" + "".join(f"{n:>22s}" for n in names) + f"{'sum of spans':>14s}")
for md in MODES:
    row, tot = [], 0.0
    for li in range(NL):
        if per[md][li]:
            p, sp = statistics.median(per[md][li]), statistics.median(span[md][li])
            tot += sp
            row.append(f"{p:9.0f} / {sp / 1000:7.1f}K")
        else:
            row.append(f"{'-':>22s}")
    print(f"{md:2d} {mname.get(md, '?'):19s}" + "".join(f"{c:>22s}" for c in row) + f"{tot / 1000:12.1f}K")
