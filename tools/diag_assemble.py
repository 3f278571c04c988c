import sys, numpy as np, torch
sys.path[:0] = ['.', 'tests/golden']
import _rgbd_import
from rgbd_amd import ops, synthetic
from oracle import dggm_pre
H, W = 64, 96
s = synthetic.make_scene(5000 + 17 * H, H, W)
pv = ops.assemble_pixel_values(torch.from_numpy(s["depth_u8"][None]).cuda(), torch.from_numpy(s["rgb_u8"][None]).cuda()).cpu().numpy()[0]
ref = np.concatenate([synthetic.rgbd_planes(s), dggm_pre.dggm_planes(s["depth_u8"])])
for c in range(10):
    d = pv[c].view(np.uint32).astype(np.int64) - ref[c].view(np.uint32).astype(np.int64)
    print(c, int((d != 0).sum()), int(np.abs(d).max()))
c = int(np.argmax([(pv[c] != ref[c]).sum() for c in range(10)]))
idx = np.argwhere(pv[c] != ref[c])[:3]
for y, x in idx:
    print(c, y, x, repr(pv[c, y, x]), repr(ref[c, y, x]), s["rgb_u8"][y, x], s["depth_u8"][y, x])
# GPU elementwise torch for comparison
v = torch.arange(256, dtype=torch.float32).cuda()
g = ((v * np.float32(1/255)) - 0.485) / 0.229
n = ((np.arange(256, dtype=np.float32) * np.float32(1/255)) - np.float32(0.485)) / np.float32(0.229)
print("torch-gpu vs numpy mismatches:", int((g.cpu().numpy() != n).sum()))
