"""The whole drop-in model's training step captured into one HIP graph (bench.full_model: the
number the bench line's full_model block reports as img_s): the capture must succeed after an
eager warm-up step — every per-batch device vector of the matcher / loss (ops.device_vec) is in
device_const's cache by then, so the capture makes no host copy — and replay with a finite loss.
(A regression here makes full_model fall back to the eager step silently: its graph_error.)"""
import math
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


@pytest.mark.timeout(300)
def test_full_model_step_captures():
    sys.path.insert(0, str(REPO))
    import bench
    res = bench.full_model(torch.device("cuda", 0), B=2, H=240, W=320, steps=1, warmup=1)
    assert "graph_error" not in res, res.get("graph_error")
    assert res["timed"] == "captured graph" and res["graph_branches"] <= 2
    assert math.isfinite(res["graph_loss"]) and math.isfinite(res["loss"])
