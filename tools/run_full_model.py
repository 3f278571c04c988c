"""bench.py's full_model block alone (eager and captured whole-model step), one JSON line."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    graph = "--no-graph" not in sys.argv
    print(json.dumps(bench.full_model(torch.device("cuda"), graph=graph)))
