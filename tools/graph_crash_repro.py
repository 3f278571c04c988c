"""Round-2 graph hazard, reproduced under a native SIGSEGV reporter: the hot path's
side-stream forks switched to the structure that crashed hipGraphLaunch (``twoside``: forks
alternate between two side streams; ``dupfork``: every fork issued twice from one point), then the
GPU tests that exposed it run in one process (parity tests first, the graph tests after).  A crash
prints the native frames (tools/native/segv_bt.so) before the process dies.

    python tools/graph_crash_repro.py twoside tests/test_gpu_parity.py tests/test_gpu_train_graph.py
"""
import ctypes
import os
import sys

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tools")]
bt = ctypes.CDLL(os.path.join(_R, "tools/native/segv_bt.so"))
import pytest  # noqa: E402

import graph_topology  # noqa: E402


class _Mode:
    def __init__(self, mode):
        self.mode = mode

    def pytest_sessionstart(self, session):
        graph_topology.set_mode(self.mode)
        assert bt.rgbd_segv_install() == 0  # after pytest's faulthandler: ours reports first


if __name__ == "__main__":
    mode, files = sys.argv[1], sys.argv[2:]
    sys.exit(pytest.main(["-m", "gpu", "-q", "-x", "-s", "-p", "no:cacheprovider", "-p", "no:faulthandler",
                          "--timeout", "300", "--timeout-method", "thread"] + files, plugins=[_Mode(mode)]))
