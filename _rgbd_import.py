"""Import shim for the product package.

The package directory is named ``rgb-d-instance-segmentation_amd`` (the layout the
build contract asks for), which is not a valid Python identifier.  ``load()``
registers it in ``sys.modules`` as ``rgbd_amd`` so that ``import rgbd_amd.ops``
works everywhere (tests, bench.py, __graft_entry__.py).
"""
import importlib.util
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent / "rgb-d-instance-segmentation_amd"


def load():
    mod = sys.modules.get("rgbd_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "rgbd_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["rgbd_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


load()
