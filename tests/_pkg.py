"""Import the package directory ``quantized-gemm-for-transformer-inference_amd`` (not a Python
identifier) as module ``qgemm_amd``."""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "quantized-gemm-for-transformer-inference_amd")


def package(build: bool = False):
    mod = sys.modules.get("qgemm_amd")
    if mod is None:
        spec = importlib.util.spec_from_file_location(
            "qgemm_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
        mod = importlib.util.module_from_spec(spec)
        sys.modules["qgemm_amd"] = mod
        spec.loader.exec_module(mod)
    if build:
        # always the incremental make (a no-op when up to date), so a stale build/ is never tested as-is;
        # on a box without hipcc the shipped binary must then carry this tree's source hash
        if _have_hipcc():
            mod.build()
        mod.check_binary()
    return mod


def _have_hipcc():
    import shutil
    return shutil.which("hipcc") is not None or os.path.exists("/opt/rocm/bin/hipcc")
