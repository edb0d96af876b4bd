"""Import helper: the package directory is ``lidar-visual-odometry_amd/`` (not a valid Python
identifier), so it is loaded by path and registered as the module ``lvo_amd``."""
import importlib.util
import os
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(_REPO, "lidar-visual-odometry_amd")


def load():
    if "lvo_amd" in sys.modules:
        return sys.modules["lvo_amd"]
    spec = importlib.util.spec_from_file_location("lvo_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["lvo_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


lvo = load()
abi = lvo.abi
synth = lvo.synth
