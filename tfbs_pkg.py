"""Import helper: the package directory is named `find-tfbs_amd` (not a Python
identifier), so it is loaded by path and registered as `find_tfbs_amd`."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "find-tfbs_amd")


def load():
    mod = sys.modules.get("find_tfbs_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location("find_tfbs_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["find_tfbs_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
