"""Import helper for the ``craniofacialsd-vae_amd/`` package directory.

The directory name carries a hyphen (the layout the build contract asks
for), which Python's import statement cannot spell, so it is registered in
``sys.modules`` as ``craniofacialsd_vae_amd``; afterwards ordinary
``from craniofacialsd_vae_amd import engine`` imports work.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "craniofacialsd-vae_amd")
NAME = "craniofacialsd_vae_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
