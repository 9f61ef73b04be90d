"""Import shim for the product package.

The package directory is ``stable-diffusion-from-scratch_amd/`` (not a valid
Python identifier), so it is registered under the importable name ``sd_amd``.
``load()`` is idempotent; after it, ``import sd_amd`` and YAML targets such as
``sd_amd.openai_model.model.UNetModel`` resolve normally.
"""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stable-diffusion-from-scratch_amd")
NAME = "sd_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
