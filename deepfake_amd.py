"""Import alias for the package directory ``deepfake-video-detection_amd/``.

The directory name carries hyphens (it is the repository's required layout) and
therefore cannot be named in an ``import`` statement.  Importing this module
loads that directory as the package ``deepfake_amd`` and replaces this module in
``sys.modules``, so ``import deepfake_amd`` / ``from deepfake_amd.x import y``
work from the repository root.
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "deepfake-video-detection_amd")
_spec = importlib.util.spec_from_file_location(
    "deepfake_amd", os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR]
)
_mod = importlib.util.module_from_spec(_spec)
sys.modules["deepfake_amd"] = _mod
_spec.loader.exec_module(_mod)
