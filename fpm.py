"""Import shim: ``import fpm`` loads the package living in ``fingerprint-matching-code_amd/``.

The package directory name contains hyphens (it is fixed by the build layout), so it cannot be
imported by name.  This module replaces itself in ``sys.modules`` with that package.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fingerprint-matching-code_amd")
_spec = importlib.util.spec_from_file_location(
    "fpm", os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules["fpm"] = _mod
_spec.loader.exec_module(_mod)
