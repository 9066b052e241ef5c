"""Import alias for the framework package.

The package directory is named
``performance-comparison-of-tensorflow-pytorch-and-their-distributed-counterparts_amd`` (the
project layout the build plan asks for), which is not a valid Python identifier.  Importing
``pcmp`` loads that directory as a regular package named ``pcmp`` so that
``import pcmp.models`` / ``from pcmp.ops import conv2d`` work everywhere (tests, entry points,
``bench.py``).  The module replaces itself in ``sys.modules`` with the real package object.
"""
import importlib.util
import pathlib
import sys

PKG_DIR = (pathlib.Path(__file__).resolve().parent
           / "performance-comparison-of-tensorflow-pytorch-and-their-distributed-counterparts_amd")

_spec = importlib.util.spec_from_file_location(
    __name__, PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
