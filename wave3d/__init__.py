"""``import wave3d`` from a source checkout: the framework package lives in
``3d-wave-equation-mpi-cuda_amd/`` (a directory name that is not a Python identifier).

This stub imports that directory as the package ``wave3d`` with the standard importlib
machinery (a file-location spec with its own ``submodule_search_locations``) and puts the real
module in ``sys.modules``, so ``wave3d.__spec__`` / ``__file__`` / ``__path__`` and every
submodule (``wave3d.models.wave`` ...) are ordinary package attributes — pickling and other
introspection see a normal package. An installed copy (``pip install .``, pyproject.toml maps
the same directory to ``wave3d``) does not need this stub.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_ROOT = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                      "3d-wave-equation-mpi-cuda_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_ROOT, "__init__.py"),
                                     submodule_search_locations=[_ROOT])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
