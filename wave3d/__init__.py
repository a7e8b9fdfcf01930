"""Import shim: ``import wave3d`` loads the framework package that lives in
``3d-wave-equation-mpi-cuda_amd/`` (a directory name that is not a Python identifier).

The shim re-points this package's ``__path__`` at that directory and executes its
``__init__``, so ``wave3d.models``, ``wave3d.ops``, ``wave3d.parallel`` and
``wave3d.utils`` resolve to the real subpackages.
"""
import os as _os

_ROOT = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                      "3d-wave-equation-mpi-cuda_amd")
__path__ = [_ROOT]
__file__ = _os.path.join(_ROOT, "__init__.py")
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, "exec"))
