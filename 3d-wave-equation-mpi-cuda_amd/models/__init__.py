"""Problem definitions ("model family" of this framework) and the solver front-end."""
from .wave import WaveProblem, WaveSolver, RunResult, PI_REF, CFL_LIMIT  # noqa: F401
from . import presets  # noqa: F401
