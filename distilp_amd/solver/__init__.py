"""Public solver API (reference: src/distilp/solver/__init__.py:5-13)."""

from .coefficients import HALDAResult, ILPResult
from .fleets import halda_solve_fleets  # noqa: F401
from .halda import halda_solve, halda_solve_batch  # noqa: F401

__all__ = ["halda_solve", "halda_solve_batch", "halda_solve_fleets", "HALDAResult", "ILPResult"]

__version__ = "0.1.2"  # the reference's solver module reports 0.1.2 (solver/__init__.py:13)
