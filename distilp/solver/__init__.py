"""Alias of distilp_amd.solver (reference API: distilp.solver.halda_solve / HALDAResult)."""

from distilp_amd.solver import HALDAResult, ILPResult, halda_solve, halda_solve_batch  # noqa: F401

__all__ = ["halda_solve", "HALDAResult"]

__version__ = "0.1.2"
