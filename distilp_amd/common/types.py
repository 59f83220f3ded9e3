"""Literal aliases shared by the profile schemas.

Mirrors `src/distilp/common/types.py:3-4` of the reference, written as plain
`typing.Literal` aliases so the package imports on Python 3.10 (the reference
uses PEP 695 `type X = ...`, which needs 3.12).
"""

from typing import Literal

ModelPhase = Literal["merged", "prefill", "decode"]
QuantizationLevel = Literal["Q4_K", "Q5_K", "Q6_K", "Q8_0", "BF16", "F16", "F32"]

__all__ = ["ModelPhase", "QuantizationLevel"]
