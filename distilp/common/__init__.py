"""Alias of distilp_amd.common (reference: distilp.common schemas)."""

from distilp_amd.common import (  # noqa: F401
    DeviceProfile,
    ModelPhase,
    ModelProfile,
    ModelProfilePhased,
    ModelProfileSplit,
    QuantizationLevel,
)

__all__ = ["DeviceProfile", "ModelProfile", "ModelProfilePhased", "ModelProfileSplit", "QuantizationLevel",
           "ModelPhase"]
