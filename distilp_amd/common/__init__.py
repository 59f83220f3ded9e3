"""Profile schemas: the solver's input contract (reference `src/distilp/common/__init__.py`)."""

from .types import ModelPhase, QuantizationLevel
from .device import DeviceProfile
from .model import ModelProfile, ModelProfilePhased, ModelProfileSplit

__all__ = [
    "DeviceProfile",
    "ModelProfile",
    "ModelProfilePhased",
    "ModelProfileSplit",
    "QuantizationLevel",
    "ModelPhase",
]
