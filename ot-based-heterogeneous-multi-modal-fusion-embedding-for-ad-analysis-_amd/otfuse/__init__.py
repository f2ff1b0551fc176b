"""otfuse — MI355X-native (gfx950) Sinkhorn OT fusion path.

Drop-in for the OT alignment step of the reference MRI/PET fusion scripts:
``otfuse.pot`` mirrors the POT calls and ``get_feature_coupling_pot``,
``otfuse.perturbot`` mirrors the ``perturbot.match`` transport-plan API,
``otfuse.fusion`` is the device-resident OT block of the model's forward, and
``otfuse.ops`` exposes the HIP kernels (C ABI: include/otfuse.h) on torch tensors.
"""
from . import ops, synthetic  # noqa: F401
from ._lib import LIB_PATH, OtfError, lib  # noqa: F401

__version__ = "0.1.0"


def version() -> str:
    return lib().otf_version().decode()
