"""ffm_amd -- MI355X-native batched floor-field stepper (SoraKurihara/FFM hot path).

The product is the HIP library ``ffm_amd/_lib/libffm_amd.so`` (C ABI in
``include/ffm_amd.h``); ``ffm_amd.engine`` binds it and
``ffm_amd.model.ffm_core`` mirrors the reference's ``model/ffm_core.py``
class on top of it.
"""
from .data import make_room, l1_sff, free_cells  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    if name in ("Engine", "load_library"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
