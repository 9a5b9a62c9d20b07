"""adiabatic_raytracer_amd -- MI355X (gfx950) engine for the hot path of
SamWitte/Adiabatic_RayTracer: batched photon/axion segments around a neutron star
(RT.propagate), resonance crossings and their conversion probability (get_Prob_nonAD),
conversion-surface sampling and the binned flux, all on hand-written HIP kernels in
libart.so (include/art.h). `Engine` (device-resident torch tensors) is imported lazily."""
from ._lib import (ART_AXION, ART_PHOTON, ART_RK4, ART_VERN6, STATUS_NAMES, ArtError,  # noqa: F401
                   load as load_library)
from .raytracer import (Find_Conversion_Surface, Params, Propagated, func_axion, func_photon,  # noqa: F401
                        get_Prob_nonAD, params_from_mvars, propagate, propagate_batch, sample_conversion_points,
                        vern6_tableau)

__all__ = ["Params", "propagate", "propagate_batch", "get_Prob_nonAD", "Find_Conversion_Surface",
           "sample_conversion_points", "Engine", "func_photon", "func_axion"]


def __getattr__(name):
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name in ("trees", "scan", "shard", "engine"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
