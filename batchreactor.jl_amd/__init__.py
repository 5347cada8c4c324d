"""batchreactor.jl_amd -- MI355X-native (gfx950) engine for BatchReactor.jl's hot path.

Host mirror of the reference interface (Python here; the Julia ccall module is
julia/BatchReactorHIP.jl) over the C-ABI library libbrhip.so (include/brhip.h).
Load it as a package with ``_pkgload.load()`` (the directory name is not an identifier).
"""
from .mechanism import (CONV_DOC_COVG, CONV_FALLOFF_XM, CONV_KC_UNIT_SLIP, CONV_REFERENCE, CONV_TROE_C4,
                        Mechanism, MechanismError, read_batch_xml, read_chemkin, read_surface_xml, read_therm)
from .engine import Engine, STAT_FIELDS, integrate_multi
from .reactor import (Chemistry, ConstantParams, ODEProblem, UserDefinedState, batch_reactor, batch_reactor_ensemble,
                      batch_reactor_programmatic, compile_mechanism, julia_string)
from . import _lib

__all__ = ["Mechanism", "MechanismError", "Engine", "Chemistry", "ConstantParams", "ODEProblem", "UserDefinedState",
           "julia_string", "integrate_multi", "batch_reactor", "batch_reactor_ensemble",
           "batch_reactor_programmatic", "compile_mechanism", "read_batch_xml", "read_chemkin",
           "read_surface_xml", "read_therm", "STAT_FIELDS", "CONV_KC_UNIT_SLIP", "CONV_FALLOFF_XM",
           "CONV_DOC_COVG", "CONV_TROE_C4", "CONV_REFERENCE"]
