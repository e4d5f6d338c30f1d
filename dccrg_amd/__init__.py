"""dccrg_amd — MI355X-native neighbor-stencil + remote-neighbor halo path of
dccrg (distributed cartesian cell-refinable grid).

The compute path is the HIP/RCCL library ``libdccrgx.so`` (C ABI:
include/dccrgx.h); this package is the Python mirror of the reference's
``dccrg::Dccrg`` host interface on top of it.
"""
from ._lib import DccrgError, header_symbols, lib  # noqa: F401
from .grid import Dccrg, Field, VariableField  # noqa: F401
from .poisson import Poisson_Solve  # noqa: F401

__all__ = ["Dccrg", "Field", "VariableField", "Poisson_Solve", "DccrgError", "lib", "header_symbols"]
