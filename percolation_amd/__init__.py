"""percolation_amd -- MI355X-native cluster labeling + Kirchhoff conductance.

Drop-in engine for the IsaiahSteinke/Percolation conductance path: the
Fortran drivers (percolation_amd/fortran/) and this Python mirror both call
libperc.so (include/perc.h), whose hot path is hand-written HIP for gfx950.
"""
from . import _lib
from ._lib import (DOT_FAST, DOT_LITERAL, DOT_LITERAL_HOST, FMT_AUTO, FMT_CSR, FMT_STENCIL, FMT_STENCIL_SPLIT,
                   FMT_STENCIL_TILED, MARCH_ALT, MARCH_DEFAULT, MARCH_QFREE, MARCH_SLOTS, MARCH_STRIPS,
                   MARCH_NIBBLE, MARCH_TAG, SOLVE_RESIDENT, PercError, lib)
from .api import (Context, bond_cond_grid, bond_list, bondc, nbonds, nearestn, pb_grid, site,
                  sitebond, shuffled_ids, trial_seeds)

__all__ = ["DOT_FAST", "DOT_LITERAL", "DOT_LITERAL_HOST", "FMT_AUTO", "FMT_CSR", "FMT_STENCIL", "FMT_STENCIL_SPLIT",
           "FMT_STENCIL_TILED", "MARCH_ALT", "MARCH_DEFAULT", "MARCH_QFREE", "MARCH_SLOTS", "MARCH_STRIPS",
           "MARCH_NIBBLE", "MARCH_TAG", "SOLVE_RESIDENT", "Context", "PercError", "bond_list", "bondc", "lib", "nbonds", "nearestn", "pb_grid",
           "site", "sitebond", "shuffled_ids", "trial_seeds", "bond_cond_grid"]
