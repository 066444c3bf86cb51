"""nfdpf -- MI355X (gfx950) hot path of normalizing-flow differentiable particle filters.

Host side of libnfdpf.so: ctypes binding (``_lib``), parameter packing (``pack``), torch
wrappers of each C-ABI entry point (``ops``) and the filtering driver (``engine``).  The
reference-compatible modules (``DPFs``, ``nf``, ``model``, ``resamplers``, ``utils``,
``losses``, ``arguments``, ``dataset``) sit next to this package and call into it.
"""
from ._lib import NfdpfError, load  # noqa: F401
