"""shud_rhs — host-side mirror of the SHUD RHS plugin surface (DankerMu/SHUD-up src/Model/f.cpp).

The compute path is the HIP library ../libshud_rhs.so (C-ABI: include/shud_rhs.h).  This package only
loads it (runtime.py), prepares SoA inputs (model.py, shudio.py, synth.py) and partitions meshes for
multi-GPU runs (partition.py).  There is no CPU fallback: importing runtime without the built library
raises.
"""
from . import abi  # noqa: F401
from .model import ShudModel  # noqa: F401
