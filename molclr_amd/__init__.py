"""molclr_amd — MI355X-native MolCLR contrastive pre-training hot path.

Drop-in counterparts of the reference modules (CameronDiao/MolCLR):

* ``molclr_amd.ginet_molclr.GINet``  <- models/ginet_molclr.py
* ``molclr_amd.gcn_molclr.GCN``      <- models/gcn_molclr.py
* ``molclr_amd.nt_xent.NTXentLoss``  <- utils/nt_xent.py
* ``molclr_amd.molclr.MolCLR``       <- molclr.py (trainer loop)

Every op runs on the HIP kernels of ``libmolclr_hip.so`` (C ABI:
include/molclr.h), built in-tree by ``python -m molclr_amd.build``.
"""
from .data import Batch, Data, DeviceGraph, collate_pairs, device_graph  # noqa: F401

__version__ = "0.1.0"


def lib():
    """The loaded C-ABI library (raises if it has not been built)."""
    from . import _lib
    return _lib.load()
