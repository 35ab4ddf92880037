"""``aug: mix`` data module: the counterpart of dataset/dataset_mix.py.

main() imports ``MoleculeDatasetWrapper`` from the module that
``config['aug']`` names (molclr.py:184-191).  This one is
molclr_amd.dataset's wrapper with ``aug='mix'``: the subgraph-removal plus
atom / bond masking views (dataset/dataset_mix.py:86-217) are built on the
GPU from the resident molecules, which are featurised with explicit
hydrogens (``Chem.AddHs``, dataset_mix.py:87-88).
"""
from __future__ import annotations

from .dataset import MoleculeDatasetWrapper as _Wrapper
from .shards import read_smiles  # noqa: F401

__all__ = ["MoleculeDatasetWrapper", "read_smiles"]


class MoleculeDatasetWrapper(_Wrapper):
    def __init__(self, batch_size, num_workers, valid_size, data_path, **kwargs):
        kwargs.setdefault("aug", "mix")
        if kwargs["aug"] != "mix":
            raise ValueError("this module builds aug=mix views")
        super().__init__(batch_size, num_workers, valid_size, data_path, **kwargs)
