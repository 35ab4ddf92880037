"""ORACLE — test infrastructure only.

CPU restatement of the CameronDiao/MolCLR pre-training path used as the parity
checker for the HIP kernels.  Only ``tests/``, ``__graft_entry__.smoke()`` and
the ``cpu_baseline`` leg of ``bench.py`` may import it; the product package
``molclr_amd`` never does (it has no CPU path at all).
"""
