"""The C-ABI library builds, loads and exports every symbol include/molclr.h
declares (no compute calls: argument validation returns before any HIP call)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "molclr.h"


def declared_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(molclr_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from molclr_amd import _lib
    from molclr_amd.build import build
    build()
    return _lib.load()


def test_header_declares_the_path():
    syms = declared_symbols()
    for s in ("molclr_graph_build", "molclr_gine_aggregate_fwd", "molclr_gine_aggregate_bwd",
              "molclr_gemm_f32", "molclr_ntxent_fwd", "molclr_ntxent_bwd", "molclr_adam_step"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_signatures_cover_header():
    from molclr_amd._lib import SIGNATURES
    assert sorted(SIGNATURES) == declared_symbols()


def test_version_and_error_plumbing(lib):
    assert b"gfx950" in lib.molclr_version()
    # bad epilogue -> MOLCLR_ERR_ARG before any device work
    rc = lib.molclr_gemm_f32(None, None, None, 4, 4, 4, 4, 4, 4, 0, 0, 99, None, None, 0, None, 0, None)
    assert rc == -1
    assert b"epilogue" in lib.molclr_last_error()
    rc = lib.molclr_gine_aggregate_fwd(None, None, None, None, None, None, None, 10, 301, None)
    assert rc == -1 and b"multiple of 4" in lib.molclr_last_error()
    rc = lib.molclr_edge_tables_combine(17, None, None, None, 300, None)
    assert rc == -1 and b"layers" in lib.molclr_last_error()
    rc = lib.molclr_graph_build(None, None, None, (1 << 24) + 1, 0, 1, None, None, None, None, None,
                                None, None, None, None, None, None, 0, None)
    assert rc == -1 and b"neighbour-slot" in lib.molclr_last_error()


def test_workspace_queries(lib):
    assert lib.molclr_graph_build_workspace_bytes(100, 300) >= 300 * 4 * 4
    assert lib.molclr_gemm_f32_workspace_bytes(300, 600, 15000) > 0   # split-K weight gradient
    assert lib.molclr_gemm_f32_workspace_bytes(15000, 600, 300) == 0  # no split needed
    assert lib.molclr_ntxent_workspace_bytes(1024, 1024, 256) > 0


def test_product_path_has_no_cpu_fallback():
    """The product package never imports the oracle."""
    for p in (ROOT / "molclr_amd").rglob("*.py"):
        assert "oracle" not in re.sub(r'""".*?"""', "", p.read_text(), flags=re.S).replace(
            "# oracle", ""), p


def test_torch_ops_registered():
    """import molclr_amd.torch_ops registers the operator seam
    in the torch.ops.molclr namespace (no device needed to register)."""
    import torch

    import molclr_amd.torch_ops as tops
    for name in tops.OPS:
        assert hasattr(torch.ops.molclr, name), name
    schema = str(torch.ops.molclr.gine_aggregate.default._schema)
    assert schema.startswith("molclr::gine_aggregate(Tensor h, Tensor E1, Tensor E2")
