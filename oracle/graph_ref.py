"""ORACLE — test infrastructure only (see oracle/__init__.py).

numpy restatement of the integer work on the path, for bit-exact checks of
``molclr_graph_build`` (graph.hip):

* the destination CSR is the order in which the reference's scatter-add
  accumulates messages: PyG's ``add_self_loops`` appends the loops after the
  real edges (models/ginet_molclr.py:31) and torch_scatter's CPU
  ``scatter_add_`` walks edges in index order, so inside a destination row the
  real in-edges come in edge order and the self loop last — a STABLE sort of
  edge ids by destination;
* the source CSC is the same for index_select's backward (``index_add_`` in
  edge order, keyed by source);
* bond-type / bond-dir counts per destination include the self loop
  (edge attr [4, 0], ginet_molclr.py:34-37);
* graph offsets are the ``ptr`` of PyG's collate (nodes of graph g are
  contiguous, batch ascending);
* the neighbour slots (``nbr`` / ``nbr_t``, a layout of this build, see
  include/molclr.h) restate the first 4 entries of every CSR / CSC row packed
  with the combined edge-table index ``bt * 3 + bd`` and the row degree.
"""
from __future__ import annotations

import numpy as np


def graph_build(edge_index: np.ndarray, edge_attr: np.ndarray, batch: np.ndarray,
                num_nodes: int, num_graphs: int) -> dict:
    ei = np.asarray(edge_index, dtype=np.int64)
    ea = np.asarray(edge_attr, dtype=np.int64)
    N = int(num_nodes)
    src, dst = ei[0], ei[1]
    perm = np.argsort(dst, kind="stable")
    indeg = np.bincount(dst, minlength=N)
    rowptr = np.concatenate([[0], np.cumsum(indeg)]).astype(np.int32)
    col = src[perm].astype(np.int32)
    ecode = (ea[perm, 0] | (ea[perm, 1] << 3)).astype(np.uint8)
    perm_t = np.argsort(src, kind="stable")
    outdeg = np.bincount(src, minlength=N)
    rowptr_t = np.concatenate([[0], np.cumsum(outdeg)]).astype(np.int32)
    col_t = dst[perm_t].astype(np.int32)
    ecount = np.zeros((N, 8), dtype=np.int32)
    np.add.at(ecount, (dst, ea[:, 0]), 1)
    np.add.at(ecount, (dst, 5 + ea[:, 1]), 1)
    ecount[:, 4] += 1  # self loop: bond type 4
    ecount[:, 5] += 1  # self loop: bond dir 0
    b = np.asarray(batch, dtype=np.int64)
    graph_ptr = np.searchsorted(b, np.arange(num_graphs + 1), side="left").astype(np.int32)
    graph_ptr[num_graphs] = N
    ecomb = (ecode & 7).astype(np.uint32) * 3 + (ecode >> 3).astype(np.uint32)
    nbr = neighbour_slots(rowptr, col.astype(np.uint32) | (ecomb << 24))
    nbr_t = neighbour_slots(rowptr_t, col_t.astype(np.uint32))
    return dict(rowptr=rowptr, col=col, ecode=ecode, rowptr_t=rowptr_t, col_t=col_t,
                nbr=nbr, nbr_t=nbr_t, ecount=ecount.reshape(-1), graph_ptr=graph_ptr)


SLOTS, OVERFLOW = 4, 7


def neighbour_slots(rowptr: np.ndarray, packed: np.ndarray) -> np.ndarray:
    """[N*4] u32 view as int32: row i's first 4 packed entries, degree (or 7
    when > 4) in bits 29..31 of word 0."""
    N = len(rowptr) - 1
    out = np.zeros((N, SLOTS), dtype=np.uint32)
    deg = np.diff(rowptr)
    for s in range(SLOTS):
        rows = np.nonzero(deg > s)[0]
        out[rows, s] = packed[rowptr[rows] + s]
    out[:, 0] |= np.where(deg > SLOTS, OVERFLOW, deg).astype(np.uint32) << 29
    return out.reshape(-1).view(np.int32)
