"""On-device node-mask augmentation + collate (molclr_mask_views) vs the host.

    python tools/augment_bench.py [B] [reps]

Times both views of a B-molecule batch from a resident store of 16 B
molecules (HIP events around `reps` back-to-back calls of the two kernels'
launches, i.e. per batch pair), checks one pair against the oracle, and times
the host paths on the same molecules: the numpy restatement used by the
synthetic loader (mask_view + collate) and the reference's per-molecule loop
(oracle.augment_ref.reference_mask_view, dataset.py:117-131, without RDKit).
Prints one JSON line.
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from molclr_amd.augment import DeviceMoleculeStore  # noqa: E402
from molclr_amd.dataset import SyntheticPairBatches, collate_views, mask_view  # noqa: E402
from oracle.augment_ref import mask_views as oracle_views, reference_mask_view  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda", 0)
    mols = SyntheticPairBatches(B, seed=0).molecules(16 * B)
    store = DeviceMoleculeStore.from_molecules(mols, dev)
    rng = np.random.default_rng(1)
    ids = [rng.permutation(16 * B)[:B].astype(np.int64) for _ in range(16)]
    ids_d = [torch.from_numpy(v).to(dev) for v in ids]
    # parity on one pair
    host = store.host_store()
    bi, bj = store.mask_views(ids_d[0], 5, check=True, host_ids=ids[0])
    for b, v in ((bi, 0), (bj, 1)):
        r = oracle_views(host, ids[0], 5, v)
        assert np.array_equal(b.x.cpu().numpy(), r["x"])
        assert np.array_equal(b.edge_index.cpu().numpy(), r["edge_index"])
        assert np.array_equal(b.edge_attr.cpu().numpy(), r["edge_attr"])
    for i in range(10):
        store.mask_views(ids_d[i % 16], i, host_ids=ids[i % 16])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for i in range(reps):
        store.mask_views(ids_d[i % 16], i, host_ids=ids[i % 16])
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    gpu = e0.elapsed_time(e1) / reps * 1e-3
    N = int(bi.x.shape[0])
    E = int(bi.edge_index.shape[1])
    E_in = int(sum(2 * mols[i].num_bonds for i in ids[0]))
    # algorithmic bytes per view: read store x (16/atom) + directed edges
    # (16 index + 16 attr), write x (16) + batch (8) per atom and 32 per kept edge
    bytes_pair = 2 * (16 * N + 32 * E_in + 24 * N + 32 * E)

    # host: numpy restatement (the synthetic loader) and the reference loop
    vr = np.random.default_rng(2)
    sel = [mols[i] for i in ids[0]]
    t0 = time.perf_counter()
    collate_views([mask_view(m, vr) for m in sel])
    collate_views([mask_view(m, vr) for m in sel])
    host_np = time.perf_counter() - t0
    t0 = time.perf_counter()
    for m in sel:
        for _ in range(2):
            n, M = m.num_atoms, m.num_bonds
            mn = vr.choice(n, max(1, n // 4), replace=False).tolist()
            me = vr.choice(M, M // 4, replace=False).tolist() if M else []
            reference_mask_view(m.x.tolist(), m.edge_index.tolist(), m.edge_attr.tolist(), mn, me)
    host_ref = time.perf_counter() - t0
    print(json.dumps({
        "what": "node-mask augmentation + collate, both views of one batch",
        "batch": B, "atoms_per_view": N, "edges_in_per_view": E_in, "edges_out_per_view": E,
        "gpu_us_per_pair": round(gpu * 1e6, 2), "host_enqueue_us_per_pair": round(wall * 1e6, 2),
        "gpu_molecules_per_s": round(B / gpu), "algorithmic_bytes_per_pair": bytes_pair,
        "achieved_GBps": round(bytes_pair / gpu / 1e9, 1),
        "host_numpy_ms_per_pair": round(host_np * 1e3, 2),
        "host_numpy_molecules_per_s": round(B / host_np),
        "host_reference_loop_ms_per_pair": round(host_ref * 1e3, 2),
        "host_reference_loop_molecules_per_s": round(B / host_ref),
        "host_cores": 1,
    }))


if __name__ == "__main__":
    main()
