"""Golden fixture (3) of SURVEY.md §8(c): the reference's shipped GCN
checkpoint pushed through the oracle.

Run in the build container (where /root/reference exists):

    python tests/golden/make_gcn_pretrained.py

* reads ``ckpt/pretrained_gcn/checkpoints/model.pth`` -- trained weights for
  models/gcn_molclr.py:94-158 (GCN 5 x 300, feat_dim 512) -- with the
  non-executing loader ``torch.load(weights_only=True)``;
* builds a fixed 16-molecule batch (molclr_amd's synthetic molecule
  generator, SURVEY §8(d) distribution, node-masked view as in
  dataset/dataset.py:111-145) and stores its PyG fields;
* evaluates ``oracle.reference_cpu.RefGCN`` in float64, eval mode (running
  BatchNorm statistics of the checkpoint) and stores ``h`` [16, 512] and
  ``out`` [16, 256].

Output: ``gcn_pretrained_b16.npz`` (the state dict as float32 arrays under
``w/<key>``, the batch, and the fp64 outputs), about 4 MB.  The fixture is
data: the checkpoint's tensors and the oracle's outputs.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
REF_CKPT = Path("/root/reference/ckpt/pretrained_gcn/checkpoints/model.pth")
OUT = Path(__file__).resolve().parent / "gcn_pretrained_b16.npz"


def main():
    from molclr_amd.dataset import SyntheticPairBatches
    from oracle.reference_cpu import RefGCN
    sd = torch.load(REF_CKPT, map_location="cpu", weights_only=True)
    xi, _ = SyntheticPairBatches(16, seed=2024).next()
    ref = RefGCN(5, 300, 512).double()
    ref.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()})
    ref.eval()
    with torch.no_grad():
        h, out = ref(xi)
    arrays = {f"w/{k}": v.numpy() for k, v in sd.items()}
    arrays.update(x=xi.x.numpy(), edge_index=xi.edge_index.numpy(),
                  edge_attr=xi.edge_attr.numpy(), batch=xi.batch.numpy(),
                  h=h.numpy(), out=out.numpy())
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT} ({OUT.stat().st_size / 1e6:.1f} MB): atoms {xi.x.shape[0]}, "
          f"edges {xi.edge_index.shape[1]}, |h| {h.norm():.4f}, |out| {out.norm():.4f}")


if __name__ == "__main__":
    main()
