"""Generate the committed golden fixtures from the reference itself.

Run in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

* ``ntxent_*.npz`` — the reference's OWN ``utils/nt_xent.py`` (imported from
  /root/reference by file path; it needs only torch and numpy) evaluated on
  seeded inputs: loss and the gradients w.r.t. ``zis`` / ``zjs`` from
  ``loss.backward()``.  These pin ``oracle.reference_cpu.RefNTXentLoss`` and,
  through it, the HIP NT-Xent kernels.
* ``pretrained_gcn_manifest.json`` — key -> shape of the shipped
  ``ckpt/pretrained_gcn/checkpoints/model.pth`` (loaded with
  ``torch.load(weights_only=True)``), plus checksums of a few tensors; pins
  the GCN ``state_dict`` contract.

The reference's encoders (models/*.py) import torch_geometric, which is not
installed and is not shimmed; they are not executed here.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import sys
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent

# (name, B, C, temperature, use_cosine_similarity, normalised inputs, seed)
NTXENT_CASES = [
    ("b4_c256_cos", 4, 256, 0.1, True, True, 0),
    ("b16_c256_cos", 16, 256, 0.1, True, True, 1),
    ("b64_c256_cos", 64, 256, 0.1, True, True, 2),
    ("b64_c256_cos_raw", 64, 256, 0.1, True, False, 3),
    ("b32_c64_cos_t05", 32, 64, 0.5, True, True, 4),
    ("b32_c128_dot", 32, 128, 0.1, False, True, 5),
]


def load_reference_ntxent():
    spec = importlib.util.spec_from_file_location("ref_nt_xent", REF / "utils" / "nt_xent.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.NTXentLoss


def ntxent_inputs(B, C, normalised, seed):
    rng = np.random.default_rng(seed)
    zis = rng.standard_normal((B, C)).astype(np.float32)
    zjs = (0.6 * zis + 0.8 * rng.standard_normal((B, C))).astype(np.float32)  # correlated views
    if normalised:
        zis /= np.linalg.norm(zis, axis=1, keepdims=True)
        zjs /= np.linalg.norm(zjs, axis=1, keepdims=True)
    return zis, zjs


def make_ntxent():
    NTXentLoss = load_reference_ntxent()
    for name, B, C, T, cos, normed, seed in NTXENT_CASES:
        zis, zjs = ntxent_inputs(B, C, normed, seed)
        ti = torch.from_numpy(zis).requires_grad_(True)
        tj = torch.from_numpy(zjs).requires_grad_(True)
        crit = NTXentLoss("cpu", B, T, cos)
        loss = crit(ti, tj)
        loss.backward()
        np.savez_compressed(OUT / f"ntxent_{name}.npz", zis=zis, zjs=zjs,
                            loss=np.float32(loss.item()), dzis=ti.grad.numpy(),
                            dzjs=tj.grad.numpy(), batch_size=B, temperature=T,
                            use_cosine=cos)
        print(f"ntxent_{name}: loss={loss.item():.6f}")


def make_manifest():
    sd = torch.load(REF / "ckpt" / "pretrained_gcn" / "checkpoints" / "model.pth",
                    map_location="cpu", weights_only=True)
    manifest = {"keys": {k: list(v.shape) for k, v in sd.items()}, "checksums": {}}
    for k in ("x_embedding1.weight", "gnns.0.weight", "gnns.0.edge_embedding1.weight",
              "batch_norms.4.running_var", "out_lin.2.bias"):
        t = sd[k].detach().contiguous().numpy()
        manifest["checksums"][k] = {
            "sum": float(t.astype(np.float64).sum()),
            "sha256": hashlib.sha256(t.tobytes()).hexdigest(),
        }
    manifest["num_batches_tracked"] = int(sd["batch_norms.0.num_batches_tracked"])
    (OUT / "pretrained_gcn_manifest.json").write_text(json.dumps(manifest, indent=1))
    print(f"manifest: {len(manifest['keys'])} keys")


if __name__ == "__main__":
    if not REF.exists():
        sys.exit("the reference is not mounted; fixtures are generated in the build container")
    make_ntxent()
    make_manifest()
