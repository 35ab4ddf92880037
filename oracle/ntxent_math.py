"""ORACLE — test infrastructure only (see oracle/__init__.py).

Closed-form NT-Xent (utils/nt_xent.py:47-65) in float64, in the row-sharded
form the HIP kernels implement (ntxent.hip), with an explicit gradient:

    R = [zj; zi] (rows scaled to unit norm when cosine), S = R R^T
    lse_r  = log Σ_{c≠r} exp(S_rc / T)
    loss   = (1/2B) Σ_r (lse_r − S_{r,p(r)} / T),     p(r) = (r + B) mod 2B
    dL/dR̂_r = Σ_c W_rc R̂_c,  W_rc = (P_rc + P_cr − 2[c = p(r)]) / (2B T),  c ≠ r
    P_rc = exp(S_rc / T − lse_r)

It is checked against the reference's own outputs (tests/golden/ntxent_*.npz)
and used by the data-parallel tests to check the sharded algorithm (each rank
owns some rows, sees all gathered columns and the gathered lse).
"""
from __future__ import annotations

import numpy as np


def prep(R: np.ndarray, cosine: bool):
    R = np.asarray(R, dtype=np.float64)
    if not cosine:
        return R, np.ones(R.shape[0])
    n = np.maximum(np.linalg.norm(R, axis=1), 1e-8)
    return R / n[:, None], n


def prep_bwd(dRhat: np.ndarray, Rhat: np.ndarray, norm: np.ndarray, cosine: bool):
    if not cosine:
        return dRhat
    dot = (dRhat * Rhat).sum(1, keepdims=True)
    return (dRhat - dot * Rhat) / norm[:, None]


def rows_forward(rows_hat, gidx, cols_hat, B, T):
    """lse and per-row loss (already divided by 2B) of the owned rows."""
    S = rows_hat @ cols_hat.T / T
    n2 = cols_hat.shape[0]
    S[np.arange(len(gidx)), gidx] = -np.inf
    m = S.max(1, keepdims=True)
    lse = (m + np.log(np.exp(S - m).sum(1, keepdims=True)))[:, 0]
    pos = S[np.arange(len(gidx)), (gidx + B) % n2]
    return lse, (lse - pos) / (2 * B)


def rows_backward(rows_hat, gidx, cols_hat, lse_cols, B, T, g=1.0):
    """dL/d(rows_hat) using the gathered columns and gathered lse."""
    n2 = cols_hat.shape[0]
    S = rows_hat @ cols_hat.T / T
    lse_r = lse_cols[gidx][:, None]
    W = np.exp(S - lse_r) + np.exp(S - lse_cols[None, :])
    r = np.arange(len(gidx))
    W[r, (gidx + B) % n2] -= 2.0
    W[r, gidx] = 0.0
    W *= g / (2 * B * T)
    return W @ cols_hat


def ntxent(zis, zjs, T, cosine=True):
    """Single-process loss and (dzis, dzjs)."""
    B = zis.shape[0]
    R = np.concatenate([zjs, zis], 0)
    Rh, n = prep(R, cosine)
    gidx = np.arange(2 * B)
    lse, lr = rows_forward(Rh, gidx, Rh, B, T)
    dRh = rows_backward(Rh, gidx, Rh, lse, B, T)
    dR = prep_bwd(dRh, Rh, n, cosine)
    return lr.sum(), dR[B:], dR[:B]
