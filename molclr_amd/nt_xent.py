"""NT-Xent contrastive loss — drop-in for utils/nt_xent.py.

``NTXentLoss(device, batch_size, temperature, use_cosine_similarity)`` and
``loss = criterion(zis, zjs)`` exactly as the reference (utils/nt_xent.py:5-65,
called at molclr.py:43,66): representations ``[zjs; zis]``, cosine (or dot)
similarity, positives on the ±B diagonals, all other off-diagonal entries as
negatives, ``CrossEntropyLoss(reduction='sum') / 2B``.

The computation is one fused HIP pipeline (ntxent.hip): no (2B, 2B, C)
broadcast, no mask gather, no (2B, 2B−1) logits matrix.  Passing
``group=`` (a torch.distributed process group) makes ``batch_size`` the
GLOBAL batch: each rank passes its local (zis, zjs) and receives the loss of
the global contrastive batch (see molclr_amd.distributed).
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


class NTXentLoss(torch.nn.Module):

    def __init__(self, device, batch_size, temperature, use_cosine_similarity, group=None):
        super().__init__()
        self.batch_size = batch_size
        self.temperature = temperature
        self.device = device
        self.use_cosine_similarity = bool(use_cosine_similarity)
        self.group = group

    def _get_correlated_mask(self):
        """The reference's negatives mask (nt_xent.py:24-30), kept for API
        compatibility and tests; the fused kernel never materialises it."""
        n = 2 * self.batch_size
        diag = np.eye(n)
        l1 = np.eye(n, n, k=-self.batch_size)
        l2 = np.eye(n, n, k=self.batch_size)
        mask = torch.from_numpy(diag + l1 + l2)
        return (1 - mask).type(torch.bool)

    def forward(self, zis, zjs):
        return ops.nt_xent(zis, zjs, self.batch_size, self.temperature,
                           self.use_cosine_similarity, self.group)

    def forward_pair(self, z):
        """The loss of a paired forward's projections z = [zis; zjs]
        (GINet.forward_pair): the same value as forward(z[:B], z[B:])."""
        return ops.nt_xent_pair(z, self.batch_size, self.temperature,
                                self.use_cosine_similarity, self.group)

    def forward_pair_normalized(self, z):
        """forward_pair(F.normalize(z, dim=1)) (molclr.py:63-66) as one fused
        node: bit-identical to the two calls, fewer launches."""
        return ops.nt_xent_pair_normalized(z, self.batch_size, self.temperature,
                                           self.use_cosine_similarity, self.group)
