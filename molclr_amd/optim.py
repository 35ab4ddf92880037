"""Adam over one flat parameter buffer (molclr_adam_step, adam.hip).

Replaces ``torch.optim.Adam(model.parameters(), init_lr,
weight_decay=eval(config['weight_decay']))`` of molclr.py:84-87 with the same
update rule (coupled L2 weight decay, bias-corrected moments).  All
parameters are re-seated as views of one contiguous fp32 buffer and their
``.grad`` as views of one gradient buffer, so:

* the optimizer step is a single kernel over every parameter;
* data-parallel gradient reduction is one collective over ``flat_grad``;
* the backward kernels of molclr_amd.ops accumulate straight into the flat
  buffer (no separate autograd accumulation kernels); gradients produced by
  other ops are accumulated there by autograd as usual.  ``zero_grad``
  zeroes it in place and never sets grads to ``None``.

Learning rate and step counter live on the device, so a captured step
replays with the scheduler's current learning rate.  Parameters that receive
no gradient in a step are still decayed (their grad is zero, not ``None``),
as torch.optim.Adam does after ``zero_grad(set_to_none=False)``.
"""
from __future__ import annotations

import torch

from . import _lib, ops


def _align4(n: int) -> int:
    return (n + 3) // 4 * 4


class FusedAdam(torch.optim.Optimizer):

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdam supports a single parameter group (as molclr.py uses)")
        plist = self.param_groups[0]["params"]
        dev = plist[0].device
        if dev.type != "cuda":
            raise RuntimeError("FusedAdam runs on the GPU only")
        total = sum(_align4(p.numel()) for p in plist)
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(total, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        with torch.no_grad():
            for p in plist:
                if p.dtype != torch.float32 or p.device != dev:
                    raise ValueError("FusedAdam: all parameters must be fp32 on one device")
                n = p.numel()
                self.flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + n].view_as(p)
                p.grad = self.flat_grad[off:off + n].view_as(p)
                # molclr_amd's backward kernels add straight into this .grad
                # view (ops._grad_sink) instead of handing autograd a tensor
                p._molclr_fused_grad = True
                self.views.append((p, off, n))
                off += _align4(n)
        self.numel = total
        self._lr_dev = torch.tensor([float(lr)], dtype=torch.float32, device=dev)
        self._lr_host = float(lr)
        self._step_dev = torch.zeros(1, dtype=torch.int32, device=dev)

    @torch.no_grad()
    def zero_grad(self, set_to_none: bool = False):  # noqa: D401 - torch API
        self.flat_grad.zero_()
        for p, off, n in self.views:  # re-seat if a caller replaced .grad
            if p.grad is None or p.grad.data_ptr() != self.flat_grad[off:].data_ptr():
                p.grad = self.flat_grad[off:off + n].view_as(p)

    @torch.no_grad()
    def sync_lr(self) -> None:
        """Copy the param group's learning rate (a scheduler may have changed
        it) to the device value the kernel reads."""
        lr = float(self.param_groups[0]["lr"])
        if lr != self._lr_host:
            self._lr_dev.fill_(lr)
            self._lr_host = lr

    @torch.no_grad()
    def step(self, closure=None, sync_lr: bool = True, tick: bool = True):
        """``sync_lr=False`` while capturing a HIP graph: the replays read the
        device learning rate, which the caller syncs before each replay.
        ``tick=False``: the caller advances the device step counter itself
        (molclr_step_tail, the captured step's closing launch)."""
        loss = closure() if closure is not None else None
        ops.join_side()  # side-stream weight gradients (ops.linear_bwd) are final
        g = self.param_groups[0]
        if sync_lr:
            self.sync_lr()
        b1, b2 = g["betas"]
        _lib.call("molclr_adam_step_ex", self.flat.data_ptr(), self.flat_grad.data_ptr(),
                  self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self.numel,
                  self._lr_dev.data_ptr(), self._step_dev.data_ptr(), float(b1), float(b2),
                  float(g["eps"]), float(g["weight_decay"]), int(tick),
                  _lib.stream_of(self.flat.device))
        ops.bump_param_generation()  # cached weight planes are stale now
        return loss

    @property
    def steps_taken(self) -> int:
        return int(self._step_dev.item())
