"""Pre-training driver — drop-in for the reference's molclr.py.

Same ``MolCLR(dataset, config).train()`` loop and ``config.yaml`` schema as
molclr.py:33-195: Adam(init_lr, weight_decay=eval(weight_decay)),
CosineAnnealingLR(T_max = epochs - warm_up) stepped per epoch once
``epoch >= warm_up``, ``train_loss`` / ``cosine_lr_decay`` logged every
``log_every_n_steps``, validation every ``eval_every_n_epochs`` with the best
weights saved to ``<log_dir>/checkpoints/model.pth`` and ``model_{epoch}.pth``
every ``save_every_n_epochs``.  Quirks kept: ``weight_decay`` is a string
evaluated as a number, ``load_model: None`` is the string 'None' and a missing
checkpoint is tolerated.

Differences (all additive): the optimiser is :class:`FusedAdam` (same update
rule, one kernel); optional config keys ``world_size`` (data parallel via
torchrun), ``seed``, ``dataset.views`` ('device', the default: both views of
every batch are built on the GPU from the resident molecules, for every
``aug`` mode; 'host': the reference's DataLoader, node masking only),
``hip_graph`` (default True: each process replays the whole step from HIP
graphs captured per batch-size capacity bucket, molclr_amd.graph_step, when
the run allows it -- the paired executor pass, one process or data parallel
over RCCL; False: eager); the
scalar writer is TensorBoard when installed, otherwise a JSONL file with the
same tags.  ``data_path`` may be the reference's SMILES text file (featurised
once into a cached binary shard), a shard, or ``synthetic:<count>``.
Invalid inputs raise at the next log step (``check_inputs``), as the
reference's embedding lookup would: every step's graph status word is ORed
into a sticky device accumulator, so a bad batch between log steps is caught.
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import warnings
from datetime import datetime

import numpy as np
import torch
import yaml
from torch.optim.lr_scheduler import CosineAnnealingLR

from . import distributed as mdist
from .nt_xent import NTXentLoss
from .ops import l2_normalize


class _JsonlWriter:
    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.log_dir = log_dir
        self._f = open(os.path.join(log_dir, "scalars.jsonl"), "a")

    def add_scalar(self, tag, value, global_step=None):
        if torch.is_tensor(value):
            value = float(value.detach().item())
        self._f.write(json.dumps({"tag": tag, "value": float(value), "step": global_step}) + "\n")
        self._f.flush()


def _summary_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=log_dir)
    except Exception:  # tensorboard not installed
        return _JsonlWriter(log_dir)


def _save_config_file(model_checkpoints_folder, config):
    if not os.path.exists(model_checkpoints_folder):
        os.makedirs(model_checkpoints_folder)
        with open(os.path.join(model_checkpoints_folder, "config.yaml"), "w") as f:
            yaml.safe_dump(config, f)


class MolCLR(object):
    def __init__(self, dataset, config):
        self.config = config
        self.rank, self.world, self.device = self._get_device()
        dir_name = datetime.now().strftime('%b%d_%H-%M-%S')
        log_dir = os.path.join(config.get('log_root', 'ckpt'), dir_name)
        self.writer = _summary_writer(log_dir) if self.rank == 0 else None
        self.log_dir = log_dir
        self.dataset = dataset
        # sticky OR of every eager step's graph status word (check_inputs)
        self._status = torch.zeros(1, dtype=torch.int32, device=self.device)
        group = torch.distributed.group.WORLD if self.world > 1 else None
        global_batch = config['batch_size'] * self.world
        self.nt_xent_criterion = NTXentLoss(self.device, global_batch, group=group,
                                            **config['loss'])

    def _get_device(self):
        if not torch.cuda.is_available() or self.config.get('gpu', 'cuda:0') == 'cpu':
            raise RuntimeError("molclr_amd pre-training runs on MI355X GPUs only")
        if int(self.config.get('world_size', 1)) > 1 or int(os.environ.get('WORLD_SIZE', 1)) > 1:
            rank, world, device = mdist.init()
        else:
            device = torch.device(self.config['gpu'])
            torch.cuda.set_device(device)
            rank, world = 0, 1
        if rank == 0:
            print("Running on:", device, "world size", world)
        return rank, world, device

    def _step(self, model, xis, xjs, n_iter):
        """molclr.py:55-67.  Both views go through ONE encoder pass
        (model.forward_pair: per-view BatchNorm statistics, the reference's
        two-call semantics); F.normalize and NT-Xent on the stacked [zis; zjs]."""
        if getattr(self, "paired", True) and hasattr(model, "forward_pair"):
            _, z = model.forward_pair(xis, xjs)
            return self.nt_xent_criterion.forward_pair_normalized(z)
        ris, zis = model(xis)  # [N,C]
        rjs, zjs = model(xjs)  # [N,C]
        zis = l2_normalize(zis)
        zjs = l2_normalize(zjs)
        return self.nt_xent_criterion(zis, zjs)

    def build_model(self):
        if self.config['model_type'] == 'gin':
            from .ginet_molclr import GINet
            # fp16_precision (apex O2 in the reference, molclr.py:16-24,93-96):
            # the bf16 encoder path here, fp32 master weights
            prec = 'bf16' if self.config.get('fp16_precision', False) else 'fp32'
            model = GINet(**self.config["model"], precision=prec).to(self.device)
        elif self.config['model_type'] == 'gcn':
            from .gcn_molclr import GCN
            if self.config.get('fp16_precision', False):
                # The reference's switch only takes effect with apex installed
                # (molclr.py:14-22,93-96,121-125); without it the reference
                # prints a notice and trains in fp32.  The GCN kernels have no
                # reduced-precision storage path, so this is the reference's
                # no-apex behaviour: a warning, then fp32
                warnings.warn("fp16_precision: True with model_type: gcn -- the GCN encoder has "
                              "no reduced-precision path; training in fp32 (the reference's "
                              "behaviour without apex, molclr.py:14-22,93-96)", RuntimeWarning,
                              stacklevel=2)
            model = GCN(**self.config["model"]).to(self.device)
        else:
            raise ValueError('Undefined GNN model.')
        return self._load_pre_trained_weights(model)

    def build_optimizer(self, model):
        from .optim import FusedAdam
        # data parallel: parameters in gradient-bucket order, so each bucket of
        # the overlapped all-reduce is one slice of the flat gradient buffer
        params = mdist.bucketed_parameters(model) if self.world > 1 else model.parameters()
        optimizer = FusedAdam(params, self.config['init_lr'],
                              weight_decay=float(eval(str(self.config['weight_decay']))))
        self.reducer = None
        if self.world > 1:
            mdist.broadcast_params(optimizer.flat)
            if getattr(self, "paired", True) and hasattr(model, "forward_pair"):
                self.reducer = mdist.OverlappedGradReducer(
                    model, optimizer, torch.distributed.group.WORLD)
        scheduler = CosineAnnealingLR(optimizer, T_max=self.config['epochs'] - self.config['warm_up'],
                                      eta_min=0, last_epoch=-1)
        return optimizer, scheduler

    def _graph_step(self, model, optimizer):
        """The HIP-graph step (molclr_amd.graph_step) unless the config turns
        it off (``hip_graph: False``), when the run allows it: the paired
        executor pass at an unpadded width, one process or data parallel over
        RCCL (the collectives are captured with the step; captures happen in
        lockstep across ranks); else None (eager)."""
        if not self.config.get('hip_graph', True):
            return None
        if not getattr(self, "paired", True) or not hasattr(model, "forward_staged"):
            return None
        if not model._executor_ok() or model._dim_pad() or not mdist.graph_capturable():
            return None
        cs = getattr(self, "_captured", None)
        if cs is None or cs.model is not model or cs.optimizer is not optimizer:
            from .graph_step import CapturedTrainStep
            # data parallel: the RCCL collectives are captured with the step
            cs = self._captured = CapturedTrainStep(model, optimizer, self.nt_xent_criterion,
                                                    reducer=getattr(self, "reducer", None))
        return cs

    def train_step(self, model, optimizer, xis, xjs, n_iter):
        xis = xis.to(self.device, non_blocking=True)
        xjs = xjs.to(self.device, non_blocking=True)
        cs = self._graph_step(model, optimizer)
        if cs is not None:  # zero_grad .. Adam replayed as one HIP graph
            loss = cs(xis, xjs)
            self._last_graph = cs.last_graph
            return loss
        self._last_graph = None
        optimizer.zero_grad()
        reducer = getattr(self, "reducer", None)
        if reducer is not None:
            reducer.arm()
        loss = self._step(model, xis, xjs, n_iter)
        self._last_inputs = xis
        self._accumulate_status(xis, xjs)
        loss.backward()
        if reducer is not None:
            reducer.finish()
        elif self.world > 1:
            mdist.allreduce_grads(optimizer.flat_grad)
        optimizer.step()
        return loss

    def train(self):
        train_loader, valid_loader = self.dataset.get_data_loaders()
        model = self.build_model()
        if self.rank == 0:
            print(model)
        optimizer, scheduler = self.build_optimizer(model)

        model_checkpoints_folder = os.path.join(self.log_dir, 'checkpoints')
        if self.rank == 0:
            _save_config_file(model_checkpoints_folder, self.config)

        cs = self._graph_step(model, optimizer)
        if cs is not None and hasattr(train_loader, "on_epoch_plan"):
            # capture every graph an epoch's batches need when it is drawn
            # (node masking: exact sizes), not in the middle of the epoch;
            # data parallel: every rank captures the union of all ranks' sizes
            train_loader.on_epoch_plan = cs.prepare_sizes
        try:
            return self._train_epochs(model, optimizer, scheduler, train_loader, valid_loader,
                                      model_checkpoints_folder)
        finally:
            # graphs holding RCCL collectives go before the process group does
            if cs is not None:
                cs.close()  # its counters and status word stay readable

    def _train_epochs(self, model, optimizer, scheduler, train_loader, valid_loader,
                      model_checkpoints_folder):
        n_iter = 0
        valid_n_iter = 0
        best_valid_loss = np.inf
        for epoch_counter in range(self.config['epochs']):
            bn = 0
            for bn, (xis, xjs) in enumerate(train_loader):
                loss = self.train_step(model, optimizer, xis, xjs, n_iter)
                if n_iter % self.config['log_every_n_steps'] == 0 and self.rank == 0:
                    self.check_inputs()
                    self.writer.add_scalar('train_loss', loss, global_step=n_iter)
                    self.writer.add_scalar('cosine_lr_decay', scheduler.get_last_lr()[0],
                                           global_step=n_iter)
                    print(epoch_counter, bn, loss.item())
                n_iter += 1

            if epoch_counter % self.config['eval_every_n_epochs'] == 0:
                valid_loss = self._validate(model, valid_loader)
                if self.rank == 0:
                    print(epoch_counter, bn, valid_loss, '(validation)')
                    if valid_loss < best_valid_loss:
                        best_valid_loss = valid_loss
                        torch.save(model.state_dict(),
                                   os.path.join(model_checkpoints_folder, 'model.pth'))
                    self.writer.add_scalar('validation_loss', valid_loss, global_step=valid_n_iter)
                valid_n_iter += 1

            if (epoch_counter + 1) % self.config['save_every_n_epochs'] == 0 and self.rank == 0:
                torch.save(model.state_dict(),
                           os.path.join(model_checkpoints_folder, f'model_{epoch_counter}.pth'))

            if epoch_counter >= self.config['warm_up']:
                scheduler.step()
        return model

    def _accumulate_status(self, xi, xj) -> None:
        """OR the step's graph status words (the paired graph, or each view's
        own) into the sticky accumulator (tiny device ops, no sync)."""
        pg = getattr(xi, "_molclr_pair_graph", None)
        graphs = [pg[1]] if pg is not None else [getattr(v, "_molclr_graph", None) for v in (xi, xj)]
        for g in graphs:
            if g is not None:
                torch.bitwise_or(self._status, g.status, out=self._status)

    def check_inputs(self) -> None:
        """Raise if any step so far had invalid inputs (out-of-range edges, or
        atom features outside the embedding tables, where the reference's
        nn.Embedding raises IndexError).  Reads the sticky device status words
        of the eager steps and of the captured step (a sync: called where the
        loop syncs anyway, at the log steps)."""
        from .data import raise_for_status
        cs = getattr(self, "_captured", None)
        st = int(self._status.item()) | (int(cs.status.item()) if cs is not None else 0)
        raise_for_status(st)

    def _load_pre_trained_weights(self, model):
        try:
            checkpoints_folder = os.path.join('./ckpt', str(self.config['load_model']), 'checkpoints')
            state_dict = torch.load(os.path.join(checkpoints_folder, 'model.pth'),
                                    map_location=self.device, weights_only=True)
            model.load_state_dict(state_dict)
            print("Loaded pre-trained model with success.")
        except FileNotFoundError:
            print("Pre-trained weights not found. Training from scratch.")
        return model

    def _validate(self, model, valid_loader):
        with torch.no_grad():
            model.eval()
            valid_loss = 0.0
            counter = 0
            for (xis, xjs) in valid_loader:
                xis = xis.to(self.device)
                xjs = xjs.to(self.device)
                loss = self._step(model, xis, xjs, counter)
                self._last_inputs = xis
                self._last_graph = None
                self._accumulate_status(xis, xjs)
                valid_loss += loss.item()
                self.check_inputs()
                counter += 1
            valid_loss /= max(counter, 1)
        model.train()
        return valid_loss


def main(config_path: str = "config.yaml"):
    """molclr.py:180-195: the data module is chosen by ``config['aug']``."""
    with open(config_path, "r") as f:
        config = yaml.safe_load(f)
    print(config)

    if config['aug'] == 'node':
        from .dataset import MoleculeDatasetWrapper
    elif config['aug'] == 'subgraph':
        from .dataset_subgraph import MoleculeDatasetWrapper
    elif config['aug'] == 'mix':
        from .dataset_mix import MoleculeDatasetWrapper
    else:
        raise ValueError('Not defined molecule augmentation!')

    dataset = MoleculeDatasetWrapper(config['batch_size'], **config['dataset'])
    molclr = MolCLR(dataset, config)
    try:
        molclr.train()  # closes its captured graphs itself
    finally:
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "config.yaml")
