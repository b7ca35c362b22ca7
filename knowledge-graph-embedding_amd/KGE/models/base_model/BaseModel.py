"""Base module for KGE models (reference ``KGE/models/base_model/BaseModel.py``).

``KGEModel`` keeps the reference's public surface -- ``train`` (:58-190),
``evaluate`` (:578-618), ``get_rank`` (:620-654), ``score_hrt`` (:410-430),
``restore_model_weights`` (:656-666) -- and its per-batch step
(``__run_single_batch``, :293-330), which is dispatched by ``KGE.engine`` to
the fused HIP step (``libkge_hip.so``) or, for user-defined plugins, to the
eager autograd path with the same TF-2.5 semantics.

Deviations from the reference, all documented in DESIGN.md:
  * ``train`` without ``val_X`` works (the reference fails at :148).
  * ``get_rank`` counts in int64 (the reference's int16 overflows for E > 32767).
  * ``restore_model_weights`` checks the given weights (the reference calls
    ``_check_model_weights()`` without its argument, :665).
  * per-batch losses stay on the device; the host reads one value per epoch
    (the reference syncs every batch with ``.numpy()``, :330).
  * TensorBoard summaries are written as JSON lines under ``log_path``.
"""

import datetime
import json
import logging
import os

import numpy as np
import torch

from ... import engine
from ... import optimizers as _opt
from ...data_utils import calculate_data_size, set_tf_iterator
from ...metrics import (geometric_mean_rank, harmonic_mean_rank, hits_at_k, mean_rank, mean_reciprocal_rank,
                        median_rank, std_rank)
from ...ns_strategy import TypedStrategy, UniformStrategy

logging.getLogger().setLevel(logging.INFO)


def _world_size():
    d = torch.distributed
    return d.get_world_size() if d.is_available() and d.is_initialized() else 1


def _is_rank0():
    d = torch.distributed
    return not (d.is_available() and d.is_initialized()) or d.get_rank() == 0


def _shared_seed(seed):
    """Multi-GPU: every rank must shuffle the same global stream (each scores
    its slice of the same global batch, ``_run_single_batch``); with
    ``seed=None`` rank 0's draw is broadcast so the ranks agree."""
    if seed is not None or _world_size() == 1:
        return seed
    d = torch.distributed
    dev = engine.device() if d.get_backend() == "nccl" else torch.device("cpu")
    s = torch.tensor([int.from_bytes(os.urandom(7), "little")], dtype=torch.int64, device=dev)
    d.broadcast(s, src=0)
    return int(s.item())


class KGEModel:
    """Base class for KGE models (``BaseModel.py:23-56``)."""

    _fused_model_id = None

    def __init__(self, embedding_params, negative_ratio, corrupt_side, loss_fn, ns_strategy, n_workers):
        assert corrupt_side in ['h+t', 'h', 't'], "Invalid corrupt_side, valid options: 'h+t', 'h', 't'"
        self.embedding_params = embedding_params
        self.negative_ratio = negative_ratio
        self.corrupt_side = corrupt_side
        self.loss_fn = loss_fn
        self.ns_strategy = ns_strategy
        self._n_workers = n_workers
        self._model_weights_initial = None
        self._tape = None
        self._batch_scale = 1.0
        self._fused = None
        self._optimizer = None
        self.metadata = None

    # ------------------------------------------------------------ train
    def train(self, train_X, val_X, metadata, epochs, batch_size, early_stopping_rounds=None,
              model_weights_initial=None, restore_best_weight=True, optimizer="Adam", seed=None,
              log_path="./logs", log_projector=False):
        """Train the model (``BaseModel.py:58-190``)."""
        self.metadata = metadata
        self.batch_size = batch_size
        self._model_weights_initial = model_weights_initial
        self._optimizer = optimizer
        self.seed = seed
        self.log_path = log_path

        logging.info("[%s] Preparing for training..." % str(datetime.datetime.now()))
        train_iter, val_iter = self._prepare_for_train(train_X=train_X, val_X=val_X)
        train_loss_history, val_loss_history = [], []
        patience_count = 0
        self.best_step = None

        logging.info("[%s] Start Training..." % str(datetime.datetime.now()))
        try:
            self._train_epochs(epochs, train_iter, val_iter, early_stopping_rounds, restore_best_weight,
                               train_loss_history, val_loss_history, patience_count)
        finally:
            self._join_checkpoint()   # (also when an epoch raised: no writer outlives train())
        self.sync_weights()
        self.train_loss_history = train_loss_history
        self.val_loss_history = val_loss_history
        if log_projector:
            self._log_embeddings_projector(log_path)
        logging.info("[%s] Finished training!" % str(datetime.datetime.now()))

    def _train_epochs(self, epochs, train_iter, val_iter, early_stopping_rounds, restore_best_weight,
                      train_loss_history, val_loss_history, patience_count):
        """The epoch loop of ``BaseModel.py:100-184``.

        Single-GPU fused training without early stopping never lets the GPU
        run dry at an epoch boundary: the epoch's loss sums, status word and
        weight histograms are computed on the stream and copied into pinned
        host buffers behind its last batch, and the host reads them (logs,
        loss history, status check) only after it has queued the next epoch's
        first batches. The values and the order of everything written are the
        same as reading them at once; a device error is raised one epoch
        later. Early stopping reads the validation loss at once (its decision
        gates the next epoch)."""
        pending = None
        # a deferred epoch's results are read once this many of the next
        # epoch's batches are queued: the reads then wait for nothing (the GPU
        # has ~1.5 ms of batches ahead of the host at C2's 0.08 ms per batch)
        read_after = 15
        for i in range(epochs):
            # per-epoch loss sums stay on the device: the fused step adds each
            # batch's loss into them itself (no per-batch host work); the host
            # reads them once per epoch (the reference syncs every batch, :330)
            train_loss = torch.zeros(1, dtype=torch.float32, device=self._device)
            val_loss = torch.zeros(1, dtype=torch.float32, device=self._device)
            for b in range(self._batch_count_train):
                self._run_single_batch(next(train_iter), is_train=True, accum=train_loss)
                if val_iter is not None and b < self._batch_count_val:
                    self._run_single_batch(next(val_iter), is_train=False, accum=val_loss)
                if pending is not None and b >= read_after:
                    self._finish_epoch(pending, train_loss_history, val_loss_history)
                    pending = None
            if pending is not None:
                self._finish_epoch(pending, train_loss_history, val_loss_history)
                pending = None
            ep = self._end_epoch(i, train_loss, val_loss, val_iter is not None)
            if early_stopping_rounds is None and ep["deferred"]:
                # (pinned copies on the stream, written by a thread -- only if
                # the epoch's status word is clean: a failing epoch never
                # replaces the last good checkpoint; _finish_epoch raises it)
                self._save_checkpoint(status=ep["dev_vals"][2:3])
                pending = ep
                continue
            self._finish_epoch(ep, train_loss_history, val_loss_history)
            if early_stopping_rounds is not None:
                assert val_iter is not None, "val_X should be given if want to check early stopping."
                early_stop, patience_count = self._check_early_stopping(
                    val_loss_history, "larger", patience_count, early_stopping_rounds, i, restore_best_weight)
                if early_stop:
                    logging.info("[%s] Val loss does not improve within %i iterations, trigger early stopping."
                                 % (str(datetime.datetime.now()), early_stopping_rounds))
                    break
            else:
                self._save_checkpoint()
        if pending is not None:
            self._finish_epoch(pending, train_loss_history, val_loss_history)

    def _end_epoch(self, i, train_loss, val_loss, has_val):
        """Queue epoch i's reads behind its last batch: losses, the fused
        step's status word and the weight histograms' device statistics into
        pinned host memory, one event after them. Deferred reading only for a
        single-GPU fused step (multi-GPU keeps its collectives in step)."""
        fused = self._fused
        deferred = (self._device.type == "cuda" and isinstance(fused, engine.FusedStep) and _world_size() == 1)
        ep = {"epoch": i, "has_val": has_val, "deferred": deferred}
        if not deferred:
            self._check_device_status()
            ep["losses"] = (float(train_loss), float(val_loss))
            ep["hist"] = self._histogram_stats()
            return ep
        bufs = self.__dict__.setdefault("_epoch_bufs", {})
        dev_vals = torch.cat([train_loss, val_loss, fused.status.to(torch.float32)])
        fused.status.zero_()   # (read from the copy; a later epoch's error is its own)
        host = bufs.get("vals")
        if host is None:
            host = bufs["vals"] = torch.empty(3, dtype=torch.float32, pin_memory=True)
        host.copy_(dev_vals, non_blocking=True)
        ep["vals"] = host
        ep["dev_vals"] = dev_vals
        ep["hist"] = self._histogram_stats(pinned=bufs)
        ev = torch.cuda.Event()
        ev.record()
        ep["event"] = ev
        return ep

    def _finish_epoch(self, ep, train_loss_history, val_loss_history):
        """Epoch ep's host side: status check, loss history, logs, histograms."""
        i = ep["epoch"]
        if ep["deferred"]:
            ep["event"].synchronize()
            tl, vl, code = [float(x) for x in ep["vals"]]
            from ... import _hip
            _hip.raise_status_code(int(code), "kge_step")
        else:
            tl, vl = ep["losses"]
        train_loss = tl / self._batch_count_train
        train_loss_history.append(train_loss)
        self._log_scalar("train", train_loss, i)
        if ep["has_val"]:
            val_loss = vl / self._batch_count_val
            val_loss_history.append(val_loss)
            self._log_scalar("validation", val_loss, i)
            logging.info("epoch: %i, train loss: %f, valid loss: %f" % (i, train_loss, val_loss))
        else:
            logging.info("epoch: %i, train loss: %f" % (i, train_loss))
        self._histogram_write(i, ep["hist"])

    def _prepare_for_train(self, train_X, val_X):
        """``BaseModel.py:192-278``: batch counts, iterators, init, optimizer, sampler."""
        self._device = engine.device()
        self.seed = _shared_seed(self.seed)
        n_train = calculate_data_size(train_X)
        self._batch_count_train = int(np.ceil(n_train / self.batch_size))
        # batches gathered up to 32 at a time into a ring (one launch instead of 32)
        train_iter = set_tf_iterator(train_X, self.batch_size, shuffle=True, buffer_size=n_train,
                                     seed=self.seed, device=self._device, reuse_buffer=True,
                                     chunk=max(1, min(32, n_train // self.batch_size)))
        if val_X is not None:
            n_val = calculate_data_size(val_X)
            self._batch_count_val = int(np.ceil(n_val / self.batch_size))
            val_iter = set_tf_iterator(val_X, self.batch_size, shuffle=False, device=self._device, reuse_buffer=True)
        else:
            self._batch_count_val = 0
            val_iter = None

        self._init_embeddings(seed=self.seed)
        self._to_device()
        self._optimizer = _opt.get(self._optimizer)
        check_path = self.log_path
        os.makedirs(check_path, exist_ok=True)

        if self.ns_strategy is UniformStrategy:
            self.ns_strategy = UniformStrategy(sample_pool=np.arange(len(self.metadata["ind2ent"])),
                                               seed=self.seed)
        elif self.ns_strategy is TypedStrategy:
            self.metadata["type2inds"] = {}
            for t in np.unique(self.metadata["ind2type"]):
                indices = [i for (i, ti) in enumerate(self.metadata["ind2type"]) if ti == t]
                self.metadata["type2inds"][t] = np.array(indices)
            self.ns_strategy = TypedStrategy(pool=None, metadata={
                "type2inds": self.metadata["type2inds"], "ind2type": self.metadata["ind2type"]}, seed=self.seed)
        self._fused = None
        self.__dict__.pop("_bound", None)
        return train_iter, val_iter

    def _to_device(self):
        dev = getattr(self, "_device", None) or engine.device()
        self._device = dev
        for k, w in list(self.model_weights.items()):
            if not isinstance(w, torch.Tensor):
                w = torch.as_tensor(np.asarray(w), dtype=torch.float32)
            self.model_weights[k] = w.detach().to(device=dev, dtype=torch.float32).contiguous()

    # ------------------------------------------------------------ step
    def _plan_for(self, opt, batch_size):
        """engine.fused_plan, cached per (optimizer, batch size, plugins)."""
        key = (id(opt), batch_size, id(getattr(self, "score_fn", None)), id(self.loss_fn), id(self.ns_strategy),
               self.negative_ratio, self.corrupt_side, bool(getattr(self, "constraint", False)), engine.backend(),
               id(self.model_weights.get("ent_emb")))
        c = self.__dict__.get("_plan_key")
        if c is None or c[0] != key:
            self._plan_key = (key, engine.fused_plan(self, opt, batch_size))
        return self._plan_key[1]

    def _run_single_batch(self, batch_data, is_train, accum=None):
        """One batch (``BaseModel.py:293-330``). Returns the loss as a device
        scalar, or, given ``accum`` (device float32 [1]), adds it there and
        returns None (the fused single-device step adds it in-kernel).

        The training loop refills one batch buffer (or a ring of them, views
        of one tensor) in place, so a single-GPU fused step is bound to
        (buffer, optimizer, accum) once (``FusedStep.bind``) and later batches
        are one ``kge_step`` call with the batch's address; the binding is
        dropped when the plugins, the optimizer or the weight tensors change."""
        opt = self._optimizer if is_train else None
        if accum is not None:
            b = self.__dict__.get("_bound")
            if b is not None:
                base = batch_data._base if batch_data._base is not None else batch_data
                run = b.get((id(base), batch_data.shape, is_train, id(opt), id(accum)))
                if run is not None and run[0] == self._bind_fingerprint(opt) and batch_data.is_contiguous():
                    run[1](batch_data.data_ptr())
                    return None
        world = _world_size()
        reason = self._plan_for(opt, batch_data.shape[0] // world)
        if reason is None:
            if self._fused is None:
                if world > 1:
                    from ...sharded import ShardedStep
                    self._fused = ShardedStep(self, batch_hint=batch_data.shape[0] // world,
                                              optimizer=self._optimizer)
                else:
                    self._fused = engine.FusedStep(self)
            if world > 1:
                # every rank draws the same global batch; each scores its slice
                n = batch_data.shape[0]
                assert n % world == 0, "batch_size must be divisible by the world size"
                rank = torch.distributed.get_rank()
                batch_data = batch_data[rank * (n // world):(rank + 1) * (n // world)]
            if accum is not None and isinstance(self._fused, engine.FusedStep):
                f = self._fused
                if batch_data.device == f.device and batch_data.dtype in (torch.int32, torch.int64) and \
                        batch_data.is_contiguous():
                    run = f.bind(batch_data, is_train, opt, accum=accum)
                    b = self.__dict__.setdefault("_bound", {})
                    if len(b) >= 8:
                        b.clear()
                    # the entry holds every object whose id it is keyed or checked by
                    # (batch buffer, optimizer, accum, weights), so no id can be reused while it lives
                    base = batch_data._base if batch_data._base is not None else batch_data
                    b[(id(base), batch_data.shape, is_train, id(opt), id(accum))] = (
                        self._bind_fingerprint(opt), run, (base, opt, accum, list(self.model_weights.values())))
                    run()
                    return None
                f(batch_data, is_train, opt, accum=accum)
                return None
            loss = self._fused(batch_data, is_train, opt)
            if accum is not None:
                accum += loss.reshape(1)     # (the multi-GPU loss is final only after its all-reduce)
                return None
            return loss.clone().reshape(()).to(torch.float64)
        if world > 1:
            raise NotImplementedError("multi-GPU training needs a fused combination (%s)" % reason)
        if engine.backend() != "eager":
            engine.warn_once((type(self).__name__, reason), "eager plugin path: %s" % reason)
        loss = engine.eager_step(self, batch_data, is_train, opt)
        if accum is not None:
            accum += loss.reshape(1).to(accum.dtype)
            return None
        return loss.to(torch.float64)

    def _bind_fingerprint(self, opt):
        """What a bound step depends on besides its buffers: the plugins, the
        weight tensors and the optimizer's learning rate."""
        return (id(getattr(self, "score_fn", None)), id(self.loss_fn), id(self.ns_strategy), self.negative_ratio,
                self.corrupt_side, id(self._fused), getattr(opt, "learning_rate", None),
                tuple(map(id, self.model_weights.values())))

    def sync_weights(self):
        """Multi-GPU: gather the entity shards into ``model_weights`` (before evaluation)."""
        if self._fused is not None and hasattr(self._fused, "sync"):
            self._fused.sync()

    def _check_device_status(self):
        if self._fused is not None:
            self._fused.check_status()

    def _negative_sampling(self, X):
        """``BaseModel.py:332-358``."""
        if self.corrupt_side == 'h':
            return self._corrupt_h(X, self.negative_ratio, self.ns_strategy)
        if self.corrupt_side == 't':
            return self._corrupt_t(X, self.negative_ratio, self.ns_strategy)
        h = self._corrupt_h(X, self.negative_ratio // 2, self.ns_strategy)
        t = self._corrupt_t(X, self.negative_ratio // 2, self.ns_strategy)
        return torch.cat([h, t], dim=-1).reshape(-1, 3)

    def _corrupt_h(self, X, negative_ratio, strategy):
        """``BaseModel.py:360-383``."""
        h = strategy(X, negative_ratio=negative_ratio, side="h").to(X.device)
        r = torch.repeat_interleave(X[:, 1], negative_ratio)
        t = torch.repeat_interleave(X[:, 2], negative_ratio)
        return torch.stack([h, r, t], dim=1)

    def _corrupt_t(self, X, negative_ratio, strategy):
        """``BaseModel.py:385-408``."""
        s = strategy(X, negative_ratio=negative_ratio, side="t").to(X.device)
        h = torch.repeat_interleave(X[:, 0], negative_ratio)
        r = torch.repeat_interleave(X[:, 1], negative_ratio)
        return torch.stack([h, r, s], dim=1)

    # ------------------------------------------------------------ plugin helpers
    def _ids(self, x):
        dev = self.model_weights["ent_emb"].device
        if isinstance(x, torch.Tensor):
            return x.to(dev).to(torch.int64)
        return torch.as_tensor(np.asarray(x), dtype=torch.int64, device=dev)

    def _lookup(self, name, idx):
        """``tf.nn.embedding_lookup``; under a training tape each lookup is a
        separate leaf so its gradient is one IndexedSlices block."""
        w = self.model_weights[name]
        idx = self._ids(idx)
        if self._tape is None:
            return w[idx]
        flat = idx.reshape(-1)
        leaf = w.detach().index_select(0, flat).requires_grad_(True)
        self._tape.records.append((name, flat, leaf))
        return leaf.reshape(tuple(idx.shape) + tuple(w.shape[1:]))

    def _assign(self, name, value):
        """``Variable.assign`` inside ``_constraint_loss`` (no gradient)."""
        with torch.no_grad():
            self.model_weights[name].copy_(value)

    def score_hrt(self, h, r, t):
        """Resolve ``None`` to every entity (``BaseModel.py:410-430``)."""
        assert not (h is None and t is None), "h and t should not be None simultaneously"
        n = len(self.metadata["ind2ent"])
        if h is None:
            r, t = self._ids(r), self._ids(t)
            assert r.dim() == 0 and t.dim() == 0
            h = torch.arange(n, device=r.device)
        if t is None:
            h, r = self._ids(h), self._ids(r)
            assert h.dim() == 0 and r.dim() == 0
            t = torch.arange(n, device=h.device)
        return self._ids(h), self._ids(r), self._ids(t)

    def _init_embeddings(self, seed):
        raise NotImplementedError("subclass of KGEModel should implement _init_embeddings()")

    def _constraint_loss(self, X):
        raise NotImplementedError("subclass of KGEModel should implement _constraint_loss()")

    def _check_model_weights(self, model_weights):
        raise NotImplementedError("subclass of KGEModel should implement _check_model_weights()")

    def _uniform(self, shape, limit, gen):
        """U(-limit, limit) drawn where the model lives (the generator's device:
        a 50M-row table is never drawn on the host)."""
        dev = engine.device()
        x = torch.rand(shape, generator=gen, dtype=torch.float32, device=gen.device)
        return x.mul_(2).sub_(1).mul_(limit).to(dev)

    def _generator(self, seed):
        """The initialisers' seeded generator, on the model's device (identical
        draws on every rank of a multi-GPU run for the same seed)."""
        dev = engine.device()
        g = torch.Generator(device=dev) if dev.type == "cuda" else torch.Generator()
        if seed is not None:
            g.manual_seed(int(seed))
        else:
            g.seed()
        return g

    def _initial_weights(self):
        """Copy of ``model_weights_initial`` as device fp32 tensors."""
        dev = engine.device()
        out = {}
        for k, v in self._model_weights_initial.items():
            t = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
            out[k] = t.detach().to(device=dev, dtype=torch.float32).clone().contiguous()
        return out

    # ------------------------------------------------------------ logging / ckpt
    def _log_scalar(self, split, value, step):
        if not _is_rank0():
            return
        path = os.path.join(self.log_path, "scalar", split)
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "loss.jsonl"), "a") as f:
            f.write(json.dumps({"step": step, "loss": value}) + "\n")

    def _log_embeddings_histogram(self, step, bucket_count=30, chunk=1 << 24):
        """``tf.summary.histogram`` of every weight each epoch (``BaseModel.py:162,470-483``),
        written as JSON lines ``log_path/histogram/<name>.jsonl`` (TensorBoard is not installed):
        TensorBoard's bucketing in float64 -- ``bucket_count`` equal-width buckets from min to max
        (a value at max in the last one), or one bucket ``[x - 0.5, x + 0.5]`` when every value is
        ``x``; ``[left, right, count]`` per bucket. Statistics on the weights' device
        (``_histogram_stats``), the file on rank 0 (``_histogram_write``)."""
        self._histogram_write(step, self._histogram_stats(bucket_count, chunk))

    def _histogram_stats(self, bucket_count=30, chunk=1 << 24, pinned=None):
        """Per weight, float64 [n, min, max, count_0 .. count_{bucket_count-1}] computed on the
        weights' device with no host synchronisation, ``chunk`` values at a time (float64 only per
        chunk: a 50M-row table is never copied whole). Counts add 1.0 per value into its bucket
        (``index_add_``: exact, order-free). With row-sharded entity tables (multi-GPU sparse mode)
        each rank counts its own shard with the all-reduced min / max and the counts are
        all-reduced. ``pinned`` (a dict of reusable buffers): the vectors are copied into pinned
        host memory behind the stream's work (non-blocking) and those are returned."""
        d = torch.distributed
        parts = {}
        if self._fused is not None and hasattr(self._fused, "entity_parts"):
            parts = self._fused.entity_parts()     # {name: this rank's rows} (sparse mode only)
        out = {}
        for name, w in self.model_weights.items():
            sharded = name in parts
            x = (parts[name] if sharded else w.detach()).reshape(-1)
            dev = x.device
            n = torch.full((1,), float(x.numel()), dtype=torch.float64, device=dev)
            lo = torch.full((1,), np.inf, dtype=torch.float64, device=dev)
            hi = torch.full((1,), -np.inf, dtype=torch.float64, device=dev)
            for c0 in range(0, x.numel(), chunk):
                a, b = torch.aminmax(x[c0:c0 + chunk])
                lo = torch.minimum(lo, a.to(torch.float64).reshape(1))
                hi = torch.maximum(hi, b.to(torch.float64).reshape(1))
            if sharded:
                d.all_reduce(n)
                d.all_reduce(lo, op=d.ReduceOp.MIN)
                d.all_reduce(hi, op=d.ReduceOp.MAX)
            width = (hi - lo) / bucket_count
            width = torch.where(width > 0, width, torch.ones_like(width))   # (one value: one bucket, below)
            # bucket k = clamp(floor((x - lo) / width), 0, bc - 1) in float64; integer counts,
            # exact in any order. On the GPU: kge_histogram, one pass, lo / width read on the
            # device (torch.bincount sizes its output on the host: a device sync per weight,
            # ~20 ms of host stall per epoch on C2)
            if dev.type == "cuda" and x.dtype == torch.float32:
                from ... import _hip
                lw = torch.cat([lo, width])
                c64 = torch.zeros(bucket_count, dtype=torch.int64, device=dev)
                xc = x.contiguous()
                _hip.check(_hip.lib().kge_histogram(_hip.ptr(xc), xc.numel(), _hip.ptr(lw), bucket_count,
                                                    _hip.ptr(c64), _hip.stream_handle(dev)), "kge_histogram")
                counts = c64.to(torch.float64)
            else:
                counts = torch.zeros(bucket_count, dtype=torch.float64, device=dev)
                for c0 in range(0, x.numel(), chunk):
                    y = torch.floor((x[c0:c0 + chunk].to(torch.float64) - lo) / width)
                    k = y.nan_to_num_(0.0).clamp_(0, bucket_count - 1).to(torch.int64)
                    counts += torch.bincount(k, minlength=bucket_count).to(torch.float64)
            if sharded:
                d.all_reduce(counts)
            st = torch.cat([n, lo, hi, counts])
            if pinned is not None and dev.type == "cuda":
                key = ("hist", name)
                hb = pinned.get(key)
                if hb is None or hb.numel() != st.numel():
                    hb = pinned[key] = torch.empty(st.numel(), dtype=torch.float64, pin_memory=True)
                hb.copy_(st, non_blocking=True)
                st = hb
            out[name] = st
        return out

    def _histogram_write(self, step, stats):
        """Rank 0 appends one JSON line per weight from ``_histogram_stats``."""
        if not _is_rank0():
            return
        path = os.path.join(self.log_path, "histogram")
        os.makedirs(path, exist_ok=True)
        for name, st in stats.items():
            v = st.cpu().tolist()
            total, lo, hi, counts = v[0], v[1], v[2], v[3:]
            bucket_count = len(counts)
            if total == 0:
                buckets = []
            elif lo == hi:
                buckets = [[lo - 0.5, hi + 0.5, total]]
            else:
                edges = np.linspace(lo, hi, bucket_count + 1)
                buckets = [[float(edges[k]), float(edges[k + 1]), counts[k]] for k in range(bucket_count)]
            with open(os.path.join(path, "%s.jsonl" % name), "a") as f:
                f.write(json.dumps({"step": step, "buckets": buckets}) + "\n")

    def _save_checkpoint(self, status=None):
        """``CheckpointManager(max_to_keep=1).save()`` (``BaseModel.py:248-253``).

        Single device: the weights are copied into pinned host buffers on the
        step stream (ordered before the next batch's updates) and a writer
        thread waits for that copy and writes the file, so the next epoch's
        batches are issued without waiting for the disk. Every reader of the
        file (restore, the end of ``train``) joins the writer first.
        ``status`` (device float [1], optional): the epoch's step status word,
        copied beside the weights; the writer keeps the previous checkpoint
        when it is nonzero (the epoch failed)."""
        os.makedirs(self.log_path, exist_ok=True)
        path = os.path.join(self.log_path, "ckpt.pt")
        self.sync_weights()   # multi-GPU: the shards are the authoritative entity rows (collective)
        if _world_size() > 1:
            if _is_rank0():
                torch.save({k: v.detach().cpu() for k, v in self.model_weights.items()}, path)
            torch.distributed.barrier()   # the file exists before any rank may restore it
            return path
        self._join_checkpoint()   # (its buffers are reused below)
        on_gpu = all(v.is_cuda for v in self.model_weights.values())
        if not on_gpu:
            torch.save({k: v.detach().cpu() for k, v in self.model_weights.items()}, path)
            return path
        bufs = self.__dict__.setdefault("_ckpt_bufs", {})
        snap = {}
        for k, v in self.model_weights.items():
            b = bufs.get(k)
            if b is None or b.shape != v.shape or b.dtype != v.dtype:
                b = bufs[k] = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
            b.copy_(v.detach(), non_blocking=True)
            snap[k] = b
        st_host = None
        if status is not None:
            st_host = bufs.get("_status")
            if st_host is None:
                st_host = bufs["_status"] = torch.empty(1, dtype=torch.float32, pin_memory=True)
            st_host.copy_(status, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()

        def write():
            ev.synchronize()
            if st_host is not None and float(st_host[0]) != 0.0:
                return   # a failed epoch: the last good checkpoint stays
            # a whole file or none: written beside, then renamed onto ckpt.pt
            # (a reader never sees a half-written checkpoint)
            torch.save(snap, path + ".tmp")
            os.replace(path + ".tmp", path)

        import threading
        # not a daemon: an exiting interpreter waits for the file
        self._ckpt_thread = threading.Thread(target=write)
        self._ckpt_thread.start()
        return path

    def _join_checkpoint(self):
        t = self.__dict__.pop("_ckpt_thread", None)
        if t is not None:
            t.join()

    def _restore_checkpoint(self):
        self._join_checkpoint()
        path = os.path.join(self.log_path, "ckpt.pt")
        saved = torch.load(path, weights_only=True)
        with torch.no_grad():
            for k, v in saved.items():
                self.model_weights[k].copy_(v.to(self.model_weights[k].device))
        if self._fused is not None and hasattr(self._fused, "load"):
            self._fused.load(saved)   # multi-GPU: into every rank's shard

    def _check_early_stopping(self, metric_history, magnitude, patience_now, patience_max, step,
                              restore_best_weight=True):
        """``BaseModel.py:485-540``."""
        if step == 0:
            self._save_checkpoint()
            self.best_step = step
            return False, patience_now
        assert magnitude in ["larger", "smaller"], "magnitude must be 'larger' or 'smaller'"
        if self.best_step is None:
            self.best_step = step
        if magnitude == "larger":
            flag = metric_history[step] >= metric_history[self.best_step]
        else:
            flag = metric_history[step] <= metric_history[self.best_step]
        if flag:
            patience_now += 1
        else:
            patience_now = 0
            self.best_step = step
            self._save_checkpoint()
        if patience_now == patience_max:
            if restore_best_weight:
                self._restore_checkpoint()
            return True, patience_now
        return False, patience_now

    def _log_embeddings_projector(self, log_path):
        """Projector artefacts (``BaseModel.py:542-576``) as TSV files."""
        def write(path, rows):
            with open(path, "w") as f:
                for x in rows:
                    f.write("{}\n".format(x))
        write(os.path.join(log_path, "ent_metadata.tsv"), self.metadata["ind2ent"])
        ent = self.model_weights["ent_emb"].detach().cpu().reshape(len(self.metadata["ind2ent"]), -1).numpy()
        np.savetxt(os.path.join(log_path, "ent_emb.tsv"), ent, delimiter="\t")
        if self.model_weights.get("rel_emb") is not None:
            write(os.path.join(log_path, "rel_metadata.tsv"), self.metadata["ind2rel"])
            rel = self.model_weights["rel_emb"].detach().cpu().reshape(len(self.metadata["ind2rel"]), -1).numpy()
            np.savetxt(os.path.join(log_path, "rel_emb.tsv"), rel, delimiter="\t")

    # ------------------------------------------------------------ evaluation
    def evaluate(self, eval_X, corrupt_side, positive_X=None):
        """``BaseModel.py:578-618``."""
        X = np.asarray(eval_X) if not isinstance(eval_X, torch.Tensor) else eval_X.cpu().numpy()
        from ... import engine, ranking
        if engine.backend() != "eager" and ranking.supported(self):
            # the whole set in one pass on the device (kge_rank); the int64 array
            # goes to the metrics as is (a list of numpy scalars made each metric
            # re-convert 17.5k objects: ~10 ms of host time per FB15k-237 side)
            ranks = ranking.batched_ranks(self, X, corrupt_side, positive_X)
        else:
            ranks = [self.get_rank(X[k], positive_X, corrupt_side) for k in range(len(X))]
        return {
            "mean_rank": mean_rank(ranks),
            "mean_reciprocal_rank": mean_reciprocal_rank(ranks),
            "median_rank": median_rank(ranks),
            "geometric_mean_rank": geometric_mean_rank(ranks),
            "harmonic_mean_rank": harmonic_mean_rank(ranks),
            "std_rank": std_rank(ranks),
            "hit@1": hits_at_k(ranks, k=1),
            "hit@3": hits_at_k(ranks, k=3),
            "hit@10": hits_at_k(ranks, k=10),
        }

    def get_rank(self, x, positive_X, corrupt_side):
        """Rank of one triple among all corruptions (``BaseModel.py:620-654``):
        ``sum(scores > pos_score) + 1`` with filtered positives set to -inf."""
        x = np.asarray(x.cpu() if isinstance(x, torch.Tensor) else x).reshape(-1)
        with torch.no_grad():
            if corrupt_side == "h":
                filter_side, corrupt = 2, 0
                scores = self.score_hrt(h=None, r=x[1], t=x[2])
            elif corrupt_side == "t":
                filter_side, corrupt = 0, 2
                scores = self.score_hrt(h=x[0], r=x[1], t=None)
            else:
                raise ValueError("corrupt_side must be 'h' or 't'")
            scores = scores.reshape(-1).clone()
            if positive_X is not None:
                P = np.asarray(positive_X.cpu() if isinstance(positive_X, torch.Tensor) else positive_X)
                mask = (P[:, 1] == x[1]) & (P[:, filter_side] == x[filter_side])
                positive_e = torch.as_tensor(P[mask, corrupt].astype(np.int64), device=scores.device)
                scores[positive_e] = -np.inf
            pos_score = self.score_hrt(x[0:1], x[1:2], x[2:3]).reshape(())
            return np.int64(int(torch.sum(scores > pos_score).item()) + 1)

    def restore_model_weights(self, model_weights):
        """``BaseModel.py:656-666`` (argument checked)."""
        self._check_model_weights(model_weights)
        self.model_weights = model_weights
        self._to_device()
        self._fused = None
