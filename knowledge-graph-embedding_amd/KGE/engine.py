"""Step execution: the fused HIP step and the eager plugin path.

``KGEModel._run_single_batch`` (reference ``BaseModel.py:293-330``) calls
``run_step``. Built-in model + score + loss + sampler + SGD combinations run
as ONE call into ``libkge_hip.so`` (``kge_step``: sampling, gather, score,
loss, gradient, per-variable clip, sparse SGD update), on the current HIP
stream, with no host synchronisation. If such a combination is requested on a
GPU and the library is missing, this raises -- there is no silent fallback.

The eager path (torch autograd on the model's device, with the reference's
TF-2.5 IndexedSlices / clip_by_norm / optimizer semantics) runs:
  * user-defined Score / Loss / NegativeSampler subclasses and the models
    outside the fused scope (UM, SE, and those not yet fused),
  * everything when ``KGE_BACKEND=eager`` (host-side development and the CPU
    test-suite of the host logic).
"""

import ctypes
import os
import warnings

import torch

from . import _hip
from . import loss as _loss
from . import ns_strategy as _ns
from . import optimizers as _opt
from . import score as _score


def backend():
    return os.environ.get("KGE_BACKEND", "fused").lower()


def device():
    """Device new models live on: ``cuda:LOCAL_RANK`` when a GPU exists."""
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    return torch.device("cpu")


# ---------------------------------------------------------------- fused
_SIDE = {"h": _hip.SIDE_H, "t": _hip.SIDE_T, "h+t": _hip.SIDE_HT}


def fused_plan(model, optimizer):
    """Return None if (model, plugins, optimizer) run in ``kge_step``, else a reason."""
    if backend() == "eager":
        return "KGE_BACKEND=eager"
    if getattr(model, "_fused_model_id", None) is None:
        return "%s has no fused kernel" % type(model).__name__
    if model._fused_model_id not in (_hip.MODEL_TRANSE, _hip.MODEL_DISTMULT, _hip.MODEL_ROTATE):
        return "%s has no fused kernel in this build" % type(model).__name__
    if hasattr(model, "score_fn"):
        sd = _score.fused_descriptor(model.score_fn)
        if sd is None:
            return "custom score function"
        if model._fused_model_id == _hip.MODEL_ROTATE and sd[0] == _score.SCORE_DOT:
            return "RotatE + Dot (complex score)"
    if _loss.fused_descriptor(model.loss_fn) is None:
        return "custom loss function"
    if type(model.ns_strategy) not in (_ns.UniformStrategy, _ns.TypedStrategy):
        return "custom negative sampler"
    if optimizer is not None and not isinstance(optimizer, _opt.SGD):
        return "%s optimizer is not fused yet" % type(optimizer).__name__
    return None


class FusedStep:
    """Device buffers + descriptor for one model's ``kge_step`` calls."""

    def __init__(self, model):
        self.model = model
        dev = model.model_weights["ent_emb"].device
        if dev.type != "cuda":
            raise RuntimeError("the fused step needs the model on a GPU (got %s); set KGE_BACKEND=eager "
                               "for host-only runs" % dev)
        self.device = dev
        self.lib = _hip.lib()      # raises if libkge_hip.so is missing
        self.loss_out = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss_accum = torch.zeros(1, dtype=torch.float32, device=dev)
        self.norm2 = torch.zeros(4, dtype=torch.float32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.workspace = torch.empty(0, dtype=torch.uint8, device=dev)
        self.batch_scale = 1.0

    def describe(self, batch, is_train, optimizer, neg_ids=None, pos_score=None, neg_score=None):
        m = self.model
        t = m._fused_tables()
        d = _hip.kge_step_desc()
        d.abi_version = _hip.ABI_VERSION
        d.model = m._fused_model_id
        d.ent = _hip.table(t["ent"])
        d.rel = _hip.table(t["rel"])
        if t.get("ent_aux") is not None:
            d.ent_aux = _hip.table(t["ent_aux"])
        if t.get("rel_aux") is not None:
            d.rel_aux = _hip.table(t["rel_aux"])
        d.dim = t["dim"]
        d.dim_rel = t.get("dim_rel", t["dim"])
        d.pos = batch.data_ptr()
        d.idx_dtype = _hip.IDX_I64 if batch.dtype == torch.int64 else _hip.IDX_I32
        d.batch = int(batch.shape[0])
        d.negative_ratio = int(m.negative_ratio)
        d.corrupt_side = _SIDE[m.corrupt_side]
        if neg_ids is not None:
            d.sampler.kind = _hip.SAMPLER_GIVEN
            d.sampler.idx_dtype = d.idx_dtype
            d.neg_ids = neg_ids.data_ptr()
        else:
            planes = 2 if m.corrupt_side == "h+t" else 1
            plane = m.ns_strategy.take_planes(planes)
            d.sampler = m.ns_strategy.sampler_desc(d.idx_dtype, self.device, plane)
        if hasattr(m, "score_fn"):
            kind, p = _score.fused_descriptor(m.score_fn)
        else:
            kind, p = _score.SCORE_DOT, 0.0
        d.score_kind = kind
        d.score_p = p
        lk, margin, temp = _loss.fused_descriptor(m.loss_fn)
        d.loss_kind = lk
        d.margin = margin
        d.temperature = temp
        d.batch_scale = self.batch_scale
        d.constraint = int(bool(getattr(m, "constraint", False)))
        d.constraint_weight = float(getattr(m, "constraint_weight", 0.0))
        d.rotate_limit = float(t.get("limit", 0.0))
        if is_train:
            d.optimizer = _hip.OPT_SGD
            d.lr = optimizer.learning_rate
        else:
            d.optimizer = _hip.OPT_NONE
        d.clip_norm = 5.0
        d.loss_out = self.loss_out.data_ptr()
        d.loss_accum = self.loss_accum.data_ptr()
        d.norm2_out = self.norm2.data_ptr()
        d.status = self.status.data_ptr()
        if pos_score is not None:
            d.pos_score_out = pos_score.data_ptr()
        if neg_score is not None:
            d.neg_score_out = neg_score.data_ptr()
        return d

    def __call__(self, batch, is_train, optimizer, neg_ids=None, pos_score=None, neg_score=None,
                 prof_events=None):
        if batch.device != self.device:
            batch = batch.to(self.device)
        if batch.dtype not in (torch.int32, torch.int64):
            batch = batch.to(torch.int64)
        if not batch.is_contiguous():
            batch = batch.contiguous()
        m = self.model
        key = (int(batch.shape[0]), batch.dtype, bool(is_train), id(optimizer),
               getattr(optimizer, "learning_rate", None), neg_ids is not None,
               pos_score is not None, neg_score is not None, m.model_weights["ent_emb"].data_ptr(),
               id(m.ns_strategy), m.negative_ratio, m.corrupt_side)
        cached = getattr(self, "_cache", None)
        if cached is not None and cached[0] == key:
            d = cached[1]
            d.pos = batch.data_ptr()
            if neg_ids is not None:
                d.neg_ids = neg_ids.data_ptr()
            else:
                d.sampler.offset = m.ns_strategy.take_planes(2 if m.corrupt_side == "h+t" else 1)
            if pos_score is not None:
                d.pos_score_out = pos_score.data_ptr()
            if neg_score is not None:
                d.neg_score_out = neg_score.data_ptr()
        else:
            d = self.describe(batch, is_train, optimizer, neg_ids, pos_score, neg_score)
            need = int(self.lib.kge_step_workspace_bytes(d))
            if need == 0:   # invalid descriptor: kge_step re-validates and reports the status
                _hip.check(self.lib.kge_step(d, _hip.stream_handle(self.device)), "kge_step")
            if self.workspace.numel() < need:
                self.workspace = torch.empty(need, dtype=torch.uint8, device=self.device)
            d.workspace = self.workspace.data_ptr()
            d.workspace_bytes = self.workspace.numel()
            self._cache = (key, d)
        d.prof_events = ctypes.cast(prof_events, ctypes.c_void_p) if prof_events is not None else None
        _hip.check(self.lib.kge_step(d, _hip.stream_handle(self.device)), "kge_step")
        return self.loss_out

    def check_status(self):
        _hip.check_device_status(self.status, "kge_step")


# ---------------------------------------------------------------- eager
class Tape:
    """Records every embedding lookup as its own leaf so gradients come back
    per lookup, i.e. as TF IndexedSlices (values not de-duplicated)."""

    def __init__(self):
        self.records = []   # (name, flat idx, leaf)


def _apply(name, w, opt, idx=None, values=None, dense=None):
    """Optimizer apply for one variable (keras SGD / Adam semantics)."""
    with torch.no_grad():
        if isinstance(opt, _opt.SGD):
            if dense is not None:
                w.add_(dense * (-opt.learning_rate))
            else:
                w.index_add_(0, idx, values * (-opt.learning_rate))
            return
        # Adam
        st = opt.slots.setdefault(name, {"m": torch.zeros_like(w), "v": torch.zeros_like(w)})
        t = opt.iterations
        b1, b2 = opt.beta_1, opt.beta_2
        lr_t = opt.learning_rate * (1 - b2 ** t) ** 0.5 / (1 - b1 ** t)
        m, v = st["m"], st["v"]
        if dense is not None:
            m.add_((dense - m) * (1 - b1))
            v.add_((dense * dense - v) * (1 - b2))
        else:
            g = torch.zeros_like(w).index_add_(0, idx, values)
            uniq = torch.unique(idx)
            gu = g.index_select(0, uniq)
            m.mul_(b1).index_add_(0, uniq, gu * (1 - b1))
            v.mul_(b2).index_add_(0, uniq, (gu * gu) * (1 - b2))
        w.sub_(lr_t * m / (torch.sqrt(v) + opt.epsilon))


def eager_step(model, batch, is_train, optimizer, neg=None, batch_scale=1.0):
    """Reference step order (BaseModel.py:316-328) with TF-2.5 gradient semantics."""
    weights = model.model_weights
    if neg is None:
        neg = model._negative_sampling(batch)
    tape = Tape()
    model._tape = tape if is_train else None
    model._batch_scale = batch_scale
    try:
        if is_train:
            for w in weights.values():
                w.requires_grad_(True)
        with torch.set_grad_enabled(is_train):
            constraint_term = model._constraint_loss(batch)
            pos_score = model.score_hrt(batch[:, 0], batch[:, 1], batch[:, 2])
            neg_score = model.score_hrt(neg[:, 0], neg[:, 1], neg[:, 2])
            batch_loss = _call_loss(model.loss_fn, pos_score, neg_score, batch_scale) + constraint_term
        if not is_train:
            return batch_loss.detach().reshape(())
        names = list(weights.keys())
        params = [weights[n] for n in names]
        leaves = [r[2] for r in tape.records]
        grads = torch.autograd.grad(batch_loss, params + leaves, allow_unused=True)
        dense = dict(zip(names, grads[:len(names)]))
        slices = {}
        for (name, idx, _), g in zip(tape.records, grads[len(names):]):
            if g is None:
                continue
            slices.setdefault(name, []).append((idx, g))
    finally:
        model._tape = None
        for w in weights.values():
            w.requires_grad_(False)
    if isinstance(optimizer, _opt.Adam):
        optimizer.iterations += 1
    for name in names:
        w = weights[name]
        sl = slices.get(name, [])
        dg = dense.get(name)
        if dg is None and not sl:
            continue
        if dg is not None:
            total = dg.clone()
            for idx, g in sl:
                total.index_add_(0, idx, g)
            total = total * 5.0 / torch.maximum(_norm_or_zero(total), torch.tensor(5.0, device=total.device))
            _apply(name, w, optimizer, dense=total)
        else:
            idx = torch.cat([i for i, _ in sl])
            vals = torch.cat([g for _, g in sl])
            vals = vals * 5.0 / torch.maximum(_norm_or_zero(vals), torch.tensor(5.0, device=vals.device))
            _apply(name, w, optimizer, idx=idx, values=vals)
    return batch_loss.detach().reshape(())


def _norm_or_zero(x):
    l2 = torch.sum(x * x)
    return torch.where(l2 > 0, torch.sqrt(torch.where(l2 > 0, l2, torch.ones_like(l2))), l2)


def _call_loss(loss_fn, pos, neg, batch_scale):
    if batch_scale != 1.0 and type(loss_fn) in (_loss.PairwiseHingeLoss, _loss.BinaryCrossEntropyLoss,
                                                 _loss.SelfAdversarialNegativeSamplingLoss,
                                                 _loss.SquareErrorLoss, _loss.PairwiseLogisticLoss):
        return loss_fn(pos, neg, batch_scale=batch_scale)
    return loss_fn(pos, neg)


_warned = set()


def warn_once(key, msg):
    if key not in _warned:
        _warned.add(key)
        warnings.warn(msg, stacklevel=3)
