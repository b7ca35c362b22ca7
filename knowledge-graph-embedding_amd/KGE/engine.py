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


def fused_plan(model, optimizer, batch_size=1):
    """Return None if (model, plugins, optimizer) run in ``kge_step`` for
    batches of ``batch_size`` triples, else a reason."""
    if backend() == "eager":
        return "KGE_BACKEND=eager"
    if getattr(model, "_fused_model_id", None) is None:
        return "%s has no fused kernel" % type(model).__name__
    if model._fused_model_id not in FUSED_MODELS:
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
    if optimizer is not None and not isinstance(optimizer, (_opt.SGD, _opt.Adam)):
        return "%s optimizer has no fused apply" % type(optimizer).__name__
    return _native_plan_error(model, optimizer, batch_size)


def _native_plan_error(model, optimizer, batch_size=1):
    """Ask the library whether it has an instance for this combination
    (``kge_step_workspace_bytes`` is 0 for a plan it cannot run, with the
    reason in ``kge_last_error``: rows wider than the fragment limit, LDS
    budget, RESCAL without its regulariser, 32-bit destination codes, ...),
    with the real batch size and the optimizer's step mode (SGD in-step, Adam
    as KGE_OPT_GRAD). Cached per configuration."""
    try:
        t = model._fused_tables()
    except (AttributeError, KeyError):
        return None
    if t["ent"].device.type != "cuda":
        return None      # FusedStep raises: the fused step needs the model on a GPU
    key = (int(batch_size), tuple(t["ent"].shape), tuple(t["rel"].shape), type(optimizer).__name__,
           model.negative_ratio,
           model.corrupt_side, bool(getattr(model, "constraint", False)),
           _score.fused_descriptor(model.score_fn) if hasattr(model, "score_fn") else None,
           _loss.fused_descriptor(model.loss_fn))
    cache = model.__dict__.setdefault("_native_plan_cache", {})
    if key not in cache:
        lib = _hip.lib()      # raises if libkge_hip.so is missing (no silent fallback)
        probe = FusedStep(model)
        dev = t["ent"].device
        B = max(int(batch_size), 1)
        batch = torch.zeros((B, 3), dtype=torch.int64, device=dev)
        train = optimizer is not None
        # the SGD descriptor, switched to the gradient mode for Adam: the plan
        # check reads no buffer, so non-null placeholders stand in for the
        # dense gradient outputs (a probe must not allocate E x cols floats)
        opt = optimizer if isinstance(optimizer, _opt.SGD) or not train else _opt.SGD(0.01)
        d = probe.describe(batch, train, opt, neg_ids=batch)
        if train and not isinstance(optimizer, _opt.SGD):
            d.optimizer = _hip.OPT_GRAD
            for i in range(4):
                d.grad_out[i] = 16
        if int(lib.kge_step_workspace_bytes(d)) == 0:
            cache[key] = "kge_step: " + lib.kge_last_error().decode(errors="replace")
        else:
            cache[key] = None
    return cache[key]


FUSED_MODELS = (_hip.MODEL_TRANSE, _hip.MODEL_DISTMULT, _hip.MODEL_ROTATE, _hip.MODEL_RESCAL, _hip.MODEL_TRANSR,
                _hip.MODEL_TRANSH, _hip.MODEL_TRANSD)


def fused_names(model):
    """model_weights keys of the fused step's tables, by role."""
    t = model._fused_tables()
    out = {}
    for role in ("ent", "rel", "ent_aux", "rel_aux"):
        x = t.get(role)
        if x is None:
            continue
        out[role] = next(k for k, w in model.model_weights.items() if w is x)
    return out


def _rows_cols(t):
    return int(t.shape[0]), int(t.numel() // max(int(t.shape[0]), 1))


class FusedStep:
    """Device buffers + descriptor for one model's ``kge_step`` calls.

    SGD runs entirely inside ``kge_step`` (sparse update in its second
    kernel). Adam runs ``kge_step`` in ``KGE_OPT_GRAD`` mode (dense
    duplicate-summed gradients + per-variable slice norm^2) followed by one
    ``kge_apply`` per variable (keras sparse Adam decays every row).
    ``grad_mode=True`` always stops after the gradients (multi-GPU exchange).
    """

    def __init__(self, model, grad_mode=False, tables=None):
        self.model = model
        self.tables = tables          # optional override of model._fused_tables()
        t = self._tables()
        dev = t["ent"].device
        if dev.type != "cuda":
            raise RuntimeError("the fused step needs the model on a GPU (got %s); set KGE_BACKEND=eager "
                               "for host-only runs" % dev)
        self.device = dev
        self.lib = _hip.lib()      # raises if libkge_hip.so is missing
        self.grad_mode = grad_mode
        self.loss_out = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss_accum = torch.zeros(1, dtype=torch.float32, device=dev)
        self.norm2 = torch.zeros(4, dtype=torch.float32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.workspace = torch.empty(0, dtype=torch.uint8, device=dev)
        self.grads = None
        self.batch_scale = 1.0
        self.cw_scale = 1.0           # multi-GPU: share of a full-table regulariser this rank adds
        self.flags = 0
        self.plane_fn = None          # optional: planes -> first plane (multi-GPU offsets)
        self.shard = None             # optional (G, shard_rows, global E): the tables are gathered shards
        self.names = fused_names(model) if tables is not None else None   # weight keys by role (Adam slots)
        # split step (KGE/sharded.py, KGE_FLAG_PHASE_*): rows >= remote_from get
        # their raw gradient in place; relation gradients into rel_grad_out;
        # the update pass skipped when *abort != 0
        self.remote_from = None
        self.rel_grad_out = None
        self.abort = None
        self.grad_row_offset = 0      # grad mode: entity gradient buffers start at this table row
        # owner-side scoring (KGE/sharded.py "owner"): {world, rank, batch, rows_from,
        # records, stats, stats_out, err, global_entities} of the kge_step_desc owner fields
        self.owner = None
        self._descs = {}              # call key -> (descriptor, plan signature)
        self._ws_sig = None

    def _tables(self):
        return self.tables if self.tables is not None else self.model._fused_tables()

    def grad_roles(self):
        """Variables of the step in grad_out / norm2_out order (kge_hip.h)."""
        t = self._tables()
        return [r for r in ("ent", "rel", "rel_aux", "ent_aux") if t.get(r) is not None]

    def grad_buffers(self):
        """Dense [rows, cols] gradient buffers of the step's tables (KGE_OPT_GRAD)."""
        if self.grads is None:
            t = self._tables()
            self.grads = [torch.zeros(_rows_cols(t[k]), dtype=torch.float32, device=self.device)
                          for k in self.grad_roles()]
        return self.grads

    def _opt_code(self, is_train, optimizer):
        if not is_train:
            return _hip.OPT_NONE
        if self.grad_mode or isinstance(optimizer, _opt.Adam):
            return _hip.OPT_GRAD
        return _hip.OPT_SGD

    def _planes(self):
        m = self.model
        n = 2 if m.corrupt_side == "h+t" else 1
        if self.plane_fn is not None:
            return self.plane_fn(m.ns_strategy, n)
        return m.ns_strategy.take_planes(n)

    def describe(self, batch, is_train, optimizer, neg_ids=None, pos_score=None, neg_score=None):
        m = self.model
        t = self._tables()
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
            d.sampler = m.ns_strategy.sampler_desc(d.idx_dtype, self.device, self._planes())
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
        d.constraint_weight = float(getattr(m, "constraint_weight", 0.0)) * self.cw_scale
        d.rotate_limit = float(t.get("limit", 0.0))
        d.optimizer = self._opt_code(is_train, optimizer)
        if d.optimizer == _hip.OPT_SGD:
            d.lr = optimizer.learning_rate
        d.clip_norm = 5.0
        d.flags = self.flags
        if self.shard is not None:
            d.shard_count, d.shard_rows, d.global_entities = self.shard
        if d.optimizer == _hip.OPT_GRAD:
            g = self.grad_buffers()
            slot = {"ent": 0, "rel": 1, "rel_aux": 2, "ent_aux": 3}
            for role, buf in zip(self.grad_roles(), g):
                off = self.grad_row_offset * buf.shape[1] * 4 if role in ("ent", "ent_aux") else 0
                # (KGE_FLAG_GRAD_ROWS_TOUCHED: the step writes rows >= the offset only)
                d.grad_out[slot[role]] = buf.data_ptr() - off
        elif self.rel_grad_out is not None:
            d.grad_out[1] = self.rel_grad_out.data_ptr()
        if self.remote_from is not None:
            d.remote_rows_from = int(self.remote_from)
        if self.abort is not None:
            d.abort_flag = self.abort.data_ptr()
        if self.owner is not None:
            o = self.owner
            d.owner_world, d.owner_rank, d.owner_batch = o["world"], o["rank"], o["batch"]
            d.owner_rows_from = o.get("rows_from", 0)
            d.global_entities = o.get("global_entities", 0)
            d.owner_key_capacity = int(o.get("key_capacity", 0))
            for f in ("records", "stats", "stats_out", "err", "flags_in", "flags_out", "sticky"):
                if o.get(f) is not None:
                    setattr(d, "owner_" + f, o[f].data_ptr())
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
                 prof_events=None, accum=None):
        """One step; ``accum`` (device float32 [1], optional) receives += the
        batch loss inside the step (the training loop's per-epoch sum: no
        per-batch host work), else the step's own ``loss_accum``."""
        if batch.device != self.device:
            batch = batch.to(self.device)
        if batch.dtype not in (torch.int32, torch.int64):
            batch = batch.to(torch.int64)
        if not batch.is_contiguous():
            batch = batch.contiguous()
        d = self._desc_for(batch, is_train, optimizer, neg_ids, pos_score, neg_score)
        d.prof_events = ctypes.cast(prof_events, ctypes.c_void_p) if prof_events is not None else None
        d.loss_accum = (accum if accum is not None else self.loss_accum).data_ptr()
        _hip.check(self.lib.kge_step(d, _hip.stream_handle(self.device)), "kge_step")
        if is_train and isinstance(optimizer, _opt.Adam) and not self.grad_mode:
            self.apply_adam(optimizer)
        return self.loss_out

    def _desc_for(self, batch, is_train, optimizer, neg_ids=None, pos_score=None, neg_score=None):
        """The cached descriptor of this call shape, its per-call pointers and
        sampler planes filled in; the workspace claimed for its plan."""
        m = self.model
        t = self._tables()
        key = (int(batch.shape[0]), batch.dtype, bool(is_train), id(optimizer),
               getattr(optimizer, "learning_rate", None), neg_ids is not None,
               pos_score is not None, neg_score is not None,
               tuple((t[r].data_ptr(), tuple(t[r].shape), t[r].stride(0)) if t.get(r) is not None else None
                     for r in ("ent", "rel", "ent_aux", "rel_aux")),
               tuple((g.data_ptr(), tuple(g.shape)) for g in self.grads) if self.grads is not None else None,
               id(m.ns_strategy), m.negative_ratio, m.corrupt_side, self.batch_scale, self.cw_scale, self.flags,
               float(getattr(m, "constraint_weight", 0.0)), self.remote_from, self.grad_row_offset,
               self.rel_grad_out.data_ptr() if self.rel_grad_out is not None else None,
               self.abort.data_ptr() if self.abort is not None else None,
               tuple(sorted((k, v.data_ptr() if torch.is_tensor(v) else v) for k, v in self.owner.items()))
               if self.owner is not None else None)
        hit = self._descs.get(key)
        if hit is not None:
            d, sig = hit
            d.pos = batch.data_ptr()
            if neg_ids is not None:
                d.neg_ids = neg_ids.data_ptr()
            else:
                d.sampler.offset = self._planes()
            if pos_score is not None:
                d.pos_score_out = pos_score.data_ptr()
            if neg_score is not None:
                d.neg_score_out = neg_score.data_ptr()
            if sig != self._ws_sig:   # another cached plan ran in between
                self._refuse_split_wipe(d)
                self.workspace.zero_()
                self._ws_sig = sig
        else:
            d = self.describe(batch, is_train, optimizer, neg_ids, pos_score, neg_score)
            need = int(self.lib.kge_step_workspace_bytes(d))
            if need == 0:   # invalid descriptor: kge_step re-validates and reports the status
                _hip.check(self.lib.kge_step(d, _hip.stream_handle(self.device)), "kge_step")
            sig = int(self.lib.kge_step_plan_signature(d))
            if self.workspace.numel() < need:
                # zero-filled once: the step's tickets / destination counters
                # live in the workspace and reset themselves between calls
                self.workspace = torch.zeros(need, dtype=torch.uint8, device=self.device)
                self._descs.clear()   # (they point at the old buffer)
            elif sig != self._ws_sig:
                # a different plan lays the workspace out differently (the
                # library would refuse the stamped buffer): zeros again
                self._refuse_split_wipe(d)
                self.workspace.zero_()
            self._ws_sig = sig
            d.workspace = self.workspace.data_ptr()
            d.workspace_bytes = self.workspace.numel()
            if len(self._descs) >= 8:
                self._descs.clear()
            self._descs[key] = (d, sig)   # (the split step alternates two descriptors)
        return d

    def _refuse_split_wipe(self, d):
        """A PHASE_UPDATE call consumes the lists its PHASE_SCORE call left in
        the workspace; a plan change in between (any descriptor field in the
        signature, flags included) would zero them and make the update a
        silent no-op."""
        if (d.flags & _hip.FLAG_PHASE_UPDATE) and self._ws_sig is not None:
            raise RuntimeError("split step: the PHASE_UPDATE descriptor's plan differs from its PHASE_SCORE "
                               "call's (every field but the phase flags must match)")

    def bind(self, batch, is_train, optimizer, accum=None):
        """A callable running this step again and again on ``batch``'s buffer
        (the training loop refills it in place; the sampler's planes advance
        per call), loss added into ``accum``: the descriptor, stream and entry
        point are resolved once, so a call is one ``kge_step`` (+ keras Adam's
        apply) with no per-batch key building. Call again after changing the
        model's tables, plugins or the optimizer's learning rate."""
        if batch.device != self.device or batch.dtype not in (torch.int32, torch.int64) or \
                not batch.is_contiguous():
            raise ValueError("bind: the batch buffer must be a contiguous int32 / int64 tensor on the step's device")
        ns = self.model.ns_strategy
        off = ns.offset
        d = self._desc_for(batch, is_train, optimizer)
        ns.offset = off   # (the lookup drew planes for a call that is not made)
        sig = self._ws_sig
        d.prof_events = None
        d.loss_accum = (accum if accum is not None else self.loss_accum).data_ptr()
        dref = ctypes.byref(d)
        step = self.lib.kge_step
        st = _hip.stream_handle(self.device)
        planes = self._planes
        adam = is_train and isinstance(optimizer, _opt.Adam) and not self.grad_mode

        def run(pos=None):
            """``pos``: the batch's device address when it is another buffer of
            the bound one's shape and dtype (the training loop's ring views)."""
            if self._ws_sig != sig:   # another plan used the workspace in between
                self.workspace.zero_()
                self._ws_sig = sig
            if pos is not None:
                d.pos = pos
            d.sampler.offset = planes()
            rc = step(dref, st)
            if rc:
                _hip.check(rc, "kge_step")
            if adam:
                self.apply_adam(optimizer)
            return self.loss_out
        return run

    def _apply_desc(self, var, grad, norm2_ptr, optimizer, name, abort):
        a = _hip.kge_apply_desc()
        if abort is not None:
            a.abort_flag = abort.data_ptr()
        a.var = _hip.table(var)
        a.grad = grad.data_ptr()
        a.norm2 = norm2_ptr
        a.lr = optimizer.learning_rate
        a.clip_norm = 5.0
        if isinstance(optimizer, _opt.Adam):
            st = optimizer.slots.setdefault(name, {"m": torch.zeros_like(var), "v": torch.zeros_like(var)})
            a.optimizer = _hip.OPT_ADAM
            a.m = st["m"].data_ptr()
            a.v = st["v"].data_ptr()
            a.beta_1, a.beta_2, a.epsilon = optimizer.beta_1, optimizer.beta_2, optimizer.epsilon
            a.iteration = optimizer.iterations
        else:
            a.optimizer = _hip.OPT_SGD
        return a

    def apply(self, var, grad, norm2_ptr, optimizer, name=None, abort=None):
        """``kge_apply`` of one variable (SGD or keras Adam) with global norm^2
        at ``norm2_ptr``; nothing applied when ``abort`` (device float [1]) is nonzero."""
        a = self._apply_desc(var, grad, norm2_ptr, optimizer, name, abort)
        _hip.check(self.lib.kge_apply(a, _hip.stream_handle(self.device)), "kge_apply")

    def apply_many(self, items, optimizer, abort=None):
        """``kge_apply_many``: [(var, grad, norm2_ptr, name)] (up to 4) in one launch."""
        items = [it for it in items if it[0].numel() > 0]
        for i in range(0, len(items), 4):
            chunk = items[i:i + 4]
            arr = (_hip.kge_apply_desc * len(chunk))(*[self._apply_desc(v, g, n, optimizer, nm, abort)
                                                       for v, g, n, nm in chunk])
            _hip.check(self.lib.kge_apply_many(arr, len(chunk), _hip.stream_handle(self.device)), "kge_apply_many")

    def apply_adam(self, optimizer):
        optimizer.iterations += 1
        t = self._tables()
        names = self.names or fused_names(self.model)
        g = self.grad_buffers()
        slot = {"ent": 0, "rel": 1, "rel_aux": 2, "ent_aux": 3}
        self.apply_many([(t[role], buf, self.norm2.data_ptr() + 4 * slot[role], names[role])
                         for role, buf in zip(self.grad_roles(), g)], optimizer)

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


def eager_grads(model, batch, is_train, neg=None, batch_scale=1.0):
    """Steps 1-5 of the reference step (BaseModel.py:316-326) with TF-2.5
    gradient semantics. Returns (loss, {name: ("dense", g) | ("slices", idx, values)});
    the gradient dict is empty for a validation step."""
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
            return batch_loss.detach().reshape(()), {}
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
    out = {}
    for name in names:
        sl = slices.get(name, [])
        dg = dense.get(name)
        if dg is None and not sl:
            continue
        if dg is not None:
            total = dg.clone()
            for idx, g in sl:
                total.index_add_(0, idx, g)
            out[name] = ("dense", total)
        else:
            out[name] = ("slices", torch.cat([i for i, _ in sl]), torch.cat([g for _, g in sl]))
    return batch_loss.detach().reshape(()), out


def grad_norm2(g):
    """Squared L2 norm clip_by_norm sees: over the slice values (not de-duplicated)."""
    x = g[1] if g[0] == "dense" else g[2]
    return torch.sum(x * x)


def dense_grad(g, like):
    """Duplicate-summed dense gradient of a variable shaped like ``like``."""
    if g[0] == "dense":
        return g[1]
    return torch.zeros_like(like).index_add_(0, g[1], g[2])


def eager_step(model, batch, is_train, optimizer, neg=None, batch_scale=1.0):
    """Reference step order (BaseModel.py:316-328) with TF-2.5 gradient semantics."""
    loss, grads = eager_grads(model, batch, is_train, neg, batch_scale)
    if not is_train:
        return loss
    if isinstance(optimizer, _opt.Adam):
        optimizer.iterations += 1
    for name, g in grads.items():
        w = model.model_weights[name]
        n2 = grad_norm2(g)
        scale = 5.0 / torch.maximum(_sqrt_or_zero(n2), torch.tensor(5.0, device=w.device))
        if g[0] == "dense":
            _apply(name, w, optimizer, dense=g[1] * scale)
        else:
            _apply(name, w, optimizer, idx=g[1], values=g[2] * scale)
    return loss


def _sqrt_or_zero(l2):
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
