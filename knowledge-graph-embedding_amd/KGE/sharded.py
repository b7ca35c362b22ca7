"""Multi-GPU training step: data-parallel over triples.

The reference is single-device (``BaseModel.py:19-21``); this is the build's
one parallel strategy. One process per GPU,
``torch.distributed`` with the RCCL backend ("nccl" on ROCm) over xGMI.

Two exchanges, chosen by the entity table's size ("auto": dense up to 1 GiB):

* ``dense`` (FB15k-237 scale, where a step touches every row anyway): every
  rank keeps the whole table (identical replicas). A step is ``kge_step`` in
  ``KGE_OPT_GRAD`` mode on the local batch (in-register draws from
  rank-disjoint counter planes, loss normalised by the GLOBAL batch), then ONE
  ``all_reduce`` of one buffer [entity gradients | relation gradients |
  norm^2 x4 | loss], then the same clip + SGD / Adam apply on every rank
  (ring all-reduce hands every rank the same sums, so the replicas stay
  bit-identical). One collective per step, no gather.
* ``sparse`` (tables > 1 GiB, C5): the entity rows are sharded, row ``e`` on
  rank ``e mod G`` at local row ``e div G`` (modulo keeps FB15k-237's degree
  load within 1.05x at G = 8; id blocks give 2.24x because ``index_kg``
  numbers entities in first-appearance order). The entity tables of a model
  (``ent_emb``, TransD's ``ent_proj``) share one ``shard`` buffer, row =
  [ent | ent_aux]. Relation tables are replicated.

One sparse step (``ShardedStep.__call__``), every rank with its own B positives:
  0. ``_constraint_loss`` assigns on the owned rows (TransE / DistMult
     renormalise, TransR / TransD clip; ``BaseModel.py:319`` order) and on the
     replicated relation tables;
  1. negatives drawn with ``kge_sample`` from rank-disjoint counter planes;
  2. exchange the rows the batch needs into a local row cache: sort + unique
     of the batch's ids, one ``all_to_all_single`` of per-owner counts, one of
     the ids, the owners gather their rows, one ``all_to_all_single`` of the
     rows back -- the cache holds exactly the unique rows, in request order;
  3. ``kge_step`` in ``KGE_OPT_GRAD`` mode on the cache (ids remapped to cache
     rows, negatives given): gather, score, loss normalised by the GLOBAL
     batch (``batch_scale = G``), duplicate-summed gradient rows of the cache,
     per-variable slice norm^2;
  4. one ``all_reduce`` of [relation gradients | norm^2 x4 | loss];
  5. the cache's gradient rows go back to their owners (``all_to_all_single``
     with the request splits reversed);
  6. owners sum each row's contributions in source-rank order (unique indices
     per source: deterministic) and apply clip_by_norm with the global norm
     + SGD on the touched rows only (``kge_apply_rows``; Adam: dense keras
     Adam over the shard, ``kge_apply``); the replicated relation tables get
     the same ``kge_apply`` on every rank.
G ranks x B positives compute the step one device computes on the
concatenated G*B batch with the same negatives (up to float summation order).
"""

import ctypes
import math

import numpy as np
import torch
import torch.distributed as dist

from . import _hip
from . import engine
from . import optimizers as _opt
from .constraint import clip_constraint, normalized_embeddings

_RENORM = (_hip.MODEL_TRANSE, _hip.MODEL_DISTMULT)
_SPLIT = (_hip.MODEL_TRANSE, _hip.MODEL_DISTMULT, _hip.MODEL_ROTATE)   # the split (two-pass) SGD step
_CLIP = (_hip.MODEL_TRANSR, _hip.MODEL_TRANSD)
DENSE_TABLE_BYTES = 1 << 30   # "auto": replicated tables + one all-reduce below this entity-table size


class Exchange:
    """The step's collectives on one process group (tensor forms on RCCL; the
    gloo CPU tests of this logic get list forms with the same results). A
    gloo group given device tensors stages them through host memory (the
    multi-process tests that put several ranks on one GPU)."""

    def __init__(self, group=None, force=False):
        """``force``: issue every collective even on a one-rank group (the
        RCCL tensor forms then run as copies -- a one-GPU test of the N-rank
        code path)."""
        self.group = group
        self.force = bool(force)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.tensor_forms = dist.get_backend(group) == "nccl"

    def _host(self, t):
        return t.cpu() if (not self.tensor_forms and t.is_cuda) else t

    def all_gather(self, full, shard):
        if self.tensor_forms:
            dist.all_gather_into_tensor(full, shard, group=self.group)
            return
        f = self._host(full)
        dist.all_gather(list(f.chunk(self.world)), self._host(shard), group=self.group)
        if f is not full:
            full.copy_(f)

    def all_reduce(self, t):
        if self.world == 1 and not self.force:   # (one rank: the sum is the tensor itself)
            return
        h = self._host(t)
        dist.all_reduce(h, group=self.group)
        if h is not t:
            t.copy_(h)

    def all_to_all(self, out, inp, out_splits=None, in_splits=None):
        o = self._host(out)
        dist.all_to_all_single(o, self._host(inp.contiguous()), out_splits, in_splits, group=self.group)
        if o is not out:
            out.copy_(o)


class ShardedStep:
    """Drop-in for ``FusedStep`` across G ranks (see module docstring)."""

    def __init__(self, model, exchange=None, mode="auto", local_fast=True, loopback=False, capacity_slack=1.1,
                 capacity_floor=1024, batch_hint=None, optimizer=None, force_collectives=False):
        """``loopback`` (sparse mode): own ids too go through the exchange blocks
        (a one-GPU rehearsal of the remote path). Each owner block holds
        ceil(capacity_slack * occurrences / G) + capacity_floor rows; a step
        whose ids overflow a block is skipped on every rank and reported by
        the next check_status() (a sticky device flag, read and cleared
        there); a skipped step still advances keras Adam's iteration count
        (``optimizer.iterations``, hence lr_t), as the host counts steps
        before the device knows of the overflow. ``batch_hint`` (positives per rank per step) sizes the
        exchange blocks up front, so the owned rows are allocated once, at the
        head of the extended table (no second copy of a shard that fills HBM).
        ``optimizer`` (the training optimizer, if known): "auto" takes owner-side
        scoring only for SGD, whose steps it covers (keras Adam trains through
        the row exchange); with it unknown, an owner-mode step sizes its
        buffers for both passes up front, so an Adam step falling through to
        the row exchange never re-plans a second copy of the shard. The owner
        pass's key capacity follows ``capacity_slack`` / ``capacity_floor``
        too (at least 5/4 of the expected owned negatives + 4096).
        ``force_collectives``: take the N-rank code path (separate send /
        receive buffers, every collective issued) even on one rank -- the
        RCCL world-1 tests' way to run the tensor-form collectives."""
        self.model = model
        self.ex = exchange or Exchange()
        if force_collectives:
            self.ex.force = True
        G, g = self.ex.world, self.ex.rank
        self.G, self.g = G, g
        self.multi = G > 1 or self.ex.force   # the N-rank code path
        t = model._fused_tables()
        self.tables = t
        self.names = engine.fused_names(model)
        ent = t["ent"]
        E = int(ent.shape[0])
        self.E = E
        self.ent_shape = tuple(ent.shape)
        self.ce = ent.numel() // E
        self.aux_shape = tuple(t["ent_aux"].shape) if t.get("ent_aux") is not None else None
        self.ca = t["ent_aux"].numel() // E if self.aux_shape else 0
        C = self.ce + self.ca
        self.C = C
        self.Es = -(-E // G)
        self.valid = len(range(g, E, G))
        dev = ent.device
        self.device = dev
        self.mid = model._fused_model_id
        # full-table regularisers (RESCAL.py:190-198, TransH.py:202-211 with
        # constraint) make TF's gradients dense: every rank adds 1/G of the
        # term (loss and gradient) to its replica's gradient, the all-reduce
        # sums them, and the clip norm is taken of the reduced dense tensor
        self.full_reg = self.mid == _hip.MODEL_RESCAL or (self.mid == _hip.MODEL_TRANSH and
                                                           bool(getattr(model, "constraint", False)))
        if mode == "auto":
            if E * C * 4 <= DENSE_TABLE_BYTES or self.full_reg:
                mode = "dense"
            else:
                owner_ok = optimizer is None or isinstance(optimizer, _opt.SGD)
                mode = "owner" if self.mid in _SPLIT and owner_ok else "sparse"
        if mode not in ("dense", "sparse", "owner"):
            raise ValueError("mode must be 'auto', 'dense', 'sparse' or 'owner'")
        if mode in ("sparse", "owner") and self.full_reg:
            raise NotImplementedError("sharded step: a full-table regulariser (RESCAL, TransH with constraint) "
                                      "has a dense gradient of every row -- use the dense exchange")
        if mode == "owner" and self.mid not in _SPLIT:
            raise NotImplementedError("owner-side scoring covers TransE, DistMult and RotatE")
        self.mode = mode
        self.debug_flags = 0   # test hooks (KGE_FLAG_DEBUG_*) for the owner merge's update pass
        self.loopback = bool(loopback)
        self.slack = float(capacity_slack)
        self.cap_floor = int(capacity_floor)
        self._ext = None
        self._needs_loop = False
        self._own = None
        if mode in ("sparse", "owner"):
            # owned rows [ent | ent_aux], padded to Es rows (on a GPU: the head of
            # the extended table, the fetched blocks follow -- _ext_for)
            if batch_hint and dev.type == "cuda":
                if mode == "owner":   # blocks for the positives' rows + every rank's positive rows
                    n = 2 * int(batch_hint)
                    if not isinstance(optimizer, _opt.SGD):   # (a keras Adam step runs the row exchange)
                        n = max(n, self._occurrences(int(batch_hint)))
                    self._ext_for(n, torch.int64, fill=False, pos_rows=2 * G * int(batch_hint))
                else:
                    self._ext_for(self._occurrences(int(batch_hint)), torch.int64, fill=False)
            else:
                self.shard = torch.zeros(self.Es, C, dtype=torch.float32, device=dev)
            self.shard[:self.valid, :self.ce] = ent.reshape(E, -1)[g::G]
            if self.ca:
                self.shard[:self.valid, self.ce:] = t["ent_aux"].reshape(E, -1)[g::G]
        # the all-reduce buffer: [entity gradients (dense mode) | relation
        # gradients | norm^2 x4 | loss]
        self.rel_roles = [r for r in ("rel", "rel_aux") if t.get(r) is not None]
        ent_sizes = [E * c for c in self._ecols()] if mode == "dense" else []   # (sparse / owner: none)
        sizes = [t[r].numel() for r in self.rel_roles]
        self.red = torch.zeros(sum(ent_sizes) + sum(sizes) + 8, dtype=torch.float32, device=dev)
        o = 0
        self.gent = []
        for n, c in zip(ent_sizes, self._ecols()):
            self.gent.append(self.red[o:o + n].view(E, c))
            o += n
        self.grel = {}
        for r, n in zip(self.rel_roles, sizes):
            self.grel[r] = self.red[o:o + n].view(t[r].shape[0], -1)
            o += n
        self.norm2 = self.red[o:o + 4]
        self.loss = self.red[o + 4:o + 5]
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        # sticky overflow flags [exchange block, owner pass]: the max of every
        # step's all-reduced flags since check_status() last read them (no host
        # sync per step)
        self.xerr = torch.zeros(2, dtype=torch.float32, device=dev)
        c = getattr(model, "constraint", False)
        self.renorm = self.mid in _RENORM and bool(c)
        self.clip = self.mid in _CLIP and bool(c)
        self.hyper = self.mid == _hip.MODEL_TRANSH and bool(c)
        self.fused = None
        self._cap = 0
        if dev.type == "cuda":
            self.lib = _hip.lib()
            f = engine.FusedStep(model, grad_mode=True, tables=dict(t))
            f.norm2 = self.norm2
            f.loss_out = self.loss
            f.status = self.status
            f.batch_scale = float(G)
            if self.full_reg:
                f.cw_scale = 1.0 / G
            f.flags = _hip.FLAG_NO_TABLE_CONSTRAINT
            if mode != "dense":   # every cache row [0, U) is a batch id: no gradient zero-fill
                f.flags |= _hip.FLAG_GRAD_ROWS_TOUCHED
            else:   # the replica, global ids, in-register draws from rank-disjoint planes
                f.plane_fn = lambda ns, n: ns.take_planes(n) * G + g * n
                if self.renorm:   # the renormalisation assign inside the step (no K0 pass)
                    f.flags = _hip.FLAG_GRAD_RENORM
            self.fused = f
        elif engine.backend() != "eager":
            raise RuntimeError("ShardedStep needs GPUs (or KGE_BACKEND=eager for host-only tests)")
        # one rank: every row is local, so the fused single-device step runs on
        # the shard itself (in-kernel SGD, compact update launch) -- no cache
        self.direct = None
        if self.fused is not None and not self.multi and mode != "dense" and local_fast and not self.loopback:
            td = dict(t)
            td["ent"] = self.shard[:, :self.ce].view(self.ent_shape)
            if self.ca:
                td["ent_aux"] = self.shard[:, self.ce:]
            self.direct = engine.FusedStep(model, tables=td)

    def _ecols(self):
        return [self.ce] + ([self.ca] if self.ca else [])

    def _ent_rows(self, k):
        """Dense mode: entity table k (0 ent_emb, 1 ent_proj) as [E, cols] rows."""
        return self.tables["ent" if k == 0 else "ent_aux"].view(self.E, -1)

    # ------------------------------------------------------------ phases
    def _constrain(self):
        """_constraint_loss assigns (BaseModel.py:319): owned entity rows, and
        the replicated relation tables identically on every rank (dense mode:
        the whole replica)."""
        rows = self.shard[:self.valid, :self.ce] if self.mode != "dense" else self._ent_rows(0)
        rel = self.tables["rel"]
        if self.fused is not None:
            st = _hip.stream_handle(self.device)
            # (dense mode: kge_step renormalises the replica itself, KGE_FLAG_GRAD_RENORM)
            if self.renorm and rows.shape[0] and self.mode != "dense":
                _hip.check(self.lib.kge_constrain_rows(_hip.table(rows), 0, 1.0, st), "kge_constrain_rows")
            if self.clip:
                if rows.shape[0]:
                    _hip.check(self.lib.kge_constrain_rows(_hip.table(rows), 1, 1.0, st), "kge_constrain_rows")
                _hip.check(self.lib.kge_constrain_rows(_hip.table(rel), 1, 1.0, st), "kge_constrain_rows")
            if self.hyper:
                _hip.check(self.lib.kge_constrain_rows(_hip.table(self.tables["rel_aux"]), 0, 1.0, st),
                           "kge_constrain_rows")
            return
        with torch.no_grad():
            if self.renorm and rows.shape[0]:
                rows.copy_(normalized_embeddings(rows, p=2, value=1, axis=1))
            if self.clip:
                rows.copy_(clip_constraint(rows, p=2, value=1, axis=-1))
                rel.copy_(clip_constraint(rel, p=2, value=1, axis=-1))
            if self.hyper:
                w = self.tables["rel_aux"]
                w.copy_(normalized_embeddings(w, p=2, value=1, axis=1))

    def _draw(self, batch):
        """Negatives in the step's slot layout (h+t: alternating h / t draws,
        BaseModel.py:353-356) from rank-disjoint planes (kge_sample)."""
        m = self.model
        ns = m.ns_strategy
        two = m.corrupt_side == "h+t"
        p0 = ns.take_planes(2 if two else 1) * self.G + self.g * (2 if two else 1)
        K = int(m.negative_ratio)
        Ks = K // 2 if two else K
        B = int(batch.shape[0])
        i64 = batch.dtype == torch.int64
        outs = []
        for k, side in enumerate(("h", "t") if two else (m.corrupt_side,)):
            out = torch.empty(B * Ks, dtype=batch.dtype, device=batch.device)
            d = _hip.kge_sample_desc()
            d.sampler = ns.sampler_desc(_hip.IDX_I64 if i64 else _hip.IDX_I32, batch.device, p0 + k)
            d.X = batch.data_ptr()
            d.n = B
            d.side = _hip.SIDE_H if side == "h" else _hip.SIDE_T
            d.negative_ratio = Ks
            d.out = out.data_ptr()
            d.status = self.status.data_ptr()
            _hip.check(self.lib.kge_sample(d, _hip.stream_handle(batch.device)), "kge_sample")
            outs.append(out)
        if not two:
            return outs[0]
        return torch.stack([outs[0].view(B, Ks), outs[1].view(B, Ks)], dim=-1).reshape(-1)

    def _fetch_sparse(self, ids):
        """Unique ids -> row cache + the remap of ``ids`` to cache rows. One
        sort: unique of the owner-major key (owner, id), so the cache order is
        the request order and the inverse index is the remap."""
        G, ex, E = self.G, self.ex, self.E
        key = (ids % G) * E + ids if G > 1 else ids
        uniq, inv = torch.unique(key, return_inverse=True)
        U = int(uniq.shape[0])
        cache = self._cache_buf(U)
        if G == 1:   # every row is local: gather straight into the cache
            torch.index_select(self.shard, 0, uniq, out=cache[:U])
            return cache, inv, (None, None, uniq)
        own = torch.div(uniq, E, rounding_mode="floor")
        req = uniq - own * E
        send = torch.bincount(own, minlength=G)
        recv = torch.empty_like(send)
        ex.all_to_all(recv, send)
        sc, rc = send.tolist(), recv.tolist()
        rids = torch.empty(sum(rc), dtype=req.dtype, device=req.device)
        ex.all_to_all(rids, req, rc, sc)
        rows = torch.index_select(self.shard, 0, torch.div(rids, G, rounding_mode="floor"))
        ex.all_to_all(cache[:U], rows, sc, rc)
        return cache, inv, (sc, rc, rids)

    def _cache_buf(self, U):
        """The row cache at a FIXED capacity (the kernel's table shape, hence
        its plan and workspace layout, stays the same from step to step):
        rows [0, U) hold this step's unique rows, the rest are never referenced."""
        if U > self._cap:
            m = self.model
            keff = 2 * (int(m.negative_ratio) // 2) if m.corrupt_side == "h+t" else int(m.negative_ratio)
            self._cap = max(U, min(self.E, self._bmax * (keff + 2)))
            self._cache = torch.zeros(self._cap, self.C, dtype=torch.float32, device=self.device)
            self._gcache = [torch.zeros(self._cap, c, dtype=torch.float32, device=self.device) for c in self._ecols()]
        return self._cache

    def _local_tables(self, cache):
        """The model's tables with the entity tables replaced by cache views."""
        t = dict(self.tables)
        U = cache.shape[0]
        ent = cache[:, :self.ce]
        t["ent"] = ent if len(self.ent_shape) == 2 else ent.view((U,) + self.ent_shape[1:])
        if self.ca:
            t["ent_aux"] = cache[:, self.ce:]
        return t

    def _local_grads(self, batch, neg, is_train, optimizer, lt, gbufs, prof_events=None):
        """kge_step (KGE_OPT_GRAD) on the tables ``lt`` (the row cache, or the
        replica); gbufs receive their duplicate-summed gradient rows."""
        if self.fused is not None:
            f = self.fused
            f.tables = lt
            grads = [gbufs[0], self.grel["rel"]]
            if "rel_aux" in self.grel:
                grads.append(self.grel["rel_aux"])
            if self.ca:
                grads.append(gbufs[1])
            f.grads = grads
            f(batch, is_train, optimizer if is_train else None, neg_ids=neg, prof_events=prof_events)
            return
        # host-only (KGE_BACKEND=eager) restatement of the same phase, for the gloo tests
        m = self.model
        saved = dict(m.model_weights)
        cw = getattr(m, "constraint_weight", None)
        try:
            m.model_weights[self.names["ent"]] = lt["ent"]
            if self.ca:
                m.model_weights[self.names["ent_aux"]] = lt["ent_aux"]
            if self.full_reg:
                m.constraint_weight = cw / self.G
            loss, grads = engine.eager_grads(m, batch, is_train, neg=self._neg_triples(batch, neg),
                                             batch_scale=float(self.G))
        finally:
            m.model_weights.update(saved)
            if self.full_reg:
                m.constraint_weight = cw
        self.red.zero_()
        for b in gbufs:
            b.zero_()
        self.loss.fill_(float(loss))
        slot = {"ent": 0, "rel": 1, "rel_aux": 2, "ent_aux": 3}
        for role in ("ent", "ent_aux", "rel", "rel_aux"):
            name = self.names.get(role)
            g = grads.get(name) if name else None
            if g is None:
                continue
            self.norm2[slot[role]] = engine.grad_norm2(g)
            w = lt[role] if role in ("ent", "ent_aux") else m.model_weights[name]
            dg = engine.dense_grad(g, w).reshape(w.shape[0], -1)
            if role == "ent":
                gbufs[0].copy_(dg)
            elif role == "ent_aux":
                gbufs[1].copy_(dg)
            else:
                self.grel[role].copy_(dg)

    def _neg_triples(self, batch, neg_ids):
        m = self.model
        K = int(m.negative_ratio)
        if m.corrupt_side == "h+t":
            K = 2 * (K // 2)
        rep = torch.repeat_interleave(batch, K, dim=0).clone()
        neg_ids = neg_ids.to(rep.dtype)
        if m.corrupt_side == "h":
            rep[:, 0] = neg_ids
        elif m.corrupt_side == "t":
            rep[:, 2] = neg_ids
        else:
            rep[0::2, 0] = neg_ids[0::2]
            rep[1::2, 2] = neg_ids[1::2]
        return rep

    def _slot(self, k):
        """norm2 slot of entity table k (0 ent_emb, 3 ent_proj)."""
        return 0 if k == 0 else 3

    def _apply_sparse(self, optimizer, gbufs, sc, rc, rids):
        """Gradient rows back to their owners; the owner applies each source
        rank's rows in rank order (rows unique within a source: no write
        conflicts, deterministic; duplicates across sources are added one
        after the other, as keras SGD's scatter-add of IndexedSlices does)."""
        G, ex = self.G, self.ex
        local = G == 1
        U = rids.shape[0] if local else sum(sc)
        lidx = rids if local else torch.div(rids, G, rounding_mode="floor")
        bounds = [0, U] if local else [0]
        if not local:
            for c in rc:
                bounds.append(bounds[-1] + c)
        adam = isinstance(optimizer, _opt.Adam)
        for k, gb in enumerate(gbufs):
            cols = gb.shape[1]
            if local:
                back = gb[:U]
            else:
                back = torch.empty(bounds[-1], cols, dtype=torch.float32, device=gb.device)
                ex.all_to_all(back, gb[:U].contiguous(), rc, sc)
            lo = 0 if k == 0 else self.ce
            var = self.shard[:, lo:lo + cols]
            v = self._slot(k)
            if adam:   # keras Adam decays every row: a dense gradient of the shard
                acc = torch.zeros(self.Es, cols, dtype=torch.float32, device=gb.device)
                for s in range(len(bounds) - 1):
                    if bounds[s + 1] > bounds[s]:
                        acc.index_add_(0, lidx[bounds[s]:bounds[s + 1]], back[bounds[s]:bounds[s + 1]])
                self._apply_dense(var[:self.valid], acc[:self.valid], v, optimizer, self._shard_name(k))
                continue
            for s in range(len(bounds) - 1):
                a, b = bounds[s], bounds[s + 1]
                if b == a:
                    continue
                if self.fused is not None:
                    d = _hip.kge_apply_rows_desc()
                    d.var = _hip.table(var)
                    d.rows = lidx.data_ptr() + 8 * a
                    d.n = b - a
                    d.grad = back.data_ptr() + 4 * a * back.stride(0)
                    d.grad_ld = back.stride(0)
                    d.norm2 = self.norm2.data_ptr() + 4 * v
                    d.lr = optimizer.learning_rate
                    d.clip_norm = 5.0
                    _hip.check(self.lib.kge_apply_rows(ctypes.byref(d), _hip.stream_handle(var.device)),
                               "kge_apply_rows")
                else:
                    with torch.no_grad():
                        cs = 5.0 / max(math.sqrt(float(self.norm2[v])), 5.0)
                        li = lidx[a:b]
                        var[li] = var[li] + (back[a:b] * cs) * (-optimizer.learning_rate)

    def _shard_name(self, k):
        return self.names["ent" if k == 0 else "ent_aux"] + "#shard"

    def _apply_dense(self, var, grad, v, optimizer, name, abort=None):
        if var.shape[0] == 0:
            return
        if self.fused is not None:
            self.fused.apply(var, grad, self.norm2.data_ptr() + 4 * v, optimizer, name, abort=abort)
        else:
            _host_apply(var, grad, self.norm2[v], optimizer, name)

    def _apply_rel(self, optimizer, abort=None, extra=()):
        """The replicated relation tables' apply (+ ``extra`` [(var, grad,
        norm2 slot, name)]): one kge_apply_many launch on a GPU."""
        slot = {"rel": 1, "rel_aux": 2}
        items = list(extra) + [(self.tables[r].view(self.tables[r].shape[0], -1), self.grel[r], slot[r], self.names[r])
                               for r in self.rel_roles]
        if self.fused is not None:
            self.fused.apply_many([(v, g, self.norm2.data_ptr() + 4 * k, n) for v, g, k, n in items], optimizer,
                                  abort=abort)
            return
        for v, g, k, n in items:
            self._apply_dense(v, g, k, optimizer, n, abort=abort)

    # ------------------------------------------------------------ step
    def __call__(self, batch, is_train, optimizer, neg_ids=None, prof_events=None):
        if self.direct is not None:
            return self.direct(batch, is_train, optimizer, neg_ids=neg_ids, prof_events=prof_events)
        if isinstance(optimizer, _opt.Adam) and is_train:
            optimizer.iterations += 1
        self._constrain()
        if self.mode == "dense":
            # the replica: global ids straight into kge_step (in-kernel draws
            # on the GPU; the host restatement takes the given negatives), then
            # one all-reduce and the same apply on every rank
            self._local_grads(batch, neg_ids, is_train, optimizer, dict(self.tables), self.gent, prof_events)
            self.ex.all_reduce(self.red)
            if is_train and self.full_reg:
                # dense variables: clip_by_norm of the reduced tensor (norms
                # do not add across ranks); identical on every rank
                dense = [(0, self.gent[0])] + [(1 if r == "rel" else 2, self.grel[r]) for r in self.rel_roles]
                for slot, gbuf in dense:
                    g1 = gbuf.reshape(-1)
                    self.norm2[slot:slot + 1].copy_(torch.dot(g1, g1).reshape(1))
            if is_train:
                ents = [(self._ent_rows(k), gk, self._slot(k), self.names["ent" if k == 0 else "ent_aux"])
                        for k, gk in enumerate(self.gent)]
                self._apply_rel(optimizer, extra=ents)   # every variable in one launch
            return self.loss
        if self.mode == "owner" and (not is_train or isinstance(optimizer, _opt.SGD)):
            if self.fused is not None:
                return self._owner_device(batch, is_train, optimizer, neg_ids, prof_events)
            if neg_ids is not None:   # (the host restatement takes the caller's negatives)
                return self._owner_host(batch, is_train, optimizer, neg_ids)
        if neg_ids is None:
            neg_ids = self._draw(batch)
        if self.fused is not None:
            return self._sparse_device(batch, is_train, optimizer, neg_ids.to(batch.dtype).contiguous(), prof_events)
        Bn = int(batch.shape[0])
        ids = torch.cat([batch[:, 0], batch[:, 2], neg_ids.to(batch.dtype)]).to(torch.int64)
        self._bmax = max(getattr(self, "_bmax", 0), Bn)
        cache, remap, plan = self._fetch_sparse(ids)
        gbufs = self._gcache if self.fused is not None else [torch.zeros(cache.shape[0], c) for c in self._ecols()]
        lb = batch.clone()
        lb[:, 0] = remap[:Bn].to(batch.dtype)
        lb[:, 2] = remap[Bn:2 * Bn].to(batch.dtype)
        lneg = remap[2 * Bn:].to(batch.dtype).contiguous()
        self._local_grads(lb, lneg, is_train, optimizer, self._local_tables(cache), gbufs, prof_events)
        self.ex.all_reduce(self.red)
        if is_train:
            self._apply_sparse(optimizer, gbufs, *plan)
            self._apply_rel(optimizer)
        return self.loss

    # ------------------------------------------------------------ device sparse exchange
    def _occurrences(self, B):
        """Entity id occurrences of a B-positive step (h, t, negatives)."""
        m = self.model
        K = int(m.negative_ratio)
        return B * (2 + (2 * (K // 2) if m.corrupt_side == "h+t" else K))

    def _ext_for(self, n_occ, idx_dtype, fill=True, pos_rows=0):
        """Fixed-capacity exchange buffers for steps of up to n_occ id
        occurrences (sized once for the largest step seen, so the step's plan
        never changes): the extended table [Es owned rows | G blocks of cap
        fetched rows | pos_rows gathered positive rows (owner mode)] whose
        head IS the shard, the request / receive id blocks, send rows, the
        hash table."""
        G = self.G
        old = self._ext
        if old is not None and old["n_occ"] >= n_occ and old["pos_rows"] >= pos_rows:
            if old["dtype"] != idx_dtype:   # same blocks, id arrays of the other width
                for k in ("req_ids", "recv_ids"):
                    if k in old:
                        old[k] = torch.zeros(old[k].shape[0], dtype=idx_dtype, device=self.device)
                if not self.multi:
                    old["recv_ids"] = old["req_ids"]
                old["dtype"] = idx_dtype
            return old
        dev, C = self.device, self.C
        if old is not None:   # (re-planned: keep what the other pass sized for)
            n_occ = max(n_occ, old["n_occ"])
            pos_rows = max(pos_rows, old["pos_rows"])
        remote = self.multi or self.loopback or self._needs_loop
        cap = max(1, int(math.ceil(self.slack * n_occ / G)) + self.cap_floor) if remote else 1
        rows = self.Es + G * cap + pos_rows
        if dev.type == "cuda" and rows * C * 4 > (1 << 32):
            torch.cuda.empty_cache()   # a shard that fills HBM: hand cached blocks back first
        ext = torch.zeros(rows, C, dtype=torch.float32, device=dev)
        if fill:
            ext[:self.Es] = self.shard
        self.shard = ext[:self.Es]       # the owned rows live at the head of the extended table
        self._ext = None
        del old
        self.direct = None
        hs = 1
        while hs < 2 * n_occ:
            hs <<= 1
        self._own = None   # (its buffers point into the old table)
        if hasattr(self, "_sf"):
            self._sf = None
        # the plan's per-step zero state: two [hash table | per-owner counts]
        # halves, used by alternate steps (owner mode: each step's plan zeroes
        # the half the previous step used, kge_exchange_desc.zero_next -- no
        # fill launch), then the error flags (zeroed by the owner merge after
        # it reads them; sparse mode fills the whole buffer once per step)
        zb = -(-(G * 4) // 8) * 8
        half = hs * 8 + zb
        zero = torch.zeros(2 * half + 8, dtype=torch.uint8, device=dev)
        halves = [zero[k * half:(k + 1) * half] for k in range(2)]
        b = {"n_occ": n_occ, "dtype": idx_dtype, "cap": cap, "ext": ext, "hslots": hs, "pos_rows": pos_rows,
             "pos_base": self.Es + G * cap, "zero": zero, "halves": halves, "parity": 0,
             "htabs": [h[:hs * 8].view(torch.int64) for h in halves],
             "req_cnts": [h[hs * 8:hs * 8 + G * 4].view(torch.int32) for h in halves],
             "req_ids": torch.zeros(G * cap, dtype=idx_dtype, device=dev),
             "err": zero[2 * half:2 * half + 4].view(torch.float32),
             # [exchange plan's flag | owner pass's flag]
             "errs": zero[2 * half:2 * half + 8].view(torch.float32)}
        b["htab"], b["req_cnt"] = b["htabs"][0], b["req_cnts"][0]
        if self.multi:
            b["recv_cnt"] = torch.zeros(G, dtype=torch.int32, device=dev)
            b["recv_ids"] = torch.zeros(G * cap, dtype=idx_dtype, device=dev)
            b["send"] = torch.zeros(G * cap, C, dtype=torch.float32, device=dev)
        else:   # one rank: the owner side reads the request blocks, fetched rows land in place
            b["recv_cnt"], b["recv_ids"] = b["req_cnt"], b["req_ids"]
        self._ext = b
        return b

    def _flip(self, b):
        """Owner mode: this step's [hash table | counts] half (zeroed by the
        previous step's plan, or never used) and the half to zero now."""
        p = b["parity"] = 1 - b["parity"]
        b["htab"], b["req_cnt"] = b["htabs"][p], b["req_cnts"][p]
        if not self.multi:
            b["recv_cnt"] = b["req_cnt"]
        return b["halves"][1 - p]

    def _xrows(self, b, mode, rows, rows_ld, view, source=-1, norm2_ptr=None, lr=0.0, acc=None, ids=None,
               count=None):
        """kge_exchange_rows on this rank's owned rows ``view`` (a column view of
        the shard); POS mode: ``count`` triples ``ids`` (extended-table rows)
        -> their h, t rows of ``view`` into ``rows``."""
        d = _hip.kge_exchange_rows_desc()
        d.mode = mode
        d.idx_dtype = _hip.IDX_I64 if b["dtype"] == torch.int64 else _hip.IDX_I32
        d.shard = _hip.table(view)
        d.ids = (ids if ids is not None else b["recv_ids"]).data_ptr()
        d.cnt = b["recv_cnt"].data_ptr()
        d.world, d.rank, d.source = self.G, self.g, source
        d.cap = b["cap"] if count is None else count
        d.rows = rows.data_ptr()
        d.rows_ld = rows_ld
        d.acc = acc.data_ptr() if acc is not None else None
        d.norm2 = norm2_ptr
        d.lr = lr
        d.clip_norm = 5.0
        d.abort_flag = self.red[-1:].data_ptr()   # the all-reduced exchange error flag
        d.status = self.status.data_ptr()
        _hip.check(self.lib.kge_exchange_rows(ctypes.byref(d), _hip.stream_handle(self.device)), "kge_exchange_rows")

    def _split_fused(self):
        """The element-wise models' SGD step in two passes (KGE_FLAG_PHASE_*)."""
        if getattr(self, "_sf", None) is None:
            f = engine.FusedStep(self.model, tables=dict(self.tables))
            f.norm2 = self.norm2
            f.loss_out = self.loss
            f.status = self.status
            f.batch_scale = float(self.G)
            f.rel_grad_out = self.grel["rel"]
            self._sf = f
        return self._sf

    def _sparse_device(self, batch, is_train, optimizer, neg, prof_events):
        """One sparse step with no host synchronisation (KGE/sharded.py module
        docstring): kge_exchange_plan on the device, collectives of static
        sizes, the step on the extended table, gradients back, owner applies
        in rank order.

        Element-wise models (TransE / DistMult / RotatE) with SGD run the split
        step: score pass -> all-reduce [norm^2 | loss | error flag] -> update
        pass (owned rows updated in place with the global clip scale, fetched
        rows replaced by their raw gradients, relation gradients out) ->
        all-reduce of the relation gradients -> the fetched rows' gradients
        back to their owners. The other models, Adam and validation steps run
        one gradient-mode step with every id through the blocks (loopback):
        gradient rows back, owners apply (SGD) or accumulate them (Adam)."""
        G, g = self.G, self.g
        Bn = int(batch.shape[0])
        n_neg = int(neg.shape[0])
        split = self.mid in _SPLIT and is_train and isinstance(optimizer, _opt.SGD)
        loop = self.loopback or not split
        if loop and not self.loopback and not self.multi and (self._ext is None or self._ext["cap"] == 1):
            self._needs_loop = True    # a one-rank gradient-mode step needs the blocks
            if self._ext is not None:
                self._ext["n_occ"] = -1   # re-plan the blocks
        b = self._ext_for(2 * Bn + n_neg, batch.dtype)
        cap, ext, C = b["cap"], b["ext"], self.C
        st = _hip.stream_handle(self.device)
        # 1. plan: the triples / negatives in extended-table rows, request blocks
        b["zero"].zero_()   # htab | req_cnt | err
        lpos = torch.empty_like(batch)
        lneg = torch.empty_like(neg)
        x = _hip.kge_exchange_desc()
        x.abi_version = _hip.ABI_VERSION
        x.idx_dtype = _hip.IDX_I64 if batch.dtype == torch.int64 else _hip.IDX_I32
        x.pos, x.neg = batch.data_ptr(), neg.data_ptr()
        x.batch, x.n_neg = Bn, n_neg
        x.n_entities = self.E
        x.world, x.rank, x.loopback = G, g, int(loop)
        x.local_rows = self.Es
        x.cap = cap
        x.htab, x.hslots = b["htab"].data_ptr(), b["hslots"]
        x.pos_out, x.neg_out = lpos.data_ptr(), lneg.data_ptr()
        x.req_ids, x.req_cnt = b["req_ids"].data_ptr(), b["req_cnt"].data_ptr()
        x.err_flag = b["err"].data_ptr()
        x.status = self.status.data_ptr()
        _hip.check(self.lib.kge_exchange_plan(ctypes.byref(x), st), "kge_exchange_plan")
        # 2. requests to the owners, owners gather, rows back
        blocks = ext[self.Es:b["pos_base"]]
        if self.multi:
            self.ex.all_to_all(b["recv_cnt"], b["req_cnt"])
            self.ex.all_to_all(b["recv_ids"], b["req_ids"])
            self._xrows(b, _hip.XROWS_GATHER, b["send"], C, self.shard)
            self.ex.all_to_all(blocks, b["send"])
        elif loop:
            self._xrows(b, _hip.XROWS_GATHER, blocks, C, self.shard)
        lt = self._local_tables(ext)
        # [norm^2 x4 | loss | exchange flag | owner flag | any flag]: summed
        # across ranks, each slot counts the ranks that raised its flag (the
        # kernels' abort word is the last)
        small = self.red[-8:]
        if split:
            # 3a. score pass, global norms / loss / error, update pass
            # (prof_events [before K0, before KS, after KS, after KU]: the
            # score pass records the first three, the update pass the last --
            # KU's interval then also holds the [norm^2 | loss | flag]
            # all-reduce between the passes)
            ev_s = ev_u = None
            if prof_events is not None:
                sc = self._scratch_events()
                ev_s = (ctypes.c_void_p * 4)(prof_events[0], prof_events[1], prof_events[2], sc[0])
                ev_u = (ctypes.c_void_p * 4)(sc[0], sc[1], sc[2], prof_events[3])
            f = self._split_fused()
            f.tables = lt
            f.flags = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_PHASE_SCORE
            f(lpos, True, optimizer, neg_ids=lneg, prof_events=ev_s)
            small[5:7].copy_(b["errs"])   # (no owner pass: its flag stays 0)
            small[7:8].copy_(b["err"])
            if self.multi:
                self.ex.all_reduce(small)
            torch.maximum(self.xerr, small[5:7], out=self.xerr)
            f.flags = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_PHASE_UPDATE
            f.remote_from = self.Es
            f.abort = small[-1:]
            f(lpos, True, optimizer, neg_ids=lneg, prof_events=ev_u)
            if self.multi:
                self.ex.all_reduce(self.red[:-8])   # relation gradients
            grad_blocks = [blocks]
        else:
            # 3b. one gradient-mode step: every entity gradient row in the blocks
            f = self.fused
            f.tables = lt
            gb = self._gblocks(b)
            f.grads = [gb[0], self.grel["rel"]] + ([self.grel["rel_aux"]] if "rel_aux" in self.grel else []) + \
                ([gb[1]] if self.ca else [])
            f.grad_row_offset = self.Es   # the step addresses rows >= Es only (all ids through the blocks)
            f(lpos, is_train, optimizer if is_train else None, neg_ids=lneg, prof_events=prof_events)
            small[5:7].copy_(b["errs"])
            small[7:8].copy_(b["err"])
            if self.multi:
                self.ex.all_reduce(self.red)
            torch.maximum(self.xerr, small[5:7], out=self.xerr)
            grad_blocks = gb
        if not is_train:
            return self.loss
        # 4. the fetched rows' gradients back to their owners; owners apply
        # them source by source in rank order (SGD) or add them up (Adam: a
        # dense keras Adam of the shard)
        dense_items = []
        if self.multi or loop:
            adam = isinstance(optimizer, _opt.Adam)
            for k, gk in enumerate(grad_blocks):
                if self.multi:
                    r = b["send"] if gk.shape[1] == C else torch.empty_like(gk)
                    self.ex.all_to_all(r, gk)
                    gk = r
                lo = 0 if k == 0 else self.ce
                cols = self._ecols()[k]
                view = self.shard[:, lo:lo + cols]
                if adam:
                    acc = torch.zeros(self.Es, cols, dtype=torch.float32, device=self.device)
                    for s in range(G):
                        self._xrows(b, _hip.XROWS_ACCUM, gk, gk.stride(0), view, source=s, acc=acc)
                    dense_items.append((view[:self.valid], acc[:self.valid], self._slot(k), self._shard_name(k)))
                else:
                    for s in range(G):
                        self._xrows(b, _hip.XROWS_SGD, gk, gk.stride(0), view, source=s,
                                    norm2_ptr=self.norm2.data_ptr() + 4 * self._slot(k),
                                    lr=optimizer.learning_rate)
        self._apply_rel(optimizer, abort=small[-1:], extra=dense_items)
        return self.loss

    # ------------------------------------------------------------ owner-side scoring
    def _owner_state(self, Bn, idx_dtype, given):
        """Buffers and the two fused steps of owner mode for Bn positives per
        rank: extended table [Es | G blocks | 2 G Bn gathered positive rows],
        records, softmax stats, the all-gathered triples (and negatives)."""
        G, g = self.G, self.g
        Keff = self._keff()
        b = self._ext_for(2 * Bn, idx_dtype, pos_rows=2 * G * Bn)
        o = self._own
        if o is not None and o["B"] == Bn and o["dtype"] == idx_dtype and (o["gneg"] is not None) == given:
            return b, o
        dev = self.device
        lt = self._local_tables(b["ext"])
        fo = engine.FusedStep(self.model, tables=dict(lt))     # the owner pass (virtual batch G Bn)
        fm = engine.FusedStep(self.model, tables=dict(lt))     # the merge (this rank's Bn)
        for f in (fo, fm):
            f.status = self.status
            f.norm2 = self.norm2                  # merge: this rank's share out; updates: the all-reduced in
            f.rel_grad_out = self.grel["rel"]     # (the owner pass files no relation keys)
        fm.loss_out = self.loss
        fm.batch_scale = float(G)   # (the owner pass's batch is already the global one)
        fm.remote_from = self.Es
        fm.plane_fn = lambda ns, n: 0            # (the merge draws nothing)
        o = {"B": Bn, "dtype": idx_dtype, "fo": fo, "fm": fm, "base_plane": 0,
             "gtrip": torch.zeros(G * Bn, 3, dtype=idx_dtype, device=dev),
             "gneg": torch.zeros(G * Bn * Keff, dtype=idx_dtype, device=dev) if given else None,
             "stats": torch.zeros(G * Bn, 4, dtype=torch.float32, device=dev),
             "lpos": torch.zeros(Bn, 3, dtype=idx_dtype, device=dev),   # the batch in extended-table rows
             "runs": {},
             "err": b["errs"][1:]}   # (zeroed each step by the merge, after it reads it)
        fo.plane_fn = lambda ns, n: o["base_plane"]   # rank 0's planes of this step (set per step)
        common = {"world": G, "rank": g, "batch": Bn}
        # key positions for the owned negatives: ~Bn Keff expected (1/G of the
        # G Bn virtual positives' slots), more when ownership is skewed
        o["key_cap"] = min(G * Bn * Keff, int(math.ceil(max(1.25, self.slack) * Bn * Keff)) + max(4096, self.cap_floor))
        small = self.red[-8:]
        # (flags_out / sticky: the owner update pass folds the all-reduced flags
        # into the sticky max -- no launch of its own)
        fo.owner = dict(common, rows_from=b["pos_base"], global_entities=self.E, err=o["err"], stats=o["stats"],
                        key_capacity=o["key_cap"], flags_out=small[5:8], sticky=self.xerr)
        fo.flags = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_OWNER | _hip.FLAG_PHASE_SCORE
        # the record width of this plan, then the record buffers
        probe = fo.describe(o["gtrip"], True, _opt.SGD(0.01), neg_ids=o["gneg"])
        probe.owner_records = 16   # (non-null placeholder: the query reads no buffer)
        R = int(self.lib.kge_owner_record_floats(probe))
        if R <= 0:
            raise RuntimeError("owner-side scoring: " + self.lib.kge_last_error().decode(errors="replace"))
        o["R"] = R
        o["rec"] = torch.zeros(G * Bn, R, dtype=torch.float32, device=dev)
        o["rec_in"] = torch.zeros(G * Bn, R, dtype=torch.float32, device=dev) if self.multi else o["rec"]
        o["stats_mine"] = o["stats"][g * Bn:(g + 1) * Bn]
        fo.owner["records"] = o["rec"]
        # (flags_in -> flags_out: the merge hands the step's flags to the
        # all-reduce buffer and zeroes them)
        fm.owner = dict(common, records=o["rec_in"], stats_out=o["stats_mine"], flags_in=b["errs"],
                        flags_out=small[5:8])
        self._own = o
        return b, o

    @staticmethod
    def _owner_run(o, f, batch, is_train, optimizer, flags, abort=None):
        """One owner-mode kge_step through a bound descriptor (FusedStep.bind),
        bound on first use per (step, phase, optimizer, learning rate) and again
        whenever the step's workspace was reallocated."""
        runs = o["runs"]
        key = (id(f), flags, bool(is_train), id(optimizer), getattr(optimizer, "learning_rate", None),
               abort is not None)
        hit = runs.get(key)
        if hit is None or hit[0] != f.workspace.data_ptr():
            if len(runs) >= 16:
                runs.clear()
            f.flags, f.abort = flags, abort
            run = f.bind(batch, is_train, optimizer)
            hit = runs[key] = (f.workspace.data_ptr(), run)
        hit[1](batch.data_ptr())

    def _keff(self):
        m = self.model
        K = int(m.negative_ratio)
        return 2 * (K // 2) if m.corrupt_side == "h+t" else K

    def _owner_device(self, batch, is_train, optimizer, neg_ids, prof_events):
        """One owner-side-scoring step (KGE_FLAG_OWNER, include/kge_hip.h):
        the negatives are scored where their rows live, so only positives'
        rows, per-positive records and small stats cross ranks.

          1. this rank's positives' h / t rows fetched (the exchange plan of
             2B ids, blocks, all_to_all);
          2. every rank's positive rows and triples all-gathered;
          3. owner pass over the G B virtual positives (negatives drawn from
             each positive's own rank's planes, owned ones scored) -> records;
          4. all_to_all of the records to the positives' ranks;
          5. merge -> loss, norm^2 shares, row gradients, softmax stats;
          6. all-reduce [norm^2 | loss | error flag], all-gather the stats;
          7. owner update (coefficients, owned rows' SGD) BEFORE
          8. the positives' rows (own in place, fetched ones' raw gradients);
          9. relation gradients all-reduced, fetched rows' gradients back to
             their owners (kge_exchange_rows SGD in rank order); relations
             applied.
        Same draws, losses and updates as the single-device step on the
        concatenated G B batch (up to float summation order)."""
        G, g = self.G, self.g
        ex = self.ex
        Bn = int(batch.shape[0])
        given = neg_ids is not None
        b, o = self._owner_state(Bn, batch.dtype, given)
        cap, ext, C = b["cap"], b["ext"], self.C
        st = _hip.stream_handle(self.device)
        loop = self.loopback
        # 1. the positives' rows: plan (no negatives), requests, owners gather, rows back
        # (this step's hash table / counts were zeroed by the previous step's
        # plan, which zeroes the other half now; the flags by the last merge)
        zero_next = self._flip(b)
        lpos = o["lpos"]
        x = o.get("x")
        if x is None:   # (built once per plan: only the batch address changes per step)
            x = _hip.kge_exchange_desc()
            x.abi_version = _hip.ABI_VERSION
            x.idx_dtype = _hip.IDX_I64 if batch.dtype == torch.int64 else _hip.IDX_I32
            x.batch, x.n_neg = Bn, 0
            x.n_entities = self.E
            x.world, x.rank, x.loopback = G, g, int(loop)
            x.local_rows = self.Es
            x.cap = cap
            x.hslots = b["hslots"]
            x.pos_out, x.neg_out = lpos.data_ptr(), lpos.data_ptr()
            x.req_ids = b["req_ids"].data_ptr()
            x.err_flag = b["err"].data_ptr()
            x.status = self.status.data_ptr()
            o["x"] = x
        x.pos = x.neg = batch.data_ptr()
        x.htab, x.req_cnt = b["htab"].data_ptr(), b["req_cnt"].data_ptr()
        x.zero_next, x.zero_next_bytes = zero_next.data_ptr(), zero_next.numel()
        _hip.check(self.lib.kge_exchange_plan(ctypes.byref(x), st), "kge_exchange_plan")
        blocks = ext[self.Es:b["pos_base"]]
        if self.multi:
            ex.all_to_all(b["recv_cnt"], b["req_cnt"])
            ex.all_to_all(b["recv_ids"], b["req_ids"])
            self._xrows(b, _hip.XROWS_GATHER, b["send"], C, self.shard)
            ex.all_to_all(blocks, b["send"])
        elif loop:
            self._xrows(b, _hip.XROWS_GATHER, blocks, C, self.shard)
        # 2. every rank's positives: rows (h, t of positive v at pos_base + 2v, + 1) and triples
        P = ext[b["pos_base"]:b["pos_base"] + 2 * G * Bn]
        mine = P[2 * g * Bn:2 * (g + 1) * Bn]
        # (gathered straight into P by kge_exchange_rows' POS mode: the source
        # rows [0, pos_base) and P do not overlap)
        self._xrows(b, _hip.XROWS_POS, mine, C, ext[:b["pos_base"]], ids=lpos, count=Bn)
        gtrip = o["gtrip"]
        if self.multi:   # (one rank: P is `mine`, the virtual batch is the batch)
            ex.all_gather(P, mine)
            ex.all_gather(gtrip, batch)
        else:
            gtrip = batch
        if given:
            ex.all_gather(o["gneg"], neg_ids.to(batch.dtype).contiguous())
        else:
            m = self.model
            o["base_plane"] = m.ns_strategy.take_planes(2 if m.corrupt_side == "h+t" else 1) * G
        # 3. owner pass
        ev_s = ev_u = None
        if prof_events is not None:   # [before, owner pass, after it, after the update passes]
            sc = self._scratch_events()
            ev_s = (ctypes.c_void_p * 4)(prof_events[0], prof_events[1], prof_events[2], sc[0])
            ev_u = (ctypes.c_void_p * 4)(sc[0], sc[1], sc[2], prof_events[3])
        fo, fm = o["fo"], o["fm"]
        opt = optimizer if is_train else None
        # (steady state: the four calls' descriptors bound once -- FusedStep.bind --
        # so a call is one kge_step, no per-call key building on the host)
        fast = prof_events is None and not given and (opt is None or isinstance(opt, _opt.SGD))
        small = self.red[-8:]
        f_os = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_OWNER | _hip.FLAG_PHASE_SCORE
        f_ms = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_OWNER_MERGE | _hip.FLAG_PHASE_SCORE | self.debug_flags
        if fast:
            self._owner_run(o, fo, gtrip, is_train, opt, f_os)
        else:
            fo.flags, fo.abort = f_os, None
            fo(gtrip, is_train, opt, neg_ids=o["gneg"], prof_events=ev_s)
        # 4. records to the positives' ranks; 5. merge
        if self.multi:
            ex.all_to_all(o["rec_in"], o["rec"])
        if fast:
            self._owner_run(o, fm, lpos, is_train, opt, f_ms)
        else:
            fm.flags, fm.abort = f_ms, None
            fm(lpos, is_train, opt)
        # 6. [norm^2 x4 | loss | exchange flag | owner flag | any flag] (the
        # merge wrote the flags and zeroed them for the next step), the stats
        if self.multi:
            ex.all_reduce(small)
            ex.all_gather(o["stats"], o["stats_mine"])
        if not is_train:   # (training steps: the owner update pass keeps the sticky max)
            torch.maximum(self.xerr, small[5:7], out=self.xerr)
            return self.loss
        # 7. the owned negatives' rows, then 8. the positives' rows
        f_ou = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_OWNER | _hip.FLAG_PHASE_UPDATE
        f_mu = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_OWNER_MERGE | _hip.FLAG_PHASE_UPDATE | self.debug_flags
        if fast:
            self._owner_run(o, fo, gtrip, True, optimizer, f_ou, abort=small[-1:])
            self._owner_run(o, fm, lpos, True, optimizer, f_mu, abort=small[-1:])
        else:
            fo.flags, fo.abort = f_ou, small[-1:]
            fo(gtrip, True, optimizer, neg_ids=o["gneg"], prof_events=ev_u)
            fm.flags, fm.abort = f_mu, small[-1:]
            fm(lpos, True, optimizer)
        # 9. relation gradients; the fetched rows' gradients back to their owners
        if self.multi:
            ex.all_reduce(self.red[:-8])
        if self.multi or loop:
            gk = blocks
            if self.multi:
                ex.all_to_all(b["send"], blocks)
                gk = b["send"]
            for src in range(G):
                self._xrows(b, _hip.XROWS_SGD, gk, gk.stride(0), self.shard, source=src,
                            norm2_ptr=self.norm2.data_ptr(), lr=optimizer.learning_rate)
        self._apply_rel(optimizer, abort=small[-1:])
        return self.loss

    def _score_rows(self, H, Rr, T):
        """The model's score_hrt on gathered rows (TransE.py:127-155,
        DistMult.py:118-146, RotatE.py:126-165) -- host restatement."""
        m = self.model
        if self.mid == _hip.MODEL_DISTMULT:
            return torch.sum(H * Rr * T, dim=-1)
        if self.mid == _hip.MODEL_ROTATE:
            d = Rr.shape[-1]
            h2, t2 = H.view(-1, d, 2), T.view(-1, d, 2)
            th = Rr / m.limit * float(np.float32(np.pi))
            x = torch.complex(h2[..., 0], h2[..., 1]) * torch.complex(torch.cos(th), torch.sin(th))
            return m.score_fn(x, torch.complex(t2[..., 0], t2[..., 1]))
        return m.score_fn(H + Rr, T)

    def _owner_host(self, batch, is_train, optimizer, neg_ids):
        """Host restatement of ``_owner_device`` (KGE_BACKEND=eager, the gloo
        CPU tests): the same data flow and the same algebra as the kernels --
        the owner scores every rank's positives against the negatives it owns
        and keeps a record per positive (its own softmax maximum Ms_o, Z_o,
        loss part, hinge / logistic weight sum, slice-norm^2 partials and the
        h / r / t gradient sums at unit 1/Z); the positive's rank merges the
        records (Ms = max Ms_o, F_o = exp(Ms_o - Ms), 1/Z); the owners scale
        their rows' gradients by F_o / Z and apply them. Every per-negative
        gradient comes from torch autograd on the lookup slices (TF-2.5
        IndexedSlices), so this checks the merge, not the kernels' calculus."""
        G, g, ex = self.G, self.g, self.ex
        m = self.model
        Bn = int(batch.shape[0])
        Keff = self._keff()
        C, ce = self.C, self.ce
        lk, margin, temp = _loss_kind(m.loss_fn)
        Bg = float(G * Bn)
        relt = self.tables["rel"]
        rel2 = relt.reshape(relt.shape[0], -1)
        # 1. the positives' rows (the sparse exchange's fetch of 2 Bn ids)
        ids = torch.cat([batch[:, 0], batch[:, 2]]).to(torch.int64)
        self._bmax = max(getattr(self, "_bmax", 0), Bn)
        cache, remap, plan = self._fetch_sparse(ids)
        hrow, trow = cache[remap[:Bn], :ce], cache[remap[Bn:], :ce]
        # 2. every rank's positives and negatives
        gpos = torch.zeros(G * Bn, 2, ce, dtype=torch.float32)
        ex.all_gather(gpos.view(G * Bn * 2, ce), torch.stack([hrow, trow], 1).reshape(2 * Bn, ce).contiguous())
        gtri = torch.zeros(G * Bn, 3, dtype=torch.int64)
        ex.all_gather(gtri, batch.to(torch.int64).contiguous())
        gneg = torch.zeros(G * Bn * Keff, dtype=torch.int64)
        ex.all_gather(gneg, neg_ids.to(torch.int64).contiguous())
        # 3. the owner pass: a record per virtual positive, and its owned rows' gradients
        R = 8 + 3 * max(ce, rel2.shape[1])
        rec = torch.zeros(G * Bn, R, dtype=torch.float32)
        own_rows, own_grad, own_v = [], [], []
        jk = torch.arange(Keff)
        hc = (jk % 2 == 0) if m.corrupt_side == "h+t" else torch.full((Keff,), m.corrupt_side == "h")
        for v in range(G * Bn):
            e = gneg[v * Keff:(v + 1) * Keff]
            mine = (e % G) == g
            sel = torch.nonzero(mine).reshape(-1)
            h, t, r = gpos[v, 0], gpos[v, 1], rel2[gtri[v, 1]]
            sp = float(self._score_rows(h[None], r[None], t[None])[0])
            rec[v, 0] = -math.inf
            if sel.numel() == 0:
                continue
            ish = hc[sel]
            E = self.shard[torch.div(e[sel], G, rounding_mode="floor"), :ce]
            Hs = torch.where(ish[:, None], E, h[None].expand_as(E)).clone().requires_grad_(True)
            Ts = torch.where(ish[:, None], t[None].expand_as(E), E).clone().requires_grad_(True)
            Rs = r[None].expand(sel.numel(), -1).clone().requires_grad_(True)
            with torch.enable_grad():
                sc = self._score_rows(Hs, Rs, Ts)
                sd = sc.detach()
                if lk == "sans":
                    z = temp * sd
                    Mo = float(z.max())
                    w = torch.exp(z - Mo)
                    c = w * torch.sigmoid(sd + margin) / Bg
                    rec[v, 0], rec[v, 1] = Mo, float(w.sum())
                    rec[v, 2] = float((w * torch.nn.functional.logsigmoid(-sd - margin)).sum())
                elif lk == "hinge":
                    c = (margin + sd - sp >= 0).to(torch.float32) / (Bg * Keff)
                    rec[v, 2] = float(torch.clamp(margin + sd - sp, min=0).sum())
                elif lk == "logistic":
                    c = torch.exp(sd - sp) / (1 + torch.exp(sd - sp))
                    rec[v, 2] = float(torch.log(1 + torch.exp(sd - sp)).sum())
                elif lk == "bce":
                    c = torch.sigmoid(sd) / Bg
                    rec[v, 2] = float(torch.nn.functional.logsigmoid(-sd).sum())
                else:
                    c = sd / Bg
                    rec[v, 2] = float((sd * sd).sum())
                rec[v, 3] = float(c.sum())
                gh, gr, gt = torch.autograd.grad(torch.sum(c * sc), [Hs, Rs, Ts])
            rec[v, 4] = float((gh * gh).sum() + (gt * gt).sum())
            rec[v, 5] = float((gr * gr).sum())
            rec[v, 8:8 + ce] = gh[~ish].sum(0)
            rec[v, 8 + ce:8 + ce + gr.shape[1]] = gr.sum(0)
            rec[v, 8 + 2 * ce:8 + 3 * ce] = gt[ish].sum(0)
            own_rows.append(torch.div(e[sel], G, rounding_mode="floor"))
            own_grad.append(torch.where(ish[:, None], gh, gt))
            own_v.append(torch.full((sel.numel(),), v, dtype=torch.int64))
        # 4. records to the positives' ranks; 5. merge
        rin = torch.zeros_like(rec)
        ex.all_to_all(rin, rec)
        rin = rin.view(G, Bn, R)
        stats = torch.zeros(G * Bn, 2, dtype=torch.float32)   # (Ms, 1/Z) per virtual positive
        loss = 0.0
        n2 = [0.0, 0.0]
        ggrad = torch.zeros(Bn, 3, C if C >= rel2.shape[1] else rel2.shape[1], dtype=torch.float32)
        for i in range(Bn):
            hd = rin[:, i]
            h = hrow[i].clone().requires_grad_(True)
            r = rel2[batch[i, 1]].clone().requires_grad_(True)
            t = trow[i].clone().requires_grad_(True)
            with torch.enable_grad():
                spt = self._score_rows(h[None], r[None], t[None])[0]
                ph, pr, pt = torch.autograd.grad(spt, [h, r, t])
            sp = float(spt)
            Ms = float(hd[:, 0].max()) if lk == "sans" else 0.0
            fo = torch.exp(hd[:, 0] - Ms) if lk == "sans" else torch.ones(G)
            fo = torch.where(torch.isinf(hd[:, 0]) & (lk == "sans"), torch.zeros_like(fo), fo)
            Z = float((hd[:, 1] * fo).sum())
            invZ = (1.0 / Z if Z > 0 else 0.0) if lk == "sans" else 1.0
            cw = float(hd[:, 3].sum())
            if lk == "hinge":
                lossp, cp, wl = 0.0, -cw, 1.0 / (Bg * Keff)
            elif lk == "logistic":
                lossp, cp, wl = 0.0, -cw, 1.0
            elif lk == "bce":
                lossp = -float(torch.nn.functional.logsigmoid(torch.tensor(sp))) / Bg
                cp, wl = -float(torch.sigmoid(torch.tensor(-sp))) / Bg, -1.0 / Bg
            elif lk == "sans":
                lossp = -float(torch.nn.functional.logsigmoid(torch.tensor(sp + margin))) / Bg
                cp, wl = -float(torch.sigmoid(torch.tensor(-(sp + margin)))) / Bg, -1.0 / Bg
            else:
                lossp, cp, wl = (sp - 1.0) ** 2 * 0.5 / Bg, (sp - 1.0) / Bg, 0.5 / Bg
            fz = fo * invZ
            lneg = float(((fz if lk == "sans" else torch.ones(G)) * hd[:, 2]).sum())
            n2[0] += cp * cp * float((ph * ph).sum() + (pt * pt).sum()) + float((fz * fz * hd[:, 4]).sum())
            n2[1] += cp * cp * float((pr * pr).sum()) + float((fz * fz * hd[:, 5]).sum())
            gh = cp * ph + (fz[:, None] * hd[:, 8:8 + ce]).sum(0)
            grr = cp * pr + (fz[:, None] * hd[:, 8 + ce:8 + ce + pr.shape[0]]).sum(0)
            gt = cp * pt + (fz[:, None] * hd[:, 8 + 2 * ce:8 + 3 * ce]).sum(0)
            if self.mid == _hip.MODEL_DISTMULT and getattr(m, "constraint", False):
                lam = m.constraint_weight
                rsq = float((r.detach() ** 2).sum())
                lossp += lam * rsq / Bg
                grr = grr + (lam / Bg) * 2 * r.detach()
                n2[1] += float(((lam / Bg) * 2 * r.detach()).pow(2).sum())
            loss += lossp + wl * lneg
            ggrad[i, 0, :ce], ggrad[i, 1, :grr.shape[0]], ggrad[i, 2, :ce] = gh, grr, gt
            stats[g * Bn + i, 0], stats[g * Bn + i, 1] = Ms, invZ
        # 6. [norm^2 | loss], the stats
        self.red.zero_()
        self.norm2[0], self.norm2[1] = n2[0], n2[1]
        self.loss.fill_(loss)
        ex.all_reduce(self.red)
        mine_st = stats[g * Bn:(g + 1) * Bn].clone()
        ex.all_gather(stats, mine_st)
        if not is_train:
            return self.loss
        lr = optimizer.learning_rate
        with torch.no_grad():
            cs0 = 5.0 / max(math.sqrt(float(self.norm2[0])), 5.0)
            # 7. the owned negatives' rows: gradients at the global softmax state
            if own_rows:
                rows = torch.cat(own_rows)
                vv = torch.cat(own_v)
                gr_ = torch.cat(own_grad)
                if lk == "sans":
                    Mo = rec[vv, 0]
                    gr_ = gr_ * (torch.exp(Mo - stats[vv, 0]) * stats[vv, 1])[:, None]
                acc = torch.zeros(self.Es, ce, dtype=torch.float32).index_add_(0, rows, gr_)
                self.shard[:, :ce] += acc * (cs0 * -lr)
            # 8. the positives' rows: summed per fetched id, back to their owners
            gc = torch.zeros(cache.shape[0], ce, dtype=torch.float32)
            gc.index_add_(0, remap[:Bn], ggrad[:, 0, :ce])
            gc.index_add_(0, remap[Bn:], ggrad[:, 2, :ce])
            gbufs = [gc]
            # relation gradients: this rank's positives, then summed over ranks
            grel = torch.zeros_like(rel2).index_add_(0, batch[:, 1].to(torch.int64), ggrad[:, 1, :rel2.shape[1]])
            ex.all_reduce(grel)
            self.grel["rel"].copy_(grel.view_as(self.grel["rel"]))
        self._apply_sparse(optimizer, gbufs, *plan)
        self._apply_rel(optimizer)
        return self.loss

    def _scratch_events(self):
        """Three recorded HIP events the split step's profiling passes use as
        placeholders (handles; torch creates an event at its first record)."""
        if getattr(self, "_sc_ev", None) is None:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            for e in evs:
                e.record()
            self._sc_ev = (evs, [e.cuda_event for e in evs])
        return self._sc_ev[1]

    def _gblocks(self, b):
        """Gradient rows of the fetched blocks [G cap, cols], per entity table."""
        if "gblocks" not in b:
            b["gblocks"] = [torch.zeros(self.G * b["cap"], c, dtype=torch.float32, device=self.device)
                            for c in self._ecols()]
        return b["gblocks"]

    # ------------------------------------------------------------ state
    def release_entity_tables(self):
        """Drop the id-order entity tables the model held (the shards are
        authoritative; sync() allocates them again). Frees E x cols floats per
        table on every rank -- needed when the table is most of HBM (C5)).
        Dense mode: the tables are the replica, nothing to release."""
        if self.mode == "dense":
            return
        w = self.model.model_weights
        for role in ("ent", "ent_aux"):
            if role in self.names and self.tables.get(role) is not None:
                w[self.names[role]] = torch.empty(0, dtype=torch.float32, device=self.device)
                self.tables[role] = self.tables[role][:0]
        self._released = True

    def sync(self):
        """Gather the shards into ``model_weights`` in id order (evaluation,
        checkpoints). Dense mode: ``model_weights`` is the replica already."""
        if self.mode == "dense":
            return
        G, Es = self.G, self.Es
        full = torch.zeros(G * Es, self.C, dtype=torch.float32, device=self.device)
        self.ex.all_gather(full, self.shard)
        nat = full.view(G, Es, self.C).transpose(0, 1).reshape(G * Es, self.C)[:self.E]
        w = self.model.model_weights
        if getattr(self, "_released", False):
            w[self.names["ent"]] = torch.empty((self.E,) + self.ent_shape[1:], dtype=torch.float32,
                                               device=self.device)
            if self.ca:
                w[self.names["ent_aux"]] = torch.empty((self.E,) + self.aux_shape[1:], dtype=torch.float32,
                                                       device=self.device)
            self._released = False
        with torch.no_grad():
            w[self.names["ent"]].copy_(nat[:, :self.ce].reshape(self.ent_shape))
            if self.ca:
                w[self.names["ent_aux"]].copy_(nat[:, self.ce:].reshape(self.aux_shape))

    def entity_parts(self):
        """Sparse mode: {weight name: this rank's owned entity rows} (histograms
        reduce over the shards instead of gathering the table). Dense: {}."""
        if self.mode == "dense":
            return {}
        out = {self.names["ent"]: self.shard[:self.valid, :self.ce]}
        if self.ca:
            out[self.names["ent_aux"]] = self.shard[:self.valid, self.ce:]
        return out

    def load(self, weights):
        """Write ``weights`` (id order) into this rank's shard and the
        replicated tables (checkpoint restore)."""
        G, g = self.G, self.g
        if self.mode == "dense":
            with torch.no_grad():
                for role in ["ent"] + (["ent_aux"] if self.ca else []) + self.rel_roles:
                    self.tables[role].copy_(torch.as_tensor(weights[self.names[role]]).to(self.device)
                                            .reshape(self.tables[role].shape))
            return
        with torch.no_grad():
            ent = torch.as_tensor(weights[self.names["ent"]]).to(self.device).reshape(self.E, -1)
            self.shard[:self.valid, :self.ce] = ent[g::G]
            if self.ca:
                aux = torch.as_tensor(weights[self.names["ent_aux"]]).to(self.device).reshape(self.E, -1)
                self.shard[:self.valid, self.ce:] = aux[g::G]
            for r in self.rel_roles:
                self.tables[r].copy_(torch.as_tensor(weights[self.names[r]]).to(self.device))
        self.sync()

    def check_status(self):
        if self.direct is not None:
            self.direct.check_status()
        if self.fused is not None:
            _hip.check_device_status(self.status, "kge_step")
        if self._ext is not None:
            xf, of = self.xerr.tolist()
            if xf == 0.0 and of == 0.0:
                return
            self.xerr.zero_()
            if of != 0.0:   # (the owner pass's flag, kge_hip.h owner_err)
                raise RuntimeError("owner-side scoring: this rank's owned negatives overflowed the owner pass's "
                                   "%d key positions; the step was skipped on every rank -- raise capacity_slack "
                                   "or capacity_floor" % (self._own or {}).get("key_cap", 0))
            raise RuntimeError("sparse exchange: the step's ids overflowed an owner block (capacity %d rows); "
                               "the step was skipped on every rank -- raise capacity_slack" % self._ext["cap"])


def _loss_kind(lf):
    """(kind, margin, temperature) of a built-in loss (loss.py)."""
    from . import loss as L
    t = type(lf)
    if t is L.PairwiseHingeLoss:
        return "hinge", float(lf.margin), 1.0
    if t is L.PairwiseLogisticLoss:
        return "logistic", 0.0, 1.0
    if t is L.BinaryCrossEntropyLoss:
        return "bce", 0.0, 1.0
    if t is L.SelfAdversarialNegativeSamplingLoss:
        return "sans", float(lf.margin), float(lf.temperature)
    return "sqerr", 0.0, 1.0


def _host_apply(var, grad, norm2, optimizer, name):
    """kge_apply restated with torch ops (host-only eager backend)."""
    with torch.no_grad():
        cs = 5.0 / max(math.sqrt(float(norm2)), 5.0)
        g = grad * cs
        if isinstance(optimizer, _opt.Adam):
            st = optimizer.slots.setdefault(name, {"m": torch.zeros_like(var), "v": torch.zeros_like(var)})
            b1, b2, t = optimizer.beta_1, optimizer.beta_2, optimizer.iterations
            lr_t = optimizer.learning_rate * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
            st["m"].mul_(b1).add_(g * (1 - b1))
            st["v"].mul_(b2).add_(g * g * (1 - b2))
            var.sub_(lr_t * st["m"] / (torch.sqrt(st["v"]) + optimizer.epsilon))
        else:
            var.add_(g * (-optimizer.learning_rate))
