"""Multi-GPU training step: data-parallel over triples, entity table row-sharded.

The reference is single-device (``BaseModel.py:19-21``); this is the build's
one parallel strategy. One process per GPU,
``torch.distributed`` with the RCCL backend ("nccl" on ROCm) over xGMI.

Layout in HBM, per rank g of G:
  * ``shard``  [Es, cols]   rows [g*Es, (g+1)*Es) of ent_emb (block ownership,
                            Es = ceil(E / G)); the authoritative copy.
  * ``full``   [G*Es, cols] the gathered table the kernels read this step
                            (``model_weights['ent_emb']`` views its first E rows).
  * ``gfull``  [G*Es, cols] this rank's dense entity gradient; ``gshard`` its
                            reduce-scattered owner slice.
  * relation tables are replicated (<= 38 MB even for RESCAL / TransR);
    their gradient travels in ``red`` with the per-variable slice norm^2 and
    the loss, in ONE all-reduce.

One step (``ShardedStep.__call__``), every rank with its own positives:
  1. ``_constraint_loss`` table assigns on the owned rows (TransE / DistMult
     renormalisation, ``TransE.py:171-172``) -- before scoring, as
     ``BaseModel.py:319`` orders it;
  2. all-gather shards -> ``full``;
  3. ``kge_step`` in ``KGE_OPT_GRAD`` mode on ``full`` (sampling with a
     rank-disjoint counter plane, gather, score, loss normalised by the GLOBAL
     batch via ``batch_scale = G``, gradients, slice norm^2);
  4. all-reduce ``red`` = [rel grad | norm^2 x4 | loss];
  5. reduce-scatter ``gfull`` -> ``gshard``;
  6. ``kge_apply`` (clip_by_norm with the global norm, SGD / Adam) on the
     shard and on the replicated relation table.
G ranks x B positives therefore compute the step one device would compute
on the concatenated G*B batch (up to float summation order).

Whenever every row is touched each step (uniform negatives at FB15k-237
scale touch all 14,505 rows), this dense exchange moves the same bytes as a
de-duplicated all-to-all of requested rows, with fixed sizes and no host
sync. The collectives go through ``Exchange``, which uses the tensor forms
RCCL provides and, for the gloo CPU tests of this logic, list / all-reduce
forms with the same results.
"""

import math

import torch
import torch.distributed as dist

from . import _hip
from . import engine
from . import optimizers as _opt
from .constraint import normalized_embeddings

_RENORM = (_hip.MODEL_TRANSE, _hip.MODEL_DISTMULT)


class Exchange:
    """The step's collectives on one process group."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.tensor_forms = dist.get_backend(group) == "nccl"

    def all_gather(self, full, shard):
        if self.tensor_forms:
            dist.all_gather_into_tensor(full, shard, group=self.group)
        else:
            dist.all_gather(list(full.chunk(self.world)), shard, group=self.group)

    def reduce_scatter(self, shard, full):
        if self.tensor_forms:
            dist.reduce_scatter_tensor(shard, full, op=dist.ReduceOp.SUM, group=self.group)
        else:
            dist.all_reduce(full, group=self.group)
            shard.copy_(full.chunk(self.world)[self.rank])

    def all_reduce(self, t):
        dist.all_reduce(t, group=self.group)


class ShardedStep:
    """Drop-in for ``FusedStep`` across G ranks (see module docstring)."""

    def __init__(self, model, exchange=None):
        self.model = model
        self.ex = exchange or Exchange()
        G, g = self.ex.world, self.ex.rank
        self.names = engine.fused_names(model) if hasattr(model, "_fused_tables") else \
            {"ent": "ent_emb", "rel": _rel_name(model)}
        ent = model.model_weights[self.names["ent"]]
        rel = model.model_weights[self.names["rel"]]
        self.ent_shape = tuple(ent.shape)
        E = int(ent.shape[0])
        cols = ent.numel() // E
        Es = -(-E // G)
        dev = ent.device
        self.E, self.Es, self.lo = E, Es, g * Es
        self.valid = max(0, min(Es, E - self.lo))
        self.full = torch.zeros(G * Es, cols, dtype=torch.float32, device=dev)
        self.full[:E] = ent.reshape(E, cols)
        self.shard = self.full[self.lo:self.lo + Es].clone()
        self.gfull = torch.zeros(G * Es, cols, dtype=torch.float32, device=dev)
        self.gshard = torch.zeros(Es, cols, dtype=torch.float32, device=dev)
        model.model_weights[self.names["ent"]] = self.full[:E].view(self.ent_shape)
        R = int(rel.shape[0])
        self.rel_cols = rel.numel() // R
        nrel = R * self.rel_cols
        self.red = torch.zeros(nrel + 8, dtype=torch.float32, device=dev)
        self.grel = self.red[:nrel].view(R, self.rel_cols)
        self.norm2 = self.red[nrel:nrel + 4]
        self.loss = self.red[nrel + 4:nrel + 5]
        self.renorm = model._fused_model_id in _RENORM and bool(getattr(model, "constraint", False))
        self.fused = None
        if dev.type == "cuda":
            f = engine.FusedStep(model, grad_mode=True)
            f.grads = [self.gfull[:E], self.grel]
            f.norm2 = self.norm2
            f.loss_out = self.loss
            f.batch_scale = float(G)
            f.flags = _hip.FLAG_NO_TABLE_CONSTRAINT if self.renorm else 0
            f.plane_fn = lambda ns, n: ns.take_planes(n) * G + g * n
            self.fused = f
        elif engine.backend() != "eager":
            raise RuntimeError("ShardedStep needs GPUs (or KGE_BACKEND=eager for host-only tests)")

    # ------------------------------------------------------------ phases
    def _constrain_shard(self):
        if not self.renorm or self.valid == 0:
            return
        rows = self.shard[:self.valid]
        if self.fused is not None:
            _hip.check(self.fused.lib.kge_constrain_rows(_hip.table(rows), 0, 1.0,
                                                         _hip.stream_handle(rows.device)), "kge_constrain_rows")
        else:
            rows.copy_(normalized_embeddings(rows, p=2, value=1, axis=1))

    def _local_grads(self, batch, is_train, neg_ids, optimizer, prof_events=None):
        if self.fused is not None:
            self.fused(batch, is_train, optimizer if is_train else None, neg_ids=neg_ids, prof_events=prof_events)
            return
        # host-only (KGE_BACKEND=eager) restatement of the same phase, for the gloo tests
        loss, grads = engine.eager_grads(self.model, batch, is_train, neg=self._neg_triples(batch, neg_ids),
                                         batch_scale=float(self.ex.world))
        self.red.zero_()
        self.gfull.zero_()
        self.loss.fill_(float(loss))
        for v, role in enumerate(("ent", "rel")):
            name = self.names[role]
            g = grads.get(name)
            if g is None:
                continue
            self.norm2[v] = engine.grad_norm2(g)
            w = self.model.model_weights[name]
            dg = engine.dense_grad(g, w).reshape(w.shape[0], -1)
            (self.gfull[:self.E] if role == "ent" else self.grel).copy_(dg)

    def _neg_triples(self, batch, neg_ids):
        m = self.model
        if neg_ids is None:
            return None
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

    def _apply(self, optimizer):
        rel = self.model.model_weights[self.names["rel"]]
        if isinstance(optimizer, _opt.Adam):
            optimizer.iterations += 1
        pairs = [(self.shard[:self.valid], self.gshard[:self.valid], 0, self.names["ent"] + "#shard"),
                 (rel.view(rel.shape[0], -1), self.grel, 1, self.names["rel"])]
        for var, grad, v, name in pairs:
            if var.shape[0] == 0:
                continue
            if self.fused is not None:
                self.fused.apply(var, grad, self.norm2.data_ptr() + 4 * v, optimizer, name)
            else:
                _host_apply(var, grad, self.norm2[v], optimizer, name)

    # ------------------------------------------------------------ step
    def __call__(self, batch, is_train, optimizer, neg_ids=None, prof_events=None):
        self._constrain_shard()
        self.ex.all_gather(self.full, self.shard)
        self._local_grads(batch, is_train, neg_ids, optimizer, prof_events)
        self.ex.all_reduce(self.red)
        if is_train:
            self.ex.reduce_scatter(self.gshard, self.gfull)
            self._apply(optimizer)
        return self.loss

    def sync(self):
        """Gather the current shards so ``model_weights`` is up to date (evaluation)."""
        self.ex.all_gather(self.full, self.shard)

    def check_status(self):
        if self.fused is not None:
            self.fused.check_status()


def _rel_name(model):
    for k in ("rel_emb", "rel_inter"):
        if k in model.model_weights:
            return k
    raise ValueError("no relation table")


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
