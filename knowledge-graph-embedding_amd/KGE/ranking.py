"""Batched filtered ranking through ``kge_rank`` (row f1).

``KGEModel.evaluate`` (reference ``BaseModel.py:578-618``) ranks one triple
per iteration with ``get_rank`` (``:620-654``): score every entity on the
corrupted side, set the filtered positives to -inf, count the scores strictly
above the true triple's. Here the whole evaluation set goes to the device in
one call per (relation group, side): the host prepares each query's rows in
the model's own op order (below, one builder per built-in model), builds the
filter as a sorted (relation, kept entity) -> entity index, and the HIP
kernels score all E candidates of every query (``csrc/kge_rank.hip``).

Only the exact built-in model classes with built-in score functions take
this path; user subclasses, UM / SE and custom scores keep the reference's
per-triple loop (``BaseModel.get_rank``).
"""

import ctypes

import numpy as np
import torch

from . import _hip
from . import score as _score


def _lk(model, name, idx):
    return model.model_weights[name].detach()[idx]


def _score_desc(model):
    sd = _score.fused_descriptor(model.score_fn)
    if sd is None:
        return None
    return sd


# ---------------------------------------------------------------- builders
# Each returns a list of groups: dict(sel, mode, proj, cand, cand_aux, dim,
# clip, q0, q1, qw, score) -- `sel` the query positions of the group (None =
# all), rows in the reference's op order for that model's score_hrt.
def _q_transe(m, h, r, t, side):
    sd = _score_desc(m)
    if sd is None:
        return None
    re_ = _lk(m, "rel_emb", r)
    if side == "t":
        q0, q1 = _lk(m, "ent_emb", h) + re_, None        # TransE.py:149-155: s(h + r, t)
    else:
        q0, q1 = re_, _lk(m, "ent_emb", t)
    return [dict(sel=None, mode=_hip.RANK_TRANS, proj=_hip.RPROJ_NONE, cand=m.model_weights["ent_emb"],
                 cand_aux=None, dim=int(re_.shape[1]), clip=0, q0=q0, q1=q1, qw=None, score=sd)]


def _q_transh(m, h, r, t, side):
    sd = _score_desc(m)
    if sd is None:
        return None
    w = _lk(m, "rel_hyper", r)
    re_ = _lk(m, "rel_emb", r)

    def proj(e):   # TransH.py:180-181
        return e - torch.sum(w * e, dim=-1, keepdim=True) * w
    if side == "t":
        q0, q1 = proj(_lk(m, "ent_emb", h)) + re_, None
    else:
        q0, q1 = re_, proj(_lk(m, "ent_emb", t))
    return [dict(sel=None, mode=_hip.RANK_TRANS, proj=_hip.RPROJ_HYPER, cand=m.model_weights["ent_emb"],
                 cand_aux=None, dim=int(re_.shape[1]), clip=0, q0=q0, q1=q1, qw=w, score=sd)]


def _clip(x):
    n = torch.pow(torch.sum(torch.abs(x) ** 2, dim=-1, keepdim=True), 0.5)
    mask = (n < 1).to(x.dtype)
    return mask * x + (1 - mask) * (x / torch.clamp(n, min=1e-9))


def _q_transd(m, h, r, t, side):
    sd = _score_desc(m)
    if sd is None:
        return None
    rp = _lk(m, "rel_proj", r)
    re_ = _lk(m, "rel_emb", r)
    kr = int(re_.shape[1])

    def proj(e, ep):   # TransD.py:206-219: (r_p e_p^T + I) e, clipped
        ke = int(e.shape[1])
        eye = torch.eye(kr, ke, dtype=e.dtype, device=e.device)
        M = torch.matmul(rp.unsqueeze(-1), ep.unsqueeze(-2)) + eye
        p = torch.matmul(M, e.unsqueeze(-1)).squeeze(-1)
        return _clip(p) if m.constraint else p
    if side == "t":
        q0, q1 = proj(_lk(m, "ent_emb", h), _lk(m, "ent_proj", h)) + re_, None
    else:
        q0, q1 = re_, proj(_lk(m, "ent_emb", t), _lk(m, "ent_proj", t))
    return [dict(sel=None, mode=_hip.RANK_TRANS, proj=_hip.RPROJ_RANK1, cand=m.model_weights["ent_emb"],
                 cand_aux=m.model_weights["ent_proj"], dim=kr, clip=int(bool(m.constraint)), q0=q0, q1=q1,
                 qw=rp, score=sd)]


def _q_transr(m, h, r, t, side):
    """Queries grouped by relation: each group's candidates are the whole
    entity table projected by its M_r (one GEMM per relation)."""
    sd = _score_desc(m)
    if sd is None:
        return None
    groups = []
    ent = m.model_weights["ent_emb"].detach()
    for rr in torch.unique(r).tolist():
        sel = torch.nonzero(r == rr).reshape(-1)
        M = m.model_weights["rel_proj"].detach()[rr]
        cand = torch.matmul(ent, M)                  # TransR.py:181-189
        if m.constraint:
            cand = _clip(cand)
        re_ = _lk(m, "rel_emb", r[sel])
        if side == "t":
            q0, q1 = cand[h[sel]] + re_, None
        else:
            q0, q1 = re_, cand[t[sel]]
        groups.append(dict(sel=sel, mode=_hip.RANK_TRANS, proj=_hip.RPROJ_NONE, cand=cand.contiguous(),
                           cand_aux=None, dim=int(re_.shape[1]), clip=0, q0=q0, q1=q1, qw=None, score=sd))
    return groups


def _cplx(z):
    return torch.view_as_real(z).reshape(z.shape[0], -1)


def _q_rotate(m, h, r, t, side):
    sd = _score_desc(m)
    if sd is None or sd[0] == _score.SCORE_DOT:
        return None
    if not hasattr(m, "limit"):
        m._set_limit()
    th = _lk(m, "rel_emb", r) / m.limit * np.float32(np.pi)     # RotatE.py:150-160
    w = torch.complex(torch.cos(th), torch.sin(th))
    ent = m.model_weights["ent_emb"]
    E = ent.shape[0]
    if side == "t":
        he = _lk(m, "ent_emb", h)
        q0, q1 = _cplx(torch.complex(he[..., 0], he[..., 1]) * w), None
    else:
        q0, q1 = _cplx(w), _lk(m, "ent_emb", t).reshape(len(t), -1)
    return [dict(sel=None, mode=_hip.RANK_ROT, proj=_hip.RPROJ_NONE, cand=ent.view(E, -1), cand_aux=None,
                 dim=int(q0.shape[1]), clip=0, q0=q0, q1=q1, qw=None, score=sd)]


def _q_distmult(m, h, r, t, side):
    ri = _lk(m, "rel_inter", r)
    if side == "t":
        q0, q1 = _lk(m, "ent_emb", h) * ri, None          # DistMult.py:140-146: sum(h * r * t)
    else:
        q0, q1 = ri, _lk(m, "ent_emb", t)
    return [dict(sel=None, mode=_hip.RANK_MUL, proj=_hip.RPROJ_NONE, cand=m.model_weights["ent_emb"],
                 cand_aux=None, dim=int(ri.shape[1]), clip=0, q0=q0, q1=q1, qw=None, score=(_score.SCORE_DOT, 0.0))]


def _q_rescal(m, h, r, t, side):
    R = _lk(m, "rel_inter", r)
    if side == "t":
        q0 = torch.matmul(_lk(m, "ent_emb", h).unsqueeze(-2), R).squeeze(-2)   # RESCAL.py:166-171: h^T R t
    else:
        q0 = torch.matmul(R, _lk(m, "ent_emb", t).unsqueeze(-1)).squeeze(-1)
    return [dict(sel=None, mode=_hip.RANK_DOT, proj=_hip.RPROJ_NONE, cand=m.model_weights["ent_emb"],
                 cand_aux=None, dim=int(q0.shape[1]), clip=0, q0=q0, q1=None, qw=None, score=(_score.SCORE_DOT, 0.0))]


def _builders():
    from .models.semantic_based.DistMult import DistMult
    from .models.semantic_based.RESCAL import RESCAL
    from .models.translating_based.RotatE import RotatE
    from .models.translating_based.TransD import TransD
    from .models.translating_based.TransE import TransE
    from .models.translating_based.TransH import TransH
    from .models.translating_based.TransR import TransR
    return {TransE: _q_transe, TransH: _q_transh, TransD: _q_transd, TransR: _q_transr, RotatE: _q_rotate,
            DistMult: _q_distmult, RESCAL: _q_rescal}


RANK_Q = 8                  # csrc/kge_step.h kRankQ: queries per count workgroup
RANK_LDS_BYTES = 64 * 1024  # kge_rank's limit on the staged query rows


def query_width(model):
    """Floats per query row kge_rank stages (its rows in the model's op order)."""
    from .models.semantic_based.RESCAL import RESCAL
    from .models.translating_based.RotatE import RotatE
    w = model.model_weights
    if isinstance(model, RotatE):
        return 2 * int(w["rel_emb"].shape[1])
    if isinstance(model, RESCAL):
        return int(w["ent_emb"].shape[1])
    rel = w.get("rel_emb", w.get("rel_inter"))
    return int(rel.shape[1])


def supported(model):
    """The model class and score function have a batched ranking path that
    ``kge_rank`` accepts (the same limits it checks: staged query rows within
    its LDS budget, no complex Dot score) -- otherwise ``evaluate`` keeps the
    reference's per-triple ``get_rank`` loop."""
    b = _builders().get(type(model))
    if b is None:
        return False
    if hasattr(model, "score_fn"):
        sd = _score.fused_descriptor(model.score_fn)
        if sd is None:
            return False
        from .models.translating_based.RotatE import RotatE
        if isinstance(model, RotatE) and sd[0] == _score.SCORE_DOT:
            return False
    ent = model.model_weights.get("ent_emb") if getattr(model, "model_weights", None) else None
    if ent is None or not ent.is_cuda:
        return False
    return 3 * RANK_Q * ((query_width(model) + 3) & ~3) * 4 <= RANK_LDS_BYTES


# ---------------------------------------------------------------- filter
def filter_index(X, positive_X, side, E):
    """Per query [beg, end) into a sorted entity array: the corrupted-side
    entities of the known positives sharing the query's (relation, kept
    entity) -- BaseModel.py:646-650 (mask on r and the kept side), duplicates
    removed (tensor_scatter_nd_update writes -inf once per entity)."""
    keys, ents = filter_keys(positive_X, side, E)
    return filter_lookup(X, keys, ents, side, E) + (ents,)


def filter_lookup(X, keys, ents, side, E):
    """[beg, end) of each query's (relation, kept entity) run in ``keys``."""
    keep = 2 if side == "h" else 0
    qk = X[:, 1].to(torch.int64) * E + X[:, keep].to(torch.int64)
    beg = torch.searchsorted(keys, qk, right=False)
    end = torch.searchsorted(keys, qk, right=True)
    return beg.contiguous(), end.contiguous()


def filter_keys(positive_X, side, E):
    """The known positives as sorted, unique (relation * E + kept entity,
    corrupted entity) pairs: ``keys`` ascending, ``ents`` ascending within a
    key. Independent of the evaluation set, so ``batched_ranks`` caches it."""
    keep, corrupt = (2, 0) if side == "h" else (0, 2)
    P = positive_X.to(torch.int64)
    key = P[:, 1] * E + P[:, keep]            # < R * E: fits int64 for any table
    ent = P[:, corrupt]
    # (key, entity) pairs sorted lexicographically, then de-duplicated: one
    # sort of the combined key * E + entity while it fits int64, two stable
    # sorts once R * E^2 > 2^63
    R = int(P[:, 1].max().item()) + 1 if P.numel() else 1
    if R * E * E < (1 << 62):
        u = torch.unique(key * E + ent)   # sorted, unique
        keys, ents = u // E, u % E
    else:
        o = torch.argsort(ent, stable=True)
        key, ent = key[o], ent[o]
        o = torch.argsort(key, stable=True)
        key, ent = key[o], ent[o]
        first = torch.ones_like(key, dtype=torch.bool)
        if key.numel() > 1:
            first[1:] = (key[1:] != key[:-1]) | (ent[1:] != ent[:-1])
        keys, ents = key[first], ent[first]
    return keys.contiguous(), ents.contiguous()


# evaluate() is called once per epoch (early stopping) and per side with the
# same positive set: the sorted filter pairs are built once per (content,
# side, E, device) and kept for the last few sets. The key is the set's bytes
# hashed on the host (a 272k-triple set: ~1 ms), so an array edited in place
# is a new set.
_FILTER_CACHE = {}
_FILTER_CACHE_MAX = 4


def _fingerprint(P):
    import hashlib
    a = np.ascontiguousarray(P)
    try:
        import xxhash
        h = xxhash.xxh3_128_hexdigest(a.data)
    except ImportError:
        h = hashlib.blake2b(a.data, digest_size=16).hexdigest()
    return (a.shape, a.dtype.str, h)


def cached_filter_keys(positive_X, side, E, dev):
    P = np.asarray(positive_X.cpu() if isinstance(positive_X, torch.Tensor) else positive_X)
    key = (_fingerprint(P), side, int(E), str(dev))
    hit = _FILTER_CACHE.pop(key, None)
    if hit is None:
        PX = torch.as_tensor(P, dtype=torch.int64).to(dev).reshape(-1, 3)
        hit = filter_keys(PX, side, E)
        while len(_FILTER_CACHE) >= _FILTER_CACHE_MAX:
            _FILTER_CACHE.pop(next(iter(_FILTER_CACHE)))
    _FILTER_CACHE[key] = hit     # most recent last
    return hit


# ---------------------------------------------------------------- entry
_BITS_MAX_BYTES = 1 << 30
RESCORE_FILTER = 1 << 30   # (batched_ranks flag, not passed on: the rescoring filter pass, for A/B tests)


def batched_ranks(model, eval_X, corrupt_side, positive_X=None, flags=0):
    """Ranks of every triple of ``eval_X`` (numpy int64 [n]), the same values
    ``get_rank`` gives one triple at a time. ``flags``: KGE_RANK_FLAG_*."""
    if corrupt_side not in ("h", "t"):
        raise ValueError("corrupt_side must be 'h' or 't'")
    lib = _hip.lib()
    dev = model.model_weights["ent_emb"].device
    X = torch.as_tensor(np.asarray(eval_X.cpu() if isinstance(eval_X, torch.Tensor) else eval_X),
                        dtype=torch.int64).to(dev).reshape(-1, 3)
    n = X.shape[0]
    E = int(model.model_weights["ent_emb"].shape[0])
    h, r, t = X[:, 0], X[:, 1], X[:, 2]
    with torch.no_grad():
        groups = _builders()[type(model)](model, h, r, t, corrupt_side)
    if groups is None:
        raise NotImplementedError("no batched ranking for this model / score")
    if positive_X is not None:
        fkeys, fent = cached_filter_keys(positive_X, corrupt_side, E, dev)
        fb, fe = filter_lookup(X, fkeys, fent, corrupt_side, E)
    ranks = torch.zeros(n, dtype=torch.int64, device=dev)
    pos = torch.zeros(n, dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    true_col = 0 if corrupt_side == "h" else 2
    keep = []
    # the filter as a bitmap (ABI 8: the count pass skips the known positives,
    # no rescoring pass), n x ceil(E / 32) words while that stays under
    # _BITS_MAX_BYTES; past it the library's rescoring filter pass runs
    bits = None
    W = (E + 31) // 32
    if positive_X is not None and not (flags & RESCORE_FILTER) and 0 < n * W * 4 <= _BITS_MAX_BYTES:
        bits = torch.empty(n * W, dtype=torch.int32, device=dev)
    for g in groups:
        sel = g["sel"]
        ids = X[:, true_col] if sel is None else X[sel, true_col]
        m = int(ids.shape[0])
        rk = ranks if sel is None else torch.zeros(m, dtype=torch.int64, device=dev)
        ps = pos if sel is None else torch.zeros(m, dtype=torch.float32, device=dev)
        q0 = g["q0"].to(torch.float32).contiguous()
        q1 = g["q1"].to(torch.float32).contiguous() if g["q1"] is not None else None
        qw = g["qw"].to(torch.float32).contiguous() if g["qw"] is not None else None
        ids = ids.contiguous()
        d = _hip.kge_rank_desc()
        d.abi_version = _hip.ABI_VERSION
        d.mode = g["mode"]
        d.proj = g["proj"]
        d.corrupt_side = _hip.SIDE_H if corrupt_side == "h" else _hip.SIDE_T
        d.cand = _hip.table(g["cand"])
        if g["cand_aux"] is not None:
            d.cand_aux = _hip.table(g["cand_aux"])
        d.dim = g["dim"]
        d.clip = g["clip"]
        d.q0 = q0.data_ptr()
        d.q1 = q1.data_ptr() if q1 is not None else None
        d.qw = qw.data_ptr() if qw is not None else None
        d.ldq = q0.shape[1]
        d.true_ids = ids.data_ptr()
        d.idx_dtype = _hip.IDX_I64
        d.score_kind, d.score_p = g["score"]
        d.n = m
        d.flags = int(flags) & ~RESCORE_FILTER
        if positive_X is not None:
            gb = fb if sel is None else fb[sel].contiguous()
            ge = fe if sel is None else fe[sel].contiguous()
            d.filt_beg, d.filt_end, d.filt_ent = gb.data_ptr(), ge.data_ptr(), fent.data_ptr()
            if bits is not None:
                d.filt_bits, d.filt_bits_words = bits.data_ptr(), bits.numel()
            keep.append((gb, ge))
        d.rank_out = rk.data_ptr()
        d.pos_score_out = ps.data_ptr()
        d.status = status.data_ptr()
        _hip.check(lib.kge_rank(ctypes.byref(d), _hip.stream_handle(dev)), "kge_rank")
        if sel is not None:
            ranks[sel] = rk
            pos[sel] = ps
        keep.append((q0, q1, qw, ids, rk, ps, g["cand"]))
    _hip.check_device_status(status, "kge_rank")
    return ranks.cpu().numpy()
