"""CPU oracle for the KGE training step -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker (or the
timed CPU baseline); the product (``KGE``) never does.

What it restates (reference = melissakou/knowledge-graph-embedding, TF 2.5):
  * negative draws: the counter-based spec of ``include/kge_hip.h``
    (Philox4x32-10, pinned by the Random123 known-answer vectors in
    ``tests/golden/philox_kat.json``) in the corruption layout of
    ``BaseModel.py:332-408`` (h-side draws, then t-side; 'h+t' rows
    alternate h-corrupt / t-corrupt per positive);
  * the input stream: ``data_utils.py:176-196``'s shuffle -> repeat ->
    batch under the per-epoch permutation spec of ``kge_stream_desc``;
  * typed draws: ``utils.py:11-16`` (pool of the entity's type minus the
    entity) mapped from the same counter stream;
  * the step ``BaseModel.py:316-328``: constraint assigns, scores
    (``score.py:49-89`` per model ``score_hrt``), loss (``loss.py``), TF-2.5
    gradients with embedding lookups as IndexedSlices (values of every
    lookup kept, duplicates NOT summed; any dense contribution turns the
    variable's gradient dense -- ``backprop.aggregate_indexed_slices_gradients``),
    ``clip_by_norm(g, 5)`` per variable (``values * 5 / max(||values||, 5)``),
    keras SGD (``ResourceScatterAdd(var, idx, -lr * g)``).
  Arithmetic is float64 torch autograd on the op sequence the reference
  writes (each op's TF gradient rule coincides with torch's: clip passes on
  the closed interval, abs'(0) = 0, |z|'(0) = 0, reduce_max splits ties).

PARITY UNPINNED: the reference's own tests pin only properties (shape, sign,
finiteness), TF 2.5 is not installed and cannot be imported here, and the
reference's negatives are unseeded (irreproducible). The restatement is
cross-checked against finite differences and the reference's property tests
(``tests/test_oracle.py``); golden vectors under ``tests/golden`` are
generated from it by ``tests/golden/make_golden.py``.
"""

import math

import numpy as np
import torch

F64 = torch.float64

# ---------------------------------------------------------------- Philox
_M0, _M1 = 0xD2511F53, 0xCD9E8D57
_W0, _W1 = 0x9E3779B9, 0xBB67AE85


def philox4x32_10(ctr, key):
    """Scalar reference Philox4x32-10 (Salmon et al. 2011; Random123)."""
    c = [int(x) & 0xFFFFFFFF for x in ctr]
    k0, k1 = int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & 0xFFFFFFFF
            k1 = (k1 + _W1) & 0xFFFFFFFF
        p0 = _M0 * c[0]
        p1 = _M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF,
             ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF, p0 & 0xFFFFFFFF]
    return c


def _philox_vec(b, plane, seed):
    """Vectorised over block indices b (numpy uint64)."""
    b = np.asarray(b, dtype=np.uint64)
    m = np.uint64(0xFFFFFFFF)
    c = [b & m, b >> np.uint64(32), np.full_like(b, plane & 0xFFFFFFFF), np.full_like(b, (plane >> 32) & 0xFFFFFFFF)]
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & 0xFFFFFFFF
            k1 = (k1 + _W1) & 0xFFFFFFFF
        p0 = np.uint64(_M0) * c[0]
        p1 = np.uint64(_M1) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ np.uint64(k0), p1 & m, (p0 >> np.uint64(32)) ^ c[3] ^ np.uint64(k1), p0 & m]
    return np.stack(c, axis=-1)


def draw_bits(seed, plane, n, i64):
    """Raw bits of draw indices n: u32 word n%4 of block n//4 (int32 ids), or
    w[2q] | w[2q+1] << 32 of block n//2 (int64 ids)."""
    n = np.asarray(n, dtype=np.uint64)
    if i64:
        w = _philox_vec(n // np.uint64(2), plane, seed)
        q = (n % np.uint64(2)).astype(np.int64)
        lo = w[np.arange(len(n)), 2 * q]
        hi = w[np.arange(len(n)), 2 * q + 1]
        return lo | (hi << np.uint64(32))
    w = _philox_vec(n // np.uint64(4), plane, seed)
    return w[np.arange(len(n)), (n % np.uint64(4)).astype(np.int64)]


def _side_draws(ref_ent, k, seed, plane, i64, sampler, E, typed=None):
    """k draws per positive for one side (ns_strategy.py:57-62 / utils.py:11-16)."""
    B = len(ref_ent)
    n = np.arange(B * k)
    bits = draw_bits(seed, plane, n, i64)
    if sampler == "uniform":
        return (bits % np.uint64(E)).astype(np.int64)
    ent_type, offsets, members, pos_in_type = typed
    x = np.repeat(np.asarray(ref_ent, dtype=np.int64), k)
    ty = ent_type[x]
    beg, cnt = offsets[ty], offsets[ty + 1] - offsets[ty]
    assert (cnt > 1).all(), "empty typed pool"
    kk = (bits % (cnt - 1).astype(np.uint64)).astype(np.int64)
    kk = kk + (kk >= pos_in_type[x])
    return members[beg + kk].astype(np.int64)


def negatives(pos, K, side, E, seed, plane, i64=True, sampler="uniform", typed=None):
    """Negative entity ids in the reference layout, [B * K_eff]."""
    pos = np.asarray(pos, dtype=np.int64)
    if side == "h":
        return _side_draws(pos[:, 0], K, seed, plane, i64, sampler, E, typed)
    if side == "t":
        return _side_draws(pos[:, 2], K, seed, plane, i64, sampler, E, typed)
    k = K // 2
    B = len(pos)
    hs = _side_draws(pos[:, 0], k, seed, plane, i64, sampler, E, typed).reshape(B, k)
    ts = _side_draws(pos[:, 2], k, seed, plane + 1, i64, sampler, E, typed).reshape(B, k)
    return np.stack([hs, ts], axis=-1).reshape(-1)   # alternate h, t per slot


def uniform_negatives(pos, K, side, E, seed, plane, i64=True):
    return negatives(pos, K, side, E, seed, plane, i64)


def typed_tables(ind2type):
    """CSR form of type2inds built as BaseModel.py:258-263 does."""
    ind2type = list(ind2type)
    types = list(np.unique(ind2type))
    tid = {t: i for i, t in enumerate(types)}
    members, offsets = [], [0]
    pos_in = np.zeros(len(ind2type), np.int64)
    for t in types:
        inds = [i for (i, ti) in enumerate(ind2type) if ti == t]
        for k, e in enumerate(inds):
            pos_in[e] = k
        members += inds
        offsets.append(len(members))
    return (np.array([tid[t] for t in ind2type], np.int64), np.array(offsets, np.int64),
            np.array(members, np.int64), pos_in)


def corrupt(pos, neg_ids, K, side):
    """[B*K_eff, 3] negative triples (BaseModel.py:360-408)."""
    pos = np.asarray(pos, dtype=np.int64)
    Keff = 2 * (K // 2) if side == "h+t" else K
    rep = np.repeat(pos, Keff, axis=0).copy()
    neg_ids = np.asarray(neg_ids, dtype=np.int64)
    if side == "h":
        rep[:, 0] = neg_ids
    elif side == "t":
        rep[:, 2] = neg_ids
    else:
        j = np.tile(np.arange(Keff), len(pos))
        hmask = (j % 2) == 0
        rep[hmask, 0] = neg_ids[hmask]
        rep[~hmask, 2] = neg_ids[~hmask]
    return rep


# ---------------------------------------------------------------- input stream
def stream_rows(n, seed, start, batch, shuffle):
    """Source rows of stream positions [start, start + batch): the
    ``shuffle(n, seed, reshuffle_each_iteration=True).repeat().batch()``
    stream of ``data_utils.py:176-196`` under the per-epoch permutation spec
    of ``kge_stream_desc`` (include/kge_hip.h), one position at a time with
    the scalar Philox above. Small cases only (pure Python)."""
    w = 2
    while w < 64 and (1 << w) < n:
        w += 2
    h = w // 2
    mask = (1 << h) - 1

    def feistel(x, epoch):
        L, R = x >> h, x & mask
        for r in range(4):
            f = philox4x32_10((R, r, epoch & 0xFFFFFFFF, epoch >> 32), (seed & 0xFFFFFFFF, seed >> 32))[0]
            L, R = R, (L ^ f) & mask
        return (L << h) | R

    out = []
    for p in range(start, start + batch):
        e, k = divmod(p, n)
        if shuffle:
            k = feistel(k, e)
            while k >= n:
                k = feistel(k, e)
        out.append(k)
    return out


# ---------------------------------------------------------------- scores / losses
def score_fn(kind, p, x, y):
    """score.py:49-89."""
    if kind == "dot":
        return torch.sum(x * y, dim=-1)
    diff = torch.abs(x - y)
    if math.isinf(p):
        lp = -torch.amax(diff, dim=-1)
    else:
        R = torch.clamp(torch.sum(torch.pow(diff, p), dim=-1), min=1e-9)
        # p = 2: sqrt, the correctly rounded form of pow(R, 1/2) (a host's
        # vectorised powf may differ by an ulp, which decides a hinge term
        # that sits exactly on its margin in the float32 mode)
        lp = -(torch.sqrt(R) if p == 2 else torch.pow(R, 1.0 / p))
    if kind == "lp":
        return lp
    return -torch.pow(lp, 2)


def loss_fn(spec, pos, neg, batch_scale=1.0):
    """loss.py:49-204; spec = ('hinge', m) | ('logistic',) | ('bce',) | ('sans', m, T) | ('sqerr',)."""
    name = spec[0]
    B = pos.shape[0]
    K = int(neg.shape[0] / B)
    Bg = B * batch_scale
    if name == "hinge":
        p = torch.repeat_interleave(pos, K)
        return torch.sum(torch.clamp(spec[1] + neg - p, min=0)) / (p.shape[0] * batch_scale)
    if name == "logistic":
        p = torch.repeat_interleave(pos, K)
        return torch.sum(torch.log(1 + torch.exp(neg - p)))
    if name == "bce":
        return -(torch.sum(torch.nn.functional.logsigmoid(pos)) + torch.sum(torch.nn.functional.logsigmoid(-neg))) / Bg
    if name == "sans":
        m, T = spec[1], spec[2]
        n = neg.reshape(B, K)
        prob = torch.softmax(T * n, dim=-1).detach()
        return -(torch.sum(torch.nn.functional.logsigmoid(pos + m)) +
                 torch.sum(prob * torch.nn.functional.logsigmoid(-n - m))) / Bg
    if name == "sqerr":
        return (torch.sum((pos - 1.0) ** 2) + torch.sum(neg ** 2)) / 2 / Bg
    raise ValueError(name)


def _norm_rows(X, axis):
    return X / torch.pow(torch.sum(torch.abs(X) ** 2, dim=axis, keepdim=True), 0.5)


def _clip_rows(X):
    n = torch.pow(torch.sum(torch.abs(X) ** 2, dim=-1, keepdim=True), 0.5)
    mask = (n < 1).to(X.dtype)
    return mask * X + (1 - mask) * (X / torch.clamp(n, min=1e-9) * 1)


# ---------------------------------------------------------------- models
class _Lookups:
    def __init__(self, W, train):
        self.W, self.train, self.rec = W, train, []

    def __call__(self, name, idx):
        idx = torch.as_tensor(idx, dtype=torch.int64)
        if not self.train:
            return self.W[name][idx]
        leaf = self.W[name].detach()[idx.reshape(-1)].clone().requires_grad_(True)
        self.rec.append((name, idx.reshape(-1), leaf))
        return leaf.reshape(tuple(idx.shape) + tuple(self.W[name].shape[1:]))


def _score_hrt(model, W, L, h, r, t, score, cfg):
    kind, p = score
    if model == "TransE":
        return score_fn(kind, p, L("ent_emb", h) + L("rel_emb", r), L("ent_emb", t))
    if model == "DistMult":
        return torch.sum(L("ent_emb", h) * L("rel_inter", r) * L("ent_emb", t), dim=-1)
    if model == "RotatE":
        he, re_, te = L("ent_emb", h), L("rel_emb", r), L("ent_emb", t)
        th = re_ / cfg["limit"] * np.float32(np.pi).item()
        x = torch.complex(he[..., 0], he[..., 1]) * torch.complex(torch.cos(th), torch.sin(th))
        return score_fn(kind, p, x, torch.complex(te[..., 0], te[..., 1]))
    if model == "TransH":
        he, re_, w, te = L("ent_emb", h), L("rel_emb", r), L("rel_hyper", r), L("ent_emb", t)
        hp = he - torch.sum(w * he, -1, keepdim=True) * w
        tp = te - torch.sum(w * te, -1, keepdim=True) * w
        return score_fn(kind, p, hp + re_, tp)
    if model == "TransR":
        he, re_, te, M = L("ent_emb", h), L("rel_emb", r), L("ent_emb", t), L("rel_proj", r)
        hp = torch.matmul(he.unsqueeze(-2), M).squeeze(-2)
        tp = torch.matmul(te.unsqueeze(-2), M).squeeze(-2)
        if cfg["constraint"]:
            hp, tp = _clip_rows(hp), _clip_rows(tp)
        return score_fn(kind, p, hp + re_, tp)
    if model == "TransD":
        he, re_, te = L("ent_emb", h), L("rel_emb", r), L("ent_emb", t)
        hpj, rpj, tpj = L("ent_proj", h), L("rel_proj", r), L("ent_proj", t)
        kr, ke = re_.shape[-1], he.shape[-1]
        eye = torch.eye(kr, ke, dtype=he.dtype)
        hm = torch.matmul(rpj.unsqueeze(-1), hpj.unsqueeze(-2)) + eye
        tm = torch.matmul(rpj.unsqueeze(-1), tpj.unsqueeze(-2)) + eye
        hp = torch.matmul(hm, he.unsqueeze(-1)).squeeze(-1)
        tp = torch.matmul(tm, te.unsqueeze(-1)).squeeze(-1)
        if cfg["constraint"]:
            hp, tp = _clip_rows(hp), _clip_rows(tp)
        return score_fn(kind, p, hp + re_, tp)
    if model == "RESCAL":
        he, te, Rm = L("ent_emb", h), L("ent_emb", t), L("rel_inter", r)
        return torch.matmul(torch.matmul(he.unsqueeze(-2), Rm), te.unsqueeze(-1)).reshape(-1)
    raise ValueError(model)


def filtered_ranks(model, weights, X, side, positive_X=None, score=("lp", 2.0), limit=None, constraint=False,
                   tie_tol=1e-5):
    """BaseModel.get_rank (BaseModel.py:620-654) for every triple of X, in
    float64: every entity scored on the corrupted side (score_hrt with h or t
    None), the known positives sharing the query's (r, kept entity) set to
    -inf (:646-650), rank = 1 + #(scores > the true triple's score) (:652-654;
    counted in int64, the reference's int16 overflows past 32,767).
    Also returns, per query, the candidates within tie_tol * max(1, |s_true|)
    of the true score: an fp32 evaluation may order those either way."""
    W = {k: torch.tensor(np.asarray(v), dtype=F64) for k, v in weights.items()}
    L = _Lookups(W, False)
    cfg = {"constraint": constraint, "constraint_weight": 1.0, "limit": limit}
    E = W["ent_emb"].shape[0]
    X = np.asarray(X, dtype=np.int64).reshape(-1, 3)
    P = None if positive_X is None else np.asarray(positive_X, dtype=np.int64).reshape(-1, 3)
    keep, corr = (2, 0) if side == "h" else (0, 2)
    every = np.arange(E)
    ranks, ties = [], []
    with torch.no_grad():
        for x in X:
            h = every if side == "h" else np.full(E, x[0])
            t = every if side == "t" else np.full(E, x[2])
            s = _score_hrt(model, W, L, h, np.full(E, x[1]), t, score, cfg).numpy().copy()
            ps = float(_score_hrt(model, W, L, x[0:1], x[1:2], x[2:3], score, cfg).reshape(-1)[0])
            near = int(np.sum(np.abs(s - ps) <= tie_tol * max(1.0, abs(ps))))
            if P is not None:
                m = (P[:, 1] == x[1]) & (P[:, keep] == x[keep])
                s[P[m, corr]] = -np.inf
            ranks.append(int(np.sum(s > ps)) + 1)
            ties.append(near)
    return np.array(ranks, dtype=np.int64), np.array(ties, dtype=np.int64)


def _constraint(model, W, L, X, cfg, batch_scale):
    """Per-model _constraint_loss: assigns (no grad) + returned term."""
    if not cfg["constraint"]:
        return 0.0
    lam = cfg.get("constraint_weight", 1.0)
    with torch.no_grad():
        if model in ("TransE", "DistMult"):
            W["ent_emb"].copy_(_norm_rows(W["ent_emb"], 1))
        if model in ("TransR", "TransD"):
            W["ent_emb"].copy_(_clip_rows(W["ent_emb"]))
            W["rel_emb"].copy_(_clip_rows(W["rel_emb"]))
        if model == "TransH":
            W["rel_hyper"].copy_(_norm_rows(W["rel_hyper"], 1))
    if model == "DistMult":
        r = L("rel_inter", X[:, 1])
        reg = torch.sum(torch.abs(r) ** 2, dim=-1)
        return lam * torch.sum(reg) / (reg.shape[0] * batch_scale)
    if model == "TransH":
        e = W["ent_emb"]
        norm = torch.pow(torch.sum(torch.abs(e) ** 2, -1, keepdim=True), 0.5)
        scale = torch.sum(torch.clamp(norm ** 2 - 1, min=0))
        orth = torch.sum(W["rel_hyper"] * W["rel_emb"], -1)
        orth = torch.pow(orth / torch.linalg.norm(W["rel_emb"], dim=-1), 2) - 1e-18
        return lam * (scale + torch.sum(torch.clamp(orth, min=0)))
    if model == "RESCAL":
        e_norm = torch.mean(torch.sum(torch.abs(W["ent_emb"]) ** 2, -1))
        r_norm = torch.mean(torch.sum(torch.abs(W["rel_inter"]) ** 2, dim=(1, 2)))
        return lam * (e_norm + r_norm)
    return 0.0


def train_step(model, weights, pos, neg_ids, score=("lp", 2.0), loss=("hinge", 1.0), lr=0.01, constraint=True,
               constraint_weight=1.0, side="h+t", train=True, batch_scale=1.0, limit=None,
               clip_norm=5.0, dtype=F64, optimizer="sgd", adam=(0.9, 0.999, 1e-7), adam_state=None):
    """One reference step with injected negatives. Returns dict with loss,
    pos_score, neg_score, weights (numpy, updated) and norm2 per variable.

    optimizer "sgd": keras SGD (sparse ResourceScatterAdd of -lr * g).
    optimizer "adam": keras Adam (OptimizerV2, TF 2.5), BaseModel.py:243-246
    (the reference's default optimizer), applied at :328. ``adam_state`` =
    {"t": steps done so far, "slots": {name: (m, v)}} carries the slots and
    ``optimizer.iterations`` from one call to the next (None: the first step,
    zero slots); the returned dict holds the advanced state under "adam".
    Per variable, with t = iterations + 1:
      sparse (IndexedSlices; _resource_apply_sparse_duplicate_indices sums the
      duplicates first): m = b1 m over every row, then scatter-add (1-b1) g;
      v likewise with (1-b2) g^2;
      dense (ResourceApplyAdam): m += (g - m)(1-b1), v += (g^2 - v)(1-b2);
      both: var -= lr_t m / (sqrt(v) + eps), lr_t = lr sqrt(1-b2^t) / (1-b1^t),
      over every row."""
    W = {k: torch.tensor(np.asarray(v), dtype=dtype) for k, v in weights.items()}
    names = list(W.keys())
    pos = np.asarray(pos, dtype=np.int64)
    B = len(pos)
    Keff = len(neg_ids) // max(B, 1)
    negt = corrupt(pos, neg_ids, Keff, side)
    cfg = {"constraint": constraint, "constraint_weight": constraint_weight, "limit": limit}
    L = _Lookups(W, train)
    if train:
        for w in W.values():
            w.requires_grad_(True)
    with torch.set_grad_enabled(train):
        cterm = _constraint(model, W, L, torch.as_tensor(pos), cfg, batch_scale)
        ps = _score_hrt(model, W, L, pos[:, 0], pos[:, 1], pos[:, 2], score, cfg)
        ns = _score_hrt(model, W, L, negt[:, 0], negt[:, 1], negt[:, 2], score, cfg)
        lval = loss_fn(loss, ps, ns, batch_scale) + cterm
    out = {"loss": float(lval.detach()), "pos_score": ps.detach().numpy(), "neg_score": ns.detach().numpy(),
           "norm2": {}}
    if optimizer == "adam" and train:
        st = adam_state or {"t": 0, "slots": {}}
        t_adam = st["t"] + 1
        slots = {k: (torch.as_tensor(np.asarray(m), dtype=dtype).clone(), torch.as_tensor(np.asarray(v), dtype=dtype).clone())
                 for k, (m, v) in st["slots"].items()}
    if train:
        leaves = [x[2] for x in L.rec]
        grads = torch.autograd.grad(lval, [W[n] for n in names] + leaves, allow_unused=True)
        dense = dict(zip(names, grads[:len(names)]))
        slices = {}
        for (n, idx, _), g in zip(L.rec, grads[len(names):]):
            if g is not None:
                slices.setdefault(n, []).append((idx, g))
        with torch.no_grad():
            for n in names:
                w = W[n]
                w.requires_grad_(False)
                dg, sl = dense.get(n), slices.get(n, [])
                if dg is None and not sl:
                    continue
                if dg is not None:
                    tot = dg.clone()
                    for idx, g in sl:
                        tot.index_add_(0, idx, g)
                    l2 = torch.sum(tot * tot)
                    out["norm2"][n] = float(l2)
                    tot = tot * clip_norm / max(math.sqrt(float(l2)), clip_norm)
                    if optimizer == "adam":
                        _adam_step(w, tot, lr, *adam, slots, n, t_adam, dense=True)
                    else:
                        w.add_(-lr * tot)
                else:
                    idx = torch.cat([i for i, _ in sl])
                    vals = torch.cat([g for _, g in sl])
                    l2 = torch.sum(vals * vals)
                    out["norm2"][n] = float(l2)
                    vals = vals * clip_norm / max(math.sqrt(float(l2)), clip_norm)
                    if optimizer == "adam":
                        _adam_step(w, torch.zeros_like(w).index_add_(0, idx, vals), lr, *adam, slots, n, t_adam,
                                   dense=False)
                    else:
                        w.index_add_(0, idx, -lr * vals)
        if optimizer == "adam":
            out["adam"] = {"t": t_adam, "slots": {k: (m.numpy(), v.numpy()) for k, (m, v) in slots.items()}}
    out["weights"] = {k: v.detach().numpy() for k, v in W.items()}
    return out


def train_step_chunked(model, weights, pos, neg_ids, score=("lp", 2.0), loss=("hinge", 1.0), lr=0.01,
                       constraint=True, constraint_weight=1.0, side="h+t", limit=None, clip_norm=5.0, dtype=F64,
                       chunk=32):
    """``train_step`` (SGD, training) in chunks of ``chunk`` positives, for
    full-size cases whose per-triple relation matrices (RESCAL / TransR at C4:
    [B (1+K), d, d] float64 = 10 GB per lookup) do not fit one autograd graph.

    Same math as ``train_step``: the constraint assigns and term once
    (``BaseModel.py:319``), then per chunk the scores and its share of the
    loss (``loss_fn`` with batch_scale = B / chunk: every loss is a sum over
    positives normalised by the whole batch, SANS' softmax is per positive),
    and its gradients. Per variable the slices are reduced on the fly: a
    variable with a dense contribution (the constraint term) accumulates the
    duplicate-summed tensor and its norm is taken of that; an IndexedSlices
    variable accumulates both the duplicate-summed rows and the sum of the
    slice values' squares (TF-2.5 clip_by_norm over the values). The apply is
    then ``clip_by_norm`` + keras SGD as in ``train_step`` (up to float64
    summation order)."""
    W = {k: torch.tensor(np.asarray(v), dtype=dtype) for k, v in weights.items()}
    names = list(W.keys())
    pos = np.asarray(pos, dtype=np.int64)
    B = len(pos)
    Keff = len(neg_ids) // max(B, 1)
    neg_ids = np.asarray(neg_ids, dtype=np.int64)
    cfg = {"constraint": constraint, "constraint_weight": constraint_weight, "limit": limit}
    acc = {n: torch.zeros_like(W[n]) for n in names}
    sq = {n: 0.0 for n in names}
    dense = set()
    touched = set()

    def collect(lval, L, leaves_only):
        for w in W.values():
            w.requires_grad_(True)
        leaves = [x[2] for x in L.rec]
        gs = torch.autograd.grad(lval, [W[n] for n in names] + leaves, allow_unused=True)
        for n, g in zip(names, gs[:len(names)]):
            if g is not None and not leaves_only:
                acc[n] += g
                dense.add(n)
                touched.add(n)
        for (n, idx, _), g in zip(L.rec, gs[len(names):]):
            if g is not None:
                acc[n].index_add_(0, idx, g)
                sq[n] += float(torch.sum(g * g))
                touched.add(n)

    L = _Lookups(W, True)
    for w in W.values():
        w.requires_grad_(True)
    cterm = _constraint(model, W, L, torch.as_tensor(pos), cfg, 1.0)
    total = 0.0
    if torch.is_tensor(cterm) and cterm.requires_grad:
        collect(cterm, L, False)
        total += float(cterm.detach())
    ps_all, ns_all = [], []
    for a in range(0, B, chunk):
        p = pos[a:a + chunk]
        c = len(p)
        negt = corrupt(p, neg_ids[a * Keff:(a + c) * Keff], Keff, side)
        L = _Lookups(W, True)
        ps = _score_hrt(model, W, L, p[:, 0], p[:, 1], p[:, 2], score, cfg)
        ns = _score_hrt(model, W, L, negt[:, 0], negt[:, 1], negt[:, 2], score, cfg)
        lval = loss_fn(loss, ps, ns, B / c)
        collect(lval, L, True)
        total += float(lval.detach())
        ps_all.append(ps.detach())
        ns_all.append(ns.detach())
    out = {"loss": total, "pos_score": torch.cat(ps_all).numpy(), "neg_score": torch.cat(ns_all).numpy(),
           "norm2": {}}
    with torch.no_grad():
        for n in names:
            w = W[n]
            w.requires_grad_(False)
            if n not in touched:
                continue
            l2 = float(torch.sum(acc[n] * acc[n])) if n in dense else sq[n]
            out["norm2"][n] = l2
            w.add_(acc[n] * (-lr * clip_norm / max(math.sqrt(l2), clip_norm)))
    out["weights"] = {k: v.detach().numpy() for k, v in W.items()}
    return out


def _adam_step(w, g, lr, b1, b2, eps, slots, name, t, dense):
    """keras Adam on one variable (TF 2.5 OptimizerV2): g is the clipped,
    duplicate-summed gradient (zero on rows no slice touched)."""
    m, v = slots.get(name, (torch.zeros_like(w), torch.zeros_like(w)))
    if dense:      # ResourceApplyAdam
        m = m + (g - m) * (1 - b1)
        v = v + (g * g - v) * (1 - b2)
    else:          # _resource_apply_sparse: decay every row, scatter-add the slices
        m = m * b1 + (1 - b1) * g
        v = v * b2 + (1 - b2) * (g * g)
    slots[name] = (m, v)
    lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    w.sub_(lr_t * m / (torch.sqrt(v) + eps))
