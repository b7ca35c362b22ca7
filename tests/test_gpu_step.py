"""GPU parity: the fused HIP step (libkge_hip.so through the C-ABI) vs the
float64 CPU oracle, on the same seeded inputs.

Tolerances (north_star: scores/ranks within 1e-5 fp32, negative ids
bit-exact): sampled ids exact; loss / scores |got - ref| <= 1e-5 * max(1, |ref|);
updated tables |got - ref| <= 1e-5 elementwise.
"""

import math
import os

import numpy as np
import pytest
import torch

from oracle import kge_oracle as orc

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _make(model_name, d, K, side, score_fn, loss_fn, E, R, sampler, constraint=True, k=None):
    from KGE.models.semantic_based.DistMult import DistMult
    from KGE.models.semantic_based.RESCAL import RESCAL
    from KGE.models.translating_based.RotatE import RotatE
    from KGE.models.translating_based.TransD import TransD
    from KGE.models.translating_based.TransE import TransE
    from KGE.models.translating_based.TransH import TransH
    from KGE.models.translating_based.TransR import TransR
    common = dict(loss_fn=loss_fn, ns_strategy=sampler)
    if model_name == "TransH":
        m = TransH({"embedding_size": d}, K, side, score_fn=score_fn, constraint=constraint, constraint_weight=0.3,
                   **common)
    elif model_name == "TransD":
        m = TransD({"ent_embedding_size": d, "rel_embedding_size": k or d}, K, side, score_fn=score_fn,
                   constraint=constraint, **common)
    elif model_name == "TransE":
        m = TransE({"embedding_size": d}, K, side, score_fn=score_fn, constraint=constraint, **common)
    elif model_name == "RotatE":
        m = RotatE({"embedding_size": d}, K, side, score_fn=score_fn, **common)
    elif model_name == "TransR":
        m = TransR({"ent_embedding_size": d, "rel_embedding_size": k or d}, K, side, score_fn=score_fn,
                   constraint=constraint, **common)
    elif model_name == "RESCAL":
        m = RESCAL({"embedding_size": d}, K, side, constraint=constraint, constraint_weight=0.5, **common)
    else:
        m = DistMult({"embedding_size": d}, K, side, constraint=constraint, **common)
    m.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    return m


def _weights(model_name, E, R, d, rng, k=None):
    if model_name == "RotatE":
        return {"ent_emb": rng.uniform(-0.5, 0.5, (E, d, 2)).astype(np.float32),
                "rel_emb": rng.uniform(-0.5, 0.5, (R, d)).astype(np.float32)}
    if model_name == "TransR":
        k = k or d
        return {"ent_emb": rng.uniform(-0.5, 0.5, (E, d)).astype(np.float32),
                "rel_emb": rng.uniform(-0.5, 0.5, (R, k)).astype(np.float32),
                "rel_proj": (np.eye(d, k)[None] + rng.uniform(-0.2, 0.2, (R, d, k))).astype(np.float32)}
    if model_name == "TransH":
        return {"ent_emb": rng.uniform(-0.5, 0.5, (E, d)).astype(np.float32),
                "rel_emb": rng.uniform(-0.5, 0.5, (R, d)).astype(np.float32),
                "rel_hyper": rng.uniform(-0.5, 0.5, (R, d)).astype(np.float32)}
    if model_name == "TransD":
        k = k or d
        return {"ent_emb": rng.uniform(-0.5, 0.5, (E, d)).astype(np.float32),
                "rel_emb": rng.uniform(-0.5, 0.5, (R, k)).astype(np.float32),
                "ent_proj": rng.uniform(-0.5, 0.5, (E, d)).astype(np.float32),
                "rel_proj": rng.uniform(-0.5, 0.5, (R, k)).astype(np.float32)}
    if model_name == "RESCAL":
        return {"ent_emb": rng.uniform(-0.5, 0.5, (E, d)).astype(np.float32),
                "rel_inter": rng.uniform(-0.2, 0.2, (R, d, d)).astype(np.float32)}
    rk = "rel_inter" if model_name == "DistMult" else "rel_emb"
    return {"ent_emb": rng.uniform(-0.5, 0.5, (E, d)).astype(np.float32),
            rk: rng.uniform(-0.5, 0.5, (R, d)).astype(np.float32)}


def _spec_score(s):
    from KGE import score
    if isinstance(s, score.Dot):
        return ("dot", 0.0)
    return ("lp" if type(s) is score.LpDistance else "lppow", float(s.p))


def _spec_loss(lf):
    from KGE import loss
    t = type(lf)
    if t is loss.PairwiseHingeLoss:
        return ("hinge", lf.margin)
    if t is loss.PairwiseLogisticLoss:
        return ("logistic",)
    if t is loss.BinaryCrossEntropyLoss:
        return ("bce",)
    if t is loss.SelfAdversarialNegativeSamplingLoss:
        return ("sans", lf.margin, lf.temperature)
    return ("sqerr",)


def _init_world1(dist, dev):
    """One-rank RCCL process group through a file store (no TCP port to race for)."""
    import tempfile
    path = os.path.join(tempfile.mkdtemp(prefix="kge_pg_"), "store")
    dist.init_process_group("nccl", init_method="file://" + path, rank=0, world_size=1, device_id=dev)


def run_case(hiplib, model_name, d, B, K, side, score_fn, loss_fn, E=50, R=7, idx=torch.int64, train=True,
             seed=11, constraint=True, typed=None, lr=0.05, opt="sgd", flags=0, k=None, pos=None, W=None,
             oracle_dtype=None, oracle_loss=None, oracle_chunk=None):
    from KGE import engine, optimizers
    from KGE.ns_strategy import TypedStrategy, UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(seed)
    W = _weights(model_name, E, R, d, rng, k) if W is None else W
    if pos is None:
        pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
    pos = np.asarray(pos, dtype=np.int64)
    if typed is None:
        sampler = UniformStrategy(np.arange(E), seed=seed)
    else:
        sampler = TypedStrategy(None, {"ind2type": typed}, seed=seed)
    m = _make(model_name, d, K, side, score_fn, loss_fn, E, R, sampler, constraint, k)
    m.model_weights = {k: torch.tensor(v, device=dev) for k, v in W.items()}
    step = engine.FusedStep(m)
    step.flags = flags
    Keff = 2 * (K // 2) if side == "h+t" else K
    ps = torch.zeros(B, dtype=torch.float32, device=dev)
    ns = torch.zeros(B * Keff, dtype=torch.float32, device=dev)
    batch = torch.tensor(pos, device=dev, dtype=idx)
    plane = sampler.offset
    # sampled ids are also returned through a standalone call of the same planes
    o = (optimizers.SGD(lr) if opt == "sgd" else optimizers.Adam(lr)) if train else None
    step(batch, train, o, pos_score=ps, neg_score=ns)
    torch.cuda.synchronize()
    step.check_status()
    i64 = idx == torch.int64
    tt = orc.typed_tables(typed) if typed is not None else None
    neg = orc.negatives(pos, K, side, E, seed=seed, plane=plane, i64=i64,
                        sampler="typed" if typed is not None else "uniform", typed=tt)
    lim = getattr(m, "limit", None)
    sc = _spec_score(getattr(m, "score_fn", None)) if model_name not in ("DistMult", "RESCAL") else ("dot", 0.0)
    lo = _spec_loss(loss_fn) if oracle_loss is None else oracle_loss
    if oracle_chunk:   # full-size cases: the same oracle step, one autograd graph per chunk of positives
        assert train and opt == "sgd"
        ref = orc.train_step_chunked(model_name, W, pos, neg, score=sc, loss=lo, lr=lr,
                                     constraint=constraint if model_name != "RotatE" else False, side=side,
                                     limit=lim, constraint_weight=getattr(m, "constraint_weight", 1.0),
                                     chunk=oracle_chunk)
    else:
        ref = orc.train_step(model_name, W, pos, neg, score=sc, loss=lo,
                             lr=lr, constraint=constraint if model_name != "RotatE" else False, side=side, train=train,
                             limit=lim, optimizer=opt, constraint_weight=getattr(m, "constraint_weight", 1.0),
                             **({} if oracle_dtype is None else {"dtype": oracle_dtype}))
    got = {k: v.cpu().numpy() for k, v in m.model_weights.items()}
    return ref, got, float(step.loss_out.item()), ps.cpu().numpy(), ns.cpu().numpy(), step, neg


def check(ref, got, loss, ps, ns):
    if math.isnan(ref["loss"]):
        assert math.isnan(loss)
    else:
        assert abs(loss - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), (loss, ref["loss"])
    np.testing.assert_allclose(ps, ref["pos_score"], rtol=TOL, atol=TOL)
    np.testing.assert_allclose(ns, ref["neg_score"], rtol=TOL, atol=TOL)
    for k in ref["weights"]:
        np.testing.assert_allclose(got[k], ref["weights"][k], rtol=0, atol=TOL, err_msg=k)


def _scores():
    from KGE import score
    return [score.LpDistance(2), score.LpDistance(1), score.LpDistance(np.inf), score.LpDistancePow(2),
            score.LpDistancePow(1), score.Dot()]


def _losses():
    from KGE import loss
    return [loss.PairwiseHingeLoss(1.0), loss.PairwiseLogisticLoss(), loss.BinaryCrossEntropyLoss(),
            loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), loss.SquareErrorLoss()]


@pytest.mark.parametrize("si", range(6))
@pytest.mark.parametrize("li", range(5))
def test_transe_matrix(hiplib, si, li):
    s, l_ = _scores()[si], _losses()[li]
    ref, got, loss, ps, ns, _, _ = run_case(hiplib, "TransE", 16, 9, 4, "h+t", s, l_)
    check(ref, got, loss, ps, ns)


@pytest.mark.parametrize("tail", [(6.0, 7.5), (5.5, 3.0), (4.0, 6.25), (7.0, 2.5), (8.0, 1.5), (3.5, 6.0)])
def test_hinge_negative_on_the_margin(hiplib, tail):
    """A negative exactly on the hinge margin (margin + s - s_pos == 0 in fp32):
    the reference's clip_by_value passes the gradient on the closed interval,
    and the step must take that one decision for the negative's own row AND
    for its positive's rows. Positive (e0, r0, e1) with h + r - t = (-3, -4)
    (s_pos = -5 exactly); tail e2 at a non-square distance in [5, 10] and
    margin = fl32(sqrt(R_neg) - 5), so (margin + s) - s_pos is exactly 0
    (Sterbenz). The oracle (float32) runs with the margin raised by 1e-5, so
    every boundary term is active there whatever its host's sqrt rounding;
    the hinge weight does not depend on the margin, so the updated rows must
    agree, and the loss within its tolerance."""
    from KGE import loss, score
    rn = np.float32(tail[0]) ** 2 + np.float32(tail[1]) ** 2
    margin = float(np.float32(np.sqrt(rn, dtype=np.float32) - np.float32(5.0)))
    assert (np.float32(margin) - np.sqrt(rn, dtype=np.float32)) - np.float32(-5.0) == 0.0
    W = {"ent_emb": np.array([[0, 0, 0, 0], [3, 4, 0, 0], [tail[0], tail[1], 0, 0]], np.float32),
         "rel_emb": np.zeros((1, 4), np.float32)}
    pos = np.tile(np.array([[0, 0, 1]], np.int64), (16, 1))
    ref, got, l_, ps, ns, _, neg = run_case(hiplib, "TransE", 4, 16, 4, "t", score.LpDistance(2),
                                            loss.PairwiseHingeLoss(margin), E=3, R=1, constraint=False, W=W,
                                            pos=pos, oracle_dtype=torch.float32,
                                            oracle_loss=("hinge", margin + 1e-5))
    assert (np.asarray(neg) == 2).any()   # the boundary tail was drawn
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("side", ["h", "t", "h+t"])
@pytest.mark.parametrize("d,K,B", [(200, 256, 4), (50, 3, 17), (64, 1, 40), (128, 64, 6), (512, 16, 3)])
def test_transe_shapes(hiplib, side, d, K, B):
    from KGE import loss, score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransE", d, B, K, side, score.LpDistance(2),
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0))
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("li", range(5))
@pytest.mark.parametrize("constraint", [True, False])
def test_distmult(hiplib, li, constraint):
    ref, got, loss, ps, ns, _, _ = run_case(hiplib, "DistMult", 24, 10, 6, "h+t", None, _losses()[li],
                                            constraint=constraint)
    check(ref, got, loss, ps, ns)


@pytest.mark.parametrize("si", range(5))
@pytest.mark.parametrize("d", [16, 256, 25])
def test_rotate(hiplib, si, d):
    from KGE import loss
    s = _scores()[si]
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "RotatE", d, 7, 6, "h+t", s,
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0))
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("li", range(5))
@pytest.mark.parametrize("side", ["h+t", "t"])
def test_rescal(hiplib, li, side):
    """RESCAL (MFMA context / projection / dR passes + dot-product stream):
    R = 3 relations over 40 positives, so relation groups span several
    16-positive tiles; d = 24 pads the 16-wide MFMA tiles."""
    ref, got, loss, ps, ns, _, _ = run_case(hiplib, "RESCAL", 24, 40, 6, side, None, _losses()[li], R=3)
    check(ref, got, loss, ps, ns)


@pytest.mark.parametrize("d,B,K,R", [(200, 24, 64, 5), (64, 70, 4, 2), (17, 9, 3, 12)])
def test_rescal_shapes(hiplib, d, B, K, R):
    """C4's RESCAL shape at reduced batch (d = 200, K = 64), a 35-positive
    relation group, and an odd d with more relations than positives."""
    from KGE import loss
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "RESCAL", d, B, K, "h+t", None, loss.SquareErrorLoss(), R=R,
                                          E=300)
    check(ref, got, l_, ps, ns)


def test_rescal_validation_and_adam(hiplib):
    from KGE import loss
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "RESCAL", 32, 12, 4, "h+t", None, loss.SquareErrorLoss(),
                                          train=False)
    check(ref, got, l_, ps, ns)
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "RESCAL", 32, 12, 4, "h+t", None,
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), opt="adam", lr=0.01)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("si", [0, 1, 2, 3, 5])
@pytest.mark.parametrize("li", [0, 3, 4])
def test_transr(hiplib, si, li):
    """TransR (three per-positive MFMA products + clip) vs the oracle: every
    score kind x hinge / SANS / square error; d != k; some rows clipped."""
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransR", 24, 10, 6, "h+t", _scores()[si], _losses()[li], k=20)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("d,k,B,K,side,constraint", [(200, 200, 6, 64, "h+t", True), (32, 48, 17, 3, "t", True),
                                                      (40, 16, 9, 5, "h", False), (17, 33, 5, 70, "h+t", True),
                                                      (100, 120, 5, 20, "h+t", True), (240, 256, 4, 40, "t", True)])
def test_transr_shapes(hiplib, d, k, B, K, side, constraint):
    """C4's TransR shape (d = k = 200, K = 64) at reduced batch; odd sizes;
    the constraint off (no clip, no table assigns). Together the cases reach
    every row-tile count (1-5: K + 0..15 rounded to 16) and column-chunk count
    (4, 8, 13, 16) the two-per-CU kernel is instantiated for."""
    from KGE import loss, score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransR", d, B, K, side, score.LpDistancePow(2),
                                          loss.PairwiseHingeLoss(1.0), k=k, constraint=constraint, E=90, R=4)
    check(ref, got, l_, ps, ns)


def _fb15k237():
    z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data",
                             "fb15k237_train.npz"))
    return z["triples"].astype(np.int64), int(z["n_entities"]), int(z["n_relations"])


def _c4_batch(B, seed):
    """B positives drawn from FB15k-237 train_indexed (E = 14,505, R = 237):
    the relation-grouped passes see ~135 live relations at B = 512 (the C4
    bench batch's count, profiles/r03e/bench_c4-rescal.json)."""
    X, E, R = _fb15k237()
    rng = np.random.default_rng(seed)
    pos = X[rng.choice(len(X), B, replace=False)]
    return pos, E, R


@pytest.mark.parametrize("B", [512, 128])
def test_rescal_c4_full_size(hiplib, B):
    """RESCAL at the C4 shape (RESCAL.py:140-200): d = 200, K = 64 'h+t',
    SquareError, constraint (dense Lp regulariser over both full tables), SGD,
    E = 14,505, R = 237, positives real FB15k-237 rows (B = 512: ~135 live
    relations; the relation rank, per-relation segments, MFMA context / dR
    strips and the fused dense apply at their bench sizes) vs the float64
    oracle, chunked by 32 positives (its per-triple R_r lookups would be
    [B (1+K), d, d] = 10 GB in one graph)."""
    from KGE import loss
    pos, E, R = _c4_batch(B, 40 + B)
    assert len(np.unique(pos[:, 1])) >= (100 if B == 512 else 50)
    rng = np.random.default_rng(B)
    W = _weights("RESCAL", E, R, 200, rng)
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "RESCAL", 200, B, 64, "h+t", None, loss.SquareErrorLoss(),
                                          E=E, R=R, pos=pos, W=W, lr=0.01, oracle_chunk=32)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("B", [512, 128])
def test_transr_c4_full_size(hiplib, B):
    """TransR at the C4 shape (TransR.py:154-211): d = k = 200, K = 64 'h+t',
    LpDistancePow(2), hinge(1), constraint (table clip + clip of every
    projected vector), SGD, E = 14,505, R = 237, real FB15k-237 positives
    (~135 live relations at B = 512: the relation rank, per-positive MFMA
    products, the dM strips and transr_proj_apply at their bench sizes) vs
    the float64 oracle, chunked by 32 positives."""
    from KGE import loss, score
    pos, E, R = _c4_batch(B, 50 + B)
    rng = np.random.default_rng(B + 1)
    W = _weights("TransR", E, R, 200, rng)
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransR", 200, B, 64, "h+t", score.LpDistancePow(2),
                                          loss.PairwiseHingeLoss(1.0), E=E, R=R, pos=pos, W=W, lr=0.01,
                                          oracle_chunk=32)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("model_name", ["RESCAL", "TransR"])
def test_c4_full_size_properties(hiplib, model_name):
    """C4 at bench size (B = 512, K = 64, d = 200, FB15k-237 positives):
    finite loss, the hinge / square-error loss >= 0, and a second identical
    step from the same state and planes reproduces the first bit for bit
    (no float atomics in the relation-grouped passes)."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    pos, E, R = _c4_batch(512, 7)
    rng = np.random.default_rng(9)
    W = _weights(model_name, E, R, 200, rng)
    outs = []
    for _ in range(2):
        if model_name == "RESCAL":
            m = _make("RESCAL", 200, 64, "h+t", None, loss.SquareErrorLoss(), E, R, UniformStrategy(np.arange(E), seed=5))
        else:
            m = _make("TransR", 200, 64, "h+t", score.LpDistancePow(2), loss.PairwiseHingeLoss(1.0), E, R,
                      UniformStrategy(np.arange(E), seed=5))
        m.model_weights = {k: torch.tensor(v, device=dev) for k, v in W.items()}
        step = engine.FusedStep(m)
        ps = torch.zeros(512, device=dev)
        ns = torch.zeros(512 * 64, device=dev)
        step(torch.tensor(pos, device=dev), True, optimizers.SGD(0.01), pos_score=ps, neg_score=ns)
        torch.cuda.synchronize()
        step.check_status()
        outs.append((float(step.loss_out.item()), {k: v.clone() for k, v in m.model_weights.items()}, ps, ns))
    l0 = outs[0][0]
    assert math.isfinite(l0) and l0 >= 0
    for k in W:
        assert bool(torch.isfinite(outs[0][1][k]).all()), k
        assert torch.equal(outs[0][1][k], outs[1][1][k]), k
        assert not np.array_equal(outs[0][1][k].cpu().numpy(), W[k]), k
    assert torch.equal(outs[0][2], outs[1][2]) and torch.equal(outs[0][3], outs[1][3])
    assert l0 == outs[1][0]


def test_transr_validation_and_adam(hiplib):
    from KGE import loss, score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransR", 32, 12, 4, "h+t", score.LpDistancePow(2),
                                          loss.PairwiseHingeLoss(1.0), train=False)
    check(ref, got, l_, ps, ns)
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransR", 32, 12, 4, "h+t", score.LpDistance(2),
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), opt="adam", lr=0.01)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("si", range(6))
@pytest.mark.parametrize("li", range(5))
def test_transh_matrix(hiplib, si, li):
    """TransH (hyperplane projection, projection-family kernel) vs the oracle,
    every score x loss; constraint on: rel_hyper renormalised, soft +
    orthogonality terms make all three gradients dense."""
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransH", 24, 10, 6, "h+t", _scores()[si], _losses()[li])
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("si", range(6))
@pytest.mark.parametrize("li", range(5))
def test_transd_matrix(hiplib, si, li):
    """TransD (rank-1 r_p e_p^T + I projection, clipped) vs the oracle, every
    score x loss, d != k (identity block of min(d, k))."""
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransD", 24, 10, 6, "h+t", _scores()[si], _losses()[li], k=20)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("model_name", ["TransE", "RotatE", "TransR", "TransH", "TransD"])
@pytest.mark.parametrize("kind,p", [("lp", 3.0), ("lppow", 1.5), ("lp", 0.5)])
@pytest.mark.parametrize("li", [0, 3])
def test_general_p(hiplib, model_name, kind, p, li):
    """LpDistance / LpDistancePow with p outside {1, 2, inf} (score.py:49-76)
    on the fused kernels (SK_PGEN) vs the oracle."""
    from KGE import score
    s = (score.LpDistance if kind == "lp" else score.LpDistancePow)(p)
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, model_name, 24, 9, 6, "h+t", s, _losses()[li],
                                          k=20 if model_name in ("TransR", "TransD") else None)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("model_name", ["TransH", "TransD"])
@pytest.mark.parametrize("d,k,B,K,side,constraint", [(200, 200, 6, 64, "h+t", True), (32, 48, 17, 3, "t", True),
                                                      (40, 16, 9, 5, "h", False), (17, 33, 5, 70, "h+t", True),
                                                      (50, 50, 12, 1, "t", False), (200, 120, 3, 256, "h+t", False),
                                                      (6, 6, 8, 9, "h+t", True)])
def test_projection_shapes(hiplib, model_name, d, k, B, K, side, constraint):
    """Row widths on every fragment layout (vec 4 / 2 / 1, one or two
    chunks), K = 1 and K = 256, slots past a batch, constraint on / off."""
    from KGE import loss, score
    if model_name == "TransH":
        k = None
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, model_name, d, B, K, side, score.LpDistancePow(2),
                                          loss.SelfAdversarialNegativeSamplingLoss(2.0, 0.5), k=k,
                                          constraint=constraint, E=90, R=4)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("model_name", ["TransH", "TransD"])
@pytest.mark.parametrize("constraint", [True, False])
def test_projection_validation_and_adam(hiplib, model_name, constraint):
    from KGE import loss, score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, model_name, 32, 12, 4, "h+t", score.LpDistancePow(2),
                                          loss.PairwiseHingeLoss(1.0), train=False, constraint=constraint, k=24)
    check(ref, got, l_, ps, ns)
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, model_name, 32, 12, 4, "h+t", score.LpDistance(2),
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), opt="adam", lr=0.01,
                                          constraint=constraint, k=24)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("model_name", ["TransH", "TransD"])
def test_projection_consecutive_steps(hiplib, model_name):
    """Three steps through one workspace (the aux pass keeps the lists for the
    main pass, which then resets them) == three oracle steps."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(17)
    E, R, d, B, K = 70, 5, 40, 13, 8
    W = _weights(model_name, E, R, d, rng)
    sampler = UniformStrategy(np.arange(E), seed=3)
    m = _make(model_name, d, K, "h+t", score.LpDistance(1), loss.PairwiseHingeLoss(1.0), E, R, sampler)
    m.model_weights = {k: torch.tensor(v, device=dev) for k, v in W.items()}
    step = engine.FusedStep(m)
    opt = optimizers.SGD(0.05)
    ref_w = W
    for it in range(3):
        pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
        plane = sampler.offset
        step(torch.tensor(pos, device=dev), True, opt)
        torch.cuda.synchronize()
        step.check_status()
        neg = orc.negatives(pos, K, "h+t", E, seed=3, plane=plane)
        ref = orc.train_step(model_name, ref_w, pos, neg, score=("lp", 1.0), loss=("hinge", 1.0), lr=0.05,
                             constraint_weight=getattr(m, "constraint_weight", 1.0))
        ref_w = ref["weights"]
        assert abs(float(step.loss_out.item()) - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), it
        for k, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[k].cpu().numpy(), v, atol=TOL, err_msg="%s step %d" % (k, it))


def test_c1_workload(hiplib):
    """C1 exactly (BASELINE configs[0], example_fit_from_numpy.py pattern):
    TransE d=50, B=128, K=1 corrupt_side='t', PairwiseHinge(1), LpDistance(2),
    uniform, constraint, SGD -- on FB15k-237 ids from data/."""
    import os
    from KGE import loss, score
    z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data",
                             "fb15k237_train.npz"))
    X = z["triples"].astype(np.int64)
    E, R = int(z["n_entities"]), int(z["n_relations"])
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransE", 50, 128, 1, "t", score.LpDistance(2),
                                          loss.PairwiseHingeLoss(1.0), E=E, R=R, lr=0.01, pos=X[:128])
    check(ref, got, l_, ps, ns)


def test_rotate_k256_cross_wave_merge(hiplib):
    """RotatE at C3's K = 256 (4 waves per positive: the cross-wave online
    softmax merge of the complex accumulators) vs the oracle."""
    from KGE import loss, score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "RotatE", 64, 5, 256, "h+t", score.LpDistance(1),
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E=400)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("B,idx", [(3, torch.int64), (9, torch.int64), (4, torch.int32)])
def test_rotate_c3_kernel_instance(hiplib, B, idx):
    """The exact instance the C3 bench times (RotatE.py:126-165): d = 256
    complex (512-float rows -> two fragment chunks, score_kernel<RotatE, 4, 2,
    SK_P1, h+t>), K = 256 'h+t' (four waves per positive: the cross-wave
    online-softmax merge), LpDistance(1), SANS(3, 1) -- vs the oracle; B = 9
    puts two positives in one workgroup and a partial last workgroup."""
    from KGE import loss, score
    ref, got, l_, ps, ns, step, _ = run_case(hiplib, "RotatE", 256, B, 256, "h+t", score.LpDistance(1),
                                             loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E=700, R=11,
                                             idx=idx, lr=0.01)
    check(ref, got, l_, ps, ns)


def test_c3_full_size_properties(hiplib):
    """C3 at its full size (B = 1024, K = 256, d = 256, E = 14,505, R = 237):
    finite loss and scores <= 0, and a second identical step from the same
    state reproduces the first bit for bit (destination-major update, no
    float atomics)."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    E, R, d, B, K = 14505, 237, 256, 1024, 256
    g = torch.Generator(device="cpu").manual_seed(3)
    lim = 5.0 / d
    ent0 = ((torch.rand(E, d, 2, generator=g) * 2 - 1) * lim).to(dev)
    rel0 = ((torch.rand(R, d, generator=g) * 2 - 1) * lim).to(dev)
    pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                       torch.randint(0, E, (B,), generator=g)], 1).to(dev)
    outs = []
    for _ in range(2):
        m = _make("RotatE", d, K, "h+t", score.LpDistance(1), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
                  E, R, UniformStrategy(np.arange(E), seed=8))
        m.model_weights = {"ent_emb": ent0.clone(), "rel_emb": rel0.clone()}
        step = engine.FusedStep(m)
        ps = torch.zeros(B, device=dev)
        ns = torch.zeros(B * K, device=dev)
        step(pos, True, optimizers.SGD(0.01), pos_score=ps, neg_score=ns)
        torch.cuda.synchronize()
        step.check_status()
        outs.append((float(step.loss_out.item()), m.model_weights["ent_emb"].clone(),
                     m.model_weights["rel_emb"].clone(), ps, ns, step.norm2.clone()))
    loss0 = outs[0][0]
    assert math.isfinite(loss0) and loss0 > 0
    assert bool((outs[0][3] <= 0).all()) and bool((outs[0][4] <= 0).all())
    assert bool(torch.isfinite(outs[0][1]).all()) and bool(torch.isfinite(outs[0][2]).all())
    assert not torch.equal(outs[0][1], ent0) and not torch.equal(outs[0][2], rel0)
    for a, b in zip(outs[0][1:], outs[1][1:]):
        assert torch.equal(a, b)
    assert loss0 == outs[1][0]


@pytest.mark.parametrize("model_name", ["TransE", "DistMult", "RotatE", "TransR", "TransH", "TransD"])
def test_compact_update_large_table(hiplib, model_name):
    """E = 6000 rows vs 8 x (5 + 3) keys: the update kernel visits only the
    destinations the step touched (compact launch), untouched rows unchanged."""
    from KGE import loss, score
    sc = None if model_name == "DistMult" else score.LpDistance(2)
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, model_name, 32, 8, 5, "h+t", sc,
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E=6000, R=9,
                                          constraint=False)
    check(ref, got, l_, ps, ns)


def test_compact_update_consecutive_steps(hiplib):
    """Three steps through one workspace in compact mode (the touched-list
    counter resets itself) == three oracle steps."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(8)
    E, R, d, B, K = 3000, 5, 40, 11, 6
    W = _weights("TransE", E, R, d, rng)
    sampler = UniformStrategy(np.arange(E), seed=6)
    m = _make("TransE", d, K, "h+t", score.LpDistance(1), loss.PairwiseHingeLoss(1.0), E, R, sampler,
              constraint=False)
    m.model_weights = {k: torch.tensor(v, device=dev) for k, v in W.items()}
    step = engine.FusedStep(m)
    opt = optimizers.SGD(0.05)
    ref_w = W
    for it in range(3):
        pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
        plane = sampler.offset
        step(torch.tensor(pos, device=dev), True, opt)
        torch.cuda.synchronize()
        step.check_status()
        neg = orc.negatives(pos, K, "h+t", E, seed=6, plane=plane)
        ref = orc.train_step("TransE", ref_w, pos, neg, score=("lp", 1.0), loss=("hinge", 1.0), lr=0.05,
                             constraint=False)
        ref_w = ref["weights"]
        for k, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[k].cpu().numpy(), v, atol=TOL, err_msg="%s step %d" % (k, it))


def test_int32_ids_and_validation_step(hiplib):
    from KGE import loss, score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransE", 32, 12, 4, "h+t", score.LpDistance(2),
                                          loss.PairwiseHingeLoss(1.0), idx=torch.int32)
    check(ref, got, l_, ps, ns)
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransE", 32, 12, 4, "h+t", score.LpDistance(2),
                                          loss.PairwiseHingeLoss(1.0), train=False)
    check(ref, got, l_, ps, ns)


def test_typed_sampler(hiplib):
    from KGE import loss, score
    E = 40
    typed = ["A"] * 15 + ["B"] * 20 + ["C"] * 5
    ref, got, l_, ps, ns, _, neg = run_case(hiplib, "TransE", 16, 10, 6, "h+t", score.LpDistance(2),
                                            loss.PairwiseHingeLoss(1.0), E=E, typed=typed)
    check(ref, got, l_, ps, ns)


def test_tiny_entity_set_overflow_path(hiplib):
    """E = 3 with many negatives: every update bucket overflows the LDS list."""
    from KGE import loss, score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransE", 16, 300, 40, "h+t", score.LpDistance(2),
                                          loss.SelfAdversarialNegativeSamplingLoss(1.0, 0.5), E=3, R=2)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("li", [0, 3])
def test_destination_list_overflow(hiplib, li):
    """KGE_FLAG_DEBUG_LIST_CAP: 4-entry destination lists, so most keys go
    through the overflow list and the update kernel's selection path."""
    from KGE import score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransE", 32, 24, 16, "h+t", score.LpDistance(2),
                                          _losses()[li], E=40, R=5, flags=2)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("model_name", ["TransE", "TransR", "TransD"])
def test_zipf_skewed_batch(hiplib, model_name):
    """Skewed keys (SURVEY 8(d) C5 shape): one entity takes 30% of the
    negative draws (~600 keys for one destination), one relation 40% of the
    positives -- lists far past their capacity go through the gather + LDS
    bitonic-sort path of the update kernel; == the oracle."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(31)
    E, R, d, B, K = 300, 6, 32, 64, 32
    k = 24 if model_name in ("TransR", "TransD") else None
    W = _weights(model_name, E, R, d, rng, k)
    rels = np.where(rng.random(B) < 0.4, 2, rng.integers(0, R, B))
    pos = np.stack([rng.integers(0, E, B), rels, rng.integers(0, E, B)], 1).astype(np.int64)
    neg = np.where(rng.random(B * K) < 0.3, 7, rng.integers(0, E, B * K)).astype(np.int64)
    sc = score.LpDistance(2) if model_name == "TransE" else score.LpDistancePow(2)
    m = _make(model_name, d, K, "h+t", sc, loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E, R,
              UniformStrategy(np.arange(E), seed=1), k=k)
    m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
    step = engine.FusedStep(m)
    step(torch.tensor(pos, device=dev), True, optimizers.SGD(0.05), neg_ids=torch.tensor(neg, device=dev))
    torch.cuda.synchronize()
    step.check_status()
    ref = orc.train_step(model_name, W, pos, neg, score=_spec_score(sc), loss=("sans", 3.0, 1.0), lr=0.05)
    assert abs(float(step.loss_out.item()) - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"]))
    for kk, v in ref["weights"].items():
        np.testing.assert_allclose(m.model_weights[kk].cpu().numpy(), v, atol=TOL, err_msg=kk)


def test_consecutive_steps_reuse_workspace(hiplib):
    """Three steps through one FusedStep (one workspace: tickets, list counters
    and the overflow counter must reset themselves) == three oracle steps."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(21)
    E, R, d, B, K = 60, 6, 48, 33, 10
    W = _weights("TransE", E, R, d, rng)
    sampler = UniformStrategy(np.arange(E), seed=4)
    m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
              E, R, sampler)
    m.model_weights = {k: torch.tensor(v, device=dev) for k, v in W.items()}
    step = engine.FusedStep(m)
    opt = optimizers.SGD(0.05)
    ref_w = W
    for it in range(3):
        pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
        plane = sampler.offset
        step(torch.tensor(pos, device=dev), True, opt)
        torch.cuda.synchronize()
        step.check_status()
        neg = orc.negatives(pos, K, "h+t", E, seed=4, plane=plane)
        ref = orc.train_step("TransE", ref_w, pos, neg, score=("lp", 2.0), loss=("sans", 3.0, 1.0), lr=0.05)
        ref_w = ref["weights"]
        assert abs(float(step.loss_out.item()) - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), it
        for k, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[k].cpu().numpy(), v, atol=TOL, err_msg="%s step %d" % (k, it))


@pytest.mark.parametrize("model_name", ["TransE", "RESCAL", "TransR", "TransH"])
def test_replan_on_dirty_workspace_is_refused(hiplib, model_name):
    """kge_hip.h workspace rules: a step whose plan differs from the one
    stamped in its workspace (a caller that re-plans -- here a new batch size
    -- without re-zeroing the buffer) is refused on the device: status word
    KGE_EWORKSPACE, loss NaN, every table unchanged. After a re-zero the same
    descriptor runs and equals the oracle."""
    import ctypes
    from KGE import _hip, engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(51)
    E, R, d, K = 40, 5, 24, 4
    k = 20 if model_name == "TransR" else None
    W = _weights(model_name, E, R, d, rng, k)
    sc = {"TransE": score.LpDistance(2), "TransR": score.LpDistancePow(2), "TransH": score.LpDistancePow(2)}.get(
        model_name)
    sampler = UniformStrategy(np.arange(E), seed=2)
    m = _make(model_name, d, K, "h+t", sc, loss.SquareErrorLoss(), E, R, sampler, k=k)
    m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
    step = engine.FusedStep(m)
    opt = optimizers.SGD(0.05)
    posA = np.stack([rng.integers(0, E, 8), rng.integers(0, R, 8), rng.integers(0, E, 8)], 1).astype(np.int64)
    step(torch.tensor(posA, device=dev), True, opt)      # plan A stamps the workspace
    torch.cuda.synchronize()
    step.check_status()
    before = {kk: v.clone() for kk, v in m.model_weights.items()}
    posB = np.stack([rng.integers(0, E, 13), rng.integers(0, R, 13), rng.integers(0, E, 13)], 1).astype(np.int64)
    bB = torch.tensor(posB, device=dev)
    plane = sampler.offset
    d_ = step.describe(bB, True, opt)        # draws planes (plane, plane + 1)
    lib = _hip.lib()
    sigA = step._ws_sig
    assert lib.kge_step_plan_signature(d_) not in (0, sigA)
    need = int(lib.kge_step_workspace_bytes(d_))
    if step.workspace.numel() < need:     # grow, keeping the stamped head
        ws = torch.zeros(need, dtype=torch.uint8, device=dev)
        ws[:step.workspace.numel()] = step.workspace
        step.workspace = ws
    d_.workspace = step.workspace.data_ptr()
    d_.workspace_bytes = step.workspace.numel()
    assert lib.kge_step(ctypes.byref(d_), _hip.stream_handle(dev)) == _hip.KGE_OK   # host validation passes
    torch.cuda.synchronize()
    assert int(step.status.item()) == _hip.KGE_EWORKSPACE
    with pytest.raises(RuntimeError, match="refused"):
        step.check_status()
    assert math.isnan(float(step.loss_out.item()))
    for kk, v in m.model_weights.items():
        assert torch.equal(v, before[kk]), kk
    # re-zeroed: the same plan B runs (same draws as the refused call) and equals the oracle
    step.workspace.zero_()
    d_.sampler.offset = plane
    assert lib.kge_step(ctypes.byref(d_), _hip.stream_handle(dev)) == _hip.KGE_OK
    torch.cuda.synchronize()
    step.check_status()
    neg = orc.negatives(posB, K, "h+t", E, seed=2, plane=plane)
    Wb = {kk: v.cpu().numpy() for kk, v in before.items()}
    ref = orc.train_step(model_name, Wb, posB, neg, score=_spec_score(sc) if sc is not None else ("dot", 0.0),
                         loss=("sqerr",), lr=0.05, constraint_weight=getattr(m, "constraint_weight", 1.0))
    assert abs(float(step.loss_out.item()) - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"]))
    for kk, v in ref["weights"].items():
        np.testing.assert_allclose(m.model_weights[kk].cpu().numpy(), v, atol=TOL, err_msg=kk)


def test_update_phase_needs_its_score_pass(hiplib):
    """include/kge_hip.h split-step rule, enforced by the library through the
    C-ABI (no engine guard in the way): a KGE_FLAG_PHASE_UPDATE call runs only
    after a PHASE_SCORE call of its plan on the same workspace, once. Refused
    on the device (status KGE_EWORKSPACE, no table written) -- on a fresh
    workspace; after the score pass's workspace was re-zeroed (the silent
    no-op of the round-4 review); and for a second update. A refusal leaves
    the workspace refused (even a score pass) until it is zeroed; then score
    + update equal the oracle's SGD step (entity rows; relation gradients go
    to grad_out[1])."""
    import ctypes
    from KGE import _hip, engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(61)
    E, R, d, B, K = 40, 5, 24, 8, 4
    W = _weights("TransE", E, R, d, rng)
    m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E, R,
              UniformStrategy(np.arange(E), seed=3), constraint=False)
    m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
    step = engine.FusedStep(m)
    step.rel_grad_out = torch.zeros(R, d, device=dev)
    lib, st = _hip.lib(), _hip.stream_handle(dev)
    opt = optimizers.SGD(0.05)
    pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
    bt = torch.tensor(pos, device=dev)
    ws = None

    def run(phase):
        nonlocal ws
        step.flags = _hip.FLAG_NO_TABLE_CONSTRAINT | phase
        dd = step.describe(bt, True, opt)
        dd.sampler.offset = 0
        if ws is None:
            ws = torch.zeros(int(lib.kge_step_workspace_bytes(dd)), dtype=torch.uint8, device=dev)
        dd.workspace, dd.workspace_bytes = ws.data_ptr(), ws.numel()
        step.status.zero_()
        assert lib.kge_step(ctypes.byref(dd), st) == _hip.KGE_OK
        torch.cuda.synchronize()
        return int(step.status.item())

    def unchanged():
        for kk, v in W.items():
            assert np.array_equal(m.model_weights[kk].cpu().numpy(), v), kk

    S, U = _hip.FLAG_PHASE_SCORE, _hip.FLAG_PHASE_UPDATE
    assert run(U) == _hip.KGE_EWORKSPACE            # fresh workspace, no score pass
    unchanged()
    ws.zero_()
    assert run(S) == _hip.KGE_OK
    ws.zero_()                                       # the score pass's lists wiped
    assert run(U) == _hip.KGE_EWORKSPACE
    unchanged()
    assert run(S) == _hip.KGE_EWORKSPACE             # refused until zeroed
    ws.zero_()
    assert run(S) == _hip.KGE_OK and run(U) == _hip.KGE_OK
    neg = orc.negatives(pos, K, "h+t", E, seed=3, plane=0)
    ref = orc.train_step("TransE", W, pos, neg, score=("lp", 2.0), loss=("sans", 3.0, 1.0), lr=0.05,
                         constraint=False)
    np.testing.assert_allclose(m.model_weights["ent_emb"].cpu().numpy(), ref["weights"]["ent_emb"], atol=TOL)
    after = m.model_weights["ent_emb"].clone()
    assert run(U) == _hip.KGE_EWORKSPACE             # a second update pass
    assert torch.equal(m.model_weights["ent_emb"], after)
    # a full (non-split) step of the same plan between the passes consumes the
    # score pass's lists and clears its token: the update pass after it is refused
    ws.zero_()
    assert run(S) == _hip.KGE_OK and run(0) == _hip.KGE_OK
    after = m.model_weights["ent_emb"].clone()
    assert run(U) == _hip.KGE_EWORKSPACE
    assert torch.equal(m.model_weights["ent_emb"], after)


def test_hinge_zero_negatives_is_nan(hiplib):
    from KGE import loss, score
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "TransE", 16, 5, 1, "h+t", score.LpDistance(2),
                                          loss.PairwiseHingeLoss(1.0))
    assert math.isnan(l_) and math.isnan(ref["loss"])


def test_sampler_bit_exact(hiplib):
    """Standalone kge_sample draws == the oracle's Philox restatement."""
    from KGE.ns_strategy import TypedStrategy, UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(5)
    E = 14505
    X = np.stack([rng.integers(0, E, 1000), rng.integers(0, 237, 1000), rng.integers(0, E, 1000)], 1)
    for dt, i64 in ((torch.int64, True), (torch.int32, False)):
        s = UniformStrategy(np.arange(E), seed=123456789)
        for side in ("h", "t"):
            plane = s.offset
            got = s(torch.tensor(X, dtype=dt, device=dev), 7, side).cpu().numpy()
            exp = orc.negatives(X, 7, side, E, seed=123456789, plane=plane, i64=i64)
            assert got.dtype == (np.int64 if i64 else np.int32)
            np.testing.assert_array_equal(got, exp)
    ind2type = list(rng.integers(0, 5, E))
    t = TypedStrategy(None, {"ind2type": ind2type}, seed=99)
    plane = t.offset
    got = t(torch.tensor(X, device=dev), 5, "t").cpu().numpy()
    exp = orc.negatives(X, 5, "t", E, seed=99, plane=plane, sampler="typed", typed=orc.typed_tables(ind2type))
    np.testing.assert_array_equal(got, exp)
    assert all(ind2type[a] == ind2type[b] and a != b for a, b in zip(got, np.repeat(X[:, 2], 5)))


def test_out_of_range_ids_raise(hiplib):
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    m = _make("TransE", 16, 2, "h+t", score.LpDistance(2), loss.PairwiseHingeLoss(1.0), 10, 3,
              UniformStrategy(np.arange(10), seed=1))
    m.model_weights = {"ent_emb": torch.rand(10, 16, device=dev), "rel_emb": torch.rand(3, 16, device=dev)}
    step = engine.FusedStep(m)
    step(torch.tensor([[0, 1, 2], [11, 0, 1]], device=dev), True, optimizers.SGD(0.1))
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        step.check_status()


def test_fb15k237_bench_shape_properties(hiplib):
    """C2 shape (B=1024, K=256, d=200, E=14505): loss finite, and a second
    identical step from the same state reproduces the first bit for bit
    (deterministic destination-major update, no float atomics)."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    E, R, d, B, K = 14505, 237, 200, 1024, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    ent0 = (torch.rand(E, d, generator=g) - 0.5).to(dev)
    rel0 = (torch.rand(R, d, generator=g) - 0.5).to(dev)
    pos = torch.stack([torch.randint(0, E, (B,), generator=g), torch.randint(0, R, (B,), generator=g),
                       torch.randint(0, E, (B,), generator=g)], 1).to(dev)
    outs = []
    for _ in range(2):
        m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
                  E, R, UniformStrategy(np.arange(E), seed=5))
        m.model_weights = {"ent_emb": ent0.clone(), "rel_emb": rel0.clone()}
        step = engine.FusedStep(m)
        step(pos, True, optimizers.SGD(0.01))
        torch.cuda.synchronize()
        step.check_status()
        outs.append((float(step.loss_out.item()), m.model_weights["ent_emb"].clone(),
                     m.model_weights["rel_emb"].clone(), step.norm2.clone()))
    assert math.isfinite(outs[0][0])
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])
    assert bool(torch.isfinite(outs[0][1]).all()) and float(outs[0][3][0]) > 0


@pytest.mark.parametrize("idx", [torch.int64, torch.int32])
def test_transe_c2_full_size(hiplib, idx):
    """C2 exactly as the bench times it (BASELINE configs[1];
    BaseModel.py:293-330, TransE.py:127-174, loss.py:174-182): TransE d = 200,
    B = 1024 real FB15k-237 positives, K = 256 'h+t' in-kernel uniform draws,
    SANS(3, 1), LpDistance(2), constraint (the full-table unit-L2
    renormalisation, fused into the score / update kernels on the SGD path),
    SGD lr 0.01, E = 14,505, R = 237, the reference initialiser's range
    U(+-6/sqrt(d)) with the rows NOT yet normalised (the first step's
    renormalisation of every row, ~18 keys per row, lists at their bench
    capacities) -- vs the float64 oracle, chunked by 128 positives, at the
    same 1e-5 bar as every other case."""
    from KGE import loss, score
    X, E, R = _fb15k237()
    rng = np.random.default_rng(1024 + (idx == torch.int32))
    pos = X[rng.choice(len(X), 1024, replace=False)]
    lim = 6.0 / np.sqrt(200)
    W = {"ent_emb": rng.uniform(-lim, lim, (E, 200)).astype(np.float32),
         "rel_emb": rng.uniform(-lim, lim, (R, 200)).astype(np.float32)}
    ref, got, l_, ps, ns, _, neg = run_case(hiplib, "TransE", 200, 1024, 256, "h+t", score.LpDistance(2),
                                            loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E=E, R=R, pos=pos,
                                            W=W, lr=0.01, idx=idx, oracle_chunk=128)
    assert len(np.unique(neg)) > 0.99 * E   # (every row has a gradient: ~18 draws per row)
    check(ref, got, l_, ps, ns)


def test_rotate_c3_full_size(hiplib):
    """C3 exactly as the bench times it (BASELINE configs[2]; RotatE.py:126-165):
    RotatE d = 256 complex, B = 1024 real FB15k-237 positives, K = 256 'h+t',
    LpDistance(1), SANS(3, 1), SGD lr 0.01, E = 14,505, R = 237, weights in the
    reference initialiser's range U(+-(gamma + 2) / d) -- vs the float64
    oracle, chunked by 128 positives, at the 1e-5 bar."""
    from KGE import loss, score
    X, E, R = _fb15k237()
    rng = np.random.default_rng(256)
    pos = X[rng.choice(len(X), 1024, replace=False)]
    lim = 5.0 / 256
    W = {"ent_emb": rng.uniform(-lim, lim, (E, 256, 2)).astype(np.float32),
         "rel_emb": rng.uniform(-lim, lim, (R, 256)).astype(np.float32)}
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, "RotatE", 256, 1024, 256, "h+t", score.LpDistance(1),
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E=E, R=R, pos=pos,
                                          W=W, lr=0.01, oracle_chunk=128)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("model_name", ["TransE", "DistMult", "RotatE"])
def test_fused_adam_first_step(hiplib, model_name):
    """kge_step(KGE_OPT_GRAD) + kge_apply(KGE_OPT_ADAM) == keras Adam (oracle)."""
    from KGE import loss, score
    sc = score.LpDistance(2) if model_name != "DistMult" else None
    ref, got, l_, ps, ns, _, _ = run_case(hiplib, model_name, 32, 12, 6, "h+t", sc,
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), opt="adam", lr=0.01)
    check(ref, got, l_, ps, ns)


@pytest.mark.parametrize("model_name,constraint", [("TransE", True), ("TransE", False), ("RESCAL", True),
                                                   ("TransH", True), ("DistMult", True), ("TransR", True)])
def test_fused_adam_three_steps(hiplib, model_name, constraint):
    """keras Adam past its first step (BaseModel.py:243-246, applied at :328):
    three consecutive steps through one FusedStep and one Adam optimizer --
    the m / v slots decay on every row (sparse variables: TransE / DistMult /
    TransR) or follow ResourceApplyAdam (dense variables: RESCAL's and
    TransH's full-table regularisers) and lr_t = lr sqrt(1-b2^t)/(1-b1^t) at
    t = 1, 2, 3 -- against the oracle carrying its own slots."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(29)
    E, R, d, B, K = 45, 4, 24, 11, 6
    k = 20 if model_name == "TransR" else None
    W = _weights(model_name, E, R, d, rng, k)
    sc = {"TransE": score.LpDistance(2), "TransH": score.LpDistancePow(2), "TransR": score.LpDistancePow(2)}.get(
        model_name)
    lf = loss.SquareErrorLoss() if model_name == "RESCAL" else loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0)
    sampler = UniformStrategy(np.arange(E), seed=12)
    m = _make(model_name, d, K, "h+t", sc, lf, E, R, sampler, constraint=constraint, k=k)
    m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
    step = engine.FusedStep(m)
    opt = optimizers.Adam(0.01)
    ref_w, state = W, None
    for it in range(3):
        pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
        plane = sampler.offset
        step(torch.tensor(pos, device=dev), True, opt)
        torch.cuda.synchronize()
        step.check_status()
        assert opt.iterations == it + 1
        neg = orc.negatives(pos, K, "h+t", E, seed=12, plane=plane)
        ref = orc.train_step(model_name, ref_w, pos, neg, score=_spec_score(sc) if sc is not None else ("dot", 0.0),
                             loss=_spec_loss(lf), lr=0.01, constraint=constraint, optimizer="adam",
                             adam_state=state, constraint_weight=getattr(m, "constraint_weight", 1.0))
        ref_w, state = ref["weights"], ref["adam"]
        assert state["t"] == it + 1
        assert abs(float(step.loss_out.item()) - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), it
        for kk, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[kk].cpu().numpy(), v, atol=TOL,
                                       err_msg="%s step %d" % (kk, it + 1))
        for kk, (ms, vs) in state["slots"].items():
            got = opt.slots[kk]
            np.testing.assert_allclose(got["m"].cpu().numpy(), ms, atol=TOL, err_msg="m %s step %d" % (kk, it + 1))
            np.testing.assert_allclose(got["v"].cpu().numpy(), vs, atol=TOL, err_msg="v %s step %d" % (kk, it + 1))


@pytest.mark.parametrize("mode,model_name,score_kind",
                         [(m, n, s) for m in ("sparse", "loopback", "dense", "local")
                          for n, s in (("TransE", "lp2"), ("TransD", "lppow2"), ("RotatE", "lp1"),
                                       ("TransR", "lppow2"), ("DistMult", None))]
                         + [("dense", "RESCAL", None), ("dense", "TransH", "lppow2")]
                         + [(m, n, s) for m in ("owner", "owner-loopback")
                            for n, s in (("TransE", "lp2"), ("RotatE", "lp1"), ("DistMult", None),
                                         ("TransE", "lpinf"), ("TransE", "lp3"))]
                         + [(m, n, s) for m in ("sparse-forced", "dense-forced", "owner-forced")
                            for n, s in (("TransE", "lp2"), ("RotatE", "lp1"))]
                         + [("sparse-forced", "TransD", "lppow2"), ("dense-forced", "RESCAL", None)])
def test_sharded_step_world1_rccl(hiplib, mode, model_name, score_kind):
    """KGE/sharded.py on the RCCL backend (world size 1): e mod G shard,
    kge_sample draws, the device sparse exchange (kge_exchange_plan ->
    fixed-capacity blocks -> split step or grad-mode step on the extended
    table -> gradient rows back -> kge_exchange_rows; "loopback": every id
    through the blocks, the remote path on one GPU) or the dense replica
    (grad-mode step, one all-reduce, kge_apply), or owner-side scoring (the
    owner pass over the virtual batch with in-kernel draws, records, merge,
    owner update then the positives' rows); two steps == two oracle steps
    with the same draws. "-forced": the N-rank code path on the one rank
    (force_collectives: separate send / receive buffers, every all_to_all /
    all_gather / all_reduce issued as an RCCL tensor-form call)."""
    import torch.distributed as dist
    from KGE import loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = _dev()
    _init_world1(dist, dev)
    try:
        rng = np.random.default_rng(3)
        E, R, d, B, K = 37, 5, 24, 16, 8
        k = 20 if model_name in ("TransD", "TransR") else None
        W = _weights(model_name, E, R, d, rng, k)
        sc = {"lp2": score.LpDistance(2), "lppow2": score.LpDistancePow(2), "lp1": score.LpDistance(1),
              "lpinf": score.LpDistance(np.inf), "lp3": score.LpDistance(3), None: None}[score_kind]
        m = _make(model_name, d, K, "h+t", sc, loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E, R,
                  UniformStrategy(np.arange(E), seed=9), k=k)
        m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
        # "sparse" forces the exchange + row cache even on one rank; "local" is
        # the one-rank shortcut (the fused step directly on the shard)
        forced = mode.endswith("-forced")
        st = ShardedStep(m, mode="dense" if mode.startswith("dense") else "owner" if mode.startswith("owner")
                         else "sparse", local_fast=mode == "local", loopback=mode.endswith("loopback"),
                         force_collectives=forced)
        assert (st.direct is not None) == (mode == "local")
        assert st.multi == forced
        ref_w = W
        opt = optimizers.SGD(0.05)
        for it in range(2):
            pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
            plane = m.ns_strategy.offset
            lv = float(st(torch.tensor(pos, device=dev), True, opt))
            torch.cuda.synchronize()
            st.check_status()
            neg = orc.negatives(pos, K, "h+t", E, seed=9, plane=plane)
            ref = orc.train_step(model_name, ref_w, pos, neg, score=_spec_score(sc) if sc is not None else ("dot", 0.0),
                                 loss=("sans", 3.0, 1.0), lr=0.05, limit=getattr(m, "limit", None),
                                 constraint=model_name != "RotatE",
                                 constraint_weight=getattr(m, "constraint_weight", 1.0))
            ref_w = ref["weights"]
            assert abs(lv - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), it
        st.sync()
        for kk, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[kk].cpu().numpy(), v, atol=TOL, err_msg=kk)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model_name,loopback", [(n, lb) for n in ("TransE", "TransD") for lb in (False, True)])
def test_sharded_sparse_adam_world1(hiplib, model_name, loopback):
    """keras Adam through the device sparse exchange (world size 1): the
    grad-mode step on the extended table, gradient rows accumulated by their
    owner (kge_exchange_rows ACCUM), dense keras Adam over the shard -- three
    steps == three oracle Adam steps."""
    import torch.distributed as dist
    from KGE import loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = _dev()
    _init_world1(dist, dev)
    try:
        rng = np.random.default_rng(31)
        E, R, d, B, K = 41, 4, 24, 9, 6
        k = 20 if model_name == "TransD" else None
        W = _weights(model_name, E, R, d, rng, k)
        sc = score.LpDistance(2) if model_name == "TransE" else score.LpDistancePow(2)
        lf = loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0)
        m = _make(model_name, d, K, "h+t", sc, lf, E, R, UniformStrategy(np.arange(E), seed=4), k=k)
        m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
        st = ShardedStep(m, mode="sparse", local_fast=False, loopback=loopback)
        opt = optimizers.Adam(0.01)
        ref_w, state = W, None
        for it in range(3):
            pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
            plane = m.ns_strategy.offset
            lv = float(st(torch.tensor(pos, device=dev), True, opt))
            torch.cuda.synchronize()
            st.check_status()
            neg = orc.negatives(pos, K, "h+t", E, seed=4, plane=plane)
            ref = orc.train_step(model_name, ref_w, pos, neg, score=_spec_score(sc), loss=_spec_loss(lf), lr=0.01,
                                 constraint=True, optimizer="adam", adam_state=state,
                                 constraint_weight=getattr(m, "constraint_weight", 1.0))
            ref_w, state = ref["weights"], ref["adam"]
            assert abs(lv - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), it
        st.sync()
        for kk, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[kk].cpu().numpy(), v, atol=TOL, err_msg=kk)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model_name", ["TransE", "TransR"])
def test_sharded_exchange_overflow_voids_step(hiplib, model_name):
    """A step whose ids overflow an owner block (capacity below the step's
    unique ids) is skipped whole -- no table changes -- and check_status()
    reports it (also when later steps succeed: the flag is sticky until read).
    The next step with room, same shapes and so the same plan and workspace
    (no re-zeroing), == the oracle: the voided step left no counters, hash
    slots or list entries behind. Negatives come from an 8-entity pool, so
    a batch of positives over those 8 entities fits the 16-row blocks."""
    import torch.distributed as dist
    from KGE import loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = _dev()
    _init_world1(dist, dev)
    try:
        rng = np.random.default_rng(37)
        E, R, d, B, K, P = 300, 4, 24, 32, 8, 8
        k = 20 if model_name == "TransR" else None
        W = _weights(model_name, E, R, d, rng, k)
        m = _make(model_name, d, K, "h+t", score.LpDistancePow(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
                  E, R, UniformStrategy(np.arange(P), seed=6), constraint=False, k=k)
        m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
        # one rank, every id through the blocks: the split step (TransE: its
        # update pass aborted) / the grad-mode step (TransR)
        st = ShardedStep(m, mode="sparse", local_fast=False, loopback=True, capacity_slack=0.05,
                         capacity_floor=0, batch_hint=B)
        assert st._ext["cap"] == 16
        opt = optimizers.SGD(0.05)
        pos = np.stack([rng.integers(P, E, B), rng.integers(0, R, B), rng.integers(P, E, B)], 1).astype(np.int64)
        st(torch.tensor(pos, device=dev), True, opt)
        torch.cuda.synchronize()
        st.sync()
        for kk, v in W.items():
            np.testing.assert_array_equal(m.model_weights[kk].cpu().numpy(), v, err_msg=kk)
        # the next steps fit (ids in [0, 8)); the overflow stays reported
        ref_w = W
        for it in range(2):
            pos = np.stack([rng.integers(0, P, B), rng.integers(0, R, B), rng.integers(0, P, B)], 1).astype(np.int64)
            plane = m.ns_strategy.offset
            lv = float(st(torch.tensor(pos, device=dev), True, opt))
            torch.cuda.synchronize()
            neg = orc.negatives(pos, K, "h+t", P, seed=6, plane=plane)
            ref = orc.train_step(model_name, ref_w, pos, neg, score=("lppow", 2.0), loss=("sans", 3.0, 1.0), lr=0.05,
                                 constraint=False)
            ref_w = ref["weights"]
            assert abs(lv - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), it
            if it == 0:
                with pytest.raises(RuntimeError, match="overflowed"):
                    st.check_status()
            else:
                st.check_status()   # read and cleared
        st.sync()
        for kk, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[kk].cpu().numpy(), v, atol=TOL, err_msg=kk)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model_name", ["TransE", "RotatE", "TransD", "TransR"])
def test_gathered_shard_layout_remap(hiplib, model_name):
    """The C-ABI's gathered-shard mapping (for callers that all-gather
    row-sharded tables) on one GPU: the entity rows laid out
    as G = 3 all-gathered shards (row (e mod 3) * Es + e div 3,
    padded), kge_step given shard_count / shard_rows / global_entities draws
    and maps global ids in-kernel; un-permuted rows == the oracle step."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    dev = _dev()
    rng = np.random.default_rng(41)
    E, R, d, B, K, G = 29, 4, 24, 10, 6, 3
    k = 20 if model_name in ("TransR", "TransD") else None
    W = _weights(model_name, E, R, d, rng, k)
    Es = -(-E // G)
    perm = np.array([(e % G) * Es + e // G for e in range(E)])

    def gathered(x):
        out = np.zeros((G * Es,) + x.shape[1:], np.float32)
        out[perm] = x
        return torch.tensor(out, device=dev)
    sc = {"TransE": score.LpDistance(2), "RotatE": score.LpDistance(1)}.get(model_name, score.LpDistancePow(2))
    m = _make(model_name, d, K, "h+t", sc, loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E, R,
              UniformStrategy(np.arange(E), seed=13), constraint=False, k=k)
    m.model_weights = {kk: (gathered(v) if kk in ("ent_emb", "ent_proj") else torch.tensor(v, device=dev))
                       for kk, v in W.items()}
    step = engine.FusedStep(m)
    step.shard = (G, Es, E)
    pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
    plane = m.ns_strategy.offset
    step(torch.tensor(pos, device=dev), True, optimizers.SGD(0.05))
    torch.cuda.synchronize()
    step.check_status()
    neg = orc.negatives(pos, K, "h+t", E, seed=13, plane=plane)
    ref = orc.train_step(model_name, W, pos, neg, score=_spec_score(sc), loss=("sans", 3.0, 1.0), lr=0.05,
                         constraint=False, limit=getattr(m, "limit", None))
    assert abs(float(step.loss_out.item()) - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"]))
    for kk, v in ref["weights"].items():
        got = m.model_weights[kk].cpu().numpy()
        if kk in ("ent_emb", "ent_proj"):
            got = got[perm]
        np.testing.assert_allclose(got, v, atol=TOL, err_msg=kk)


@pytest.mark.parametrize("mode,loopback", [("sparse", False), ("sparse", True), ("owner", False), ("owner", True)])
def test_sharded_step_c5_shard_size(hiplib, mode, loopback):
    """One GPU at the C5 per-rank shard size (6.25M rows x 512, TransE, K=256
    h+t, SANS) through the sparse exchange or owner-side scoring (the mode
    "auto" gives C5): finite loss, only touched rows change, and the sharded
    step equals the fused single-device step on the same rows (same draws)."""
    import torch.distributed as dist
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = _dev()
    _init_world1(dist, dev)
    try:
        E, R, d, B, K = 6_250_000, 1000, 512, 256, 256
        g = torch.Generator(device=dev).manual_seed(0)
        ent = (torch.rand(E, d, generator=g, device=dev) - 0.5) * 0.1
        rel = (torch.rand(R, d, generator=g, device=dev) - 0.5) * 0.1
        pos = torch.stack([torch.randint(0, E, (B,), generator=g, device=dev),
                           torch.randint(0, R, (B,), generator=g, device=dev),
                           torch.randint(0, E, (B,), generator=g, device=dev)], 1)
        outs = []
        for sharded in (True, False):
            m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
                      E, R, UniformStrategy(np.arange(E), seed=5), constraint=False)
            m.model_weights = {"ent_emb": ent.clone(), "rel_emb": rel.clone()}
            stp = ShardedStep(m, mode=mode, local_fast=False, loopback=loopback) if sharded else \
                engine.FusedStep(m)
            lv = float(stp(pos, True, optimizers.SGD(0.01)))
            torch.cuda.synchronize()
            stp.check_status()
            if sharded:
                stp.sync()
            outs.append((lv, m.model_weights["ent_emb"], m.model_weights["rel_emb"]))
            del stp
        assert math.isfinite(outs[0][0]) and abs(outs[0][0] - outs[1][0]) <= 1e-5 * max(1.0, abs(outs[1][0]))
        changed = (outs[0][1] != ent).any(dim=1)
        assert 0 < int(changed.sum()) <= B * (K + 2)
        assert float((outs[0][1] - outs[1][1]).abs().max()) <= 1e-5
        assert float((outs[0][2] - outs[1][2]).abs().max()) <= 1e-5
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model_name", ["TransE", "DistMult", "RotatE"])
def test_compact_hot_relation(hiplib, model_name):
    """Compact launch with a Zipf-hot relation: 3000 positives, 70 % of them on
    relation 0 (a relation list far past its capacity, sorted in LDS) == the
    oracle."""
    from KGE import loss, score
    E, R, B = 100000, 6, 3000
    rng = np.random.default_rng(21)
    rel = np.where(rng.random(B) < 0.7, 0, rng.integers(1, R, B))
    pos = np.stack([rng.integers(0, E, B), rel, rng.integers(0, E, B)], 1).astype(np.int64)
    sc = None if model_name == "DistMult" else score.LpDistance(2)
    ref, got, l_, ps, ns, step, _ = run_case(hiplib, model_name, 32, B, 4, "h+t", sc,
                                             loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E=E, R=R,
                                             constraint=False, pos=pos, seed=5)
    check(ref, got, l_, ps, ns)


def test_owner_update_phase_needs_its_score_pass(hiplib):
    """The owner update pass gates itself (owner_coef_kernel carries the
    split step's phase gate): replayed after a full owner step, with no owner
    score pass before it, it is refused on the device (KGE_EWORKSPACE) and
    writes no table row."""
    import torch.distributed as dist
    from KGE import _hip, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = _dev()
    _init_world1(dist, dev)
    try:
        E, R, d, B, K = 50000, 5, 24, 64, 8
        rng = np.random.default_rng(71)
        W = _weights("TransE", E, R, d, rng)
        m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
                  E, R, UniformStrategy(np.arange(E), seed=5), constraint=False)
        m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
        st = ShardedStep(m, mode="owner", local_fast=False)
        opt = optimizers.SGD(0.05)
        pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1).astype(np.int64)
        bt = torch.tensor(pos, device=dev)
        st(bt, True, opt)
        torch.cuda.synchronize()
        st.check_status()
        shard = st.shard.clone()
        o = st._own
        fo = o["fo"]
        fo.flags = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_OWNER | _hip.FLAG_PHASE_UPDATE
        fo.abort = None
        st.status.zero_()
        fo(bt, True, opt)
        torch.cuda.synchronize()
        assert int(st.status.item()) == _hip.KGE_EWORKSPACE
        assert torch.equal(st.shard, shard)
        # the merge's update pass (the segmented sum) gates itself the same way
        fm = o["fm"]
        fm.workspace.zero_()
        fm.flags = _hip.FLAG_NO_TABLE_CONSTRAINT | _hip.FLAG_OWNER_MERGE | _hip.FLAG_PHASE_UPDATE
        fm.abort = None
        st.status.zero_()
        fm(o["lpos"], True, opt)
        torch.cuda.synchronize()
        assert int(st.status.item()) == _hip.KGE_EWORKSPACE
        assert torch.equal(st.shard, shard)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("loopback", [False, True])
def test_owner_merge_hot_entities(hiplib, loopback):
    """Owner mode (world size 1, RCCL) on a table large enough for compact
    launches, with Zipf-like hot rows among the positives: 40 % of the heads
    are entity 7, 30 % of the tails entity 11, 60 % of the relations 0. At
    3 B <= 8192 keys the merge's update pass is the segmented sum
    (merge_plan / merge_chunk / merge_combine kernels); two steps == two
    oracle steps, and == (up to summation order) the same steps with every
    destination summed by the update kernel itself (KGE_FLAG_DEBUG_NO_REL_SEG).
    test_owner_merge_fallback_update covers the larger batches' path."""
    import torch.distributed as dist
    from KGE import _hip, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = _dev()
    _init_world1(dist, dev)
    try:
        E, R, d, B, K = 100000, 6, 24, 400, 8
        W = _weights("TransE", E, R, d, np.random.default_rng(17))
        outs = []
        for flags in (0, _hip.FLAG_DEBUG_NO_REL_SEG):
            rng = np.random.default_rng(18)
            m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
                      E, R, UniformStrategy(np.arange(E), seed=4), constraint=False)
            m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
            st = ShardedStep(m, mode="owner", loopback=loopback, local_fast=False)   # (not the one-rank shortcut)
            st.debug_flags = flags
            ref_w = W
            opt = optimizers.SGD(0.05)
            for it in range(2):
                h = np.where(rng.random(B) < 0.4, 7, rng.integers(0, E, B))
                t = np.where(rng.random(B) < 0.3, 11, rng.integers(0, E, B))
                r = np.where(rng.random(B) < 0.6, 0, rng.integers(0, R, B))
                pos = np.stack([h, r, t], 1).astype(np.int64)
                plane = m.ns_strategy.offset
                lv = float(st(torch.tensor(pos, device=dev), True, opt))
                torch.cuda.synchronize()
                st.check_status()
                neg = orc.negatives(pos, K, "h+t", E, seed=4, plane=plane)
                ref = orc.train_step("TransE", ref_w, pos, neg, score=("lp", 2.0), loss=("sans", 3.0, 1.0), lr=0.05,
                                     constraint=False)
                ref_w = ref["weights"]
                assert abs(lv - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), it
            st.sync()
            for kk, v in ref_w.items():
                np.testing.assert_allclose(m.model_weights[kk].cpu().numpy(), v, atol=TOL, err_msg=kk)
            outs.append({kk: v.cpu().numpy() for kk, v in m.model_weights.items()})
            del st
        for kk in outs[0]:   # (rel_seg adds four row groups' partials: equal up to summation order)
            np.testing.assert_allclose(outs[0][kk], outs[1][kk], rtol=0, atol=1e-6, err_msg=kk)
    finally:
        dist.destroy_process_group()


def test_owner_merge_fallback_update(hiplib):
    """Owner mode with 3 B > 8192 positive keys (B = 2800): the merge's update
    pass falls back to the update kernel with long destinations deferred to
    long_rows_kernel and relation rows summed by rel_seg_kernel (Zipf-hot
    heads / relation). A step whose exchange blocks overflow is void and
    leaves every relation gradient row zero (rel_seg_kernel's abort path:
    never the previous values); then two clean steps == two oracle steps."""
    import torch.distributed as dist
    from KGE import loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = _dev()
    _init_world1(dist, dev)
    try:
        E, R, d, B, K = 100000, 6, 24, 2800, 4
        W = _weights("TransE", E, R, d, np.random.default_rng(27))
        rng = np.random.default_rng(28)

        def batch():
            h = np.where(rng.random(B) < 0.3, 7, rng.integers(0, E, B))
            t = rng.integers(0, E, B)
            r = np.where(rng.random(B) < 0.6, 0, rng.integers(0, R, B))
            return np.stack([h, r, t], 1).astype(np.int64)

        def model():
            m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
                      E, R, UniformStrategy(np.arange(E), seed=8), constraint=False)
            m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
            return m
        opt = optimizers.SGD(0.05)
        # the void step: every positive row through 280-row blocks (loopback)
        m = model()
        st = ShardedStep(m, mode="owner", loopback=True, local_fast=False, capacity_slack=0.05, capacity_floor=0)
        st.grel["rel"].fill_(7.0)
        st(torch.tensor(batch(), device=dev), True, opt)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match="overflowed an owner block"):
            st.check_status()
        assert float(st.grel["rel"].abs().max()) == 0.0
        st.sync()
        for kk, v in W.items():
            np.testing.assert_array_equal(m.model_weights[kk].cpu().numpy(), v, err_msg=kk)
        del st
        m = model()
        st = ShardedStep(m, mode="owner", local_fast=False)
        ref_w = W
        for it in range(2):
            pos = batch()
            plane = m.ns_strategy.offset
            lv = float(st(torch.tensor(pos, device=dev), True, opt))
            torch.cuda.synchronize()
            st.check_status()
            neg = orc.negatives(pos, K, "h+t", E, seed=8, plane=plane)
            ref = orc.train_step("TransE", ref_w, pos, neg, score=("lp", 2.0), loss=("sans", 3.0, 1.0), lr=0.05,
                                 constraint=False)
            ref_w = ref["weights"]
            assert abs(lv - ref["loss"]) <= TOL * max(1.0, abs(ref["loss"])), it
        st.sync()
        for kk, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[kk].cpu().numpy(), v, atol=TOL, err_msg=kk)
    finally:
        dist.destroy_process_group()


def _zipf(rng, n, N, s):
    """Truncated power-law ranks in [1, N] (inverse CDF of the continuous
    Zipf(s) density) scattered over the id space by k -> (a (k-1) + b) mod N
    (the C5 generator of bench.py)."""
    u = rng.random(n)
    k = np.clip(np.floor((1.0 + u * (float(N) ** (1.0 - s) - 1.0)) ** (1.0 / (1.0 - s))), 1, N).astype(np.int64)
    a = 2654435761
    while np.gcd(a, N) != 1:
        a += 2
    return (a * (k - 1) + 40503) % N


def _touched_rows_oracle(ent, rel, steps, lr, chunk):
    """The oracle on the rows the steps touch (SGD, no constraint: nothing in
    the step reads an untouched row, TransE.py:127-174 / loss.py:174-182):
    ids renumbered into a compact table, ``train_step_chunked`` step after
    step. Returns (touched ids, updated rows, losses)."""
    ids = np.unique(np.concatenate([np.concatenate([p[:, 0], p[:, 2], n]) for p, n in steps]))
    W = {"ent_emb": ent[torch.as_tensor(ids, device=ent.device)].cpu().numpy(), "rel_emb": rel.cpu().numpy()}
    losses = []
    for p, n in steps:
        pp = p.copy()
        pp[:, 0] = np.searchsorted(ids, p[:, 0])
        pp[:, 2] = np.searchsorted(ids, p[:, 2])
        ref = orc.train_step_chunked("TransE", W, pp, np.searchsorted(ids, n), score=("lp", 2.0),
                                     loss=("sans", 3.0, 1.0), lr=lr, constraint=False, chunk=chunk)
        W = ref["weights"]
        losses.append(ref["loss"])
    return ids, W, losses


@pytest.mark.parametrize("loopback", [False, True])
def test_owner_c5_kernel_shape(hiplib, loopback):
    """Owner-side scoring (what "auto" runs for C5) at C5's kernel shape:
    TransE d = 512 (two fragment chunks per row), K = 256 'h+t' (four waves per
    positive: each owner record merges the waves' partial softmax states,
    then the merge combines the records), E = 2M rows (compact launches),
    Zipf(1.1) heads / tails and Zipf(1.2) relations over R = 1000 (hot rows:
    long_rows_kernel, rel_seg_kernel), SANS(3, 1), SGD; world-1 RCCL, with
    and without every positive row through the exchange blocks. Two steps ==
    two float64 oracle steps on the touched rows (TransE.py:127-174,
    loss.py:174-182) at the 1e-5 bar; every other row bit-unchanged."""
    import torch.distributed as dist
    from KGE import loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = _dev()
    _init_world1(dist, dev)
    try:
        E, R, d, B, K = 2_000_000, 1000, 512, 512, 256
        g = torch.Generator(device=dev).manual_seed(5)
        lim = 6.0 / math.sqrt(d)
        ent0 = torch.rand(E, d, generator=g, device=dev).mul_(2).sub_(1).mul_(lim)
        rel0 = torch.rand(R, d, generator=g, device=dev).mul_(2).sub_(1).mul_(lim)
        rng = np.random.default_rng(55 + loopback)
        m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
                  E, R, UniformStrategy(np.arange(E), seed=6), constraint=False)
        m.model_weights = {"ent_emb": ent0.clone(), "rel_emb": rel0.clone()}
        st = ShardedStep(m, mode="owner", loopback=loopback, local_fast=False, batch_hint=B)
        assert st.mode == "owner"
        opt = optimizers.SGD(0.05)
        steps, got_losses = [], []
        for _ in range(2):
            pos = np.stack([_zipf(rng, B, E, 1.1), _zipf(rng, B, R, 1.2), _zipf(rng, B, E, 1.1)], 1)
            plane = m.ns_strategy.offset
            got_losses.append(float(st(torch.tensor(pos, device=dev), True, opt)))
            torch.cuda.synchronize()
            st.check_status()
            steps.append((pos, orc.negatives(pos, K, "h+t", E, seed=6, plane=plane)))
        assert np.bincount(steps[0][0][:, 0]).max() >= 16   # (a Zipf-hot head)
        st.sync()
        ids, ref_w, ref_losses = _touched_rows_oracle(ent0, rel0, steps, 0.05, 64)
        for it, (a, b) in enumerate(zip(got_losses, ref_losses)):
            assert abs(a - b) <= TOL * max(1.0, abs(b)), (it, a, b)
        got = m.model_weights["ent_emb"]
        tid = torch.as_tensor(ids, device=dev)
        np.testing.assert_allclose(got[tid].cpu().numpy(), ref_w["ent_emb"], rtol=0, atol=TOL, err_msg="ent_emb")
        np.testing.assert_allclose(m.model_weights["rel_emb"].cpu().numpy(), ref_w["rel_emb"], rtol=0, atol=TOL,
                                   err_msg="rel_emb")
        changed = torch.nonzero((got != ent0).any(dim=1)).flatten().cpu().numpy()
        assert np.isin(changed, ids).all()
    finally:
        dist.destroy_process_group()
