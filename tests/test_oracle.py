"""CPU: the oracle pinned against the golden fixtures, finite differences and
the reference's own property tests (reference tests/test_score.py,
test_loss.py, test_constraint.py, test_metrics.py, test_ns_strategy.py)."""

import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import kge_oracle as orc

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


# ---------------------------------------------------------------- Philox
@pytest.mark.parametrize("case", _json("philox_kat.json"))
def test_philox_random123_kat(case):
    assert orc.philox4x32_10(case["ctr"], case["key"]) == case["out"]
    w = orc._philox_vec(np.array([case["ctr"][0] | (case["ctr"][1] << 32)], dtype=np.uint64),
                        case["ctr"][2] | (case["ctr"][3] << 32), case["key"][0] | (case["key"][1] << 32))
    assert [int(x) for x in w[0]] == case["out"]


def test_product_host_philox_matches_kat():
    from KGE import _philox
    for case in _json("philox_kat.json"):
        c, k = case["ctr"], case["key"]
        got = _philox.philox4x32_10(c[0], c[1], c[2], c[3], k[0], k[1])
        assert [int(x) for x in got] == case["out"]


# ---------------------------------------------------------------- sampler
def test_sampler_golden_and_layout():
    g = _json("sampler_golden.json")
    X = np.array(g["X"], dtype=np.int64)
    tt = orc.typed_tables(g["ind2type"])
    for c in g["cases"]:
        typed = c.get("typed", False)
        ids = orc.negatives(X, c["K"], c["side"], c["E"], seed=c["seed"], plane=c["plane"], i64=c["i64"],
                            sampler="typed" if typed else "uniform", typed=tt if typed else None)
        assert ids.tolist() == c["ids"]
        assert ids.min() >= 0 and ids.max() < c["E"]
        if typed:   # utils.py:11-16: same type, never the entity itself
            ref = np.repeat(X[:, 2], c["K"])
            it = np.array(g["ind2type"])
            assert (it[ids] == it[ref]).all() and (ids != ref).all()


def test_ht_layout_interleaves_h_then_t():
    """BaseModel.py:353-356: h-side draws from plane p, t-side from p+1; rows alternate."""
    X = np.array([[1, 0, 2], [3, 1, 4]])
    ids = orc.negatives(X, 4, "h+t", 100, seed=9, plane=5)
    h = orc.negatives(X, 2, "h", 100, seed=9, plane=5)
    t = orc.negatives(X, 2, "t", 100, seed=9, plane=6)
    assert ids.reshape(2, 2, 2)[:, :, 0].reshape(-1).tolist() == h.tolist()
    assert ids.reshape(2, 2, 2)[:, :, 1].reshape(-1).tolist() == t.tolist()
    trip = orc.corrupt(X, ids, 4, "h+t")
    assert trip.shape == (8, 3)
    assert (trip[0::2, 2] == np.repeat(X[:, 2], 2)).all() and (trip[1::2, 0] == np.repeat(X[:, 0], 2)).all()


def test_uniform_draws_are_uniform():
    n = 200000
    ids = orc.negatives(np.zeros((n, 3), np.int64), 1, "t", 10, seed=3, plane=0)
    cnt = np.bincount(ids, minlength=10)
    assert abs(cnt / n - 0.1).max() < 0.005


# ---------------------------------------------------------------- step golden
def _cases():
    return _json("step_golden.json")


@pytest.mark.parametrize("meta", _cases(), ids=lambda m: "%s-%s-%s" % (m["model"], m["score"][0], m["loss"][0]))
def test_step_golden(meta):
    z = np.load(os.path.join(GOLD, "step_golden.npz"))
    tag = meta["tag"]
    W = {k.split("/")[-1]: z[k] for k in z.files if k.startswith(tag + "/in/")}
    pos = z["pos"]
    E = W["ent_emb"].shape[0]
    neg = orc.negatives(pos, meta["K"], meta["side"], E, seed=meta["seed"], plane=meta["plane"])
    assert neg.tolist() == z[tag + "/neg"].tolist()
    res = orc.train_step(meta["model"], W, pos, neg, score=tuple(meta["score"]), loss=tuple(meta["loss"]),
                         lr=meta["lr"], constraint=meta["constraint"], side=meta["side"], limit=meta["limit"])
    np.testing.assert_allclose(res["loss"], z[tag + "/loss"], rtol=1e-12)
    np.testing.assert_allclose(res["pos_score"], z[tag + "/pos_score"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(res["neg_score"], z[tag + "/neg_score"], rtol=1e-12, atol=1e-14)
    for k, v in res["weights"].items():
        np.testing.assert_allclose(v, z["%s/out/%s" % (tag, k)], rtol=1e-12, atol=1e-14)
    # the fp32 restatement agrees with the fp64 one
    r32 = orc.train_step(meta["model"], W, pos, neg, score=tuple(meta["score"]), loss=tuple(meta["loss"]),
                         lr=meta["lr"], constraint=meta["constraint"], side=meta["side"], limit=meta["limit"],
                         dtype=torch.float32)
    assert abs(r32["loss"] - res["loss"]) <= 1e-5 * max(1.0, abs(res["loss"]))
    for k, v in res["weights"].items():
        np.testing.assert_allclose(r32["weights"][k], v, atol=2e-6)


# ---------------------------------------------------------------- finite differences
FD_MODELS = [("TransE", ("lp", 2.0)), ("TransH", ("lppow", 2.0)), ("TransR", ("lppow", 2.0)),
             ("TransD", ("lppow", 2.0)), ("RotatE", ("lp", 2.0)), ("DistMult", ("dot", 0.0)),
             ("RESCAL", ("dot", 0.0))]


@pytest.mark.parametrize("model,score", FD_MODELS)
@pytest.mark.parametrize("loss", [("logistic",), ("bce",), ("sqerr",)])
def test_oracle_gradient_matches_finite_differences(model, score, loss):
    """w_new = w - lr * g (clip disabled, constraints off) => g from the oracle's
    autograd chain must equal the central difference of its scalar loss
    (SANS is excluded: its softmax weights are stop_gradient, loss.py:176)."""
    from tests.golden.make_golden import case_weights
    rng = np.random.default_rng(1)
    E, R, d, B, K = 6, 3, 4, 3, 2
    W = case_weights(model, E, R, d, rng)
    pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1)
    neg = rng.integers(0, E, B * K)
    lim = 5.0 / d if model == "RotatE" else None
    kw = dict(score=score, loss=loss, constraint=False, side="h+t", limit=lim)
    lr = 1e-3
    res = orc.train_step(model, W, pos, neg, lr=lr, clip_norm=1e30, **kw)
    for name in W:
        g = (W[name] - res["weights"][name]) / lr
        flat = W[name].reshape(-1)
        for j in rng.choice(flat.size, size=min(6, flat.size), replace=False):
            h = 1e-6
            Wp = {k: v.copy() for k, v in W.items()}
            Wm = {k: v.copy() for k, v in W.items()}
            Wp[name].reshape(-1)[j] += h
            Wm[name].reshape(-1)[j] -= h
            lp = orc.train_step(model, Wp, pos, neg, train=False, **kw)["loss"]
            lm = orc.train_step(model, Wm, pos, neg, train=False, **kw)["loss"]
            fd = (lp - lm) / (2 * h)
            assert abs(fd - g.reshape(-1)[j]) <= 1e-6 * max(1.0, abs(fd)), (name, j, fd, g.reshape(-1)[j])


@pytest.mark.parametrize("model,score", FD_MODELS)
@pytest.mark.parametrize("loss", [("hinge", 1.0), ("logistic",), ("bce",), ("sans", 3.0, 1.0), ("sqerr",)])
@pytest.mark.parametrize("side", ["h+t", "t"])
def test_chunked_oracle_equals_one_graph(model, score, loss, side):
    """train_step_chunked (the full-size C4 checker) == train_step: loss,
    scores, norms and updated weights, constraints on (TransH / RESCAL dense
    terms, DistMult's batch term, renormalisation / clip assigns), with a
    chunk that does not divide B."""
    from tests.golden.make_golden import case_weights
    rng = np.random.default_rng(4)
    E, R, d, B, K = 9, 3, 5, 7, 4
    W = case_weights(model, E, R, d, rng)
    pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1)
    neg = rng.integers(0, E, B * K)
    kw = dict(score=score, loss=loss, constraint=True, side=side, limit=5.0 / d if model == "RotatE" else None,
              lr=0.3, constraint_weight=0.4)
    one = orc.train_step(model, W, pos, neg, **kw)
    ch = orc.train_step_chunked(model, W, pos, neg, chunk=3, **kw)
    assert abs(one["loss"] - ch["loss"]) <= 1e-12 * max(1.0, abs(one["loss"]))
    np.testing.assert_allclose(ch["pos_score"], one["pos_score"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(ch["neg_score"], one["neg_score"], rtol=1e-12, atol=1e-14)
    assert set(ch["norm2"]) == set(one["norm2"])
    for k in one["norm2"]:
        assert abs(ch["norm2"][k] - one["norm2"][k]) <= 1e-10 * max(1.0, one["norm2"][k]), k
    for k, v in one["weights"].items():
        np.testing.assert_allclose(ch["weights"][k], v, rtol=0, atol=1e-12, err_msg=k)


@pytest.mark.parametrize("model", ["TransE", "RESCAL", "TransH"])
def test_oracle_adam_three_steps_match_eager_plugin_path(model, monkeypatch):
    """keras Adam at t = 1, 2, 3 (BaseModel.py:243-246,328): the oracle's slot
    state carried across calls == the package's eager plugin path (a separate
    restatement: per-lookup IndexedSlices, unique-row scatter of the slots)
    on the same injected negatives; sparse (TransE) and dense (RESCAL, TransH
    regularisers) variables; and t = 2 differs from a restart at t = 1."""
    monkeypatch.setenv("KGE_BACKEND", "eager")
    from KGE import engine, loss, optimizers, score
    from KGE.models.semantic_based.RESCAL import RESCAL
    from KGE.models.translating_based.TransE import TransE
    from KGE.models.translating_based.TransH import TransH
    from KGE.ns_strategy import UniformStrategy
    from tests.golden.make_golden import case_weights
    rng = np.random.default_rng(4)
    E, R, d, B, K = 9, 3, 5, 4, 4
    W = case_weights(model, E, R, d, rng)
    ns = UniformStrategy(np.arange(E), seed=1)
    lf = loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0)
    if model == "TransE":
        m = TransE({"embedding_size": d}, K, "h+t", score_fn=score.LpDistance(2), loss_fn=lf, ns_strategy=ns)
        sc = ("lp", 2.0)
    elif model == "TransH":
        m = TransH({"embedding_size": d}, K, "h+t", score_fn=score.LpDistancePow(2), loss_fn=lf, ns_strategy=ns,
                   constraint_weight=0.3)
        sc = ("lppow", 2.0)
    else:
        m = RESCAL({"embedding_size": d}, K, "h+t", loss_fn=lf, ns_strategy=ns, constraint_weight=0.5)
        sc = ("dot", 0.0)
    m.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    m.model_weights = {k: torch.tensor(v, dtype=torch.float64) for k, v in W.items()}
    opt = optimizers.Adam(0.01)
    ref_w, state = W, None
    for it in range(3):
        pos = np.stack([rng.integers(0, E, B), rng.integers(0, R, B), rng.integers(0, E, B)], 1)
        neg = rng.integers(0, E, B * K)
        negt = torch.tensor(orc.corrupt(pos, neg, K, "h+t"))
        engine.eager_step(m, torch.tensor(pos), True, opt, neg=negt)
        ref = orc.train_step(model, ref_w, pos, neg, score=sc, loss=("sans", 3.0, 1.0), lr=0.01, optimizer="adam",
                             adam_state=state, constraint_weight=getattr(m, "constraint_weight", 1.0))
        if it == 1:   # the slots matter: a fresh optimizer at t = 1 gives a different step
            fresh = orc.train_step(model, ref_w, pos, neg, score=sc, loss=("sans", 3.0, 1.0), lr=0.01,
                                   optimizer="adam", constraint_weight=getattr(m, "constraint_weight", 1.0))
            assert max(np.abs(fresh["weights"][k] - ref["weights"][k]).max() for k in W) > 1e-4
        ref_w, state = ref["weights"], ref["adam"]
        for k, v in ref_w.items():
            np.testing.assert_allclose(m.model_weights[k].numpy(), v, rtol=1e-9, atol=1e-12, err_msg="%s %d" % (k, it))
        for k, (ms, vs) in state["slots"].items():
            np.testing.assert_allclose(opt.slots[k]["m"].numpy(), ms, rtol=1e-9, atol=1e-15)
            np.testing.assert_allclose(opt.slots[k]["v"].numpy(), vs, rtol=1e-9, atol=1e-18)


# ---------------------------------------------------------------- reference property tests
def test_scores_properties():
    """reference tests/test_score.py:7-50: Lp scores <= 0, finite, one per row (also complex)."""
    from KGE import score
    x, y = torch.randn(10, 8), torch.randn(10, 8)
    for s in (score.LpDistance(1), score.LpDistance(2), score.LpDistance(np.inf), score.LpDistancePow(2)):
        v = s(x, y)
        assert v.shape == (10,) and bool(torch.isfinite(v).all()) and bool((v <= 0).all())
        zx, zy = torch.complex(x, y), torch.complex(y, x)
        v = s(zx, zy)
        assert v.shape == (10,) and bool((v <= 0).all())
    assert score.Dot()(x, y).shape == (10,)


def test_losses_properties():
    """reference tests/test_loss.py:8-70: every loss is a finite scalar >= 0."""
    from KGE import loss
    pos, neg = torch.randn(8), torch.randn(8 * 4)
    for lf in (loss.PairwiseHingeLoss(1.0), loss.PairwiseLogisticLoss(), loss.BinaryCrossEntropyLoss(),
               loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), loss.SquareErrorLoss()):
        v = lf(pos, neg)
        assert v.dim() == 0 and math.isfinite(float(v)) and float(v) >= 0


def test_losses_match_oracle():
    from KGE import loss
    pos, neg = torch.randn(8, dtype=torch.float64), torch.randn(32, dtype=torch.float64)
    pairs = [(loss.PairwiseHingeLoss(1.0), ("hinge", 1.0)), (loss.PairwiseLogisticLoss(), ("logistic",)),
             (loss.BinaryCrossEntropyLoss(), ("bce",)),
             (loss.SelfAdversarialNegativeSamplingLoss(3.0, 0.5), ("sans", 3.0, 0.5)),
             (loss.SquareErrorLoss(), ("sqerr",))]
    for lf, spec in pairs:
        assert abs(float(lf(pos, neg)) - float(orc.loss_fn(spec, pos, neg))) < 1e-12


def test_constraint_properties():
    """reference tests/test_constraint.py:8-66."""
    from KGE import constraint
    X = torch.randn(20, 7) * 3
    n = torch.linalg.norm(constraint.normalized_embeddings(X, p=2, value=1, axis=1), dim=1)
    assert bool((torch.abs(n - 1) < 1e-6).all())
    c = constraint.clip_constraint(X, p=2, value=1.0, axis=-1)
    assert bool((torch.linalg.norm(c, dim=-1) <= 1 + 1e-6).all()) and c.shape == X.shape
    assert float(constraint.soft_constraint(X, p=2, value=1, axis=-1)) >= 0
    assert bool((constraint.Lp_regularization(X, p=2, axis=-1) >= 0).all())


def test_metrics_match_reference_kat():
    """Reference KGE/metrics.py outputs (tests/golden/metrics_kat.json)."""
    from KGE import metrics
    for c in _json("metrics_kat.json"):
        r = c["ranks"]
        assert metrics.mean_rank(r) == pytest.approx(c["mean_rank"], rel=1e-12)
        assert metrics.mean_reciprocal_rank(r) == pytest.approx(c["mean_reciprocal_rank"], rel=1e-12)
        assert metrics.median_rank(r) == pytest.approx(c["median_rank"], rel=1e-12)
        assert metrics.geometric_mean_rank(r) == pytest.approx(c["geometric_mean_rank"], rel=1e-12)
        assert metrics.harmonic_mean_rank(r) == pytest.approx(c["harmonic_mean_rank"], rel=1e-12)
        assert metrics.std_rank(r) == pytest.approx(c["std_rank"], rel=1e-12)
        for k in (1, 3, 10):
            assert metrics.hits_at_k(r, k) == pytest.approx(c["hit@%d" % k], rel=1e-12)


def test_toy_kg_indexing():
    """index_kg numpy branch (data_utils.py:41-43) on the reference's toy KG."""
    from KGE.data_utils import convert_kg_to_index, index_kg
    kg = _json("toy_kg.json")
    md = index_kg(np.array(kg["train_raw"]))
    assert [str(e) for e in md["ind2ent"]] == kg["ind2ent"]
    assert [str(r) for r in md["ind2rel"]] == kg["ind2rel"]
    tr = convert_kg_to_index(np.array(kg["train_raw"]), md["ent2ind"], md["rel2ind"])
    assert np.asarray(tr).tolist() == kg["train"]
