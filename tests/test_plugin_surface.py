"""CPU: the reference's plugin surface (reference tests/test_model.py and
tests/test_integration.py) on the host-development backend
(KGE_BACKEND=eager): every model x score x loss x sampler trains, evaluates,
ranks and scores with the reference's shapes and properties. The same matrix
runs through the fused HIP step in tests/test_gpu_models.py."""

import json
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(autouse=True)
def _eager(monkeypatch):
    monkeypatch.setenv("KGE_BACKEND", "eager")


def toy():
    with open(os.path.join(GOLD, "toy_kg.json")) as f:
        kg = json.load(f)
    train, val = np.array(kg["train"]), np.array(kg["val"])
    md = {"ind2ent": kg["ind2ent"], "ind2rel": kg["ind2rel"]}
    n = len(md["ind2ent"])
    md["ind2type"] = ["A"] * (n // 2) + ["B"] * (n - n // 2)   # test_integration.py:25-31
    return train, val, md


def build(name, score=None, loss=None, sampler=None, **kw):
    from KGE.models.semantic_based.DistMult import DistMult
    from KGE.models.semantic_based.RESCAL import RESCAL
    from KGE.models.translating_based.RotatE import RotatE
    from KGE.models.translating_based.SE import SE
    from KGE.models.translating_based.TransD import TransD
    from KGE.models.translating_based.TransE import TransE
    from KGE.models.translating_based.TransH import TransH
    from KGE.models.translating_based.TransR import TransR
    from KGE.models.translating_based.UM import UM
    cls = dict(TransE=TransE, TransH=TransH, TransR=TransR, TransD=TransD, RotatE=RotatE, UM=UM, SE=SE,
               DistMult=DistMult, RESCAL=RESCAL)[name]
    ep = {"ent_embedding_size": 16, "rel_embedding_size": 12} if name in ("TransR", "TransD") else \
        {"embedding_size": 16}
    args = dict(embedding_params=ep, negative_ratio=2, corrupt_side="h+t")
    if score is not None:
        args["score_fn"] = score
    if loss is not None:
        args["loss_fn"] = loss
    if sampler is not None:
        args["ns_strategy"] = sampler
    args.update(kw)
    return cls(**args)


MODELS = ["TransE", "TransH", "TransR", "TransD", "RotatE", "UM", "SE", "DistMult", "RESCAL"]
TRANSLATING = {"TransE", "TransH", "TransR", "TransD", "RotatE", "UM", "SE"}


def _scores(name):
    from KGE import score
    s = [score.LpDistance(p=2), score.LpDistancePow(p=2), score.Dot()]
    return s[:2] if name == "RotatE" else s   # test_integration.py: RotatE x Lp kinds only


def _losses():
    from KGE import loss
    return [loss.PairwiseHingeLoss(margin=1.0), loss.PairwiseLogisticLoss(), loss.BinaryCrossEntropyLoss(),
            loss.SquareErrorLoss(), loss.SelfAdversarialNegativeSamplingLoss(margin=1.0, temperature=1.0)]


def _samplers(md):
    from KGE import ns_strategy
    return [ns_strategy.UniformStrategy(np.arange(len(md["ind2ent"])), seed=3),
            ns_strategy.TypedStrategy(pool=None, metadata=md, seed=4)]


@pytest.mark.parametrize("name", MODELS)
def test_integration_matrix(name, tmp_path):
    """test_integration.py:22-216: every score x loss x sampler trains 1 epoch and evaluates."""
    train, val, md = toy()
    scores = _scores(name) if name in TRANSLATING else [None]
    for si, s in enumerate(scores):
        for li, l_ in enumerate(_losses()):
            for sampler in _samplers(md):
                m = build(name, s, l_, sampler)
                m.train(train_X=train, val_X=val, metadata=md, epochs=1, batch_size=4, early_stopping_rounds=None,
                        restore_best_weight=False, optimizer="Adam", seed=12345, log_path=str(tmp_path),
                        log_projector=(si == 0 and li == 0))
                r = m.evaluate(eval_X=val, corrupt_side="h")
                assert r["mean_rank"] >= 1 and 0 < r["mean_reciprocal_rank"] <= 1
                assert len(m.train_loss_history) == 1


@pytest.mark.parametrize("name", MODELS)
def test_score_hrt_shapes(name):
    """test_model.py:63-77: batch / all-heads / all-tails scoring."""
    train, val, md = toy()
    m = build(name)
    m._model_weights_initial = None
    m.metadata = md
    m._init_embeddings(seed=None)
    s = m.score_hrt(h=val[:, 0], r=val[:, 1], t=val[:, 2])
    assert len(s) == len(val) and bool(torch.isfinite(torch.as_tensor(s)).all())
    assert len(m.score_hrt(h=None, r=val[0, 1], t=val[0, 2]).reshape(-1)) == len(md["ind2ent"])
    assert len(m.score_hrt(h=val[0, 0], r=val[0, 1], t=None).reshape(-1)) == len(md["ind2ent"])


def test_rank_and_filtered_metrics():
    """test_model.py:41-61: rank >= 1, filtered <= raw; filtered metrics at least as good."""
    train, val, md = toy()
    m = build("TransE")
    m._model_weights_initial = None
    m.metadata = md
    m._init_embeddings(seed=None)
    x = val[0:1]
    allp = np.concatenate((train, val), axis=0)
    raw = m.get_rank(x=x, positive_X=None, corrupt_side="h")
    flt = m.get_rank(x=x, positive_X=allp, corrupt_side="h")
    assert isinstance(raw, np.int_) and raw >= 1 and 1 <= flt <= raw
    a = m.evaluate(eval_X=val, corrupt_side="t", positive_X=None)
    b = m.evaluate(eval_X=val, corrupt_side="t", positive_X=allp)
    assert b["mean_rank"] <= a["mean_rank"] and b["hit@10"] >= a["hit@10"]


def test_model_weights_initial_and_restore(tmp_path):
    """model_weights_initial is honoured (BaseModel.py:239-240) and restore_model_weights
    checks its argument (the reference's :665 call bug is fixed)."""
    train, val, md = toy()
    E, R = len(md["ind2ent"]), len(md["ind2rel"])
    w0 = {"ent_emb": np.random.default_rng(0).uniform(-1, 1, (E, 16)).astype(np.float32),
          "rel_emb": np.random.default_rng(1).uniform(-1, 1, (R, 16)).astype(np.float32)}
    m = build("TransE")
    from KGE import optimizers
    m.train(train_X=train, val_X=None, metadata=md, epochs=2, batch_size=4, model_weights_initial=w0,
            optimizer=optimizers.SGD(0.01), seed=1, log_path=str(tmp_path))
    assert m.model_weights["ent_emb"].shape == (E, 16)
    with pytest.raises(AssertionError):
        m.restore_model_weights({"ent_emb": torch.zeros(E, 16)})
    m.restore_model_weights({k: torch.tensor(v) for k, v in w0.items()})
    assert torch.equal(m.model_weights["ent_emb"], torch.tensor(w0["ent_emb"]))


def test_early_stopping_restores_best(tmp_path):
    train, val, md = toy()
    m = build("DistMult")
    m.train(train_X=train, val_X=val, metadata=md, epochs=4, batch_size=4, early_stopping_rounds=1,
            restore_best_weight=True, optimizer="SGD", seed=5, log_path=str(tmp_path))
    assert os.path.exists(os.path.join(str(tmp_path), "ckpt.pt"))
    assert 1 <= len(m.val_loss_history) <= 4


def test_scalar_and_histogram_logs(tmp_path):
    """Per-epoch loss scalars (BaseModel.py:444-468) and weight histograms
    (BaseModel.py:162,470-483; TensorBoard bucketing: 30 equal-width buckets
    min..max, one [x-0.5, x+0.5] bucket for a constant tensor)."""
    train, val, md = toy()
    m = build("TransH")
    m.train(train_X=train, val_X=val, metadata=md, epochs=2, batch_size=4, optimizer="SGD", seed=2,
            log_path=str(tmp_path))
    for split in ("train", "validation"):
        lines = open(os.path.join(str(tmp_path), "scalar", split, "loss.jsonl")).read().splitlines()
        assert [json.loads(x)["step"] for x in lines] == [0, 1]
    for name, w in m.model_weights.items():
        recs = [json.loads(x) for x in open(os.path.join(str(tmp_path), "histogram", name + ".jsonl"))]
        assert [r["step"] for r in recs] == [0, 1]
        b = np.array(recs[-1]["buckets"])
        x = w.detach().double().reshape(-1).numpy()
        assert b.shape == (30, 3) and b[:, 2].sum() == x.size
        assert b[0, 0] == x.min() and b[-1, 1] == x.max()
        width = (x.max() - x.min()) / 30
        ref = np.bincount(np.minimum(np.floor((x - x.min()) / width).astype(int), 29), minlength=30)
        assert (b[:, 2] == ref).all()
    m.model_weights["rel_emb"] = torch.full((3, 2), 0.25)
    m._log_embeddings_histogram(7)
    rec = [json.loads(x) for x in open(os.path.join(str(tmp_path), "histogram", "rel_emb.jsonl"))][-1]
    assert rec == {"step": 7, "buckets": [[-0.25, 0.75, 6.0]]}


def test_corrupt_side_assert():
    from KGE.models.translating_based.TransE import TransE
    with pytest.raises(AssertionError, match="Invalid corrupt_side"):
        TransE({"embedding_size": 4}, 2, "x")


def test_samplers_plugin_contract():
    """test_ns_strategy.py:10-62: n*k ids, dtype preserved, typed keeps the type."""
    train, val, md = toy()
    u, t = _samplers(md)
    for X in (torch.tensor(train, dtype=torch.int64), torch.tensor(train, dtype=torch.int32)):
        for s in (u, t):
            for side in ("h", "t"):
                out = s(X, 3, side)
                assert out.shape == (len(X) * 3,) and out.dtype == X.dtype
    out = t(torch.tensor(train), 3, "t").numpy()
    ref = np.repeat(train[:, 2], 3)
    it = np.array(md["ind2type"])
    assert (it[out] == it[ref]).all() and (out != ref).all()


def test_cpu_tensors_refused_without_eager(monkeypatch):
    """No silent CPU fallback: the product refuses CPU work unless eager is explicit."""
    monkeypatch.setenv("KGE_BACKEND", "fused")
    train, val, md = toy()
    u, _ = _samplers(md)
    with pytest.raises(RuntimeError):
        u(torch.tensor(train), 2, "h")
    if not torch.cuda.is_available():
        m = build("TransE")
        with pytest.raises(RuntimeError):
            m.train(train_X=train, val_X=None, metadata=md, epochs=1, batch_size=4, optimizer="SGD")
