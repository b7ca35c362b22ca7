"""GPU: the reference's integration matrix (tests/test_integration.py:22-216)
through KGEModel.train on cuda:0 -- built-in combinations run the fused HIP
step (libkge_hip.so), the rest the plugin path on the device -- plus the
golden toy-KG steps of tests/golden/step_golden.npz through kge_step."""

import json
import os

import numpy as np
import pytest
import torch

from tests.test_plugin_surface import MODELS, TRANSLATING, _losses, _samplers, _scores, build, toy

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(autouse=True)
def _fused(monkeypatch, hiplib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("KGE_BACKEND", "fused")


@pytest.mark.parametrize("name", MODELS)
def test_integration_matrix_gpu(name, tmp_path):
    train, val, md = toy()
    scores = _scores(name) if name in TRANSLATING else [None]
    for s in scores:
        for l_ in _losses():
            for sampler in _samplers(md):
                for opt in ("SGD", "Adam"):
                    m = build(name, s, l_, sampler)
                    m.train(train_X=train, val_X=val, metadata=md, epochs=1, batch_size=4, optimizer=opt,
                            seed=12345, log_path=str(tmp_path))
                    assert np.isfinite(m.train_loss_history[0]) or type(l_).__name__ == "PairwiseLogisticLoss"
                    r = m.evaluate(eval_X=val, corrupt_side="t")
                    assert r["mean_rank"] >= 1


def _golden_cases():
    with open(os.path.join(GOLD, "step_golden.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("meta", _golden_cases(), ids=lambda m: "%s-%s-%s" % (m["model"], m["score"][0], m["loss"][0]))
def test_step_golden_fused(meta):
    """The committed golden step vectors (toy KG, injected negatives) through kge_step."""
    from KGE import engine, loss, optimizers, score
    from KGE.ns_strategy import UniformStrategy
    z = np.load(os.path.join(GOLD, "step_golden.npz"))
    tag = meta["tag"]
    W = {k.split("/")[-1]: z[k] for k in z.files if k.startswith(tag + "/in/")}
    sc = {"lp": score.LpDistance, "lppow": score.LpDistancePow}
    s = score.Dot() if meta["score"][0] == "dot" else sc[meta["score"][0]](meta["score"][1])
    lf = {"hinge": lambda a: loss.PairwiseHingeLoss(a[1]), "logistic": lambda a: loss.PairwiseLogisticLoss(),
          "bce": lambda a: loss.BinaryCrossEntropyLoss(),
          "sans": lambda a: loss.SelfAdversarialNegativeSamplingLoss(a[1], a[2]),
          "sqerr": lambda a: loss.SquareErrorLoss()}[meta["loss"][0]](meta["loss"])
    E = W["ent_emb"].shape[0]
    m = build(meta["model"], s if meta["model"] not in ("DistMult", "RESCAL") else None, lf,
              UniformStrategy(np.arange(E), seed=1))
    m.negative_ratio = meta["K"]
    if meta["model"] in ("TransR", "TransD"):
        m.embedding_params = {"ent_embedding_size": meta["d"], "rel_embedding_size": meta["d"]}
    else:
        m.embedding_params = {"embedding_size": meta["d"]}
    m.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(W[[k for k in W if k != "ent_emb"][0]].shape[0]))}
    if meta["model"] == "RotatE":
        m.limit = meta["limit"]
    dev = torch.device("cuda", 0)
    m.model_weights = {k: torch.tensor(v, dtype=torch.float32, device=dev) for k, v in W.items()}
    reason = engine.fused_plan(m, optimizers.SGD(meta["lr"]))
    if reason is not None:
        pytest.skip("not fused in this build: %s" % reason)
    step = engine.FusedStep(m)
    pos = torch.tensor(z["pos"], device=dev)
    neg = torch.tensor(z[tag + "/neg"], device=dev)
    step(pos, True, optimizers.SGD(meta["lr"]), neg_ids=neg)
    torch.cuda.synchronize()
    step.check_status()
    assert abs(float(step.loss_out) - float(z[tag + "/loss"])) <= 1e-5 * max(1.0, abs(float(z[tag + "/loss"])))
    for k in W:
        np.testing.assert_allclose(m.model_weights[k].cpu().numpy(), z["%s/out/%s" % (tag, k)], atol=1e-5, err_msg=k)


def test_unsupported_plans_take_plugin_path():
    """Combinations the library has no instance for (kge_step_workspace_bytes
    == 0) go to the eager plugin path instead of raising: RotatE rows of 2000
    floats (d = 1000), RESCAL without its regulariser."""
    from KGE import engine, loss, optimizers, score
    from KGE.models.semantic_based.RESCAL import RESCAL
    from KGE.models.translating_based.RotatE import RotatE
    from KGE.ns_strategy import UniformStrategy
    dev = torch.device("cuda", 0)
    E, R = 30, 4
    md = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    m = RotatE({"embedding_size": 1000}, 2, "h+t", score_fn=score.LpDistance(1),
               loss_fn=loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
               ns_strategy=UniformStrategy(np.arange(E), seed=1))
    m.metadata = md
    m.model_weights = {"ent_emb": torch.rand(E, 1000, 2, device=dev), "rel_emb": torch.rand(R, 1000, device=dev)}
    assert "exceeds" in engine.fused_plan(m, optimizers.SGD(0.01))
    m2 = RESCAL({"embedding_size": 8}, 2, "h+t", loss_fn=loss.SquareErrorLoss(), constraint=False,
                ns_strategy=UniformStrategy(np.arange(E), seed=1))
    m2.metadata = md
    m2.model_weights = {"ent_emb": torch.rand(E, 8, device=dev), "rel_inter": torch.rand(R, 8, 8, device=dev)}
    assert "constraint" in engine.fused_plan(m2, optimizers.SGD(0.01))
    X = np.stack([np.arange(8) % E, np.arange(8) % R, (np.arange(8) * 7) % E], 1)
    for mm in (m, m2):
        mm.model_weights = {k: v.cpu() for k, v in mm.model_weights.items()}
        with pytest.warns(UserWarning, match="eager plugin path"):
            mm.train(train_X=X, val_X=X, metadata=md, epochs=1, batch_size=4, optimizer="SGD",
                     seed=1, model_weights_initial=None)
        assert np.isfinite(mm.train_loss_history[0])


@pytest.mark.parametrize("opt_name", ["SGD", "Adam"])
def test_train_bound_fast_path_equals_step_sequence(opt_name, tmp_path):
    """KGEModel.train (BaseModel.py:58-190) on its fast path -- each batch one
    bound kge_step on the reused batch buffer, epoch reads deferred behind the
    next epoch's first batches -- equals the plain sequence of FusedStep calls
    on the same stream of batches: identical weights bit for bit, identical
    per-epoch losses; every epoch's histogram line equals the host bucketing
    of that epoch's weights; the checkpoint holds the final weights."""
    import json as _json
    from KGE import engine, loss, optimizers, score
    from KGE.models.translating_based.TransE import TransE
    from KGE.ns_strategy import UniformStrategy
    z = np.load(os.path.join(os.path.dirname(GOLD), "..", "data", "fb15k237_train.npz"))
    X = z["triples"][:700].astype(np.int64)
    E, R = int(z["n_entities"]), int(z["n_relations"])
    md = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    epochs, B = 3, 64

    def model():
        return TransE({"embedding_size": 32}, 4, "h+t", score_fn=score.LpDistance(2),
                      loss_fn=loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), ns_strategy=UniformStrategy,
                      constraint=True)
    m = model()
    m.train(train_X=X, val_X=None, metadata=md, epochs=epochs, batch_size=B, optimizer=opt_name, seed=11,
            log_path=str(tmp_path))
    assert m.__dict__.get("_bound"), "the fast path was not taken"
    # the same run, one FusedStep call per batch
    m2 = model()
    m2.metadata, m2.batch_size, m2._model_weights_initial, m2._optimizer = md, B, None, opt_name
    m2.seed, m2.log_path = 11, str(tmp_path / "ref")
    it, _ = m2._prepare_for_train(X, None)
    f = engine.FusedStep(m2)
    opt = m2._optimizer
    nb = int(np.ceil(len(X) / B))
    losses = []
    hist = []
    for e in range(epochs):
        acc = torch.zeros(1, device=f.device)
        for _ in range(nb):
            f(next(it), True, opt, accum=acc)
        losses.append(float(acc) / nb)
        hist.append({k: v.detach().cpu().numpy().astype(np.float64).reshape(-1) for k, v in m2.model_weights.items()})
    torch.cuda.synchronize()
    for k in m.model_weights:
        assert torch.equal(m.model_weights[k], m2.model_weights[k]), k
    assert m.train_loss_history == losses
    for k in m.model_weights:
        lines = [_json.loads(x) for x in open(tmp_path / "histogram" / ("%s.jsonl" % k))]
        assert [x["step"] for x in lines] == list(range(epochs))
        for e, line in enumerate(lines):
            x = hist[e][k]
            lo, hi = x.min(), x.max()
            w = (hi - lo) / 30
            idx = np.minimum(np.floor((x - lo) / w), 29).astype(np.int64)
            cnt = np.bincount(idx, minlength=30)
            edges = np.linspace(lo, hi, 31)
            assert line["buckets"] == [[float(edges[j]), float(edges[j + 1]), float(cnt[j])] for j in range(30)], (k, e)
    ck = torch.load(tmp_path / "ckpt.pt", weights_only=True)
    for k in m.model_weights:
        assert torch.equal(ck[k], m.model_weights[k].cpu()), k


@pytest.mark.gpu
@pytest.mark.parametrize("n,bc", [(0, 30), (1, 30), (1000, 1), (257, 30), (3_000_001, 30), (70_000, 256)])
def test_histogram_kernel_matches_host_bucketing(n, bc):
    """kge_histogram (the per-epoch weight histograms, BaseModel.py's
    tf.summary.histogram calls): counts equal numpy's clamp(floor((x - lo) /
    width)) bucketing exactly, values below lo / above the last edge clamp, a
    NaN counts in bucket 0, lo / width are read on the device, counts
    accumulate into the caller's buffer."""
    from KGE import _hip
    g = np.random.default_rng(n + bc)
    x = g.standard_normal(n).astype(np.float32)
    if n > 2:
        x[0], x[1] = np.nan, 1e30
    lo, width = -1.25, 2.5 / bc
    xd = torch.from_numpy(x).cuda()
    lw = torch.tensor([lo, width], dtype=torch.float64, device="cuda")
    c = torch.full((bc,), 5, dtype=torch.int64, device="cuda")
    _hip.check(_hip.lib().kge_histogram(_hip.ptr(xd), n, _hip.ptr(lw), bc, _hip.ptr(c), _hip.stream_handle()),
               "kge_histogram")
    y = np.floor((x.astype(np.float64) - lo) / width)
    k = np.where(np.isnan(y), 0, np.clip(np.nan_to_num(y, nan=0.0), 0, bc - 1)).astype(np.int64)
    want = np.bincount(k, minlength=bc) + 5
    assert np.array_equal(c.cpu().numpy(), want)
    with pytest.raises(ValueError):
        _hip.check(_hip.lib().kge_histogram(_hip.ptr(xd), n, _hip.ptr(lw), 257, _hip.ptr(c), _hip.stream_handle()),
                   "kge_histogram")
