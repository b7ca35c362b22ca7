"""GPU: batched filtered ranking (kge_rank, csrc/kge_rank.hip) vs the
reference's per-triple get_rank (BaseModel.py:620-654) restated in torch on
the same weights. Ranks are integers; they must be equal except where the
per-triple path's own scores tie the true triple's within fp32 rounding
(|s_e - s_true| <= 1e-5 max(1, |s_true|)), where a rank may move by at most
the number of such near-ties."""

import os

import numpy as np
import pytest
import torch

from tests.test_plugin_surface import build, toy

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _fused(monkeypatch, hiplib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("KGE_BACKEND", "fused")


def _per_triple(m, X, side, positive_X):
    """Reference loop: ranks and the near-tie count of each query."""
    ranks, ties = [], []
    for x in X:
        ranks.append(int(m.get_rank(x, positive_X, side)))
        with torch.no_grad():
            s = (m.score_hrt(h=None, r=x[1], t=x[2]) if side == "h" else m.score_hrt(h=x[0], r=x[1], t=None))
            s = s.reshape(-1).double()
            p = m.score_hrt(x[0:1], x[1:2], x[2:3]).reshape(()).double()
        ties.append(int(torch.sum(torch.abs(s - p) <= 1e-5 * max(1.0, abs(float(p)))).item()))
    return np.array(ranks), np.array(ties)


def _check(got, ref, ties):
    assert got.dtype == np.int64 and got.shape == ref.shape
    assert (got >= 1).all()
    bad = np.abs(got - ref) > ties
    assert not bad.any(), (np.nonzero(bad)[0][:10], got[bad][:10], ref[bad][:10], ties[bad][:10])


MODELS = ["TransE", "TransH", "TransR", "TransD", "RotatE", "DistMult", "RESCAL"]


@pytest.mark.parametrize("name", MODELS)
@pytest.mark.parametrize("side", ["h", "t"])
def test_rank_toy_matches_get_rank(name, side, tmp_path):
    from KGE import ranking, score
    train, val, md = toy()
    sc = None if name in ("DistMult", "RESCAL") else (score.LpDistance(1) if name == "RotatE" else score.LpDistance(2))
    m = build(name, sc)
    m.train(train_X=train, val_X=val, metadata=md, epochs=2, batch_size=4, optimizer="SGD", seed=7,
            log_path=str(tmp_path))
    assert ranking.supported(m)
    X = np.concatenate([train, val])
    for positive_X in (None, X):
        got = ranking.batched_ranks(m, X, side, positive_X)
        ref, ties = _per_triple(m, X, side, positive_X)
        _check(got, ref, ties)


@pytest.mark.parametrize("name,si", [("TransE", 1), ("TransE", 2), ("TransE", 3), ("TransH", 4), ("TransD", 5),
                                     ("RotatE", 2), ("TransR", 3), ("TransE", 6), ("RotatE", 6), ("TransD", 7)])
def test_rank_score_kinds(name, si, tmp_path):
    """Every score kind the kernel instantiates (p = 1, 2, inf, Pow, Dot)."""
    from KGE import ranking, score
    train, val, md = toy()
    s = [score.LpDistance(2), score.LpDistance(1), score.LpDistance(np.inf), score.LpDistancePow(2),
         score.LpDistancePow(1), score.Dot(), score.LpDistance(3), score.LpDistancePow(1.5)][si]
    m = build(name, s)
    m.train(train_X=train, val_X=val, metadata=md, epochs=1, batch_size=4, optimizer="SGD", seed=3,
            log_path=str(tmp_path))
    X = np.concatenate([train, val])
    for side in ("h", "t"):
        got = ranking.batched_ranks(m, X, side, X)
        ref, ties = _per_triple(m, X, side, X)
        _check(got, ref, ties)


def test_evaluate_uses_kernel_and_metrics(tmp_path):
    """evaluate() on the fused backend returns the reference's metric dict
    computed from the kernel's ranks (same as the per-triple loop)."""
    from KGE import ranking
    train, val, md = toy()
    m = build("TransE")
    m.train(train_X=train, val_X=val, metadata=md, epochs=1, batch_size=4, optimizer="SGD", seed=1,
            log_path=str(tmp_path))
    r = m.evaluate(eval_X=val, corrupt_side="t", positive_X=np.concatenate([train, val]))
    ranks = ranking.batched_ranks(m, val, "t", np.concatenate([train, val]))
    assert r["mean_rank"] == pytest.approx(float(np.mean(ranks)))
    assert r["hit@10"] == pytest.approx(float(np.mean(ranks <= 10)))


def test_rank_fb15k237_slice_transe_d200():
    """FB15k-237 graph (E = 14,541), TransE d = 200 with random weights: 300
    triples ranked against all entities, filtered by the whole training set,
    both sides, vs the per-triple path."""
    from KGE import ranking, score
    from KGE.models.translating_based.TransE import TransE
    z = np.load(os.path.join(ROOT, "data", "fb15k237_train.npz"))
    T = z["triples"].astype(np.int64)
    E, R = int(z["n_entities"]), int(z["n_relations"])
    m = TransE({"embedding_size": 200}, 1, "t", score_fn=score.LpDistance(2))
    m.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    g = torch.Generator().manual_seed(0)
    dev = torch.device("cuda", 0)
    m.model_weights = {"ent_emb": ((torch.rand(E, 200, generator=g) - 0.5) * 0.2).to(dev),
                       "rel_emb": ((torch.rand(R, 200, generator=g) - 0.5) * 0.2).to(dev)}
    X = T[np.random.default_rng(1).choice(len(T), 300, replace=False)]
    PX = torch.as_tensor(T, device=dev)
    for side in ("h", "t"):
        got = ranking.batched_ranks(m, X, side, PX)
        ref, ties = _per_triple(m, X, side, T)
        _check(got, ref, ties)
        assert (got > 1).any()


@pytest.mark.parametrize("name,si", [("TransE", 0), ("TransE", 1), ("TransE", 2), ("TransE", 3), ("TransE", 4),
                                     ("TransE", 5), ("DistMult", None), ("RESCAL", None), ("TransR", 0)])
def test_rank_tiled_pass_equals_lane_pass(name, si):
    """The register-tiled count pass and the lane-per-candidate pass score with
    the same ops in the same order: identical ranks, integer for integer, on a
    FB15k-237-sized candidate set (E = 14,541) with 333 queries per side,
    filtered by the whole training set -- including ranks decided by ties.
    Each pass with the filter as a bitmap (the default, ABI 8) and with the
    rescoring filter pass: the same four rank vectors."""
    from KGE import _hip, ranking, score
    from tests.test_plugin_surface import build
    z = np.load(os.path.join(ROOT, "data", "fb15k237_train.npz"))
    T = z["triples"].astype(np.int64)
    E, R = int(z["n_entities"]), int(z["n_relations"])
    sc = None if si is None else [score.LpDistance(2), score.LpDistance(1), score.LpDistance(np.inf),
                                  score.LpDistancePow(2), score.Dot(), score.LpDistance(3)][si]
    m = build(name, sc)
    m.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    m._model_weights_initial = None
    m._init_embeddings(seed=5)
    m._to_device()
    X = T[np.random.default_rng(2).choice(len(T), 333, replace=False)]
    # a few duplicated candidate rows: exact ties with the true entity's score
    with torch.no_grad():
        w = m.model_weights["ent_emb"]
        w[(X[:20, 0] + 1) % E] = w[X[:20, 0]]
        w[(X[:20, 2] + 1) % E] = w[X[:20, 2]]
    PX = torch.as_tensor(T, device=w.device)
    for side in ("h", "t"):
        tiled = ranking.batched_ranks(m, X, side, PX)
        lane = ranking.batched_ranks(m, X, side, PX, flags=_hip.RANK_FLAG_LANE_PASS)
        assert np.array_equal(tiled, lane), np.nonzero(tiled != lane)[0][:10]
        for f in (ranking.RESCORE_FILTER, ranking.RESCORE_FILTER | _hip.RANK_FLAG_LANE_PASS):
            rs = ranking.batched_ranks(m, X, side, PX, flags=f)
            assert np.array_equal(tiled, rs), (f, np.nonzero(tiled != rs)[0][:10])


def test_rank_filter_bitmap_abi():
    """kge_rank's bitmap filter through the C-ABI: a bitmap shorter than
    n * ceil(E / 32) words is refused; an out-of-range filter id sets
    KGE_ERANGE in the status word (as the rescoring pass does); words past a
    query's filter are cleared whatever the buffer held."""
    import ctypes
    from KGE import _hip
    dev = torch.device("cuda", 0)
    E, D, n = 70, 8, 3
    g = torch.Generator().manual_seed(3)
    cand = torch.rand(E, D, generator=g).to(dev)
    q0 = torch.rand(n, D, generator=g).to(dev)
    ids = torch.tensor([1, 5, 69], dtype=torch.int64, device=dev)
    fent = torch.tensor([1, 2, 40, 5, 69, 0], dtype=torch.int64, device=dev)
    fb = torch.tensor([0, 3, 4], dtype=torch.int64, device=dev)
    fe = torch.tensor([3, 4, 6], dtype=torch.int64, device=dev)
    W = (E + 31) // 32
    bits = torch.full((n * W,), -1, dtype=torch.int32, device=dev)
    rk = torch.zeros(n, dtype=torch.int64, device=dev)
    ps = torch.zeros(n, dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    d = _hip.kge_rank_desc()
    d.abi_version = _hip.ABI_VERSION
    d.mode, d.proj, d.corrupt_side = _hip.RANK_TRANS, _hip.RPROJ_NONE, _hip.SIDE_T
    d.cand = _hip.table(cand)
    d.dim = D
    d.q0, d.ldq = q0.data_ptr(), D
    d.true_ids, d.idx_dtype = ids.data_ptr(), _hip.IDX_I64
    d.score_kind, d.score_p = 0, 2.0   # KGE_SCORE_LP
    d.n = n
    d.filt_beg, d.filt_end, d.filt_ent = fb.data_ptr(), fe.data_ptr(), fent.data_ptr()
    d.rank_out, d.pos_score_out, d.status = rk.data_ptr(), ps.data_ptr(), status.data_ptr()
    d.filt_bits, d.filt_bits_words = bits.data_ptr(), n * W - 1
    lib = _hip.lib()
    assert lib.kge_rank(ctypes.byref(d), _hip.stream_handle(dev)) == _hip.KGE_EINVAL
    d.filt_bits_words = n * W
    assert lib.kge_rank(ctypes.byref(d), _hip.stream_handle(dev)) == _hip.KGE_OK
    torch.cuda.synchronize()
    got = bits.view(n, W).cpu().numpy().view(np.uint32)
    want = np.zeros((n, W), dtype=np.uint32)
    for q, ents in enumerate([[1, 2, 40], [5], [69, 0]]):
        for e in ents:
            want[q, e >> 5] |= np.uint32(1 << (e & 31))
    assert np.array_equal(got, want)
    assert int(status.item()) == 0
    # the ranks with and without the bitmap
    with_bits = rk.cpu().numpy().copy()
    d.filt_bits, d.filt_bits_words = None, 0
    assert lib.kge_rank(ctypes.byref(d), _hip.stream_handle(dev)) == _hip.KGE_OK
    torch.cuda.synchronize()
    assert np.array_equal(with_bits, rk.cpu().numpy())
    # an id past the table
    fent[2] = E
    d.filt_bits, d.filt_bits_words = bits.data_ptr(), n * W
    assert lib.kge_rank(ctypes.byref(d), _hip.stream_handle(dev)) == _hip.KGE_OK
    torch.cuda.synchronize()
    assert int(status.item()) == _hip.KGE_ERANGE


def _oracle_weights(m):
    return {k: v.detach().cpu().numpy() for k, v in m.model_weights.items()}


def _oracle_score(m):
    from tests.test_gpu_step import _spec_score
    sc = getattr(m, "score_fn", None)
    return _spec_score(sc) if sc is not None else ("dot", 0.0)


@pytest.mark.parametrize("name", MODELS)
def test_rank_toy_matches_oracle(name, tmp_path):
    """kge_rank vs the float64 restatement of get_rank in oracle/ (not the
    package's own per-triple path): every model, both sides, unfiltered and
    filtered by every known triple; ranks equal up to the oracle's near-ties."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import kge_oracle as orc
    from KGE import ranking, score
    train, val, md = toy()
    sc = None if name in ("DistMult", "RESCAL") else (score.LpDistance(1) if name == "RotatE" else score.LpDistance(2))
    m = build(name, sc)
    m.train(train_X=train, val_X=val, metadata=md, epochs=2, batch_size=4, optimizer="SGD", seed=7,
            log_path=str(tmp_path))
    X = np.concatenate([train, val])
    W = _oracle_weights(m)
    for side in ("h", "t"):
        for positive_X in (None, X):
            got = ranking.batched_ranks(m, X, side, positive_X)
            ref, ties = orc.filtered_ranks(name, W, X, side, positive_X, score=_oracle_score(m),
                                           limit=getattr(m, "limit", None),
                                           constraint=bool(getattr(m, "constraint", False)))
            _check(got, ref, ties)


@pytest.mark.parametrize("name", ["TransE", "DistMult", "RotatE"])
def test_rank_fb15k237_slice_matches_oracle(name):
    """FB15k-237 (E = 14,541), d = 200 random weights, 200 triples per side
    filtered by the whole training set: kge_rank == the float64 oracle up to
    near-ties."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import kge_oracle as orc
    from KGE import ranking, score
    z = np.load(os.path.join(ROOT, "data", "fb15k237_train.npz"))
    T = z["triples"].astype(np.int64)
    E, R = int(z["n_entities"]), int(z["n_relations"])
    sc = None if name == "DistMult" else score.LpDistance(2)
    m = build(name, sc, embedding_params={"embedding_size": 200})
    m.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    m._model_weights_initial = None
    m._init_embeddings(seed=11)
    m._to_device()
    X = T[np.random.default_rng(4).choice(len(T), 200, replace=False)]
    W = _oracle_weights(m)
    PX = torch.as_tensor(T, device=m.model_weights["ent_emb"].device)
    for side in ("h", "t"):
        got = ranking.batched_ranks(m, X, side, PX)
        ref, ties = orc.filtered_ranks(name, W, X, side, T, score=_oracle_score(m),
                                       limit=getattr(m, "limit", None),
                                       constraint=bool(getattr(m, "constraint", False)))
        _check(got, ref, ties)
        assert (got > 1).any()
