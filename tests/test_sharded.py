"""CPU (gloo, world size 2): the multi-GPU step (KGE/sharded.py) -- e mod G
row ownership, negatives per rank, the sparse exchange (unique ids ->
all_to_all of ids and rows -> local row cache -> gradient rows back ->
owner-side sum + apply) and the dense one (replicated tables, one
all-reduce of [gradients | norms | loss], the same apply on every rank),
global-batch loss normalisation, global clip norm -- gives the
single-device step on the concatenated batch. The local gradient phase runs
the host restatement (KGE_BACKEND=eager); on GPUs it is kge_step."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import kge_oracle as orc

E, R, D, B, K = 13, 4, 8, 5, 4   # E odd: ranks own 7 and 6 rows


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(name, W, loss):
    from KGE import loss as L
    from KGE import score
    from KGE.models.semantic_based.DistMult import DistMult
    from KGE.models.semantic_based.RESCAL import RESCAL
    from KGE.models.translating_based.RotatE import RotatE
    from KGE.models.translating_based.TransH import TransH
    from KGE.models.translating_based.TransD import TransD
    from KGE.models.translating_based.TransE import TransE
    from KGE.ns_strategy import UniformStrategy
    lf = {"sans": L.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), "hinge": L.PairwiseHingeLoss(1.0),
          "bce": L.BinaryCrossEntropyLoss(), "sqerr": L.SquareErrorLoss()}[loss]
    ns = UniformStrategy(np.arange(E), seed=1)
    if name == "TransE":
        m = TransE({"embedding_size": D}, K, "h+t", score_fn=score.LpDistance(2), loss_fn=lf, ns_strategy=ns,
                   constraint=True)
    elif name == "TransD":
        m = TransD({"ent_embedding_size": D, "rel_embedding_size": 6}, K, "h+t", score_fn=score.LpDistancePow(2),
                   loss_fn=lf, ns_strategy=ns, constraint=True)
    elif name == "RotatE":
        m = RotatE({"embedding_size": D}, K, "h+t", score_fn=score.LpDistance(1), loss_fn=lf, ns_strategy=ns)
        m.limit = 0.7
    elif name == "RESCAL":
        m = RESCAL({"embedding_size": D}, K, "h+t", loss_fn=lf, ns_strategy=ns, constraint=True,
                   constraint_weight=0.1)
    elif name == "TransH":
        m = TransH({"embedding_size": D}, K, "h+t", score_fn=score.LpDistancePow(2), loss_fn=lf, ns_strategy=ns,
                   constraint=True, constraint_weight=0.1)
    else:
        m = DistMult({"embedding_size": D}, K, "h+t", loss_fn=lf, ns_strategy=ns, constraint=True,
                     constraint_weight=0.1)
    m.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    m.model_weights = {k: torch.tensor(v, dtype=torch.float32) for k, v in W.items()}
    return m


def _case(seed, name):
    rng = np.random.default_rng(seed)
    if name == "TransD":
        W = {"ent_emb": rng.uniform(-0.5, 0.5, (E, D)), "rel_emb": rng.uniform(-0.5, 0.5, (R, 6)),
             "ent_proj": rng.uniform(-0.5, 0.5, (E, D)), "rel_proj": rng.uniform(-0.5, 0.5, (R, 6))}
    elif name == "RotatE":
        W = {"ent_emb": rng.uniform(-0.5, 0.5, (E, D, 2)), "rel_emb": rng.uniform(-0.5, 0.5, (R, D))}
    elif name == "RESCAL":
        W = {"ent_emb": rng.uniform(-0.5, 0.5, (E, D)), "rel_inter": rng.uniform(-0.3, 0.3, (R, D, D))}
    elif name == "TransH":
        W = {"ent_emb": rng.uniform(-0.5, 0.5, (E, D)), "rel_emb": rng.uniform(-0.5, 0.5, (R, D)),
             "rel_hyper": rng.uniform(-0.5, 0.5, (R, D))}
    else:
        rk = "rel_emb" if name == "TransE" else "rel_inter"
        W = {"ent_emb": rng.uniform(-0.5, 0.5, (E, D)), rk: rng.uniform(-0.5, 0.5, (R, D))}
    pos = np.stack([rng.integers(0, E, 2 * B), rng.integers(0, R, 2 * B), rng.integers(0, E, 2 * B)], 1)
    neg = rng.integers(0, E, 2 * B * K)
    return W, pos, neg


def _worker(rank, port, name, loss, opt, steps, mode, out):
    os.environ["KGE_BACKEND"] = "eager"
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=2)
    from KGE import optimizers
    from KGE.sharded import ShardedStep
    W, pos, neg = _case(0, name)
    m = _model(name, W, loss)
    o = optimizers.SGD(0.05) if opt == "sgd" else optimizers.Adam(0.01)
    if mode == "auto-large":
        # "auto" on a table past the dense threshold, told the optimizer (as
        # KGEModel.train does): owner-side scoring only for SGD steps
        import KGE.sharded as S
        S.DENSE_TABLE_BYTES = 0
        st = ShardedStep(m, optimizer=o)
        mode = "owner" if opt == "sgd" and name in ("TransE", "DistMult", "RotatE") else "sparse"
    else:
        st = ShardedStep(m, mode=mode)
    assert st.valid == len(range(rank, E, 2))
    if mode == "dense":
        assert not hasattr(st, "shard") and len(st.gent) == (2 if name == "TransD" else 1)
    assert st.mode == mode
    for s in range(steps):
        b = torch.tensor(pos[rank * B:(rank + 1) * B])
        n = torch.tensor(neg[rank * B * K:(rank + 1) * B * K])
        loss_v = float(st(b, True, o, neg_ids=n))
    st.sync()
    if mode == "dense":   # every rank holds the same replica
        for v in m.model_weights.values():
            t = v.detach().clone()
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            assert torch.equal(t, v.detach())
    if rank == 0:
        out.put(({k: v.detach().numpy().copy() for k, v in m.model_weights.items()}, loss_v))
    dist.barrier()
    dist.destroy_process_group()


def _run(name, loss, opt, steps, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, name, loss, opt, steps, mode, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("mode", ["sparse", "dense", "owner"])
@pytest.mark.parametrize("name,loss", [("TransE", "sans"), ("TransE", "hinge"), ("DistMult", "bce"),
                                       ("TransD", "hinge"), ("RotatE", "sans")])
def test_sharded_sgd_equals_single_device_oracle(name, loss, mode):
    """"owner": owner-side scoring (each rank scores every rank's positives
    against the negatives it owns; records merged at the positive's rank) in
    its host restatement -- the same flow and merge algebra as the kernels."""
    if mode == "owner" and name == "TransD":
        pytest.skip("owner-side scoring covers TransE, DistMult and RotatE")
    got, got_loss = _run(name, loss, "sgd", 1, mode)
    W, pos, neg = _case(0, name)
    spec = {"sans": ("sans", 3.0, 1.0), "hinge": ("hinge", 1.0), "bce": ("bce",)}[loss]
    sc = {"TransE": ("lp", 2.0), "DistMult": ("dot", 0.0), "TransD": ("lppow", 2.0), "RotatE": ("lp", 1.0)}[name]
    ref = orc.train_step(name, W, pos, neg, score=sc, loss=spec, lr=0.05, constraint=name != "RotatE",
                         constraint_weight=0.1, side="h+t", limit=0.7)
    assert abs(got_loss - ref["loss"]) <= 1e-5 * max(1.0, abs(ref["loss"]))
    for k, v in ref["weights"].items():
        np.testing.assert_allclose(got[k], v, atol=2e-6, err_msg=k)


@pytest.mark.parametrize("name,loss", [("RESCAL", "sqerr"), ("TransH", "sans"), ("TransH", "hinge")])
@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_sharded_full_table_regulariser_dense_mode(name, loss, opt):
    """RESCAL / TransH with constraint (dense gradients of every row,
    RESCAL.py:190-198, TransH.py:202-211) across 2 ranks in the dense
    exchange: each rank adds half of the regulariser, the all-reduce sums it,
    the clip norm is the reduced tensor's -- two steps == two single-device
    steps at 2B (oracle for SGD, the eager path for Adam)."""
    got, got_loss = _run(name, loss, opt, 2, "dense")
    W, pos, neg = _case(0, name)
    spec = {"sans": ("sans", 3.0, 1.0), "hinge": ("hinge", 1.0), "sqerr": ("sqerr",)}[loss]
    sc = {"RESCAL": ("dot", 0.0), "TransH": ("lppow", 2.0)}[name]
    ref_w, state = W, None
    for _ in range(2):
        ref = orc.train_step(name, ref_w, pos, neg, score=sc, loss=spec, lr=0.05 if opt == "sgd" else 0.01,
                             constraint=True, constraint_weight=0.1, side="h+t", optimizer=opt, adam_state=state)
        ref_w, state = ref["weights"], ref.get("adam")
    assert abs(got_loss - ref["loss"]) <= 1e-5 * max(1.0, abs(ref["loss"]))
    for k, v in ref_w.items():
        np.testing.assert_allclose(got[k], v, atol=2e-6, err_msg=k)


def test_sparse_mode_refuses_full_table_regulariser():
    os.environ["KGE_BACKEND"] = "eager"
    try:
        import torch.distributed as dist
        from KGE.sharded import ShardedStep
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % _port(), rank=0, world_size=1)
        try:
            W, _, _ = _case(0, "RESCAL")
            m = _model("RESCAL", W, "sqerr")
            assert ShardedStep(m).mode == "dense"   # auto picks the dense exchange at any size
            with pytest.raises(NotImplementedError):
                ShardedStep(m, mode="sparse")
        finally:
            dist.destroy_process_group()
    finally:
        os.environ.pop("KGE_BACKEND", None)


@pytest.mark.parametrize("mode", ["sparse", "dense", "auto-large"])
def test_sharded_adam_equals_single_device_eager(mode):
    """Two Adam steps across 2 ranks == two steps of the single-process eager
    path at 2B ("auto-large": "auto" above the dense threshold with keras Adam
    takes the row exchange, not owner-side scoring)."""
    os.environ["KGE_BACKEND"] = "eager"
    try:
        from KGE import engine, optimizers
        got, _ = _run("TransE", "sans", "adam", 2, mode)
        W, pos, neg = _case(0, "TransE")
        m = _model("TransE", W, "sans")
        o = optimizers.Adam(0.01)
        negt = torch.tensor(orc.corrupt(pos, neg, K, "h+t"))
        for _ in range(2):
            engine.eager_step(m, torch.tensor(pos), True, o, neg=negt)
    finally:
        os.environ.pop("KGE_BACKEND", None)
    for k, v in m.model_weights.items():
        np.testing.assert_allclose(got[k], v.numpy(), atol=2e-6, err_msg=k)


def test_auto_mode_follows_the_optimizer():
    """ShardedStep "auto" above the dense-table threshold: owner-side scoring
    for TransE / DistMult / RotatE with SGD (or an unknown optimizer), the
    row exchange for keras Adam and for the other models."""
    os.environ["KGE_BACKEND"] = "eager"
    try:
        import torch.distributed as dist
        import KGE.sharded as S
        from KGE import optimizers
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % _port(), rank=0, world_size=1)
        old = S.DENSE_TABLE_BYTES
        S.DENSE_TABLE_BYTES = 0
        try:
            W, _, _ = _case(0, "TransE")
            m = _model("TransE", W, "sans")
            assert S.ShardedStep(m, optimizer=optimizers.SGD(0.1)).mode == "owner"
            assert S.ShardedStep(m, optimizer=optimizers.Adam(0.01)).mode == "sparse"
            assert S.ShardedStep(m).mode == "owner"
            W, _, _ = _case(0, "TransD")
            assert S.ShardedStep(_model("TransD", W, "hinge"), optimizer=optimizers.SGD(0.1)).mode == "sparse"
        finally:
            S.DENSE_TABLE_BYTES = old
            dist.destroy_process_group()
    finally:
        os.environ.pop("KGE_BACKEND", None)
