"""Two ranks on ONE GPU (gloo, device tensors staged through the host): the
device-resident multi-GPU step with real remote rows -- kge_exchange_plan's
owner blocks, the owners' gathers, the split step's raw gradients of fetched
rows sent back and applied by their owner (kge_exchange_rows), the grad-mode
path (TransD, Adam), the dense replica (one all-reduce) -- equals the
single-device oracle step on the concatenated batch with the same negatives
(the CPU twin of this file is tests/test_sharded.py, on the host
restatement)."""

import math

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import kge_oracle as orc
from tests.test_sharded import B, E, K, _case, _model, _port

pytestmark = pytest.mark.gpu


def _worker(rank, port, name, loss, opt, steps, mode, loopback, out):
    import torch.distributed as dist
    import __graft_entry__  # noqa: F401  (sys.path; the parent's hiplib fixture built the library)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=2)
    from KGE import optimizers
    from KGE.sharded import ShardedStep
    dev = torch.device("cuda", 0)
    W, pos, neg = _case(0, name)
    m = _model(name, W, loss)
    m.model_weights = {k: v.to(dev) for k, v in m.model_weights.items()}
    st = ShardedStep(m, mode=mode, loopback=loopback, batch_hint=B)
    assert st.mode == mode and st.fused is not None
    o = optimizers.SGD(0.05) if opt == "sgd" else optimizers.Adam(0.01)
    for _ in range(steps):
        b = torch.tensor(pos[rank * B:(rank + 1) * B], device=dev)
        n = torch.tensor(neg[rank * B * K:(rank + 1) * B * K], device=dev)
        loss_v = float(st(b, True, o, neg_ids=n))
    torch.cuda.synchronize()
    st.check_status()
    st.sync()
    if rank == 0:
        out.put(({k: v.detach().cpu().numpy().copy() for k, v in m.model_weights.items()}, loss_v))
    dist.barrier()
    dist.destroy_process_group()


def _run(name, loss, opt, steps, mode, loopback=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, name, loss, opt, steps, mode, loopback, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        res = q.get(timeout=100)
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    for p in ps:
        assert p.exitcode == 0
    return res


_SCORE = {"TransE": ("lp", 2.0), "DistMult": ("dot", 0.0), "TransD": ("lppow", 2.0), "RotatE": ("lp", 1.0),
          "RESCAL": ("dot", 0.0), "TransH": ("lppow", 2.0)}
_LOSS = {"sans": ("sans", 3.0, 1.0), "hinge": ("hinge", 1.0), "bce": ("bce",), "sqerr": ("sqerr",)}


@pytest.mark.parametrize("name,loss,opt,mode,loopback", [
    ("TransE", "sans", "sgd", "sparse", False),     # split step, remote rows' gradients back to owners
    ("RotatE", "sans", "sgd", "sparse", False),
    ("DistMult", "bce", "sgd", "sparse", True),     # loopback: own rows through the blocks too
    ("TransD", "hinge", "sgd", "sparse", False),    # grad-mode step on the extended table
    ("TransE", "sans", "adam", "sparse", False),    # owner ACCUM + dense keras Adam of the shard
    ("TransE", "sans", "sgd", "dense", False),      # replica + one all-reduce
    ("RESCAL", "sqerr", "sgd", "dense", False),     # full-table regulariser, 1/G per rank
    ("TransE", "sans", "sgd", "owner", False),      # owner-side scoring: records, merge, owner update
    ("TransE", "hinge", "sgd", "owner", True),
    ("RotatE", "sans", "sgd", "owner", False),
    ("DistMult", "bce", "sgd", "owner", False),
])
def test_two_ranks_one_gpu_equal_oracle(hiplib, name, loss, opt, mode, loopback):
    steps = 2
    got, got_loss = _run(name, loss, opt, steps, mode, loopback)
    W, pos, neg = _case(0, name)
    ref_w, state = W, None
    for _ in range(steps):
        ref = orc.train_step(name, ref_w, pos, neg, score=_SCORE[name], loss=_LOSS[loss],
                             lr=0.05 if opt == "sgd" else 0.01, constraint=name != "RotatE", constraint_weight=0.1,
                             side="h+t", limit=0.7, optimizer=opt, adam_state=state)
        ref_w, state = ref["weights"], ref.get("adam")
    assert math.isfinite(got_loss)
    assert abs(got_loss - ref["loss"]) <= 1e-5 * max(1.0, abs(ref["loss"]))
    for k, v in ref_w.items():
        np.testing.assert_allclose(got[k], v, atol=1e-5, err_msg=k)


# owner-side scoring at a bench-like shape: two ranks on one GPU, in-kernel draws
OE, OR, OD, OB, OK = 60_000, 40, 200, 128, 64


def _owner_case():
    rng = np.random.default_rng(77)
    lim = 6.0 / np.sqrt(OD)
    W = {"ent_emb": rng.uniform(-lim, lim, (OE, OD)).astype(np.float32),
         "rel_emb": rng.uniform(-lim, lim, (OR, OD)).astype(np.float32)}
    pos = [np.stack([rng.integers(0, OE, 2 * OB), rng.integers(0, OR, 2 * OB), rng.integers(0, OE, 2 * OB)], 1)
           for _ in range(2)]
    return W, pos


def _owner_worker(rank, port, out):
    import torch.distributed as dist
    import __graft_entry__  # noqa: F401
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=2)
    from KGE import loss, optimizers, score
    from KGE.models.translating_based.TransE import TransE
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = torch.device("cuda", 0)
    W, pos = _owner_case()
    m = TransE({"embedding_size": OD}, OK, "h+t", score_fn=score.LpDistance(2),
               loss_fn=loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
               ns_strategy=UniformStrategy(np.arange(OE), seed=3), constraint=True)
    m.metadata = {"ind2ent": list(range(OE)), "ind2rel": list(range(OR))}
    m.model_weights = {k: torch.tensor(v, device=dev) for k, v in W.items()}
    st = ShardedStep(m, mode="owner", batch_hint=OB)
    assert st.mode == "owner" and st.fused is not None
    o = optimizers.SGD(0.05)
    losses = []
    for p in pos:
        losses.append(float(st(torch.tensor(p[rank * OB:(rank + 1) * OB], device=dev), True, o)))
    torch.cuda.synchronize()
    st.check_status()
    st.sync()
    if rank == 0:
        out.put(({k: v.detach().cpu().numpy().copy() for k, v in m.model_weights.items()}, losses))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_one_gpu_owner_bench_shape(hiplib):
    """Owner-side scoring across two ranks at d = 200, K = 64 'h+t' (C2 / C4's
    row width and a multi-wave negative count), 2 x 128 positives, 60k
    entities (ranks own 30k rows each), renormalisation constraint, SGD, the
    negatives drawn IN the owner pass from each positive's own rank's counter
    planes (offset + q * 2, KGE/sharded.py) -- two steps == two single-device
    oracle steps on the concatenated batch with those draws."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_owner_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        got, got_losses = q.get(timeout=150)
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    for p in ps:
        assert p.exitcode == 0
    W, pos = _owner_case()
    ref_w = W
    for s, P in enumerate(pos):
        base = s * 2 * 2        # take_planes(2) * G
        neg = np.concatenate([orc.negatives(P[q * OB:(q + 1) * OB], OK, "h+t", OE, seed=3, plane=base + 2 * q)
                              for q in range(2)])
        ref = orc.train_step("TransE", ref_w, P, neg, score=("lp", 2.0), loss=("sans", 3.0, 1.0), lr=0.05,
                             constraint=True, side="h+t")
        ref_w = ref["weights"]
        assert abs(got_losses[s] - ref["loss"]) <= 1e-5 * max(1.0, abs(ref["loss"])), s
    for k, v in ref_w.items():
        np.testing.assert_allclose(got[k], v, atol=1e-5, err_msg=k)


def _overflow_worker(rank, port, mode, out):
    import torch.distributed as dist
    import __graft_entry__  # noqa: F401
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=2)
    from KGE import loss, optimizers, score
    from KGE.models.translating_based.TransE import TransE
    from KGE.ns_strategy import UniformStrategy
    from KGE.sharded import ShardedStep
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(91)
    E_, R_, d_, B_, K_ = 4000, 5, 24, 32, 4
    W = {"ent_emb": rng.uniform(-0.3, 0.3, (E_, d_)).astype(np.float32),
         "rel_emb": rng.uniform(-0.3, 0.3, (R_, d_)).astype(np.float32)}
    m = TransE({"embedding_size": d_}, K_, "h+t", score_fn=score.LpDistance(2),
               loss_fn=loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0),
               ns_strategy=UniformStrategy(np.arange(E_), seed=3), constraint=False)
    m.metadata = {"ind2ent": list(range(E_)), "ind2rel": list(range(R_))}
    m.model_weights = {k: torch.tensor(v, device=dev) for k, v in W.items()}
    # blocks of a few rows: both ranks' steps request far more remote rows
    st = ShardedStep(m, mode=mode, batch_hint=B_, capacity_slack=0.05, capacity_floor=0,
                     optimizer=optimizers.SGD(0.05))
    pos = np.stack([rng.integers(0, E_, B_), rng.integers(0, R_, B_), rng.integers(0, E_, B_)], 1)
    st(torch.tensor(pos, device=dev), True, optimizers.SGD(0.05))
    torch.cuda.synchronize()
    msg = ""
    try:
        st.check_status()
    except RuntimeError as e:
        msg = str(e)
    st.sync()
    unchanged = bool(np.array_equal(m.model_weights["ent_emb"].cpu().numpy(), W["ent_emb"]))
    out.put((rank, msg, unchanged))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["sparse", "owner"])
def test_two_ranks_both_overflow_exchange(hiplib, mode):
    """Both ranks overflow an exchange block in the same step: the step is
    void on both (no table row changes) and check_status() names the
    exchange block on both -- the per-kind flags are summed across ranks in
    their own slots, so two exchange overflows are not read as the owner
    pass's key overflow."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_overflow_worker, args=(r, port, mode, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=100) for _ in range(2)]
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    for p in ps:
        assert p.exitcode == 0
    for rank, msg, unchanged in res:
        assert "overflowed an owner block" in msg, (rank, msg)
        assert unchanged, rank
