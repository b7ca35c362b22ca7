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
