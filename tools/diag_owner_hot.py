import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
import __graft_entry__ as ge
ge.build()
from test_gpu_step import _dev, _init_world1, _weights, _make, orc
import torch.distributed as dist
from KGE import _hip, loss, optimizers, score
from KGE.ns_strategy import UniformStrategy
from KGE.sharded import ShardedStep
dev = _dev(); _init_world1(dist, dev)
E, R, d, B, K = 100000, 6, 24, 400, 8
W = _weights("TransE", E, R, d, np.random.default_rng(17))
for loopback in (False, True):
  for flags in (0, _hip.FLAG_DEBUG_NO_REL_SEG):
    rng = np.random.default_rng(18)
    m = _make("TransE", d, K, "h+t", score.LpDistance(2), loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0), E, R, UniformStrategy(np.arange(E), seed=4), constraint=False)
    m.model_weights = {kk: torch.tensor(v, device=dev) for kk, v in W.items()}
    st = ShardedStep(m, mode="owner", loopback=loopback, local_fast=False); st.debug_flags = flags
    ref_w = W; opt = optimizers.SGD(0.05)
    for it in range(2):
        h = np.where(rng.random(B) < 0.4, 7, rng.integers(0, E, B)); t = np.where(rng.random(B) < 0.3, 11, rng.integers(0, E, B)); r = np.where(rng.random(B) < 0.6, 0, rng.integers(0, R, B))
        pos = np.stack([h, r, t], 1).astype(np.int64); plane = m.ns_strategy.offset
        lv = float(st(torch.tensor(pos, device=dev), True, opt)); torch.cuda.synchronize(); st.check_status()
        neg = orc.negatives(pos, K, "h+t", E, seed=4, plane=plane)
        ref = orc.train_step("TransE", ref_w, pos, neg, score=("lp", 2.0), loss=("sans", 3.0, 1.0), lr=0.05, constraint=False)
        ref_w = ref["weights"]
        st.sync()
        msg = []
        for kk, v in ref_w.items():
            got = m.model_weights[kk].cpu().numpy(); dd = np.abs(got - v)
            rows = np.unique(np.nonzero(dd > 1e-5)[0])
            msg.append("%s maxdiff %.3g rows %s" % (kk, dd.max(), rows[:10]))
        print("loop", loopback, "flags", flags, "step", it, "loss", lv, ref["loss"], "|", "; ".join(msg), flush=True)
    del st
dist.destroy_process_group()
