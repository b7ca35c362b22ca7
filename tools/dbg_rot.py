import sys, numpy as np, torch
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/knowledge-graph-embedding_amd'); sys.path.insert(0,'/root/repo/tests')
import __graft_entry__ as g; g.build()
import test_gpu_step as T
from KGE import loss, score
from oracle import kge_oracle as orc
for d in (16,):
    ref, got, l_, ps, ns, step, neg = T.run_case(None, "RotatE", d, 7, 6, "h+t", score.LpDistance(np.inf),
                                          loss.SelfAdversarialNegativeSamplingLoss(3.0, 1.0))
    rng = np.random.default_rng(11)
    W = T._weights("RotatE", 50, 7, d, rng)
    pos = np.stack([rng.integers(0, 50, 7), rng.integers(0, 7, 7), rng.integers(0, 50, 7)], 1)
    diff = np.abs(got["ent_emb"] - ref["weights"]["ent_emb"])
    rows = np.unique(np.where(diff > 1e-5)[0])
    print("bad rows", rows, "max", diff.max())
    for r in rows:
        print("row", r, "cols", np.where(diff[r] > 1e-5), "as pos h:", np.where(pos[:,0]==r)[0], "pos t:", np.where(pos[:,2]==r)[0])
        nn = np.where(neg == r)[0]
        print("   as neg slots", nn, "kinds", ["HC" if (s%6)%2==0 else "TC" for s in nn])
        print("   got", got["ent_emb"][r].reshape(-1)[:8], "\n   ref", ref["weights"]["ent_emb"][r].reshape(-1)[:8], "\n   orig", W["ent_emb"][r].reshape(-1)[:8])
    print("loss", l_, ref["loss"])
    print("neg score max diff", np.abs(ns-ref["neg_score"]).max())
