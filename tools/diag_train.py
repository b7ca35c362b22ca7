"""c2-train fixed vs per-batch cost: train() wall at 1 / 2 / 4 epochs and the
host time of its one-off phases (prepare, first bind, final checkpoint join)."""
import math, os, sys, tempfile, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench
import torch
from KGE import optimizers
from KGE.models.translating_based.TransE import TransE
from KGE.ns_strategy import UniformStrategy

class A: workload = "c2"; batch = None; neg = None; dim = None
w = bench.spec("c2", A())
triples, E, R = bench.load_graph()
B = w["B"]
nb = int(math.ceil(len(triples) / B))
meta = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
model = TransE({"embedding_size": w["d"]}, w["K"], w["side"], score_fn=w["score"], loss_fn=w["loss"],
               ns_strategy=UniformStrategy, constraint=w["constraint"])
t = {}
def timed(name, fn):
    def run(*a, **k):
        t0 = time.perf_counter(); r = fn(*a, **k); t[name] = t.get(name, 0) + time.perf_counter() - t0; return r
    return run
for n in ("_prepare_for_train", "_join_checkpoint", "sync_weights", "_save_checkpoint", "_finish_epoch",
          "_histogram_stats", "_end_epoch", "_init_embeddings"):
    setattr(model, n, timed(n, getattr(model, n)))
with tempfile.TemporaryDirectory() as d:
    for ep in (1, 1, 2, 4, 8):
        t.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model.train(train_X=triples, val_X=None, metadata=meta, epochs=ep, batch_size=B,
                    optimizer=optimizers.SGD(0.01), seed=12345, log_path=d)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print("epochs %d wall %.2f ms  per batch %.5f ms  | %s" % (ep, wall * 1e3, wall * 1e3 / (ep * nb),
              " ".join("%s %.2f" % (k, v * 1e3) for k, v in sorted(t.items()))), flush=True)
