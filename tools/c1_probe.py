"""GPU probe: where a launch-bound step (C1) spends its wall time -- host call
time of one FusedStep call, and steps/s with and without a sync per step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "knowledge-graph-embedding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from KGE import _hip, engine  # noqa: E402


class A:
    batch = None; neg = None; dim = None


_hip.load()
dev = torch.device("cuda", 0)
w = bench.spec(sys.argv[1] if len(sys.argv) > 1 else "c1", A)
triples, E, R = bench.load_graph()
model, opt = bench.build_model(w, E, R, 0, dev)
step = engine.FusedStep(model)
B = w["B"]
idx = torch.randint(0, len(triples), (400 * B,))
batches = torch.from_numpy(triples)[idx].reshape(400, B, 3).to(dev)
for s in range(20):
    step(batches[s], True, opt)
torch.cuda.synchronize()
t0 = time.perf_counter()
host = 0.0
for s in range(200):
    h0 = time.perf_counter()
    step(batches[s], True, opt)
    host += time.perf_counter() - h0
torch.cuda.synchronize()
t1 = time.perf_counter()
print("async: %.4f ms/step, host call %.4f ms" % ((t1 - t0) * 5, host * 5))
t0 = time.perf_counter()
for s in range(200):
    step(batches[s], True, opt)
    torch.cuda.synchronize()
print("synced: %.4f ms/step" % ((time.perf_counter() - t0) * 5))
import cProfile, pstats  # noqa: E402
pr = cProfile.Profile()
pr.enable()
for s in range(100):
    step(batches[s], True, opt)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumtime").print_stats(12)
