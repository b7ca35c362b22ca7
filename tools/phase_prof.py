"""Per-phase wall-clock breakdown of the fused step kernels (profiling build).

    python tools/phase_prof.py build          # here (CPU): KGE/_lib/libkge_hip_prof.so
    python tools/phase_prof.py run [--steps N] [--dim D] [--neg K] [--batch B]   # on the GPU box

The profiling build compiles the same sources with -DKGE_PHASE_PROF: thread 0
of every workgroup adds the s_memrealtime ticks spent in each phase to a
device counter (KGE_PROF points in csrc/kge_step.hip). Printed: mean ticks and
microseconds per workgroup per phase, i.e. where one workgroup's time goes.
"""

import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "knowledge-graph-embedding_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "KGE", "_lib", os.environ.get("KGE_PROF_LIB", "libkge_hip_prof.so"))

SCORE_PHASES = {0: "ids+sample", 1: "ctx+stream (gather/fwd/reduce/bwd)", 2: "wave state->LDS", 3: "merge",
                4: "gpos+finalize+bin", 5: "partials+last-WG reduce"}
UPDATE_PHASES = {16: "dest rows (sort+sum+apply)"}


def build(extra=()):
    objs = []
    for src in ("kge_step.hip", "kge_abi.hip", "kge_transr.hip", "kge_rel.hip", "kge_stream.hip", "kge_exchange.hip"):
        obj = os.path.join("/tmp", "prof_" + src.replace(".hip", ".o"))
        # the bench's instance only (KGE_ONLY_ONE): seconds instead of minutes
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-DKGE_PHASE_PROF",
                        "-DKGE_ONLY_ONE"] + list(extra) + ["-c", os.path.join(CSRC, src), "-o", obj], check=True)
        objs.append(obj)
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", LIB], check=True)
    print("built", LIB)


def run(args):
    import numpy as np
    import torch
    from KGE import _hip, engine, loss, optimizers, score
    from KGE.models.translating_based.TransE import TransE
    from KGE.ns_strategy import UniformStrategy

    lib = _hip.load(LIB)
    raw = ctypes.CDLL(LIB)
    raw.kge_prof_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    z = np.load(os.path.join(ROOT, "data", "fb15k237_train.npz"))
    triples, E, R = z["triples"].astype(np.int64), int(z["n_entities"]), int(z["n_relations"])
    B, K, d = args.batch, args.neg, args.dim
    dev = torch.device("cuda", 0)
    big = args.entities > 0
    if big:   # synthetic table (the C2-50M point): no constraint, ids drawn on the device
        E = args.entities
    model = TransE({"embedding_size": d}, K, "h+t", score_fn=score.LpDistance(p=2),
                   loss_fn=loss.SelfAdversarialNegativeSamplingLoss(margin=3, temperature=1),
                   ns_strategy=UniformStrategy(np.arange(E), seed=12345), constraint=not big)
    if big:
        gd = torch.Generator(device=dev).manual_seed(1)
        model.metadata = {"ind2ent": range(E), "ind2rel": list(range(R))}
        model.model_weights = {"ent_emb": (torch.rand((E, d), generator=gd, device=dev) - 0.5) * 0.2,
                               "rel_emb": (torch.rand((R, d), generator=gd, device=dev) - 0.5) * 0.2}
    else:
        model.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
        model._model_weights_initial = None
        model._init_embeddings(seed=12345)
        model._to_device()
    step = engine.FusedStep(model)
    opt = optimizers.SGD(learning_rate=0.01)
    if big:
        gb = torch.Generator(device=dev).manual_seed(2)
        n = args.steps + 5
        batches = torch.stack([torch.randint(0, E, (n, B), generator=gb, device=dev),
                               torch.randint(0, R, (n, B), generator=gb, device=dev),
                               torch.randint(0, E, (n, B), generator=gb, device=dev)], -1)
    else:
        batches = torch.from_numpy(triples[np.random.default_rng(0).integers(0, len(triples), (args.steps + 5, B))]).to(dev)
    buf = (ctypes.c_ulonglong * 64)()
    for s in range(5):
        step(batches[s], True, opt)
    torch.cuda.synchronize()
    raw.kge_prof_read(buf, 64)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for s in range(args.steps):
        step(batches[5 + s], True, opt)
    t1.record()
    torch.cuda.synchronize()
    print("step time (incl. profiling atomics): %.4f ms" % (t0.elapsed_time(t1) / args.steps))
    step.check_status()
    raw.kge_prof_read(buf, 64)
    ticks = list(buf)
    geo = step.geometry() if hasattr(step, "geometry") else None
    nwg_s = (B + 7) // 8 if geo is None else geo[0]
    print("wall clock: 100 MHz ticks (10 ns); per-workgroup means over %d steps" % args.steps)
    for name, phases, nwg in (("score", SCORE_PHASES, args.score_wgs or B), ("update", UPDATE_PHASES, args.update_wgs)):
        tot = sum(ticks[k] for k in phases)
        print("%s kernel (%s workgroups/step assumed)" % (name, nwg))
        for k, label in phases.items():
            per = ticks[k] / max(1, args.steps * nwg)
            print("  %2d %-20s %10.1f ticks/WG  %7.2f us/WG  %5.1f%%" % (k, label, per, per / 100.0,
                                                                        100.0 * ticks[k] / max(1, tot)))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--neg", type=int, default=256)
    ap.add_argument("--dim", type=int, default=200)
    ap.add_argument("--score-wgs", type=int, default=0)
    ap.add_argument("--entities", type=int, default=0, help="synthetic table of this many rows (0: FB15k-237)")
    ap.add_argument("--update-wgs", type=int, default=3686)
    a = ap.parse_args()
    build(os.environ.get("KGE_PROF_FLAGS", "").split()) if a.cmd == "build" else run(a)
