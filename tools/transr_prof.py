"""Per-phase wall-clock breakdown of the TransR kernel (profiling build).

    python tools/transr_prof.py build     # here (CPU): KGE/_lib/libkge_hip_trprof.so
    python tools/transr_prof.py run       # on the GPU box: C4 TransR steps

Thread 0 of each workgroup adds the s_memrealtime ticks of each phase
(KGE_PROF points 32..42 in csrc/kge_transr.hip) to a device counter.
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
LIB = os.path.join(PKG, "KGE", "_lib", os.environ.get("KGE_TRPROF_LIB", "libkge_hip_trprof.so"))
PHASES = {32: "ids", 33: "gather X", 34: "row stats + GEMM1", 35: "clip", 36: "scores", 37: "loss coefs",
          38: "grads (regs)", 39: "S rows + sums", 40: "GEMM2", 41: "GEMM3", 42: "keys"}
# transr2_kernel (two per CU, the default; --v1 times transr_kernel)
# (in execution order: KGE_PROF(k) in csrc/kge_transr2.h closes the phase named here)
PHASES2 = {32: "ids", 33: "gather X", 34: "row stats + GEMM1", 35: "clip + h/t rows", 36: "scores", 37: "loss coefs",
           38: "passes A-C", 39: "(drain)", 44: "Q rows + barrier", 40: "GEMM2 norms", 43: "S' rows + GEMM2",
           41: "GEMM3 + dM stores", 42: "keys"}


def build(extra=()):
    """The library's objects as build() made them, with kge_transr.hip and the
    P2 unit of kge_transr2 recompiled with -DKGE_PHASE_PROF."""
    import __graft_entry__ as g
    g.build()
    prof = {"kge_transr.hip", "kge_transr2_p2.hip"}
    objs, procs = [], []
    for src in g.SOURCES:
        if src not in prof:
            objs.append(os.path.join(ROOT, "build", "obj", "%s.%s.o" % (src[:-4], g._obj_key(src))))
            continue
        obj = os.path.join("/tmp", "trprof_" + src.replace(".hip", ".o"))
        cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-DKGE_PHASE_PROF"] + list(extra) + [
               "-c", os.path.join(CSRC, src), "-o", obj]
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    for p in procs:
        assert p.wait() == 0
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", LIB], check=True)
    print("built", LIB)


def run(args):
    if args.v1:
        os.environ["KGE_TRANSR_V1"] = "1"
    phases = PHASES if args.v1 else PHASES2
    import numpy as np
    import torch
    sys.argv = [sys.argv[0]]
    import bench
    from KGE import _hip, engine
    _hip.load(LIB)
    raw = ctypes.CDLL(LIB)
    read = raw.kge_trprof_read if args.v1 else raw.kge_trprof2_read   # (each unit counts its own kernel)
    read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda", 0)
    a = argparse.Namespace(batch=args.batch, neg=None, dim=None)
    w = bench.spec("c4-transr", a)
    triples, E, R = bench.load_graph()
    m, opt = bench.build_model(w, E, R, 0, dev)
    step = engine.FusedStep(m)
    B = w["B"]
    batches = torch.from_numpy(triples[np.random.default_rng(0).integers(0, len(triples), (args.steps + 5, B))]).to(dev)
    buf = (ctypes.c_ulonglong * 64)()
    for s in range(5):
        step(batches[s], True, opt)
    torch.cuda.synchronize()
    read(buf, 64)
    for s in range(args.steps):
        step(batches[5 + s], True, opt)
    torch.cuda.synchronize()
    step.check_status()
    read(buf, 64)
    ticks = list(buf)
    tot = sum(ticks[k] for k in phases)
    print("TransR kernel %s, B=%d workgroups/step, per-workgroup means over %d steps (10 ns ticks)" % ("v1" if args.v1 else "v2", B, args.steps))
    for k, label in phases.items():
        per = ticks[k] / max(1, args.steps * B)
        print("  %2d %-20s %10.1f ticks/WG  %7.2f us/WG  %5.1f%%" % (k, label, per, per / 100.0,
                                                                    100.0 * ticks[k] / max(1, tot)))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--v1", action="store_true", help="time the one-workgroup-per-CU kernel")
    a = ap.parse_args()
    build() if a.cmd == "build" else run(a)
