"""bench.py -- KGE training-step throughput on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): TransE, d=200,
batch 1024 positives x 256 negatives ('h+t'), LpDistance(2),
SelfAdversarialNegativeSamplingLoss(3, 1), uniform sampling, constraint=True
(entity rows renormalised every step), SGD lr=0.01, on the FB15k-237 training
graph (272,115 triples, E=14,505, R=237; ids shipped in data/). One "step" =
one call of the fused kge_step (sample -> gather -> score -> loss -> grad ->
clip -> sparse SGD update) on a batch already resident in HBM.

Other legs (``--workload``; one JSON line each, same schema):
  c1         TransE d=50, B=128, K=1, hinge(1), corrupt_side='t' (launch-bound)
  c3         RotatE d=256, B=1024, K=256, SANS(3,1), LpDistance(1)
  c4-rescal  RESCAL d=200, B=512, K=64, SquareError, constraint (dense regulariser)
  c4-transr  TransR d=k=200, B=512, K=64, LpDistancePow(2), hinge(1), constraint (fp32 MFMA)
  c2-50m     the C2 step on a synthetic 50M-entity table (HBM-honest point; SURVEY 8(d) Caveat)
  c5         TransE d=512 on a synthetic 50M-entity / 1000-relation graph with Zipf(1.1) heads /
             tails and Zipf(1.2) relations, entity table row-sharded (e mod N)
             through KGE/sharded.py's sparse all-to-all exchange at every N (N = 1 included)
  c1-train / c2-train
             the C1 / C2 configuration through the reference's entry point KGEModel.train
             (example_fit_from_numpy.py:22-30 call pattern, BaseModel.py:58-190): wall time of
             whole epochs per batch (device input stream, step, per-epoch loss read, histogram,
             checkpoint), next to the same model's bare FusedStep time
  eval       KGEModel.evaluate (BaseModel.py:578-654) of the C2 model on FB15k-237 valid_indexed
             (17,526 triples), filtered by train + valid, corrupt_side 'h' and 't' (kge_rank)

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU, each with its own 1024-positive batch (weak scaling, the
global batch is N*1024). C2's small table is replicated with one gradient
all-reduce per step; C5's is row-sharded with the sparse exchange
(KGE/sharded.py).

Prints ONE JSON line (rank 0). The default C2 line at one GPU also carries
roofline.hbm_point: the same step on a 50M-entity table, measured live
(FB15k-237's table sits in the Infinity Cache; that one cannot).
"""

import argparse
import ctypes
import json
import math
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "knowledge-graph-embedding_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

# The contract is ONE JSON line on stdout, but RCCL prints its banner and
# warnings (e.g. the iommu=pt notice) there: the process's fd 1 goes to stderr
# for the whole run and only the result line is written to the real stdout.
os.environ["NCCL_DEBUG"] = "WARN"
_RESULT_OUT = os.fdopen(os.dup(1), "w")
sys.stdout.flush()
os.dup2(2, 1)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TF = 157.3   # MI355X dense fp32 matrix peak (MI355X_MICROARCH.md)

WORKLOADS = ("c2", "c1", "c3", "c4-rescal", "c4-transr", "c2-50m", "c5", "c1-train", "c2-train", "eval")
F32_VALU_PEAK_TF = 157.3   # MI355X fp32 vector peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=WORKLOADS)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--neg", type=int, default=None)
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hbm-point", action="store_true",
                    help="c2 at one GPU: skip the live C2-50M (HBM-honest) KS measurement in roofline.hbm_point")
    ap.add_argument("--epochs", type=int, default=2, help="c1-train / c2-train: timed epochs (after one warm-up)")
    ap.add_argument("--force-exchange", action="store_true",
                    help="one GPU: run the multi-GPU step (c5: all-to-all exchange + row cache instead of the "
                         "one-rank shortcut; other workloads: the sharded step with its exchange) as a rehearsal")
    ap.add_argument("--exchange", default="auto", choices=("auto", "dense", "sparse", "owner"),
                    help="multi-GPU step (KGE/sharded.py): auto = dense replica up to 1 GiB of entity rows, else "
                         "owner-side scoring (TransE / DistMult / RotatE) or the sparse row exchange")
    ap.add_argument("--loopback", action="store_true",
                    help="with --force-exchange: every id (own ones too) through the exchange blocks -- the "
                         "remote path's kernels and copies on one GPU")
    return ap.parse_args()


def load_graph():
    z = np.load(os.path.join(ROOT, "data", "fb15k237_train.npz"))
    return z["triples"].astype(np.int64), int(z["n_entities"]), int(z["n_relations"])


# ---------------------------------------------------------------- workloads
def spec(name, args):
    """(model ctor kwargs, B, K, d, side, E override) of a workload."""
    from KGE import loss, score
    w = {
        "c2": dict(model="TransE", B=1024, K=256, d=200, side="h+t", constraint=True,
                   score=score.LpDistance(p=2), loss=loss.SelfAdversarialNegativeSamplingLoss(margin=3, temperature=1),
                   desc="C2: TransE d=%(d)d, batch=%(B)d, %(K)d negs h+t, SANS(3,1), LpDistance(2), uniform, "
                        "constraint, SGD"),
        "c1": dict(model="TransE", B=128, K=1, d=50, side="t", constraint=True, score=score.LpDistance(p=2),
                   loss=loss.PairwiseHingeLoss(margin=1),
                   desc="C1: TransE d=%(d)d, batch=%(B)d, %(K)d neg/pos corrupt_side='t', hinge(1), LpDistance(2), "
                        "uniform, constraint, SGD"),
        "c3": dict(model="RotatE", B=1024, K=256, d=256, side="h+t", constraint=False, score=score.LpDistance(p=1),
                   loss=loss.SelfAdversarialNegativeSamplingLoss(margin=3, temperature=1),
                   desc="C3: RotatE d=%(d)d (complex), batch=%(B)d, %(K)d negs h+t, SANS(3,1), LpDistance(1), "
                        "uniform, SGD"),
        "c4-rescal": dict(model="RESCAL", B=512, K=64, d=200, side="h+t", constraint=True, score=None,
                          loss=loss.SquareErrorLoss(),
                          desc="C4: RESCAL d=%(d)d, batch=%(B)d, %(K)d negs h+t, SquareError, constraint "
                               "(dense Lp regulariser), uniform, SGD"),
        "c4-transr": dict(model="TransR", B=512, K=64, d=200, side="h+t", constraint=True,
                          score=score.LpDistancePow(p=2), loss=loss.PairwiseHingeLoss(margin=1),
                          desc="C4: TransR d=k=%(d)d, batch=%(B)d, %(K)d negs h+t, LpDistancePow(2), hinge(1), "
                               "constraint (clip), uniform, SGD"),
        "c2-50m": dict(model="TransE", B=1024, K=256, d=200, side="h+t", constraint=False,
                       score=score.LpDistance(p=2),
                       loss=loss.SelfAdversarialNegativeSamplingLoss(margin=3, temperature=1), E=50_000_000,
                       desc="C2 step on a synthetic %(E)d-entity table: TransE d=%(d)d, batch=%(B)d, %(K)d negs h+t, "
                            "SANS(3,1), LpDistance(2), uniform ids, no constraint (a full-table renormalisation "
                            "would be an 80 GB pass per step), SGD"),
        "c5": dict(model="TransE", B=1024, K=256, d=512, side="h+t", constraint=False,
                   score=score.LpDistance(p=2),
                   loss=loss.SelfAdversarialNegativeSamplingLoss(margin=3, temperature=1), E=50_000_000, R=1000,
                   zipf=True, sharded=True,
                   desc="C5: TransE d=%(d)d on a synthetic %(E)d-entity graph (Zipf(1.1) heads/tails, Zipf(1.2) "
                        "relations, R=1000), batch=%(B)d per GPU, %(K)d negs h+t, SANS(3,1), LpDistance(2), "
                        "uniform negatives, no constraint, SGD; entity rows sharded e mod N, sparse all-to-all "
                        "exchange"),
    }[name]
    if args.batch:
        w["B"] = args.batch
    if args.neg is not None:
        w["K"] = args.neg
    if args.dim:
        w["d"] = args.dim
    return w


def zipf_ids(n, N, s, g, dev):
    """Truncated power-law ranks k in [1, N] (inverse CDF of the continuous
    Zipf(s) density) mapped through the bijection k -> (a (k-1) + b) mod N,
    a coprime to N: heavy hitters scattered over the id space."""
    u = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    k = torch.pow(1.0 + u * (float(N) ** (1.0 - s) - 1.0), 1.0 / (1.0 - s)).floor().clamp_(1, N).to(torch.int64)
    a = 2654435761
    while np.gcd(a, N) != 1:
        a += 2
    return (a * (k - 1) + 40503) % N


def build_model(w, E, R, rank, dev):
    from KGE import optimizers
    from KGE.models.semantic_based.RESCAL import RESCAL
    from KGE.models.translating_based.RotatE import RotatE
    from KGE.models.translating_based.TransE import TransE
    from KGE.models.translating_based.TransR import TransR
    from KGE.ns_strategy import UniformStrategy
    d, K = w["d"], w["K"]
    ns = UniformStrategy(np.arange(E), seed=12345 + rank)   # range(E): no device pool
    kw = dict(loss_fn=w["loss"], ns_strategy=ns)
    if w["model"] == "TransE":
        m = TransE({"embedding_size": d}, K, w["side"], score_fn=w["score"], constraint=w["constraint"], **kw)
    elif w["model"] == "RotatE":
        m = RotatE({"embedding_size": d}, K, w["side"], score_fn=w["score"], **kw)
    elif w["model"] == "RESCAL":
        m = RESCAL({"embedding_size": d}, K, w["side"], constraint=w["constraint"], **kw)
    else:
        m = TransR({"ent_embedding_size": d, "rel_embedding_size": d}, K, w["side"], score_fn=w["score"],
                   constraint=w["constraint"], **kw)
    m.metadata = {"ind2ent": range(E), "ind2rel": range(R)}
    m._model_weights_initial = None
    if E > 10_000_000:
        # the reference initialiser, drawn on the device (a host draw of 40 GB would dominate)
        g = torch.Generator(device=dev).manual_seed(12345)
        lim = 6.0 / np.sqrt(d)
        # (in place: no second E x d temporary -- C5's table is a third of HBM)
        m.model_weights = {"ent_emb": torch.rand((E, d), generator=g, device=dev).mul_(2).sub_(1).mul_(lim),
                           "rel_emb": torch.rand((R, d), generator=g, device=dev).mul_(2).sub_(1).mul_(lim)}
    else:
        m._init_embeddings(seed=12345)          # identical init on every rank
        m._to_device()
    return m, optimizers.SGD(learning_rate=0.01)


# ---------------------------------------------------------------- accounting
def transe_bytes(B, K, d, E):
    """1 read + 1 write of every touched row occurrence."""
    step = 4 * d * (6 * B + 2 * B * K) + 12 * B
    score = 4 * d * (3 * B + B * K) + 12 * B          # KS: positive rows + one sampled row per negative
    update = 4 * d * (3 * B + B * K)                   # KU: the write-back half
    constrain = 2 * 4 * E * d                          # K0: full-table renormalisation
    return step, score, update, constrain


def transe_update_bytes(B, K, d, E, batch, fused):
    """What KU actually moves: every row it rewrites read and
    written once -- all E entity rows when the constraint is fused (each is
    renormalised), else the distinct touched rows (the batch's own entities
    plus the expected distinct uniform draws) -- plus the batch's distinct
    relation rows; and, served from L2, one context row (snapshot / own-row
    gradient) + coefficient + list entry per key."""
    ents = torch.unique(torch.cat([batch[:, 0], batch[:, 2]])).numel()
    rels = torch.unique(batch[:, 1]).numel()
    keys = B * K + 3 * B
    if fused:
        ent_rows = E
    else:
        ent_rows = ents + (E - ents) * (1.0 - math.exp(-B * K / E))
    rows = 8 * d * (ent_rows + rels)
    context = 4 * d * keys + 12 * B * K + 4 * 3 * B
    return int(rows), int(context)


def accounting(w, B, K, d, E, R, batch):
    """Algorithmic work per step / per dominant-kernel launch."""
    m = w["model"]
    if m == "TransE":
        step, score, upd, con = transe_bytes(B, K, d, E)
        rows, context = transe_update_bytes(B, K, d, E, batch, w["constraint"])
        # update_kernel against HBM: the rows it rewrites; its per-key context
        # rows / coefficients / list entries (L2-resident, written by the score
        # kernel just before) are reported beside it, not counted as HBM bytes
        return {"bound": "hbm", "step": step, "kernels": {"score_kernel": score, "update_kernel": rows},
                "update_split": {"rows_bytes": rows, "context_bytes": context}}
    if m == "RotatE":
        # entity rows 2d floats (8d bytes), relation rows d phases (4d bytes)
        read = B * (2 * 8 * d + 4 * d) + B * K * 8 * d + 12 * B
        return {"bound": "hbm", "step": 2 * read - 12 * B, "kernels": {"score_kernel": read,
                                                                        "update_kernel": read - 12 * B}}
    if m == "RESCAL":
        ur = int(torch.unique(batch[:, 1]).numel())
        sparse = 2 * (4 * d * (2 * B + B * K) + 4 * d * d * ur)
        dense = 2 * 4 * (E * d + R * d * d)
        # score_kernel: the positives' rows, one row per negative, the ids,
        # and every live relation's R_r once (the in-kernel context / post
        # products u = R^T h, v = R t, R A, R^T B; repeats are cache hits)
        return {"bound": "hbm", "step": sparse + dense, "distinct_relations": ur,
                "kernels": {"score_kernel": 4 * d * (3 * B + B * K) + 12 * B + 4 * d * d * ur}}
    # TransR: three products per positive: P = X M (K+2 rows), S M^T (2K+4
    # slice rows: every slice's ||M g||^2 is a clip_by_norm term), X^T S' (K+2)
    flops = 2.0 * d * d * (4 * K + 8) * B
    return {"bound": "mfma", "step_flops": flops, "kernels": {"transr2_kernel": flops},
            "survey_flops": 6.0 * d * d * (K + 2) * B}


def hbm_point(args, dev, R):
    """roofline.hbm_point: the C2 step on a 50M-entity table (SURVEY 8(d)
    Caveat: FB15k-237's 11.6 MB table lives in the Infinity Cache, a 40 GB one
    cannot), measured live: 30 timed steps, then 30 with HIP events on the
    step's stream for the KS / KU split."""
    from KGE import engine
    w = spec("c2-50m", args)
    E, B, K, d = w["E"], w["B"], w["K"], w["d"]
    model, opt = build_model(w, E, R, 0, dev)
    step = engine.FusedStep(model)
    g = torch.Generator(device=dev).manual_seed(2000)
    n_w, n_t = 5, 30
    batches = torch.stack([torch.randint(0, E, (n_w + n_t, B), generator=g, device=dev),
                           torch.randint(0, R, (n_w + n_t, B), generator=g, device=dev),
                           torch.randint(0, E, (n_w + n_t, B), generator=g, device=dev)], -1)
    for s_ in range(n_w):
        step(batches[s_], True, opt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s_ in range(n_t):
        step(batches[n_w + s_], True, opt)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n_t
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(n_t)]
    for row in evs:
        for e in row:
            e.record()
    torch.cuda.synchronize()
    handles = [(ctypes.c_void_p * 4)(*[e.cuda_event for e in row]) for row in evs]
    for s_ in range(n_t):
        step(batches[n_w + s_], True, opt, prof_events=handles[s_])
    torch.cuda.synchronize()
    step.check_status()
    ks = float(np.mean([r[1].elapsed_time(r[2]) for r in evs]))
    ku = float(np.mean([r[2].elapsed_time(r[3]) for r in evs]))
    acc = accounting(w, B, K, d, E, R, batches[n_w])
    # HBM-honest rates: KU's context rows are re-read from L2 (rows_bytes only)
    rows = acc["update_split"]["rows_bytes"] / (ku * 1e-3) / 1e9
    ach = {"score_kernel": acc["kernels"]["score_kernel"] / (ks * 1e-3) / 1e9, "update_kernel": rows}
    dom = "update_kernel" if ku > ks else "score_kernel"   # the longer launch of the step
    out = {"workload": "c2-50m: " + w["desc"] % dict(B=B, K=K, d=d, E=E), "ms_per_step": round(ms, 5),
           "kernel": dom, "achieved": round(ach[dom], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach[dom] / HBM_PEAK_GBS, 4), "score_kernel_ms": round(ks, 5), "update_kernel_ms": round(ku, 5),
           "score_kernel_GBps": round(ach["score_kernel"], 1), "update_kernel_GBps": round(ach["update_kernel"], 1),
           "update_rows_GBps": round(rows, 1),
           "step_GBps": round((acc["kernels"]["score_kernel"] + acc["update_split"]["rows_bytes"]) / (ms * 1e-3) / 1e9, 1)}
    pmc = pmc_traffic("c2-50m")
    out["traffic"] = pmc["kernels"][dom].get("hbm_bytes_per_launch") \
        if pmc and dom in pmc.get("kernels", {}) else None
    out["traffic_source"] = pmc["_source"] if out["traffic"] is not None else None
    del step, model, batches
    torch.cuda.empty_cache()
    return out


def copy_peak(dev, gib=2.0, reps=20):
    """The box's HBM copy rate (the measured peak as a second
    denominator): kge_copy16 (a float4 streaming copy, csrc/kge_stream.hip)
    of a 2 GiB buffer into another -- 16x the Infinity Cache, so every byte
    comes from and goes to HBM -- timed with HIP events on the stream it
    runs on; read + write bytes over the mean of 20 copies."""
    from KGE import _hip
    lib = _hip.lib()
    n = int(gib * (1 << 30)) // 4
    src = torch.ones(n, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    st = _hip.stream_handle(dev)
    for _ in range(3):
        _hip.check(lib.kge_copy16(src.data_ptr(), dst.data_ptr(), n // 4, st), "kge_copy16")
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        _hip.check(lib.kge_copy16(src.data_ptr(), dst.data_ptr(), n // 4, st), "kge_copy16")
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / reps
    assert bool(torch.equal(src[-4:], dst[-4:]))
    del src, dst
    torch.cuda.empty_cache()
    return {"GBps": round(2 * n * 4 / (ms * 1e-3) / 1e9, 1), "ms_per_copy": round(ms, 4),
            "method": "kge_copy16 float4 copy, %.0f GiB -> %.0f GiB, %d copies, read + write bytes" % (gib, gib, reps)}


# ---------------------------------------------------------------- CPU baseline
def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def host_cores():
    """Every core this process may use (torch.set_num_threads over
    all of them): the affinity mask, capped by the cgroup's CPU quota (the
    GPU box: 256 CPUs in the mask, cpu.max "1600000 100000" = 16 CPUs of
    time -- more threads than that only get throttled). OMP_NUM_THREADS is
    recorded beside it, not obeyed."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cgroup_cpu_max()
    if q:
        quota, _, period = q.partition(" ")
        if quota.isdigit() and period.isdigit() and int(period) > 0:
            n = min(n, max(1, int(quota) // int(period)))
    return n


def cgroup_cpu_max():
    """The cgroup v2 CPU quota ("max 100000" = unlimited), if readable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            return f.read().strip()
    except OSError:
        return None


def cpu_baseline(triples, E, R, B, K, d, budget_s):
    """Time the CPU restatement (oracle, fp32 torch autograd on the host) on a
    bounded sample: whole C2 steps until ~budget_s seconds of CPU work, with
    every core, then a shorter single-thread sample."""
    from oracle import kge_oracle as orc
    threads = host_cores()
    rng = np.random.default_rng(0)

    def run(nthreads, budget):
        torch.set_num_threads(nthreads)
        W = {"ent_emb": rng.uniform(-6 / np.sqrt(d), 6 / np.sqrt(d), (E, d)).astype(np.float32),
             "rel_emb": rng.uniform(-6 / np.sqrt(d), 6 / np.sqrt(d), (R, d)).astype(np.float32)}
        n, t_total = 0, 0.0
        while t_total < budget:
            pos = triples[rng.integers(0, len(triples), B)]
            neg = orc.uniform_negatives(pos, K, "h+t", E, seed=12345, plane=2 * n)
            t0 = time.perf_counter()
            out = orc.train_step("TransE", W, pos, neg, score=("lp", 2.0), loss=("sans", 3.0, 1.0), lr=0.01,
                                 constraint=True, dtype=torch.float32)
            t_total += time.perf_counter() - t0
            W = {k: v.astype(np.float32) for k, v in out["weights"].items()}
            n += 1
        return n, t_total

    n, t = run(threads, budget_s)
    n1, t1 = run(1, max(budget_s / 3, 3.0))
    torch.set_num_threads(threads)
    return {"value": n * B / t, "unit": "positive-triples/s", "cores": threads, "kind": "port",
            "single_thread_value": n1 * B / t1, "cpu_model": cpu_model(), "nproc": threads,
            "cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "env_omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cgroup_cpu_max": cgroup_cpu_max(),
            "sample": "%d whole C2 steps (B=%d, K=%d, d=%d, FB15k-237) of the fp32 torch-CPU restatement "
                      "(oracle/kge_oracle.py) on %d threads, %.1f s; single thread: %d steps, %.1f s"
                      % (n, B, K, d, threads, t, n1, t1)}


def _round_key(name):
    """profiles/ run directories in build order: r05b < r05z < r05aa < r06."""
    import re
    m = re.match(r"r(\d+)([a-z]*)$", name)
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else None


def pmc_traffic(workload):
    """HBM bytes per launch of the leg's kernels from the newest committed
    rocprofv3 --pmc summary, profiles/<run>/pmc_traffic_<workload>.json
    (tools/pmc_traffic.py; <run> = r<round><suffix>, newest by round then
    suffix), or None. NOT measured in this run: the counters need their own
    rocprofv3 --pmc pass; the line names the file (``traffic_source``)."""
    pdir = os.path.join(ROOT, "profiles")
    name = "pmc_traffic_%s.json" % workload
    try:
        runs = sorted((d for d in os.listdir(pdir) if _round_key(d) and os.path.exists(os.path.join(pdir, d, name))),
                      key=_round_key)
    except OSError:
        return None
    if not runs:
        return None
    rel = "profiles/%s/%s" % (runs[-1], name)
    try:
        with open(os.path.join(ROOT, rel)) as f:
            out = json.load(f)
    except (OSError, ValueError):
        return None
    out["_source"] = "%s (rocprofv3 --pmc, committed; not this run)" % rel
    return out


# ---------------------------------------------------------------- entry-point legs
def _emit(out):
    _RESULT_OUT.write(json.dumps(out) + "\n")
    _RESULT_OUT.flush()


def train_leg(args, dev):
    """c1-train / c2-train: KGEModel.train as the reference's example calls it
    (example_fit_from_numpy.py:22-30: index -> Model(...).train(train_X, ...,
    epochs, batch_size, optimizer, seed)), on FB15k-237 train_indexed with
    metadata ind2ent = range(E). One warm-up train() call of
    one epoch, then one timed call of --epochs epochs; ms_per_step = its wall
    time / batches. A second call of 2 x --epochs gives the marginal per-batch
    cost (the difference) and the one-off cost. The same model's bare
    FusedStep is timed after it."""
    import tempfile
    from KGE import engine, optimizers
    from KGE.models.translating_based.TransE import TransE
    from KGE.ns_strategy import UniformStrategy
    base = args.workload.split("-")[0]
    w = spec(base, args)
    triples, E, R = load_graph()
    B, K, d = w["B"], w["K"], w["d"]
    meta = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    model = TransE({"embedding_size": d}, K, w["side"], score_fn=w["score"], loss_fn=w["loss"],
                   ns_strategy=UniformStrategy, constraint=w["constraint"])
    per_epoch = {"histogram": 0.0, "checkpoint": 0.0, "batch_host": 0.0, "epoch_host": 0.0, "prepare": 0.0}

    def timed(name, fn):
        def run(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            per_epoch[name] += time.perf_counter() - t
            return r
        return run
    model._histogram_stats = timed("histogram", model._histogram_stats)     # (device statistics, issued)
    model._finish_epoch = timed("epoch_host", model._finish_epoch)          # (host reads, logs, files)
    model._prepare_for_train = timed("prepare", model._prepare_for_train)   # (init, iterators, sampler)
    model._save_checkpoint = timed("checkpoint", model._save_checkpoint)
    # host time spent issuing each batch (no sync inside: the GPU runs behind)
    model._run_single_batch = timed("batch_host", model._run_single_batch)
    nb = int(math.ceil(len(triples) / B))
    with tempfile.TemporaryDirectory() as logdir:
        model.train(train_X=triples, val_X=None, metadata=meta, epochs=1, batch_size=B,
                    optimizer=optimizers.SGD(0.01), seed=12345, log_path=logdir)
        torch.cuda.synchronize()
        for k in per_epoch:
            per_epoch[k] = 0.0
        t0 = time.perf_counter()
        model.train(train_X=triples, val_X=None, metadata=meta, epochs=args.epochs, batch_size=B,
                    optimizer=optimizers.SGD(0.01), seed=12345, log_path=logdir)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        # the same call at twice the epochs: the difference is the per-batch cost
        # of a longer run (each epoch's histograms, checkpoint and logs included),
        # the rest one-off (prepare, init, first bind, the last checkpoint's write)
        t0 = time.perf_counter()
        model.train(train_X=triples, val_X=None, metadata=meta, epochs=2 * args.epochs, batch_size=B,
                    optimizer=optimizers.SGD(0.01), seed=12345, log_path=logdir)
        torch.cuda.synchronize()
        wall2 = time.perf_counter() - t0
    steps = args.epochs * nb
    marginal_ms = (wall2 - wall) * 1e3 / steps
    ms = wall * 1e3 / steps
    # the bare fused step of the same model on the same batches (the c1 / c2 legs' number)
    step = engine.FusedStep(model)
    opt = optimizers.SGD(0.01)
    g = torch.Generator().manual_seed(7)
    idx = torch.randint(0, len(triples), (220, B), generator=g)
    batches = torch.from_numpy(triples)[idx].to(dev)
    for s in range(20):
        step(batches[s], True, opt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(20, 220):
        step(batches[s], True, opt)
    torch.cuda.synchronize()
    fused_ms = (time.perf_counter() - t0) * 1e3 / 200
    ep_total = 3 * args.epochs   # (the per_epoch sums cover both timed calls)
    hist_ms = per_epoch["histogram"] * 1e3 / ep_total
    ckpt_ms = per_epoch["checkpoint"] * 1e3 / ep_total
    ephost_ms = per_epoch["epoch_host"] * 1e3 / ep_total
    _emit({"metric": "positive-triples/sec through KGEModel.train (wall, whole epochs) at d=%d, FB15k-237" % d,
           "value": round(B / (ms * 1e-3), 1), "unit": "positive-triples/s", "n_gpus": 1, "steps": steps,
           "warmup": nb, "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f32", "data": "FB15k-237 train_indexed (real graph), reference init",
           "config": {"workload": "%s through KGEModel.train: %s" % (base.upper(), w["desc"] % dict(B=B, K=K, d=d)),
                      "epochs": args.epochs, "batches_per_epoch": nb, "global_batch": B, "negatives": K, "dim": d,
                      "parallelism": "dp1"},
           "train_entry": {"ms_per_batch_wall": round(ms, 5),
                           "ms_per_batch_marginal": round(marginal_ms, 5),
                           "one_off_ms": round(wall * 1e3 - marginal_ms * steps, 3),
                           "host_issue_ms_per_batch": round(per_epoch["batch_host"] * 1e3 / (3 * steps), 5),
                           "fused_step_ms": round(fused_ms, 5),
                           "per_epoch_ms": {"histogram_issue": round(hist_ms, 3), "checkpoint_issue": round(ckpt_ms, 3),
                                            "epoch_host_incl_gpu_wait": round(ephost_ms, 3)},
                           "prepare_ms": round(per_epoch["prepare"] * 1e3 / 2, 3)},
           "roofline": None, "cpu_baseline": None})


def eval_leg(args, dev):
    """eval: KGEModel.evaluate (BaseModel.py:578-618, get_rank :620-654) of the
    C2 TransE model (reference init, d=200) on FB15k-237 valid_indexed, the
    filter = train + valid positives; both corrupt sides, whole set per call
    (kge_rank). Roofline: rank_count_kernel is VALU-bound (3 flops per
    candidate element: subtract, fused square-accumulate) -- n x E x d x 3
    flops per side against the fp32 vector peak."""
    from KGE import ranking
    from KGE.models.translating_based.TransE import TransE
    from KGE.ns_strategy import UniformStrategy
    w = spec("c2", args)
    triples, E, R = load_graph()
    V = np.load(os.path.join(ROOT, "data", "fb15k237_valid.npz"))["triples"].astype(np.int64)
    d = w["d"]
    model = TransE({"embedding_size": d}, w["K"], w["side"], score_fn=w["score"], loss_fn=w["loss"],
                   ns_strategy=UniformStrategy(np.arange(E), seed=1), constraint=w["constraint"])
    model.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    model._model_weights_initial = None
    model._init_embeddings(seed=12345)
    model._to_device()
    assert ranking.supported(model)
    P = np.concatenate([triples.astype(np.int64), V])
    model.evaluate(V[:512], "t", P)       # warm-up (library load, kernels)
    torch.cuda.synchronize()
    sides = {}
    for side in ("h", "t"):
        t0 = time.perf_counter()
        res = model.evaluate(V, side, P)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        ranking.batched_ranks(model, V, side, P)
        ev[1].record()
        torch.cuda.synchronize()
        sides[side] = {"evaluate_s": round(wall, 5), "device_ms": round(ev[0].elapsed_time(ev[1]), 4),
                       "mrr": round(res["mean_reciprocal_rank"], 6), "hit@10": round(res["hit@10"], 6)}
    n = len(V)
    tot = sides["h"]["evaluate_s"] + sides["t"]["evaluate_s"]
    dev_ms = sides["h"]["device_ms"] + sides["t"]["device_ms"]
    flops = 2 * n * E * d * 3.0
    cpu = None
    if not args.no_cpu_baseline:
        # the reference's per-triple get_rank loop restated on the host (torch CPU, same model)
        cm = TransE({"embedding_size": d}, w["K"], w["side"], score_fn=w["score"], loss_fn=w["loss"],
                    ns_strategy=UniformStrategy(np.arange(E), seed=1), constraint=w["constraint"])
        cm.metadata = model.metadata
        cm.model_weights = {k: v.detach().cpu() for k, v in model.model_weights.items()}
        threads = host_cores()
        torch.set_num_threads(threads)
        k, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < min(args.cpu_seconds, 10.0):
            cm.get_rank(V[k % n], P, "t")
            k += 1
        cpu = {"value": k / (time.perf_counter() - t0), "unit": "ranked-triples/s", "cores": threads,
               "kind": "port", "sample": "%d triples of FB15k-237 valid through the per-triple get_rank loop "
                                         "(BaseModel.py:620-654 restated, torch CPU), filtered, side 't'" % k}
    _emit({"metric": "filtered ranked triples/sec (KGEModel.evaluate, both sides) at d=%d, FB15k-237 valid" % d,
           "value": round(2 * n / tot, 1), "unit": "ranked-triples/s", "n_gpus": 1, "steps": 2, "warmup": 1,
           "ms_per_step": round(tot * 1e3 / 2, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f32",
           "data": "FB15k-237 valid_indexed (%d triples), filter train + valid; reference-init weights" % n,
           "config": {"workload": "evaluate(): TransE d=%d LpDistance(2), E=%d candidates per query, both sides"
                                  % (d, E), "sides": sides, "parallelism": "dp1"},
           "roofline": {"bound": "valu", "kernel": "rank_count_kernel (+ pos / filter passes)",
                        "achieved": round(flops / (dev_ms * 1e-3) / 1e12, 2), "peak": F32_VALU_PEAK_TF,
                        "unit": "TFLOP/s", "frac": round(flops / (dev_ms * 1e-3) / 1e12 / F32_VALU_PEAK_TF, 4),
                        "flops": flops, "traffic": None},
           "cpu_baseline": cpu})


# ---------------------------------------------------------------- main
def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # KGE_BENCH_BACKEND=gloo: a rehearsal of the N-rank path on fewer GPUs
    # (ranks share devices, tensors staged through the host; timings are not
    # the xGMI numbers) -- the driver's runs use RCCL ("nccl")
    backend = os.environ.get("KGE_BENCH_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local % ndev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local % ndev))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)

    from KGE import _hip, engine
    _hip.load()   # the shipped gfx950 library; raises if missing
    if args.workload in ("c1-train", "c2-train"):
        return train_leg(args, dev)
    if args.workload == "eval":
        return eval_leg(args, dev)

    w = spec(args.workload, args)
    triples, E, R = load_graph()
    synthetic = "E" in w
    if synthetic:
        E = w["E"]
        R = w.get("R", R)
    B, K, d = w["B"], w["K"], w["d"]
    sharded = world > 1 or w.get("sharded", False) or args.force_exchange
    if sharded and world == 1:
        # one-rank process group: the same sharded step (and its exchange) as at N > 1
        import tempfile
        import torch.distributed as dist
        store = os.path.join(tempfile.mkdtemp(prefix="kge_pg_"), "store")   # file store: no port to race for
        dist.init_process_group("nccl", init_method="file://" + store, rank=0, world_size=1, device_id=dev)
    model, opt = build_model(w, E, R, rank, dev)
    if sharded:
        from KGE.sharded import ShardedStep
        step = ShardedStep(model, mode=args.exchange, local_fast=not args.force_exchange, loopback=args.loopback,
                           batch_hint=B, optimizer=opt)
        if E > 10_000_000:
            step.release_entity_tables()   # the shard is the only copy the step needs
    else:
        step = engine.FusedStep(model)

    # batches resident in HBM before timing: a shuffled stream per rank
    nb = args.warmup + args.steps
    if w.get("zipf"):
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        batches = torch.stack([zipf_ids(nb * B, E, 1.1, g, dev), zipf_ids(nb * B, R, 1.2, g, dev),
                               zipf_ids(nb * B, E, 1.1, g, dev)], -1).reshape(nb, B, 3).contiguous()
    elif synthetic:
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        batches = torch.stack([torch.randint(0, E, (nb, B), generator=g, device=dev),
                               torch.randint(0, R, (nb, B), generator=g, device=dev),
                               torch.randint(0, E, (nb, B), generator=g, device=dev)], -1)
    else:
        g = torch.Generator().manual_seed(1000 + rank)
        idx = torch.cat([torch.randperm(len(triples), generator=g) for _ in range((nb * B) // len(triples) + 1)])
        batches = torch.from_numpy(triples)[idx[:nb * B]].reshape(nb, B, 3).to(dev)

    for s in range(args.warmup):
        step(batches[s], True, opt)
    torch.cuda.synchronize()
    step.check_status()

    # timed region: exactly K steps, nothing else on the stream
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(batches[args.warmup + s], True, opt)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    step.check_status()
    ms = (t1 - t0) * 1e3 / args.steps

    # per-kernel breakdown: a second pass over the same batches with HIP events
    # recorded on the step's own stream [before K0, before KS, after KS, after
    # the update kernels]; the events cost a few us per step, so this pass
    # never feeds `value`
    n_prof = min(args.steps, 100)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(n_prof)]
    for row in evs:
        for e in row:
            e.record()
    torch.cuda.synchronize()
    handles = [(ctypes.c_void_p * 4)(*[e.cuda_event for e in row]) for row in evs]
    for s in range(n_prof):
        step(batches[args.warmup + s], True, opt, prof_events=handles[s])
    torch.cuda.synchronize()
    step.check_status()
    k0 = float(np.mean([r[0].elapsed_time(r[1]) for r in evs]))
    ks = float(np.mean([r[1].elapsed_time(r[2]) for r in evs]))
    ku = float(np.mean([r[2].elapsed_time(r[3]) for r in evs]))
    if sharded:
        t = torch.tensor([ms], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        ms = float(t.item())
    if rank != 0:
        torch.distributed.destroy_process_group()
        return

    acc = accounting(w, B, K, d, E, R, batches[args.warmup])
    names = list(acc["kernels"])
    # event groups: KS group = the score pass (+ context / rank passes);
    # KU group = update + apply passes
    group_ms = {names[0]: ks}
    if len(names) > 1:
        group_ms[names[1]] = ku
    if acc["bound"] == "hbm":
        kern = {k: {"ms": round(group_ms[k], 5), "GBps": round(acc["kernels"][k] / (group_ms[k] * 1e-3) / 1e9, 1)}
                for k in group_ms}
        dom = max(group_ms, key=group_ms.get)   # the longer launch (group) of the step
        ach = acc["kernels"][dom] / (group_ms[dom] * 1e-3) / 1e9
        pmc = pmc_traffic(args.workload)
        traffic = None
        if pmc and dom in pmc.get("kernels", {}):
            traffic = pmc["kernels"][dom].get("hbm_bytes_per_launch")
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": pmc["_source"] if traffic is not None else None,
                "step": {"alg_bytes": acc["step"], "ms_per_step": round(ms, 5),
                         "achieved": round(acc["step"] / (ms * 1e-3) / 1e9, 1),
                         "frac": round(acc["step"] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
                "kernels": kern}
        if "distinct_relations" in acc:
            roof["distinct_relations"] = acc["distinct_relations"]
        if "update_split" in acc and "update_kernel" in kern:
            ku_s = group_ms["update_kernel"] * 1e-3
            kern["update_kernel"].update({k: v for k, v in acc["update_split"].items()})
            kern["update_kernel"]["GBps_rows"] = round(acc["update_split"]["rows_bytes"] / ku_s / 1e9, 1)
            kern["update_kernel"]["GBps_context_l2"] = round(acc["update_split"]["context_bytes"] / ku_s / 1e9, 1)
    else:
        dom = names[0]
        tf = acc["kernels"][dom] / (ks * 1e-3) / 1e12
        pmc = pmc_traffic(args.workload)
        traffic = (pmc or {}).get("kernels", {}).get(dom, {}).get("hbm_bytes_per_launch")
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(tf, 2), "peak": F32_MFMA_PEAK_TF,
                "unit": "TFLOP/s", "frac": round(tf / F32_MFMA_PEAK_TF, 4), "traffic": traffic,
                "traffic_source": pmc["_source"] if traffic is not None else None,
                "flops_per_launch": acc["kernels"][dom], "survey_flops_per_step": acc["survey_flops"],
                "step": {"ms_per_step": round(ms, 5), "achieved": round(acc["step_flops"] / (ms * 1e-3) / 1e12, 2)},
                "kernels": {dom: {"ms": round(ks, 5)}, "update+apply": {"ms": round(ku, 5)},
                            "constraint": {"ms": round(k0, 5)}}}
    if acc["bound"] == "hbm":
        # the measured copy peak beside the 8 TB/s spec
        cp = copy_peak(dev)
        roof["peak_measured"] = cp["GBps"]
        roof["frac_measured"] = round(roof["achieved"] / cp["GBps"], 4)
        roof["peak_measured_method"] = cp["method"]
        roof["step"]["frac_measured"] = round(roof["step"]["achieved"] / cp["GBps"], 4)
    if world == 1 and args.workload == "c2" and not args.force_exchange and not args.no_hbm_point \
            and acc["bound"] == "hbm":
        roof["hbm_point"] = hbm_point(args, dev, R)
        roof["hbm_point"]["frac_measured"] = round(roof["hbm_point"]["achieved"] / roof["peak_measured"], 4)
    cpu = None
    if world == 1 and args.workload == "c2" and not args.no_cpu_baseline:
        cpu = cpu_baseline(triples, E, R, B, K, d, args.cpu_seconds)
    value = world * B / (ms * 1e-3)
    out = {
        "metric": "positive-triples/sec (batch x neg scored) at d=%d, %s" % (d, "FB15k-237" if not synthetic else
                                                                              "synthetic %d entities" % E),
        "value": round(value, 1), "unit": "positive-triples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": ("synthetic %s ids over %d entities / %d relations; random-init weights"
                 % ("Zipf" if w.get("zipf") else "uniform", E, R)) if synthetic
        else "FB15k-237 train_indexed ids (real graph); random-init weights",
        "config": {"workload": w["desc"] % dict(B=B, K=K, d=d, E=E), "global_batch": world * B,
                   "negatives": K, "dim": d, "parallelism": "dp%d" % world,
                   "scored_triples_per_s": round(value * (1 + K), 1)},
        "roofline": roof, "cpu_baseline": cpu,
    }
    if sharded:
        out["config"]["exchange"] = "local (one rank: fused step on the shard)" if step.direct is not None \
            else step.mode + (" (loopback: every id through the blocks)" if args.loopback else "")
    _RESULT_OUT.write(json.dumps(out) + "\n")
    _RESULT_OUT.flush()
    if sharded:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
