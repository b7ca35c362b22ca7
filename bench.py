"""bench.py -- KGE training-step throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): TransE, d=200,
batch 1024 positives x 256 negatives ('h+t'), LpDistance(2),
SelfAdversarialNegativeSamplingLoss(3, 1), uniform sampling, constraint=True
(entity rows renormalised every step), SGD lr=0.01, on the FB15k-237 training
graph (272,115 triples, E=14,505, R=237; ids shipped in data/). One "step" =
one call of the fused kge_step (sample -> gather -> score -> loss -> grad ->
clip -> sparse SGD update) on a batch already resident in HBM.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU, each with its own 1024-positive batch (weak scaling, the
global batch is N*1024); the entity table is row-sharded across the ranks
(KGE/sharded.py: all-gather of the shards, fused gradient step, RCCL
reduce-scatter of the entity gradient + all-reduce of the relation gradient,
global clip norm and loss, sharded SGD apply).

Prints ONE JSON line (rank 0).
"""

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "knowledge-graph-embedding_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--neg", type=int, default=256)
    ap.add_argument("--dim", type=int, default=200)
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def load_graph():
    z = np.load(os.path.join(ROOT, "data", "fb15k237_train.npz"))
    return z["triples"].astype(np.int64), int(z["n_entities"]), int(z["n_relations"])


def algorithmic_bytes(B, K, d, E):
    """1 read + 1 write of every touched row occurrence."""
    step = 4 * d * (6 * B + 2 * B * K) + 12 * B
    score = 4 * d * (3 * B + B * K) + 12 * B          # KS: positive rows + one sampled row per negative
    update = 4 * d * (3 * B + B * K)                   # KU: the write-back half
    constrain = 2 * 4 * E * d                          # K0: full-table renormalisation
    return step, score, update, constrain


def cpu_baseline(triples, E, R, B, K, d, budget_s):
    """Time the CPU restatement (oracle, fp32 torch autograd on the host) on a
    bounded sample: whole C2 steps until ~budget_s seconds of CPU work."""
    from oracle import kge_oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    threads = min(threads, os.cpu_count() or threads)
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    W = {"ent_emb": rng.uniform(-6 / np.sqrt(d), 6 / np.sqrt(d), (E, d)).astype(np.float32),
         "rel_emb": rng.uniform(-6 / np.sqrt(d), 6 / np.sqrt(d), (R, d)).astype(np.float32)}
    n, t_total = 0, 0.0
    while t_total < budget_s:
        pos = triples[rng.integers(0, len(triples), B)]
        neg = orc.uniform_negatives(pos, K, "h+t", E, seed=12345, plane=2 * n)
        t0 = time.perf_counter()
        out = orc.train_step("TransE", W, pos, neg, score=("lp", 2.0), loss=("sans", 3.0, 1.0), lr=0.01,
                             constraint=True, dtype=torch.float32)
        t_total += time.perf_counter() - t0
        W = {k: v.astype(np.float32) for k, v in out["weights"].items()}
        n += 1
        if n >= 1 and t_total > budget_s:
            break
    return {"value": n * B / t_total, "unit": "positive-triples/s", "cores": threads, "kind": "port",
            "sample": "%d whole C2 steps (B=%d, K=%d, d=%d, FB15k-237) of the fp32 torch-CPU restatement "
                      "(oracle/kge_oracle.py), %.1f s" % (n, B, K, d, t_total)}


def pmc_traffic():
    """HBM bytes per launch of the score kernel from the committed rocprofv3
    --pmc summary (tools/pmc_traffic.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from KGE import _hip, engine, loss, optimizers, score
    from KGE.models.translating_based.TransE import TransE
    from KGE.ns_strategy import UniformStrategy
    _hip.load()   # the shipped gfx950 library; raises if missing

    triples, E, R = load_graph()
    B, K, d = args.batch, args.neg, args.dim
    model = TransE({"embedding_size": d}, K, "h+t", score_fn=score.LpDistance(p=2),
                   loss_fn=loss.SelfAdversarialNegativeSamplingLoss(margin=3, temperature=1),
                   ns_strategy=UniformStrategy(np.arange(E), seed=12345 + rank), constraint=True)
    model.metadata = {"ind2ent": list(range(E)), "ind2rel": list(range(R))}
    model._model_weights_initial = None
    model._init_embeddings(seed=12345)          # identical init on every rank
    model._to_device()
    opt = optimizers.SGD(learning_rate=0.01)
    if world > 1:
        from KGE.sharded import ShardedStep
        step = ShardedStep(model)
    else:
        step = engine.FusedStep(model)

    # batches resident in HBM before timing: a shuffled stream per rank
    nb = args.warmup + args.steps
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

    # per-kernel breakdown for the roofline: a second pass over the same
    # batches with HIP events recorded on the step's own stream between the
    # kernels [before K0, before KS, before KU, after KU]; the events cost a
    # few us per step, so this pass never feeds `value`
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
    # single-GPU SGD + constraint: the renormalisation is fused into KS / KU
    # (no K0 launch; its event pair brackets nothing) and KU also reads and
    # writes every entity row
    fused = world == 1
    if fused:
        k0 = 0.0
    if world > 1:
        t = torch.tensor([ms], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        ms = float(t.item())
    if rank != 0:
        torch.distributed.destroy_process_group()
        return

    step_b, score_b, upd_b, con_b = algorithmic_bytes(B, K, d, E)
    kern = {"constrain_rows_kernel": {"ms": k0, "alg_bytes": con_b},
            "score_kernel": {"ms": ks, "alg_bytes": score_b},
            "update_kernel": {"ms": ku, "alg_bytes": upd_b + (con_b if fused else 0)}}
    if fused:
        del kern["constrain_rows_kernel"]
    for v in kern.values():
        v["GBps"] = v["alg_bytes"] / (v["ms"] * 1e-3) / 1e9
    dom = max(kern, key=lambda k: kern[k]["ms"])
    pmc = pmc_traffic()
    traffic = None
    if pmc and dom in pmc.get("kernels", {}):
        traffic = pmc["kernels"][dom].get("hbm_bytes_per_launch")
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(kern[dom]["GBps"], 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(kern[dom]["GBps"] / HBM_PEAK_GBS, 4), "traffic": traffic,
            "step": {"alg_bytes": step_b, "kernel_ms": round(k0 + ks + ku, 5),
                     "achieved": round(step_b / ((k0 + ks + ku) * 1e-3) / 1e9, 1),
                     "frac": round(step_b / ((k0 + ks + ku) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "kernels": {k: {"ms": round(v["ms"], 5), "GBps": round(v["GBps"], 1)} for k, v in kern.items()}}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(triples, E, R, B, K, d, args.cpu_seconds)
    value = world * B / (ms * 1e-3)
    out = {
        "metric": "positive-triples/sec (batch x neg scored) at d=200, FB15k-237",
        "value": round(value, 1), "unit": "positive-triples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "FB15k-237 train_indexed ids (real graph); random-init weights",
        "config": {"workload": "C2: TransE d=%d, batch=%d, %d negs h+t, SANS(3,1), LpDistance(2), uniform, "
                               "constraint, SGD" % (d, B, K), "global_batch": world * B,
                   "negatives": K, "dim": d, "parallelism": "dp%d" % world,
                   "scored_triples_per_s": round(value * (1 + K), 1)},
        "roofline": roof, "cpu_baseline": cpu,
    }
    print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
