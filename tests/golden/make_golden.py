"""Regenerate the committed golden fixtures under tests/golden/.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

Fixtures and where their expected values come from:
  philox_kat.json    published Random123 known-answer vectors for
                     Philox4x32-10 (kat_vectors, Salmon et al. 2011).
                     The constants are written below; nothing is computed.
  metrics_kat.json   outputs of the REFERENCE's own KGE/metrics.py
                     (/root/reference/KGE/metrics.py:5-25, loaded by path;
                     it needs only numpy/scipy) on fixed rank lists.
  toy_kg.json        the reference's test fixture KG (tests/data.py:5-28),
                     indexed with the numpy branch of index_kg
                     (data_utils.py:41-43: sorted np.unique) -- data only.
  sampler_golden.json  negative ids of the counter-based sampler spec
                     (include/kge_hip.h) for fixed (seed, plane) -- oracle.
  step_golden.npz    one training step (BaseModel.py:316-328) per model and
                     plugin combination on the toy KG with seeded weights and
                     injected negatives: float64 oracle outputs (loss, scores,
                     updated tables, per-variable gradient norm^2).
The reference's own tests pin only properties, so the step
vectors are the oracle's (PARITY UNPINNED against TF, which is absent);
they freeze the restatement so that regressions in either side show up.
"""

import importlib.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import kge_oracle as orc  # noqa: E402

REF = "/root/reference"

# Random123 kat_vectors, philox4x32 10 rounds: (counter, key, expected)
PHILOX_KAT = [
    ([0x00000000, 0x00000000, 0x00000000, 0x00000000], [0x00000000, 0x00000000],
     [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff], [0xffffffff, 0xffffffff],
     [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]

# reference tests/data.py:5-28 (data: the toy KG triples)
TOY_TRAIN = [
    ["DaVinci", "painted", "MonaLisa"], ["Lily", "is_interested_in", "DaVinci"], ["Lily", "is_a", "Person"],
    ["Lily", "is_a_friend_of", "James"], ["James", "like", "MonaLisa"], ["James", "has_visited", "Louvre"],
    ["James", "has_lived_in", "TourEiffel"], ["James", "is_born_on", "Jan,1,1984"],
    ["LaJocondeAWashinton", "is_about", "MonaLisa"], ["MonaLis", "is_in", "Louvre"], ["Paris", "is_a", "Place"],
    ["TourEiffel", "is_located_in", "Paris"]]
TOY_VAL = [["DaVinci", "is_a", "Person"], ["James", "is_a", "Person"], ["Louvre", "is_located_in", "Paris"]]

# (model, score spec, loss spec) combinations frozen in step_golden.npz
STEP_CASES = [
    ("TransE", ("lp", 2.0), ("hinge", 1.0)), ("TransE", ("lp", 1.0), ("sans", 3.0, 1.0)),
    ("TransE", ("lp", float("inf")), ("logistic",)), ("TransE", ("lppow", 2.0), ("bce",)),
    ("TransE", ("dot", 0.0), ("sqerr",)),
    ("TransH", ("lppow", 2.0), ("hinge", 1.0)), ("TransR", ("lppow", 2.0), ("hinge", 1.0)),
    ("TransD", ("lppow", 2.0), ("hinge", 1.0)), ("RotatE", ("lp", 1.0), ("sans", 3.0, 1.0)),
    ("RotatE", ("lp", 2.0), ("hinge", 1.0)), ("DistMult", ("dot", 0.0), ("hinge", 1.0)),
    ("DistMult", ("dot", 0.0), ("bce",)), ("RESCAL", ("dot", 0.0), ("sqerr",)),
]


def toy_kg():
    tr = np.array(TOY_TRAIN)
    ents = list(np.unique(np.append(tr[:, 0], tr[:, 2])))
    rels = list(np.unique(tr[:, 1]))
    e2i = {e: i for i, e in enumerate(ents)}
    r2i = {r: i for i, r in enumerate(rels)}

    def conv(X):
        return [[e2i.get(h), r2i.get(r), e2i.get(t)] for h, r, t in X]

    return {"ind2ent": [str(e) for e in ents], "ind2rel": [str(r) for r in rels],
            "train": conv(TOY_TRAIN), "val": conv(TOY_VAL), "train_raw": TOY_TRAIN, "val_raw": TOY_VAL}


def case_weights(model, E, R, d, rng):
    """Seeded initial weights with the reference's weight keys and shapes."""
    u = lambda *s: rng.uniform(-0.5, 0.5, s)  # noqa: E731
    if model == "TransE":
        return {"ent_emb": u(E, d), "rel_emb": u(R, d)}
    if model == "TransH":
        return {"ent_emb": u(E, d), "rel_emb": u(R, d), "rel_hyper": u(R, d)}
    if model == "TransR":
        return {"ent_emb": u(E, d), "rel_emb": u(R, d), "rel_proj": np.eye(d)[None].repeat(R, 0) + 0.1 * u(R, d, d)}
    if model == "TransD":
        return {"ent_emb": u(E, d), "rel_emb": u(R, d), "ent_proj": u(E, d), "rel_proj": u(R, d)}
    if model == "RotatE":
        return {"ent_emb": u(E, d, 2), "rel_emb": u(R, d)}
    if model == "DistMult":
        return {"ent_emb": u(E, d), "rel_inter": u(R, d)}
    if model == "RESCAL":
        return {"ent_emb": u(E, d), "rel_inter": u(R, d, d)}
    raise ValueError(model)


def step_cases(kg):
    pos = np.array(kg["train"], dtype=np.int64)
    E, R, d, K = len(kg["ind2ent"]), len(kg["ind2rel"]), 8, 4
    out = {}
    meta = []
    for ci, (model, score, loss) in enumerate(STEP_CASES):
        rng = np.random.default_rng(1000 + ci)
        W = case_weights(model, E, R, d, rng)
        W = {k: v.astype(np.float32).astype(np.float64) for k, v in W.items()}
        neg = orc.negatives(pos, K, "h+t", E, seed=777 + ci, plane=0, i64=True)
        limit = (3.0 + 2.0) / d if model == "RotatE" else None   # RotatE.py:88-93 with gamma=3
        res = orc.train_step(model, W, pos, neg, score=score, loss=loss, lr=0.05, constraint=True,
                             side="h+t", limit=limit)
        tag = "c%02d" % ci
        for k, v in W.items():
            out["%s/in/%s" % (tag, k)] = v
        for k, v in res["weights"].items():
            out["%s/out/%s" % (tag, k)] = v
        out[tag + "/neg"] = neg
        out[tag + "/pos_score"] = res["pos_score"]
        out[tag + "/neg_score"] = res["neg_score"]
        out[tag + "/loss"] = np.array(res["loss"])
        meta.append({"tag": tag, "model": model, "score": list(score), "loss": list(loss), "d": d, "K": K,
                     "side": "h+t", "lr": 0.05, "constraint": True, "limit": limit, "seed": 777 + ci, "plane": 0,
                     "norm2": res["norm2"]})
    out["pos"] = pos
    return out, meta


def sampler_cases():
    rng = np.random.default_rng(5)
    E = 14505
    X = np.stack([rng.integers(0, E, 64), rng.integers(0, 237, 64), rng.integers(0, E, 64)], 1)
    ind2type = [int(x) for x in rng.integers(0, 5, E)]
    cases = []
    for side in ("h", "t", "h+t"):
        for i64 in (True, False):
            cases.append({"side": side, "i64": i64, "K": 6, "seed": 123456789, "plane": 3, "E": E,
                          "ids": orc.negatives(X, 6, side, E, seed=123456789, plane=3, i64=i64).tolist()})
    tt = orc.typed_tables(ind2type)
    cases.append({"side": "t", "i64": True, "K": 5, "seed": 99, "plane": 0, "E": E, "typed": True,
                  "ids": orc.negatives(X, 5, "t", E, seed=99, plane=0, sampler="typed", typed=tt).tolist()})
    return {"X": X.tolist(), "ind2type": ind2type, "cases": cases}


def metrics_kat():
    spec = importlib.util.spec_from_file_location("ref_metrics", os.path.join(REF, "KGE", "metrics.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    lists = [[1, 2, 3, 10, 100], [7], [1, 1, 1, 2], [5, 1000, 13, 4, 4, 98, 2, 1, 1, 77]]
    out = []
    for r in lists:
        out.append({"ranks": r, "mean_rank": float(m.mean_rank(r)), "mean_reciprocal_rank": float(m.mean_reciprocal_rank(r)),
                    "median_rank": float(m.median_rank(r)), "geometric_mean_rank": float(m.geometric_mean_rank(r)),
                    "harmonic_mean_rank": float(m.harmonic_mean_rank(r)), "std_rank": float(m.std_rank(r)),
                    "hit@1": float(m.hits_at_k(r, 1)), "hit@3": float(m.hits_at_k(r, 3)),
                    "hit@10": float(m.hits_at_k(r, 10))})
    return out


def main():
    with open(os.path.join(HERE, "philox_kat.json"), "w") as f:
        json.dump([{"ctr": c, "key": k, "out": o} for c, k, o in PHILOX_KAT], f, indent=1)
    kg = toy_kg()
    with open(os.path.join(HERE, "toy_kg.json"), "w") as f:
        json.dump(kg, f, indent=1)
    with open(os.path.join(HERE, "sampler_golden.json"), "w") as f:
        json.dump(sampler_cases(), f)
    arrays, meta = step_cases(kg)
    np.savez_compressed(os.path.join(HERE, "step_golden.npz"), **arrays)
    with open(os.path.join(HERE, "step_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    if os.path.exists(os.path.join(REF, "KGE", "metrics.py")):
        with open(os.path.join(HERE, "metrics_kat.json"), "w") as f:
            json.dump(metrics_kat(), f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
