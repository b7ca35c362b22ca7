"""Rank metrics over the integer ranks ``kge_rank`` returns.

Same names and values as the reference's ``KGE/metrics.py:5-25`` (pinned by
``tests/golden/metrics_kat.json``, produced by that file). Ranks arrive as an
int64 array from the device; every metric is one float64 reduction over it,
so an evaluation set of any size is summarised without a Python loop.
"""

import numpy as np


def _ranks(ranks):
    r = np.asarray(ranks, dtype=np.float64).ravel()
    if r.size == 0:
        raise ValueError("no ranks to summarise")
    return r


def mean_reciprocal_rank(ranks):
    return float(np.mean(np.reciprocal(_ranks(ranks))))


def mean_rank(ranks):
    return float(np.mean(_ranks(ranks)))


def median_rank(ranks):
    return float(np.median(_ranks(ranks)))


def geometric_mean_rank(ranks):
    """exp(mean(log r)); ranks are >= 1 so the log is finite."""
    return float(np.exp(np.mean(np.log(_ranks(ranks)))))


def harmonic_mean_rank(ranks):
    r = _ranks(ranks)
    return float(r.size / np.sum(np.reciprocal(r)))


def std_rank(ranks):
    """Population standard deviation (ddof = 0), as the reference's ``np.std``."""
    return float(np.std(_ranks(ranks)))


def hits_at_k(ranks, k):
    assert k >= 1, "k needs >= 1"
    return float(np.count_nonzero(_ranks(ranks) <= k) / np.size(ranks))


def summary(ranks, ks=(1, 3, 10)):
    """Every metric above in one dict (the keys ``evaluate`` reports)."""
    out = {"mean_rank": mean_rank(ranks), "mean_reciprocal_rank": mean_reciprocal_rank(ranks),
           "median_rank": median_rank(ranks), "geometric_mean_rank": geometric_mean_rank(ranks),
           "harmonic_mean_rank": harmonic_mean_rank(ranks), "std_rank": std_rank(ranks)}
    for k in ks:
        out["hit@%d" % k] = hits_at_k(ranks, k)
    return out
