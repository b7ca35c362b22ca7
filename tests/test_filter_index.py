"""CPU: ranking.filter_index (the filter lists of BaseModel.py:646-650) against
a plain-Python restatement, on both of its sort paths (one combined-key sort;
two stable sorts when R * E^2 would overflow int64)."""

import numpy as np
import torch

from KGE import ranking


def _reference(X, P, side):
    keep, corrupt = (2, 0) if side == "h" else (0, 2)
    lists = {}
    for row in P.tolist():
        lists.setdefault((row[1], row[keep]), set()).add(row[corrupt])
    return [sorted(lists.get((x[1], x[keep]), ())) for x in X.tolist()]


def _check(X, P, E, side):
    beg, end, ents = ranking.filter_index(X, P, side, E)
    ref = _reference(X, P, side)
    for i, want in enumerate(ref):
        got = ents[int(beg[i]):int(end[i])].tolist()
        assert got == want, (i, got, want)


def test_filter_index_combined_key_path():
    g = np.random.default_rng(0)
    E, R = 50, 7
    P = torch.as_tensor(np.stack([g.integers(0, E, 400), g.integers(0, R, 400), g.integers(0, E, 400)], 1))
    X = torch.cat([P[:60], torch.as_tensor(np.stack([g.integers(0, E, 40), g.integers(0, R, 40),
                                                     g.integers(0, E, 40)], 1))])
    for side in ("h", "t"):
        _check(X, P, E, side)


def test_filter_index_two_sort_path():
    """Entity ids near 2^31 with many relations: R * E^2 > 2^62 takes the
    lexicographic two-sort path; same lists."""
    g = np.random.default_rng(1)
    E = 2 ** 31 - 1
    ents = g.choice(E, 30, replace=False)
    P = torch.as_tensor(np.stack([ents[g.integers(0, 30, 300)], g.integers(0, 5, 300),
                                  ents[g.integers(0, 30, 300)]], 1))
    P[0, 1] = 2 ** 20   # many relations
    X = P[:80].clone()
    for side in ("h", "t"):
        _check(X, P, E, side)


def test_cached_filter_keys_follow_the_content():
    """The cached pairs equal a fresh build; an in-place edit of the positive
    set is a new key (content hash), not a stale hit."""
    g = np.random.default_rng(2)
    E, R = 40, 5
    P = np.stack([g.integers(0, E, 300), g.integers(0, R, 300), g.integers(0, E, 300)], 1)
    ranking._FILTER_CACHE.clear()
    k1, e1 = ranking.cached_filter_keys(P, "t", E, "cpu")
    k2, e2 = ranking.cached_filter_keys(P.copy(), "t", E, "cpu")
    assert k1 is k2 and e1 is e2
    fk, fe = ranking.filter_keys(torch.as_tensor(P), "t", E)
    assert torch.equal(k1, fk) and torch.equal(e1, fe)
    P[0] = [E - 1, R - 1, E - 1]
    k3, e3 = ranking.cached_filter_keys(P, "t", E, "cpu")
    fk, fe = ranking.filter_keys(torch.as_tensor(P), "t", E)
    assert k3 is not k1 and torch.equal(k3, fk) and torch.equal(e3, fe)
    for i in range(6):
        ranking.cached_filter_keys(P[i:], "h", E, "cpu")
    assert len(ranking._FILTER_CACHE) == ranking._FILTER_CACHE_MAX
