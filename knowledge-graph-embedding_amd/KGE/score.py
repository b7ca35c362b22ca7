"""Score functions (plugin surface of ``KGE/score.py`` in the reference).

Each built-in score keeps the reference's ``__call__(x, y)`` contract on torch
tensors (used by ``score_hrt`` for evaluation and by the eager plugin path for
user-defined combinations) and additionally exposes a ``kind`` / ``p``
descriptor that the fused HIP step (``libkge_hip.so``) consumes.

Reference semantics restated here:

* ``LpDistance(p)``     -- ``score.py:49-63``:
  ``-pow(clip(sum(|x-y|^p), 1e-9, inf), 1/p)``; ``p=inf`` -> ``-max|x-y|``.
  The clip is on the *sum*, so its gradient is 0 when the sum is < 1e-9.
* ``LpDistancePow(p)``  -- ``score.py:65-76``: ``-(LpDistance(p)(x, y))**2``.
* ``Dot()``             -- ``score.py:78-89``: ``sum(x*y)``.

On complex inputs (RotatE) ``|.|`` is the complex modulus, as in TF.
"""

import math

import torch

# kind codes shared with include/kge_hip.h (KGE_SCORE_*)
SCORE_LP = 0
SCORE_LP_POW = 1
SCORE_DOT = 2


def _abs(z):
    return torch.abs(z)


class Score:
    """Base class for scores (``score.py:29-46``)."""

    kind = None

    def __init__(self):
        raise NotImplementedError("subclass of Score should implement __init__() to init score parameters")

    def __call__(self, x, y):
        raise NotImplementedError("subclass of Score should implement __call__() to calculate score")


class LpDistance(Score):
    """Negative Lp distance ``-||x - y||_p`` (``score.py:49-63``)."""

    kind = SCORE_LP

    def __init__(self, p):
        self.p = p

    def __call__(self, x, y):
        diff = _abs(x - y)
        if self.p == math.inf or self.p == float("inf"):
            return -torch.amax(diff, dim=-1)
        s = torch.sum(torch.pow(diff, self.p), dim=-1)
        return -torch.pow(torch.clamp(s, min=1e-9), 1.0 / self.p)


class LpDistancePow(Score):
    """Negative squared Lp distance ``-||x - y||_p^2`` (``score.py:65-76``)."""

    kind = SCORE_LP_POW

    def __init__(self, p):
        self.p = p

    def __call__(self, x, y):
        return -torch.pow(LpDistance(p=self.p)(x, y), 2)


class Dot(Score):
    """Dot product ``sum(x * y)`` (``score.py:78-89``)."""

    kind = SCORE_DOT

    def __init__(self):
        self.p = 0

    def __call__(self, x, y):
        return torch.sum(x * y, dim=-1)


def fused_descriptor(score_fn):
    """Return ``(kind, p)`` for a built-in score, or ``None`` for a custom one.

    Only exact built-in classes are fused: a user subclass may override
    ``__call__`` and must go through the eager plugin path.
    """
    if type(score_fn) in (LpDistance, LpDistancePow):
        p = score_fn.p
        p = float("inf") if p == math.inf else float(p)
        if not p > 0:       # p <= 0 / NaN: the plugin path (TF's own behaviour)
            return None
        return score_fn.kind, p
    if type(score_fn) is Dot:
        return SCORE_DOT, 0.0
    return None
