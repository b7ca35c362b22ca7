"""Constraint / regulariser helpers (reference ``KGE/constraint.py:4-126``).

Torch restatements used by the eager plugin path and by ``_init_embeddings``;
the fused HIP step implements the same formulas in ``csrc/kge_step.hip``
(``constrain_rows_kernel``: normalise / clip rows), fused into the score / update
kernels (``csrc/kge_step_impl.h``, ``fuse_norm``), ``csrc/kge_proj.hip`` (TransH soft /
orthogonality terms) and ``csrc/kge_rel.hip`` (RESCAL Lp regulariser).
"""

import math

import torch


def _norm(X, p, axis):
    if p == math.inf:
        return torch.amax(torch.abs(X), dim=axis, keepdim=True)
    return torch.pow(torch.sum(torch.pow(torch.abs(X), p), dim=axis, keepdim=True), 1.0 / p)


def normalized_embeddings(X, p, value, axis):
    """``X / ||X||_p * value`` along ``axis`` (``constraint.py:4-31``)."""
    return X / _norm(X, p, axis) * value


def soft_constraint(X, p, value, axis):
    """``sum(clip(||X||_p^p - value, 0, inf))`` (``constraint.py:34-67``)."""
    norm = _norm(X, p, axis)
    return torch.sum(torch.clamp(torch.pow(norm, p) - value, min=0))


def clip_constraint(X, p, value, axis):
    """Rescale rows whose p-norm exceeds ``value`` (``constraint.py:70-99``)."""
    norm = _norm(X, p, axis)
    mask = (norm < value).to(X.dtype)
    return mask * X + (1 - mask) * (X / torch.clamp(norm, min=1e-9) * value)


def Lp_regularization(X, p, axis):
    """``sum(|X|^p)`` along ``axis`` (``constraint.py:102-126``)."""
    return torch.sum(torch.pow(torch.abs(X), p), dim=axis)
