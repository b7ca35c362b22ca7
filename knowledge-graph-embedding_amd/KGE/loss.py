"""Loss functions (plugin surface of ``KGE/loss.py`` in the reference).

``Loss.__call__(pos_score [B], neg_score [B*K]) -> scalar`` on torch tensors,
plus a ``kind`` descriptor consumed by the fused HIP step.

Reference formulas restated (TF-2.5 semantics):

* ``PairwiseHingeLoss(margin)``  -- ``loss.py:79-82``:
  ``sum(clip(margin + s_neg - repeat(s_pos, K), 0, inf)) / (B*K)``.
  The divisor is the *repeated* length ``B*K``.
* ``PairwiseLogisticLoss()``     -- ``loss.py:110-113``:
  ``sum(log(1 + exp(s_neg - repeat(s_pos, K))))`` (no mean, naive formula).
* ``BinaryCrossEntropyLoss()``   -- ``loss.py:138-143``:
  ``-(sum(logsig(s_pos)) + sum(logsig(-s_neg))) / B``.
* ``SelfAdversarialNegativeSamplingLoss(margin, temperature)`` -- ``loss.py:174-182``:
  ``p = stop_grad(softmax(T * s_neg.reshape(B, K)))``;
  ``-(sum(logsig(s_pos + m)) + sum(p * logsig(-s_neg - m))) / B``.
* ``SquareErrorLoss()``          -- ``loss.py:200-204``:
  ``(sum((s_pos - 1)^2) + sum(s_neg^2)) / 2 / B``.

``batch_scale`` (default 1) multiplies the positive count used in the
divisors; the multi-GPU path sets it to the world size so that G ranks of B
positives normalise exactly like one device at G*B.
"""

import torch
import torch.nn.functional as F

# kind codes shared with include/kge_hip.h (KGE_LOSS_*)
LOSS_HINGE = 0
LOSS_LOGISTIC = 1
LOSS_BCE = 2
LOSS_SANS = 3
LOSS_SQERR = 4


class Loss:
    """Base class for losses (``loss.py:28-46``)."""

    kind = None

    def __init__(self):
        raise NotImplementedError("subclass of Loss should implement __init__() to init loss parameters")

    def __call__(self, pos_score, neg_score):
        raise NotImplementedError("subclass of Loss should implement __call__() to calculate loss")


def _ratio(pos_score, neg_score):
    return int(neg_score.shape[0] / pos_score.shape[0])


class PairwiseHingeLoss(Loss):
    """Margin ranking loss (``loss.py:49-82``)."""

    kind = LOSS_HINGE

    def __init__(self, margin):
        self.margin = margin

    def __call__(self, pos_score, neg_score, batch_scale=1):
        pos = torch.repeat_interleave(pos_score, _ratio(pos_score, neg_score))
        total = torch.sum(torch.clamp(self.margin + neg_score - pos, min=0))
        return total / (pos.shape[0] * batch_scale)


class PairwiseLogisticLoss(Loss):
    """Pairwise logistic loss (``loss.py:85-113``); no normalisation."""

    kind = LOSS_LOGISTIC

    def __init__(self):
        pass

    def __call__(self, pos_score, neg_score, batch_scale=1):
        pos = torch.repeat_interleave(pos_score, _ratio(pos_score, neg_score))
        return torch.sum(torch.log(1 + torch.exp(neg_score - pos)))


class BinaryCrossEntropyLoss(Loss):
    """Binary cross entropy on triple scores as logits (``loss.py:116-143``)."""

    kind = LOSS_BCE

    def __init__(self):
        pass

    def __call__(self, pos_score, neg_score, batch_scale=1):
        pos_ll = torch.sum(F.logsigmoid(pos_score))
        neg_ll = torch.sum(F.logsigmoid(-neg_score))
        return -(pos_ll + neg_ll) / (pos_score.shape[0] * batch_scale)


class SelfAdversarialNegativeSamplingLoss(Loss):
    """Self-adversarial negative sampling loss (``loss.py:146-182``)."""

    kind = LOSS_SANS

    def __init__(self, margin, temperature):
        self.margin = margin
        self.temperature = temperature

    def __call__(self, pos_score, neg_score, batch_scale=1):
        neg = neg_score.reshape(pos_score.shape[0], _ratio(pos_score, neg_score))
        neg_prob = torch.softmax(self.temperature * neg, dim=-1).detach()
        pos_ll = torch.sum(F.logsigmoid(pos_score + self.margin))
        neg_ll = torch.sum(neg_prob * F.logsigmoid(-neg - self.margin))
        return -(pos_ll + neg_ll) / (pos_score.shape[0] * batch_scale)


class SquareErrorLoss(Loss):
    """Square error against labels 1 / 0 (``loss.py:185-204``)."""

    kind = LOSS_SQERR

    def __init__(self):
        pass

    def __call__(self, pos_score, neg_score, batch_scale=1):
        pos_loss = torch.sum(torch.pow(pos_score - 1.0, 2))
        neg_loss = torch.sum(torch.pow(neg_score - 0.0, 2))
        return (pos_loss + neg_loss) / 2 / (pos_score.shape[0] * batch_scale)


def fused_descriptor(loss_fn):
    """``(kind, margin, temperature)`` for a built-in loss, else ``None``."""
    t = type(loss_fn)
    if t is PairwiseHingeLoss:
        return LOSS_HINGE, float(loss_fn.margin), 0.0
    if t is PairwiseLogisticLoss:
        return LOSS_LOGISTIC, 0.0, 0.0
    if t is BinaryCrossEntropyLoss:
        return LOSS_BCE, 0.0, 0.0
    if t is SelfAdversarialNegativeSamplingLoss:
        return LOSS_SANS, float(loss_fn.margin), float(loss_fn.temperature)
    if t is SquareErrorLoss:
        return LOSS_SQERR, 0.0, 0.0
    return None
