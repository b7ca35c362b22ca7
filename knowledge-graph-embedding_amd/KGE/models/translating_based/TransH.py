"""TransH (reference ``KGE/models/translating_based/TransH.py``).

Hyperplane projection ``e_perp = e - (w_r . e) w_r``; ``f = s(h_perp + r, t_perp)``
with default ``LpDistancePow(p=2)``; ``constraint=True`` renormalises
``rel_hyper`` each step and adds the soft (entity norm) and orthogonality
penalties over the full tables (``TransH.py:188-213``).
"""

import numpy as np
import torch

from ... import _hip
from ...constraint import normalized_embeddings, soft_constraint
from ...loss import PairwiseHingeLoss
from ...ns_strategy import UniformStrategy
from ...score import LpDistancePow
from ..base_model.TranslatingModel import TranslatingModel


class TransH(TranslatingModel):
    _fused_model_id = _hip.MODEL_TRANSH

    def __init__(self, embedding_params, negative_ratio, corrupt_side, score_fn=LpDistancePow(p=2),
                 loss_fn=PairwiseHingeLoss(margin=1), ns_strategy=UniformStrategy, constraint=True,
                 constraint_weight=1.0, n_workers=1):
        super(TransH, self).__init__(embedding_params, negative_ratio, corrupt_side, score_fn, loss_fn,
                                     ns_strategy, n_workers)
        self.constraint = constraint
        self.constraint_weight = constraint_weight

    def _init_embeddings(self, seed):
        """``TransH.py:95-128``: U(+-sqrt(6/k))."""
        if self._model_weights_initial is None:
            assert self.embedding_params.get("embedding_size") is not None, \
                "'embedding_size' should be given in embedding_params when using TransH"
            k = self.embedding_params["embedding_size"]
            limit = np.sqrt(6.0 / k)
            g = self._generator(seed)
            E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
            self.model_weights = {"ent_emb": self._uniform([E, k], limit, g),
                                  "rel_emb": self._uniform([R, k], limit, g),
                                  "rel_hyper": self._uniform([R, k], limit, g)}
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()

    def _check_model_weights(self, model_weights):
        k = self.embedding_params["embedding_size"]
        E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
        assert model_weights.get("ent_emb") is not None, "entity embedding should be given in model_weights with key 'ent_emb'"
        assert model_weights.get("rel_emb") is not None, "relation embedding should be given in model_weights with key 'rel_emb'"
        assert model_weights.get("rel_hyper") is not None, "relation hyperplane should be given in model_weights with key 'rel_hyper'"
        assert list(model_weights["ent_emb"].shape) == [E, k], "shape of 'ent_emb' should be (len(metadata['ind2ent']), embedding_params['embedding_size'])"
        assert list(model_weights["rel_emb"].shape) == [R, k], "shape of 'rel_emb' should be (len(metadata['ind2rel']), embedding_params['embedding_size'])"
        assert list(model_weights["rel_hyper"].shape) == [R, k], "shape of 'rel_hyper' should be (len(metadata['ind2rel']), embedding_params['embedding_size'])"

    def _fused_tables(self):
        return {"ent": self.model_weights["ent_emb"], "rel": self.model_weights["rel_emb"],
                "rel_aux": self.model_weights["rel_hyper"], "dim": self.embedding_params["embedding_size"]}

    def score_hrt(self, h, r, t):
        """``TransH.py:149-185``."""
        h, r, t = super(TransH, self).score_hrt(h, r, t)
        h_emb = self._lookup("ent_emb", h)
        r_emb = self._lookup("rel_emb", r)
        r_hyper = self._lookup("rel_hyper", r)
        t_emb = self._lookup("ent_emb", t)
        h_proj = h_emb - torch.sum(r_hyper * h_emb, dim=-1, keepdim=True) * r_hyper
        t_proj = t_emb - torch.sum(r_hyper * t_emb, dim=-1, keepdim=True) * r_hyper
        return self.score_fn(h_proj + r_emb, t_proj)

    def _constraint_loss(self, X):
        """``TransH.py:188-213``."""
        if self.constraint:
            self._assign("rel_hyper", normalized_embeddings(X=self.model_weights["rel_hyper"].detach(), p=2, axis=1, value=1))
            w = self.model_weights
            scale = soft_constraint(w["ent_emb"], p=2, axis=-1, value=1)
            orthogonal = torch.sum(w["rel_hyper"] * w["rel_emb"], dim=-1)
            orthogonal = torch.pow(orthogonal / torch.linalg.norm(w["rel_emb"], dim=-1), 2) - 1e-18
            orthogonal = torch.sum(torch.clamp(orthogonal, min=0))
            return self.constraint_weight * (scale + orthogonal)
        return 0
