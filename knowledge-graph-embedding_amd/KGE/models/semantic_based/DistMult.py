"""DistMult (reference ``KGE/models/semantic_based/DistMult.py``).

``f = sum(h * r * t)``; default ``PairwiseHingeLoss(margin=1)``,
``constraint=True``: unit-L2 entity rows every step plus
``constraint_weight * mean_i ||r_{X_i}||^2`` over the batch relations.
Fused: ``kge_step`` with ``KGE_MODEL_DISTMULT``.
"""

import numpy as np
import torch

from ... import _hip
from ...constraint import Lp_regularization, normalized_embeddings
from ...loss import PairwiseHingeLoss
from ...ns_strategy import UniformStrategy
from ..base_model.SemanticModel import SemanticModel


class DistMult(SemanticModel):
    _fused_model_id = _hip.MODEL_DISTMULT

    def __init__(self, embedding_params, negative_ratio, corrupt_side, loss_fn=PairwiseHingeLoss(margin=1),
                 ns_strategy=UniformStrategy, constraint=True, constraint_weight=1.0, n_workers=1):
        super(DistMult, self).__init__(embedding_params, negative_ratio, corrupt_side, loss_fn, ns_strategy,
                                       n_workers)
        self.constraint = constraint
        self.constraint_weight = constraint_weight

    def _init_embeddings(self, seed):
        """``DistMult.py:68-100``: U(+-sqrt(6/k)) for both tables."""
        if self._model_weights_initial is None:
            assert self.embedding_params.get("embedding_size") is not None, \
                "'embedding_size' should be given in embedding_params when using DistMult"
            k = self.embedding_params["embedding_size"]
            limit = np.sqrt(6.0 / k)
            g = self._generator(seed)
            self.model_weights = {
                "ent_emb": self._uniform([len(self.metadata["ind2ent"]), k], limit, g),
                "rel_inter": self._uniform([len(self.metadata["ind2rel"]), k], limit, g),
            }
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()

    def _check_model_weights(self, model_weights):
        assert model_weights.get("ent_emb") is not None, "entity embedding should be given in model_weights with key 'ent_emb'"
        assert model_weights.get("rel_inter") is not None, "relation interaction matrix should be given in model_weights with key 'rel_inter'"
        assert list(model_weights["ent_emb"].shape) == [len(self.metadata["ind2ent"]), self.embedding_params["embedding_size"]], \
            "shape of 'ent_emb' should be (len(metadata['ind2ent']), embedding_params['embedding_size'])"
        assert list(model_weights["rel_inter"].shape) == [len(self.metadata["ind2rel"]), self.embedding_params["embedding_size"]], \
            "shape of 'rel_inter' should be (len(metadata['ind2rel']), embedding_params['embedding_size'])"

    def _fused_tables(self):
        return {"ent": self.model_weights["ent_emb"], "rel": self.model_weights["rel_inter"],
                "dim": self.embedding_params["embedding_size"]}

    def score_hrt(self, h, r, t):
        """``DistMult.py:118-146``."""
        h, r, t = super(DistMult, self).score_hrt(h, r, t)
        h_emb = self._lookup("ent_emb", h)
        t_emb = self._lookup("ent_emb", t)
        r_inter = self._lookup("rel_inter", r)
        return torch.sum(h_emb * r_inter * t_emb, dim=-1)

    def _constraint_loss(self, X):
        """``DistMult.py:148-167``."""
        if self.constraint:
            self._assign("ent_emb", normalized_embeddings(X=self.model_weights["ent_emb"].detach(), p=2, axis=1, value=1))
            r_inter = self._lookup("rel_inter", X[:, 1])
            reg = Lp_regularization(r_inter, p=2, axis=-1)
            return self.constraint_weight * torch.sum(reg) / (reg.shape[0] * self._batch_scale)
        return 0
