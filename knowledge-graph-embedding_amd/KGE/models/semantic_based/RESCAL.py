"""RESCAL (reference ``KGE/models/semantic_based/RESCAL.py``).

``f = h^T R_r t`` with ``R_r`` of shape ``[k, k]``; default ``SquareErrorLoss``;
``constraint=True`` normalises entity rows and each ``R_r`` (Frobenius) at
init and adds ``constraint_weight * (mean_e ||e||^2 + mean_r ||R_r||_F^2)``
over the full tables each step (dense gradients, ``RESCAL.py:176-200``).
"""

import numpy as np
import torch

from ... import _hip
from ...constraint import Lp_regularization, normalized_embeddings
from ...loss import SquareErrorLoss
from ...ns_strategy import UniformStrategy
from ..base_model.SemanticModel import SemanticModel


class RESCAL(SemanticModel):
    _fused_model_id = _hip.MODEL_RESCAL

    def __init__(self, embedding_params, negative_ratio, corrupt_side, loss_fn=SquareErrorLoss(),
                 ns_strategy=UniformStrategy, constraint=True, constraint_weight=1.0, n_workers=1):
        super(RESCAL, self).__init__(embedding_params, negative_ratio, corrupt_side, loss_fn, ns_strategy,
                                     n_workers)
        self.constraint = constraint
        self.constraint_weight = constraint_weight

    def _init_embeddings(self, seed):
        """``RESCAL.py:67-115``."""
        k = self.embedding_params.get("embedding_size")
        if self._model_weights_initial is None:
            assert k is not None, "'embedding_size' should be given in embedding_params when using RESCAL"
            E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
            g = self._generator(seed)
            self.model_weights = {"ent_emb": self._uniform([E, k], np.sqrt(6.0 / k), g),
                                  "rel_inter": self._uniform([R, k, k], np.sqrt(3.0 / k), g)}
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()
        if self.constraint:
            w = self.model_weights
            w["ent_emb"].copy_(normalized_embeddings(X=w["ent_emb"], p=2, axis=-1, value=1))
            w["rel_inter"].copy_(normalized_embeddings(X=w["rel_inter"], p=2, axis=(1, 2), value=1))

    def _check_model_weights(self, model_weights):
        k = self.embedding_params["embedding_size"]
        E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
        assert model_weights.get("ent_emb") is not None, "entity embedding should be given in model_weights with key 'ent_emb'"
        assert model_weights.get("rel_inter") is not None, "relation interaction matrix should be given in model_weights with key 'rel_inter'"
        assert list(model_weights["ent_emb"].shape) == [E, k], "shape of 'ent_emb' should be (len(metadata['ind2ent']), embedding_params['embedding_size'])"
        assert list(model_weights["rel_inter"].shape) == [R, k, k], "shape of 'rel_inter' should be (len(metadata['ind2rel']), embedding_params['embedding_size'], embedding_params['embedding_size'])"

    def _fused_tables(self):
        return {"ent": self.model_weights["ent_emb"], "rel": self.model_weights["rel_inter"],
                "dim": self.embedding_params["embedding_size"]}

    def score_hrt(self, h, r, t):
        """``RESCAL.py:140-174``."""
        h, r, t = super(RESCAL, self).score_hrt(h, r, t)
        h_emb = self._lookup("ent_emb", h).unsqueeze(-1)
        t_emb = self._lookup("ent_emb", t).unsqueeze(-1)
        r_inter = self._lookup("rel_inter", r)
        return torch.matmul(torch.matmul(h_emb.transpose(-1, -2), r_inter), t_emb).reshape(-1)

    def _constraint_loss(self, X):
        """``RESCAL.py:176-200``."""
        if self.constraint:
            w = self.model_weights
            e_norm = torch.mean(Lp_regularization(w["ent_emb"], p=2, axis=-1))
            r_norm = torch.mean(Lp_regularization(w["rel_inter"], p=2, axis=(1, 2)))
            return self.constraint_weight * (e_norm + r_norm)
        return 0
