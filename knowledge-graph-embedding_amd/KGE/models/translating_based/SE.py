"""SE (reference ``KGE/models/translating_based/SE.py``); eager plugin path
only (outside the fused scope)."""

import numpy as np
import torch

from ...constraint import normalized_embeddings
from ...loss import PairwiseHingeLoss
from ...ns_strategy import UniformStrategy
from ...score import LpDistance
from ..base_model.TranslatingModel import TranslatingModel


class SE(TranslatingModel):
    def __init__(self, embedding_params, negative_ratio, corrupt_side, score_fn=LpDistance(p=1),
                 loss_fn=PairwiseHingeLoss(margin=1), ns_strategy=UniformStrategy, constraint=True, n_workers=1):
        super(SE, self).__init__(embedding_params, negative_ratio, corrupt_side, score_fn, loss_fn, ns_strategy,
                                 n_workers)
        self.constraint = constraint

    def _init_embeddings(self, seed):
        if self._model_weights_initial is None:
            assert self.embedding_params.get("embedding_size") is not None, "'embedding_size' should be given in embedding_params when using SE"
            k = self.embedding_params["embedding_size"]
            E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
            g = self._generator(seed)
            self.model_weights = {"ent_emb": self._uniform([E, k], np.sqrt(6.0 / k), g),
                                  "rel_proj_h": self._uniform([R, k, k], np.sqrt(3.0 / k), g),
                                  "rel_proj_t": self._uniform([R, k, k], np.sqrt(3.0 / k), g)}
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()

    def _check_model_weights(self, model_weights):
        k = self.embedding_params["embedding_size"]
        E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
        for key in ("ent_emb", "rel_proj_h", "rel_proj_t"):
            assert model_weights.get(key) is not None, "%s should be given in model_weights" % key
        assert list(model_weights["ent_emb"].shape) == [E, k]
        assert list(model_weights["rel_proj_h"].shape) == [R, k, k]
        assert list(model_weights["rel_proj_t"].shape) == [R, k, k]

    def score_hrt(self, h, r, t):
        h, r, t = super(SE, self).score_hrt(h, r, t)
        h_emb = self._lookup("ent_emb", h).unsqueeze(-1)
        t_emb = self._lookup("ent_emb", t).unsqueeze(-1)
        ph = self._lookup("rel_proj_h", r)
        pt = self._lookup("rel_proj_t", r)
        return self.score_fn(torch.matmul(ph, h_emb).squeeze(-1), torch.matmul(pt, t_emb).squeeze(-1))

    def _constraint_loss(self, X):
        if self.constraint:
            self._assign("ent_emb", normalized_embeddings(X=self.model_weights["ent_emb"].detach(), p=2, axis=1, value=1))
        return 0
