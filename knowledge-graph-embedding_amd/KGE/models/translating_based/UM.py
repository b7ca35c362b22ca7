"""UM (reference ``KGE/models/translating_based/UM.py``); eager plugin path
only (outside the fused scope)."""

import numpy as np

from ...constraint import normalized_embeddings
from ...loss import PairwiseHingeLoss
from ...ns_strategy import UniformStrategy
from ...score import LpDistancePow
from ..base_model.TranslatingModel import TranslatingModel


class UM(TranslatingModel):
    def __init__(self, embedding_params, negative_ratio, corrupt_side, score_fn=LpDistancePow(p=2),
                 loss_fn=PairwiseHingeLoss(margin=1), ns_strategy=UniformStrategy, constraint=True, n_workers=1):
        super(UM, self).__init__(embedding_params, negative_ratio, corrupt_side, score_fn, loss_fn, ns_strategy,
                                 n_workers)
        self.constraint = constraint

    def _init_embeddings(self, seed):
        if self._model_weights_initial is None:
            assert self.embedding_params.get("embedding_size") is not None, "'embedding_size' should be given in embedding_params when using UM"
            k = self.embedding_params["embedding_size"]
            g = self._generator(seed)
            self.model_weights = {"ent_emb": self._uniform([len(self.metadata["ind2ent"]), k], np.sqrt(6.0 / k), g)}
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()

    def _check_model_weights(self, model_weights):
        assert model_weights.get("ent_emb") is not None, "entity embedding should be given in model_weights with key 'ent_emb'"
        assert list(model_weights["ent_emb"].shape) == [len(self.metadata["ind2ent"]), self.embedding_params["embedding_size"]], \
            "shape of 'ent_emb' should be (len(metadata['ind2ent']), embedding_params['embedding_size'])"

    def score_hrt(self, h, r, t):
        h, r, t = super(UM, self).score_hrt(h, r, t)
        return self.score_fn(self._lookup("ent_emb", h), self._lookup("ent_emb", t))

    def _constraint_loss(self, X):
        if self.constraint:
            self._assign("ent_emb", normalized_embeddings(X=self.model_weights["ent_emb"].detach(), p=2, axis=-1, value=1))
        return 0
