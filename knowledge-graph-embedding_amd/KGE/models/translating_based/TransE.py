"""TransE (reference ``KGE/models/translating_based/TransE.py``).

``f(h, r, t) = s(e_h + r_r, e_t)``; default ``LpDistance(p=2)``,
``PairwiseHingeLoss(margin=1)``, uniform sampling, ``constraint=True``
(unit-L2 entity rows every step, relation rows normalised once at init).
Fused: ``kge_step`` with ``KGE_MODEL_TRANSE``.
"""

import numpy as np

from ... import _hip
from ...constraint import normalized_embeddings
from ...loss import PairwiseHingeLoss
from ...ns_strategy import UniformStrategy
from ...score import LpDistance
from ..base_model.TranslatingModel import TranslatingModel


class TransE(TranslatingModel):
    _fused_model_id = _hip.MODEL_TRANSE

    def __init__(self, embedding_params, negative_ratio, corrupt_side, score_fn=LpDistance(p=2),
                 loss_fn=PairwiseHingeLoss(margin=1), ns_strategy=UniformStrategy, constraint=True, n_workers=1):
        super(TransE, self).__init__(embedding_params, negative_ratio, corrupt_side, score_fn, loss_fn,
                                     ns_strategy, n_workers)
        self.constraint = constraint

    def _init_embeddings(self, seed):
        """``TransE.py:77-109``: U(+-6/sqrt(k)); relation rows normalised if constraint.
        (With ``model_weights_initial`` the reference raises NameError at :109; here the
        given ``rel_emb`` is normalised.)"""
        if self._model_weights_initial is None:
            assert self.embedding_params.get("embedding_size") is not None, \
                "'embedding_size' should be given in embedding_params when using TransE"
            k = self.embedding_params["embedding_size"]
            limit = 6.0 / np.sqrt(k)
            g = self._generator(seed)
            self.model_weights = {
                "ent_emb": self._uniform([len(self.metadata["ind2ent"]), k], limit, g),
                "rel_emb": self._uniform([len(self.metadata["ind2rel"]), k], limit, g),
            }
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()
        if self.constraint:
            w = self.model_weights["rel_emb"]
            w.copy_(normalized_embeddings(X=w, p=2, value=1, axis=1))

    def _check_model_weights(self, model_weights):
        assert model_weights.get("ent_emb") is not None, "entity embedding should be given in model_weights with key 'ent_emb'"
        assert model_weights.get("rel_emb") is not None, "relation embedding should be given in model_weights with key 'rel_emb'"
        assert list(model_weights["ent_emb"].shape) == [len(self.metadata["ind2ent"]), self.embedding_params["embedding_size"]], \
            "shape of 'ent_emb' should be (len(metadata['ind2ent']), embedding_params['embedding_size'])"
        assert list(model_weights["rel_emb"].shape) == [len(self.metadata["ind2rel"]), self.embedding_params["embedding_size"]], \
            "shape of 'rel_emb' should be (len(metadata['ind2rel']), embedding_params['embedding_size'])"

    def _fused_tables(self):
        return {"ent": self.model_weights["ent_emb"], "rel": self.model_weights["rel_emb"],
                "dim": self.embedding_params["embedding_size"]}

    def score_hrt(self, h, r, t):
        """``TransE.py:127-155``."""
        h, r, t = super(TransE, self).score_hrt(h, r, t)
        h_emb = self._lookup("ent_emb", h)
        r_emb = self._lookup("rel_emb", r)
        t_emb = self._lookup("ent_emb", t)
        return self.score_fn(h_emb + r_emb, t_emb)

    def _constraint_loss(self, X):
        """``TransE.py:157-174``: renormalise every entity row."""
        if self.constraint:
            self._assign("ent_emb", normalized_embeddings(X=self.model_weights["ent_emb"].detach(), p=2, axis=1, value=1))
        return 0
