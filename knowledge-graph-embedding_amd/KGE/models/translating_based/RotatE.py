"""RotatE (reference ``KGE/models/translating_based/RotatE.py``).

Entities are ``[E, k, 2]`` (re, im), relations ``[R, k]`` phases scaled to
``[-pi, pi]`` by ``r / limit * pi``; ``f = s(h o e^{i theta}, t)`` with
default ``LpDistance(p=1)`` over the complex modulus and
``SelfAdversarialNegativeSamplingLoss(margin=3, temperature=1)``.
Fused: ``kge_step`` with ``KGE_MODEL_ROTATE``.
"""

import numpy as np
import torch

from ... import _hip
from ...loss import SelfAdversarialNegativeSamplingLoss
from ...ns_strategy import UniformStrategy
from ...score import LpDistance
from ..base_model.TranslatingModel import TranslatingModel


class RotatE(TranslatingModel):
    _fused_model_id = _hip.MODEL_ROTATE

    def __init__(self, embedding_params, negative_ratio, corrupt_side, score_fn=LpDistance(p=1),
                 loss_fn=SelfAdversarialNegativeSamplingLoss(margin=3, temperature=1),
                 ns_strategy=UniformStrategy, n_workers=1):
        super(RotatE, self).__init__(embedding_params, negative_ratio, corrupt_side, score_fn, loss_fn,
                                     ns_strategy, n_workers)

    def _set_limit(self):
        margin = self.loss_fn.margin if hasattr(self.loss_fn, "margin") else 6.0
        self.limit = (margin + 2.0) / self.embedding_params["embedding_size"]

    def _init_embeddings(self, seed):
        """``RotatE.py:73-108``: U(+-(margin+2)/k). (The reference's initial-weights
        branch raises AttributeError, :107-108; here it is honoured.)"""
        assert self.embedding_params.get("embedding_size") is not None, \
            "'embedding_size' should be given in embedding_params when using RotatE"
        self._set_limit()
        if self._model_weights_initial is None:
            k = self.embedding_params["embedding_size"]
            g = self._generator(seed)
            self.model_weights = {
                "ent_emb": self._uniform([len(self.metadata["ind2ent"]), k, 2], self.limit, g),
                "rel_emb": self._uniform([len(self.metadata["ind2rel"]), k], self.limit, g),
            }
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()

    def _check_model_weights(self, model_weights):
        assert model_weights.get("ent_emb") is not None, "entity embedding should be given in model_weights with key 'ent_emb'"
        assert model_weights.get("rel_emb") is not None, "relation embedding should be given in model_weights with key 'rel_emb'"
        assert list(model_weights["ent_emb"].shape) == [len(self.metadata["ind2ent"]), self.embedding_params["embedding_size"], 2], \
            "shape of 'ent_emb' should be (len(metadata['ind2ent']), embedding_params['embedding_size'], 2)"
        assert list(model_weights["rel_emb"].shape) == [len(self.metadata["ind2rel"]), self.embedding_params["embedding_size"]], \
            "shape of 'rel_emb' should be (len(metadata['ind2rel']), embedding_params['embedding_size'])"

    def _fused_tables(self):
        if not hasattr(self, "limit"):
            self._set_limit()
        return {"ent": self.model_weights["ent_emb"], "rel": self.model_weights["rel_emb"],
                "dim": self.embedding_params["embedding_size"], "limit": self.limit}

    def score_hrt(self, h, r, t):
        """``RotatE.py:126-165``."""
        if not hasattr(self, "limit"):
            self._set_limit()
        h, r, t = super(RotatE, self).score_hrt(h, r, t)
        h_emb = self._lookup("ent_emb", h)
        r_emb = self._lookup("rel_emb", r)
        t_emb = self._lookup("ent_emb", t)
        if h_emb.dim() == 2:
            h_emb = h_emb.unsqueeze(0)
        if t_emb.dim() == 2:
            t_emb = t_emb.unsqueeze(0)
        r_emb = r_emb / self.limit * np.float32(np.pi)
        hadamard = torch.complex(h_emb[..., 0], h_emb[..., 1]) * torch.complex(torch.cos(r_emb), torch.sin(r_emb))
        return self.score_fn(hadamard, torch.complex(t_emb[..., 0], t_emb[..., 1]))

    def _constraint_loss(self, X):
        return 0
