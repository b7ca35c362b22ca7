"""TransR (reference ``KGE/models/translating_based/TransR.py``).

``h_perp = h^T M_r`` with ``M_r`` of shape ``[ent_k, rel_k]`` (initialised to
identity), projected vectors clipped to norm <= 1 when ``constraint``; default
``LpDistancePow(p=2)``; ``constraint`` also clips every entity / relation row
each step (``TransR.py:193-211``).
"""

import numpy as np
import torch

from ... import _hip
from ...constraint import clip_constraint
from ...loss import PairwiseHingeLoss
from ...ns_strategy import UniformStrategy
from ...score import LpDistancePow
from ..base_model.TranslatingModel import TranslatingModel


class TransR(TranslatingModel):
    _fused_model_id = _hip.MODEL_TRANSR

    def __init__(self, embedding_params, negative_ratio, corrupt_side, score_fn=LpDistancePow(p=2),
                 loss_fn=PairwiseHingeLoss(margin=1), ns_strategy=UniformStrategy, constraint=True, n_workers=1):
        super(TransR, self).__init__(embedding_params, negative_ratio, corrupt_side, score_fn, loss_fn,
                                     ns_strategy, n_workers)
        self.constraint = constraint

    def _init_embeddings(self, seed):
        """``TransR.py:95-133``."""
        if self._model_weights_initial is None:
            assert self.embedding_params.get("ent_embedding_size") is not None, "'ent_embedding_size' should be given in embedding_params when using TransR"
            assert self.embedding_params.get("rel_embedding_size") is not None, "'rel_embedding_size' should be given in embedding_params when using TransR"
            ke, kr = self.embedding_params["ent_embedding_size"], self.embedding_params["rel_embedding_size"]
            E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
            g = self._generator(seed)
            ent = self._uniform([E, ke], np.sqrt(6.0 / ke), g)
            rel = self._uniform([R, kr], np.sqrt(6.0 / kr), g)
            proj = torch.eye(ke, kr, dtype=torch.float32).unsqueeze(0).repeat(R, 1, 1).to(ent.device)
            self.model_weights = {"ent_emb": ent, "rel_emb": rel, "rel_proj": proj}
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()

    def _check_model_weights(self, model_weights):
        ke, kr = self.embedding_params["ent_embedding_size"], self.embedding_params["rel_embedding_size"]
        E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
        assert model_weights.get("ent_emb") is not None, "entity embedding should be given in model_weights with key 'ent_emb'"
        assert model_weights.get("rel_emb") is not None, "relation embedding should be given in model_weights with key 'rel_emb'"
        assert model_weights.get("rel_proj") is not None, "relation projection matrix should be given in model_weights with key 'rel_proj'"
        assert list(model_weights["ent_emb"].shape) == [E, ke], "shape of 'ent_emb' should be (len(metadata['ind2ent']), embedding_params['ent_embedding_size'])"
        assert list(model_weights["rel_emb"].shape) == [R, kr], "shape of 'rel_emb' should be (len(metadata['ind2rel']), embedding_params['rel_embedding_size'])"
        assert list(model_weights["rel_proj"].shape) == [R, ke, kr], "shape of 'rel_emb' should be (len(metadata['ind2rel']), embedding_params['ent_embedding_size'], embedding_params['rel_embedding_size'])"

    def _fused_tables(self):
        return {"ent": self.model_weights["ent_emb"], "rel": self.model_weights["rel_emb"],
                "rel_aux": self.model_weights["rel_proj"], "dim": self.embedding_params["ent_embedding_size"],
                "dim_rel": self.embedding_params["rel_embedding_size"]}

    def score_hrt(self, h, r, t):
        """``TransR.py:154-191``."""
        h, r, t = super(TransR, self).score_hrt(h, r, t)
        h_emb = self._lookup("ent_emb", h)
        r_emb = self._lookup("rel_emb", r)
        t_emb = self._lookup("ent_emb", t)
        r_proj = self._lookup("rel_proj", r)
        h_proj = torch.matmul(h_emb.unsqueeze(-2), r_proj).squeeze(-2)
        t_proj = torch.matmul(t_emb.unsqueeze(-2), r_proj).squeeze(-2)
        if self.constraint:
            h_proj = clip_constraint(X=h_proj, p=2, axis=-1, value=1)
            t_proj = clip_constraint(X=t_proj, p=2, axis=-1, value=1)
        return self.score_fn(h_proj + r_emb, t_proj)

    def _constraint_loss(self, X):
        """``TransR.py:193-211``."""
        if self.constraint:
            self._assign("ent_emb", clip_constraint(X=self.model_weights["ent_emb"].detach(), p=2, axis=-1, value=1))
            self._assign("rel_emb", clip_constraint(X=self.model_weights["rel_emb"].detach(), p=2, axis=-1, value=1))
        return 0
