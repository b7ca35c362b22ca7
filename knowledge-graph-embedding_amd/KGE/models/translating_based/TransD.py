"""TransD (reference ``KGE/models/translating_based/TransD.py``).

``M = r_p e_p^T + I``, ``e_perp = M e`` (clipped to norm <= 1 when
``constraint``), ``f = s(h_perp + r, t_perp)``; default ``LpDistancePow(p=2)``;
``constraint`` clips every entity / relation row each step.
"""

import numpy as np
import torch

from ... import _hip
from ...constraint import clip_constraint
from ...loss import PairwiseHingeLoss
from ...ns_strategy import UniformStrategy
from ...score import LpDistancePow
from ..base_model.TranslatingModel import TranslatingModel


class TransD(TranslatingModel):
    _fused_model_id = _hip.MODEL_TRANSD

    def __init__(self, embedding_params, negative_ratio, corrupt_side, score_fn=LpDistancePow(p=2),
                 loss_fn=PairwiseHingeLoss(margin=1), ns_strategy=UniformStrategy, constraint=True, n_workers=1):
        super(TransD, self).__init__(embedding_params, negative_ratio, corrupt_side, score_fn, loss_fn,
                                     ns_strategy, n_workers)
        self.constraint = constraint

    def _init_embeddings(self, seed):
        """``TransD.py:105-146``."""
        if self._model_weights_initial is None:
            assert self.embedding_params.get("ent_embedding_size") is not None, "'ent_embedding_size' should be given in embedding_params when using TransR"
            assert self.embedding_params.get("rel_embedding_size") is not None, "'rel_embedding_size' should be given in embedding_params when using TransR"
            ke, kr = self.embedding_params["ent_embedding_size"], self.embedding_params["rel_embedding_size"]
            E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
            g = self._generator(seed)
            le, lr = np.sqrt(6.0 / ke), np.sqrt(6.0 / kr)
            self.model_weights = {"ent_emb": self._uniform([E, ke], le, g),
                                  "rel_emb": self._uniform([R, kr], lr, g),
                                  "ent_proj": self._uniform([E, ke], le, g),
                                  "rel_proj": self._uniform([R, kr], lr, g)}
        else:
            self._check_model_weights(self._model_weights_initial)
            self.model_weights = self._initial_weights()

    def _check_model_weights(self, model_weights):
        ke, kr = self.embedding_params["ent_embedding_size"], self.embedding_params["rel_embedding_size"]
        E, R = len(self.metadata["ind2ent"]), len(self.metadata["ind2rel"])
        for k in ("ent_emb", "rel_emb", "ent_proj", "rel_proj"):
            assert model_weights.get(k) is not None, "%s should be given in model_weights" % k
        assert list(model_weights["ent_emb"].shape) == [E, ke], "shape of 'ent_emb' should be (len(metadata['ind2ent']), embedding_params['ent_embedding_size'])"
        assert list(model_weights["rel_emb"].shape) == [R, kr], "shape of 'rel_emb' should be (len(metadata['ind2rel']), embedding_params['rel_embedding_size'])"
        assert list(model_weights["ent_proj"].shape) == [E, ke], "shape of 'ent_proj' should be (len(metadata['ind2ent']), embedding_params['ent_embedding_size'])"
        assert list(model_weights["rel_proj"].shape) == [R, kr], "shape of 'rel_proj' should be (len(metadata['ind2rel']), embedding_params['rel_embedding_size'])"

    def _fused_tables(self):
        return {"ent": self.model_weights["ent_emb"], "rel": self.model_weights["rel_emb"],
                "ent_aux": self.model_weights["ent_proj"], "rel_aux": self.model_weights["rel_proj"],
                "dim": self.embedding_params["ent_embedding_size"],
                "dim_rel": self.embedding_params["rel_embedding_size"]}

    def score_hrt(self, h, r, t):
        """``TransD.py:170-222``."""
        h, r, t = super(TransD, self).score_hrt(h, r, t)
        ke, kr = self.embedding_params["ent_embedding_size"], self.embedding_params["rel_embedding_size"]
        h_emb = self._lookup("ent_emb", h).unsqueeze(-1)
        r_emb = self._lookup("rel_emb", r)
        t_emb = self._lookup("ent_emb", t).unsqueeze(-1)
        h_p = self._lookup("ent_proj", h).unsqueeze(-1)
        r_p = self._lookup("rel_proj", r).unsqueeze(-1)
        t_p = self._lookup("ent_proj", t).unsqueeze(-1)
        if h_p.dim() < 3:
            h_p = h_p.unsqueeze(0)
        if r_p.dim() < 3:
            r_p = r_p.unsqueeze(0)
        if t_p.dim() < 3:
            t_p = t_p.unsqueeze(0)
        eye = torch.eye(kr, ke, dtype=torch.float32, device=r_p.device)
        h_m = torch.matmul(r_p, h_p.transpose(1, 2)) + eye
        t_m = torch.matmul(r_p, t_p.transpose(1, 2)) + eye
        h_proj = torch.matmul(h_m, h_emb).squeeze(-1)
        t_proj = torch.matmul(t_m, t_emb).squeeze(-1)
        if self.constraint:
            h_proj = clip_constraint(X=h_proj, p=2, axis=-1, value=1)
            t_proj = clip_constraint(X=t_proj, p=2, axis=-1, value=1)
        return self.score_fn(h_proj + r_emb, t_proj)

    def _constraint_loss(self, X):
        """``TransD.py:224-242``."""
        if self.constraint:
            self._assign("ent_emb", clip_constraint(X=self.model_weights["ent_emb"].detach(), p=2, axis=-1, value=1))
            self._assign("rel_emb", clip_constraint(X=self.model_weights["rel_emb"].detach(), p=2, axis=-1, value=1))
        return 0
