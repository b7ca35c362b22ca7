"""Translating-based model base (reference ``TranslatingModel.py:5-70``)."""

from .BaseModel import KGEModel


class TranslatingModel(KGEModel):
    """Adds the ``score_fn`` plugin (``TranslatingModel.py:46-70``)."""

    def __init__(self, embedding_params, negative_ratio, corrupt_side, score_fn, loss_fn, ns_strategy,
                 n_workers):
        super(TranslatingModel, self).__init__(embedding_params, negative_ratio, corrupt_side, loss_fn,
                                               ns_strategy, n_workers)
        self.score_fn = score_fn
