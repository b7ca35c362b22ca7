"""Semantic-based model base (reference ``SemanticModel.py:5-64``)."""

from .BaseModel import KGEModel


class SemanticModel(KGEModel):
    def __init__(self, embedding_params, negative_ratio, corrupt_side, loss_fn, ns_strategy, n_workers):
        super(SemanticModel, self).__init__(embedding_params, negative_ratio, corrupt_side, loss_fn,
                                            ns_strategy, n_workers)
