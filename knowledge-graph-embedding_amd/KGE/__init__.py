"""KGE -- MI355X-native knowledge-graph-embedding training.

Drop-in for the plugin surface of melissakou/knowledge-graph-embedding
(``KGE.models.*``, ``KGE.score``, ``KGE.loss``, ``KGE.ns_strategy``,
``KGE.constraint``, ``KGE.metrics``, ``KGE.data_utils``) on PyTorch-ROCm
tensors; the training step runs as hand-written HIP kernels
(``libkge_hip.so``, C-ABI in ``include/kge_hip.h``).
"""

__version__ = "0.1.0"
