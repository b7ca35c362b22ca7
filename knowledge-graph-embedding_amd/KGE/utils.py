"""Misc helpers (reference ``KGE/utils.py:6-25``)."""

import os
import shutil
import stat

import numpy as np


def check_path_exist_and_create(path):
    """Recreate ``path`` empty (``utils.py:6-9``)."""
    if os.path.exists(path):
        rmtree(path)
    os.makedirs(path)


def ns_with_same_type(x, metadata, negative_ratio):
    """Host restatement of ``utils.py:11-16``: ``negative_ratio`` draws (with
    replacement, numpy global RNG) from ``type2inds[ind2type[x]]`` minus ``x``.

    Kept for API compatibility; the fused path draws the same distribution on
    device with the counter-based sampler (``ns_strategy.TypedStrategy``).
    """
    sample_pool = metadata["type2inds"][metadata["ind2type"][x]]
    sample_pool = np.delete(sample_pool, np.where(sample_pool == x), axis=0)
    return np.random.choice(sample_pool, size=negative_ratio)


def rmtree(top):
    """Remove a directory tree even where files are read-only (``utils.py:18-25``):
    a failed unlink gets write permission and is retried once."""
    def _retry(func, path, _exc):
        os.chmod(path, stat.S_IWUSR | stat.S_IRUSR | stat.S_IXUSR)
        func(path)
    shutil.rmtree(top, onerror=_retry)
