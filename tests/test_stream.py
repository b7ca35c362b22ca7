"""CPU: the device input stream's spec (``data_utils.py:176-196``
shuffle -> repeat -> batch): the host numpy restatement used on CPU devices
(``KGE/_philox.stream_rows``) against the oracle's scalar restatement, the
per-epoch permutation property, the batcher's stream semantics (exact batch
sizes, epoch straddling, reshuffle per epoch, dtypes of the loaders) and the
C-ABI entry's argument checks (no GPU call)."""

import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import kge_oracle as O

SEED = 0x9E3779B97F4A7C15


def _host():
    from KGE import _philox
    return _philox.stream_rows


@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 256, 1000, 65537])
@pytest.mark.parametrize("shuffle", [0, 1])
def test_host_stream_matches_oracle(n, shuffle):
    for start in (0, n - 1, 3 * n + 2):
        cnt = min(2 * n + 3, 700)
        assert list(_host()(n, SEED, start, cnt, shuffle)) == O.stream_rows(n, SEED, start, cnt, shuffle)


@pytest.mark.parametrize("n", [1, 4, 5, 4097, 272115])
def test_every_epoch_is_a_permutation(n):
    f = _host()
    seen = []
    for e in range(3):
        r = f(n, 12345, e * n, n, 1)
        assert (np.sort(r) == np.arange(n)).all()
        seen.append(r)
    if n > 4:   # reshuffle_each_iteration: epochs differ, seeds differ
        assert not (seen[0] == seen[1]).all()
        assert not (f(n, 1, 0, n, 1) == f(n, 2, 0, n, 1)).all()


def test_no_shuffle_is_epoch_order():
    assert list(_host()(5, SEED, 3, 9, 0)) == [3, 4, 0, 1, 2, 3, 4, 0, 1]


def test_batcher_stream_semantics():
    from KGE.data_utils import set_tf_iterator
    X = np.arange(7 * 3, dtype=np.int64).reshape(7, 3)
    it = set_tf_iterator(X, 3, shuffle=True, buffer_size=7, seed=5)
    got = torch.cat([next(it) for _ in range(7)])          # 21 rows = 3 epochs exactly
    assert got.dtype == torch.int64 and got.shape == (21, 3)
    rows = got[:, 0].numpy() // 3
    for e in range(3):
        assert sorted(rows[7 * e:7 * e + 7]) == list(range(7))   # batches straddle epochs
    assert list(rows) == list(_host()(7, 5, 0, 21, 1))
    again = set_tf_iterator(X, 3, shuffle=True, buffer_size=7, seed=5)
    assert torch.equal(next(again), got[:3])
    it = set_tf_iterator(X, 4, shuffle=False)
    assert next(it)[:, 0].tolist() == [0, 3, 6, 9] and next(it)[:, 0].tolist() == [12, 15, 18, 0]


def test_batcher_loaders_and_errors(tmp_path):
    from KGE.data_utils import set_tf_iterator
    X = np.array([[0, 1, 2], [3, 4, 5]], dtype=np.int64)
    np.save(tmp_path / "t.npy", X)
    assert torch.equal(next(set_tf_iterator(str(tmp_path / "t.npy"), 2, shuffle=False)), torch.from_numpy(X))
    d = tmp_path / "csv"
    d.mkdir()
    np.savetxt(d / "a.csv", X, fmt="%d", delimiter=",")
    b = next(set_tf_iterator(str(d), 2, shuffle=False))
    assert b.dtype == torch.int32 and b.tolist() == X.tolist()   # CsvDataset int32 (data_utils.py:182)
    with pytest.raises(ValueError):
        set_tf_iterator(np.zeros((0, 3), np.int64), 2, shuffle=False)
    with pytest.raises(AssertionError):
        set_tf_iterator(X, 2, shuffle=True)   # buffer_size required (data_utils.py:188)


@pytest.mark.parametrize("field,value,msg", [
    ("n_rows", 0, "n_rows"), ("idx_dtype", 5, "idx_dtype"), ("start", -1, "start"), ("shuffle", 2, "shuffle"),
    ("abi_version", 1, "abi_version")])
def test_stream_abi_rejects_without_gpu(hiplib, field, value, msg):
    from KGE import _hip
    buf = (ctypes.c_int64 * 6)()
    d = _hip.kge_stream_desc()
    d.abi_version = _hip.ABI_VERSION
    d.idx_dtype = _hip.IDX_I64
    d.triples = ctypes.addressof(buf)
    d.n_rows = 2
    d.batch = 1
    d.shuffle = 1
    d.out = ctypes.addressof(buf)
    setattr(d, field, value)
    assert hiplib.kge_stream_batch(ctypes.byref(d), None) == _hip.KGE_EINVAL
    assert msg in hiplib.kge_last_error().decode()


def test_batcher_ring_only_where_it_applies():
    """DeviceBatcher(chunk=G) gathers G batches per launch only on the GPU
    (shuffled, reused buffer, G B <= n: tests/test_gpu_stream.py); on the CPU
    it is the batch-by-batch stream, the same rows."""
    from KGE.data_utils import DeviceBatcher
    host = torch.arange(700 * 3, dtype=torch.int64).reshape(700, 3)
    cpu = torch.device("cpu")
    a = DeviceBatcher(host, 64, shuffle=True, seed=5, device=cpu, reuse_buffer=True, chunk=10)
    b = DeviceBatcher(host, 64, shuffle=True, seed=5, device=cpu)
    assert a.chunk == 1
    for _ in range(25):
        assert torch.equal(next(a), next(b))
