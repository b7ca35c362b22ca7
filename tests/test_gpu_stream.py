"""GPU: the device input stream (kge_stream_batch, csrc/kge_stream.hip; SURVEY
§8 f2, data_utils.py:176-196) against the oracle's scalar restatement at small
sizes, the host numpy restatement at FB15k-237 size, and size-independent
properties at full size (every epoch a permutation; batches = data rows).
Integer work: bit-exact."""

import numpy as np
import pytest
import torch

from oracle import kge_oracle as O

pytestmark = pytest.mark.gpu
SEED = 0x0123456789ABCDEF


@pytest.fixture(autouse=True)
def _gpu(hiplib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _stream(data, start, batch, shuffle, seed=SEED):
    import ctypes
    from KGE import _hip
    L = _hip.load()
    out = torch.full((batch, 3), -1, dtype=data.dtype, device=data.device)
    d = _hip.kge_stream_desc()
    d.abi_version = _hip.ABI_VERSION
    d.idx_dtype = _hip.IDX_I64 if data.dtype == torch.int64 else _hip.IDX_I32
    d.triples = data.data_ptr()
    d.n_rows = data.shape[0]
    d.start = start
    d.batch = batch
    d.seed = seed
    d.shuffle = shuffle
    d.out = out.data_ptr()
    _hip.check(L.kge_stream_batch(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
               "kge_stream_batch")
    torch.cuda.synchronize()
    return out


def _triples(n, dtype):
    return (torch.arange(n * 3, dtype=torch.int64).reshape(n, 3) % (2 ** 31 - 1)).to(dtype).cuda()


@pytest.mark.parametrize("dtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("n", [1, 2, 7, 64, 1001])
@pytest.mark.parametrize("shuffle", [0, 1])
def test_stream_matches_oracle(dtype, n, shuffle):
    data = _triples(n, dtype)
    for start in (0, n - 1, 5 * n + 3):
        cnt = min(3 * n + 5, 600)
        out = _stream(data, start, cnt, shuffle)
        rows = torch.tensor(O.stream_rows(n, SEED, start, cnt, shuffle), device="cuda")
        assert torch.equal(out, data[rows])


def test_stream_fb15k237_size_matches_host():
    """272,115 rows (FB15k-237 train), a 2^20-row batch straddling 4 epochs."""
    from KGE import _philox
    n = 272115
    data = _triples(n, torch.int64)
    start = 5 * n - 7
    out = _stream(data, start, 1 << 20, 1)
    rows = torch.from_numpy(_philox.stream_rows(n, SEED, start, 1 << 20, 1)).cuda()
    assert torch.equal(out, data[rows])


def test_stream_full_size_epoch_is_permutation():
    """3,000,017 rows: one epoch's source rows (column 0 / 3) sort to 0..n-1,
    the next epoch's differ."""
    n = 3_000_017
    data = _triples(n, torch.int64)
    e2 = _stream(data, 2 * n, n, 1)[:, 0] // 3
    assert torch.equal(torch.sort(e2).values, torch.arange(n, device="cuda"))
    e3 = _stream(data, 3 * n, n, 1)[:, 0] // 3
    assert not torch.equal(e2, e3)
    assert torch.equal(_stream(data, 2 * n + 11, 1000, 0)[:, 0] // 3, torch.arange(11, 1011, device="cuda"))


def test_device_batcher_matches_cpu_batcher():
    from KGE.data_utils import set_tf_iterator
    X = np.random.default_rng(0).integers(0, 1000, (1234, 3))
    gpu = set_tf_iterator(X, 500, shuffle=True, buffer_size=len(X), seed=9, device=torch.device("cuda", 0))
    cpu = set_tf_iterator(X, 500, shuffle=True, buffer_size=len(X), seed=9)
    for _ in range(6):   # 3000 rows: straddles two epoch boundaries
        g = next(gpu)
        assert g.is_cuda and g.dtype == torch.int64
        assert torch.equal(g.cpu(), next(cpu))


def _stream_perm(data, start, batch, seed=SEED, cache=None):
    """kge_stream_permutation + kge_stream_batch_perm (the DeviceBatcher path)."""
    import ctypes
    from KGE import _hip
    L = _hip.load()
    n = data.shape[0]
    out = torch.full((batch, 3), -1, dtype=data.dtype, device=data.device)
    d = _hip.kge_stream_desc()
    d.abi_version = _hip.ABI_VERSION
    d.idx_dtype = _hip.IDX_I64 if data.dtype == torch.int64 else _hip.IDX_I32
    d.triples = data.data_ptr()
    d.n_rows = n
    d.start = start
    d.batch = batch
    d.seed = seed
    d.shuffle = 1
    d.out = out.data_ptr()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    e0, e1 = start // n, (start + batch - 1) // n
    perms = {}
    for e in (e0, e1):
        perms[e] = torch.full((n,), -1, dtype=torch.int32, device=data.device)
        _hip.check(L.kge_stream_permutation(ctypes.byref(d), e, ctypes.c_void_p(perms[e].data_ptr()), st),
                   "kge_stream_permutation")
    _hip.check(L.kge_stream_batch_perm(ctypes.byref(d), ctypes.c_void_p(perms[e0].data_ptr()),
                                       ctypes.c_void_p(perms[e1].data_ptr()), e0, st), "kge_stream_batch_perm")
    torch.cuda.synchronize()
    return out, perms


@pytest.mark.parametrize("dtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("n", [1, 7, 1001, 272115])
def test_stream_perm_path_equals_per_row_walk(dtype, n):
    """The materialised-permutation path gives kge_stream_batch's rows, bit for
    bit, for batches inside one epoch and straddling two."""
    data = _triples(n, dtype)
    for start, cnt in ((0, n), (3 * n + n // 2, n), (7 * n - 1, 1), (2 * n + 1, max(1, n // 3))):
        out, perms = _stream_perm(data, start, cnt)
        assert torch.equal(out, _stream(data, start, cnt, 1))
        for e, p in perms.items():   # each table is a permutation of [0, n)
            assert torch.equal(torch.sort(p.long()).values, torch.arange(n, device="cuda"))


def test_stream_perm_matches_oracle_small():
    n = 64
    data = _triples(n, torch.int64)
    out, _ = _stream_perm(data, 5 * n + 3, 50)
    rows = torch.tensor(O.stream_rows(n, SEED, 5 * n + 3, 50, 1), device="cuda")
    assert torch.equal(out, data[rows])


def test_stream_perm_rejects_bad_epochs():
    import ctypes
    from KGE import _hip
    L = _hip.load()
    n = 100
    data = _triples(n, torch.int64)
    out = torch.empty((60, 3), dtype=torch.int64, device="cuda")
    perm = torch.empty(n, dtype=torch.int32, device="cuda")
    d = _hip.kge_stream_desc()
    d.abi_version = _hip.ABI_VERSION
    d.idx_dtype = _hip.IDX_I64
    d.triples = data.data_ptr()
    d.n_rows = n
    d.start = 70          # straddles epochs 0 and 1
    d.batch = 60
    d.seed = SEED
    d.shuffle = 1
    d.out = out.data_ptr()
    p = ctypes.c_void_p(perm.data_ptr())
    assert L.kge_stream_batch_perm(ctypes.byref(d), p, None, 0, None) == _hip.KGE_EINVAL     # perm_hi missing
    assert L.kge_stream_batch_perm(ctypes.byref(d), p, p, 1, None) == _hip.KGE_EINVAL        # wrong epoch_lo
    d.shuffle = 0
    assert L.kge_stream_permutation(ctypes.byref(d), 0, p, None) == _hip.KGE_EINVAL


def test_device_batcher_uses_perm_path_and_matches_host():
    """DeviceBatcher (the train() iterator) on FB15k-237 size: three epochs of
    batches equal the host restatement, through the materialised tables."""
    from KGE import _philox
    from KGE.data_utils import DeviceBatcher
    n = 272115
    host = (torch.arange(n * 3, dtype=torch.int64).reshape(n, 3))
    it = DeviceBatcher(host, 100000, shuffle=True, seed=SEED, device=torch.device("cuda"), reuse_buffer=True)
    for b in range(9):
        out = next(it).clone()
        rows = torch.from_numpy(_philox.stream_rows(n, SEED, b * 100000, 100000, 1)).cuda()
        assert torch.equal(out, host.cuda()[rows])
    assert len(it._perms) <= 2


@pytest.mark.parametrize("n,B,G", [(272115, 1024, 32), (700, 64, 10), (1000, 100, 7)])
def test_device_batcher_ring_equals_batch_by_batch(n, B, G):
    """DeviceBatcher(chunk=G) (train()'s ring: G batches per gather launch)
    hands out the same batches as chunk=1, across epoch boundaries, as views
    of one ring tensor in order."""
    from KGE.data_utils import DeviceBatcher
    host = torch.arange(n * 3, dtype=torch.int64).reshape(n, 3)
    dev = torch.device("cuda")
    a = DeviceBatcher(host, B, shuffle=True, seed=SEED, device=dev, reuse_buffer=True, chunk=G)
    b = DeviceBatcher(host, B, shuffle=True, seed=SEED, device=dev, reuse_buffer=True)
    assert a.chunk == G
    steps = max(3 * G + 1, 3 * n // B + 2)
    for s in range(steps):
        x, y = next(a), next(b)
        assert x._base is a._ring and x.is_contiguous()
        assert torch.equal(x, y), s
    assert len(a._perms) <= 2
