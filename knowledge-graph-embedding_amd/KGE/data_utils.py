"""Data utilities (reference ``KGE/data_utils.py:12-196``).

``index_kg`` / ``convert_kg_to_index`` / ``train_test_split_no_unseen`` /
``calculate_data_size`` keep the reference's behaviour on numpy arrays and CSV
folders. ``set_tf_iterator`` is replaced by a device-resident batcher with the
same stream semantics as ``tf.data ... shuffle(n, seed,
reshuffle_each_iteration=True).repeat().batch(B)`` (``data_utils.py:176-196``):
every batch has exactly ``batch_size`` rows and batches straddle epoch
boundaries; CSV folders give int32 triples, numpy input keeps its dtype
(int64), as ``CsvDataset(record_defaults=[tf.int32]*3)`` /
``from_tensor_slices`` do.
"""

import logging
import os

import numpy as np
import pandas as pd
import torch

from .utils import check_path_exist_and_create


def index_kg(kg_data):
    """Index a KG (``data_utils.py:23-62``).

    numpy input: sorted ``np.unique`` of entities / relations. CSV folder:
    first-appearance order over files (``pd.unique``), files in
    ``os.listdir`` order.
    """
    if isinstance(kg_data, np.ndarray):
        entities = list(np.unique(np.append(kg_data[:, 0], kg_data[:, 2])))
        relations = list(np.unique(kg_data[:, 1]))
    else:
        ent_parts, rel_parts = [], []
        for f in os.listdir(kg_data):
            tmp = pd.read_csv(os.path.join(kg_data, f), header=None, dtype=str)
            ent_parts += [tmp.iloc[:, 0], tmp.iloc[:, 2]]
            rel_parts.append(tmp.iloc[:, 1])
        entities = list(pd.unique(pd.concat(ent_parts, ignore_index=True))) if ent_parts else []
        relations = list(pd.unique(pd.concat(rel_parts, ignore_index=True))) if rel_parts else []

    ent2ind = {e: i for i, e in enumerate(entities)}
    ind2ent = [e for e in entities]
    rel2ind = {r: i for i, r in enumerate(relations)}
    ind2rel = [r for r in relations]
    return {"ent2ind": ent2ind, "ind2ent": ind2ent, "rel2ind": rel2ind, "ind2rel": ind2rel}


def convert_kg_to_index(kg_data, ent2ind, rel2ind):
    """Map string triples to ids (``data_utils.py:65-99``)."""
    if isinstance(kg_data, np.ndarray):
        h = list(map(ent2ind.get, list(kg_data[:, 0])))
        r = list(map(rel2ind.get, list(kg_data[:, 1])))
        t = list(map(ent2ind.get, list(kg_data[:, 2])))
        return np.array([h, r, t]).T
    filenames = os.listdir(kg_data)
    check_path_exist_and_create(kg_data + "_indexed")
    for f in filenames:
        tmp = pd.read_csv(kg_data + "/" + f, header=None, dtype=str)
        tmp.iloc[:, 0] = tmp.iloc[:, 0].map(ent2ind)
        tmp.iloc[:, 1] = tmp.iloc[:, 1].map(rel2ind)
        tmp.iloc[:, 2] = tmp.iloc[:, 2].map(ent2ind)
        tmp.to_csv(kg_data + "_indexed/" + f, index=False, header=False)
    logging.info("indexed_kg has been save to %s" % kg_data + "_indexed")


def train_test_split_no_unseen(X, test_size, seed):
    """Split so every test entity / relation is also in train (``data_utils.py:102-159``)."""
    if isinstance(test_size, float):
        test_size = int(len(X) * test_size)

    e, e_cnt = np.unique(np.append(X[:, 0], X[:, 2]), return_counts=True)
    r, r_cnt = np.unique(X[:, 1], return_counts=True)
    e_dict = dict(zip(e, e_cnt))
    r_dict = dict(zip(r, r_cnt))

    test_id = np.array([], dtype=int)
    train_id = np.arange(len(X))
    loop_count = 0
    max_loop = len(X) * 10
    rnd = np.random.RandomState(seed)
    while len(test_id) < test_size:
        i = rnd.choice(train_id)
        if e_dict[X[i, 0]] > 1 and r_dict[X[i, 1]] > 1 and e_dict[X[i, 2]] > 1:
            e_dict[X[i, 0]] -= 1
            r_dict[X[i, 1]] -= 1
            e_dict[X[i, 2]] -= 1
            test_id = np.unique(np.append(test_id, i))
        loop_count += 1
        if loop_count == max_loop:
            logging.error("Cannot split a test set with desired size, please reduce the test size")
            return
    train_id = np.setdiff1d(train_id, test_id)
    return X[train_id], X[test_id]


def calculate_data_size(X):
    """Number of triples in an array or CSV folder (``data_utils.py:162-173``)."""
    if isinstance(X, str):
        total = 0
        for f in os.listdir(X):
            total += len(pd.read_csv(os.path.join(X, f), header=None))
        return total
    return len(X)


def load_triples(data):
    """numpy / tensor / ``.npy`` file / CSV folder -> host int tensor [n, 3].

    CSV folders are read as int32 (the reference's CsvDataset defaults,
    ``data_utils.py:182``); arrays keep an integer dtype (numpy default int64).
    """
    if isinstance(data, str) and data.endswith(".npy") and os.path.isfile(data):
        data = np.load(data, allow_pickle=False)
    if isinstance(data, str):
        parts = [pd.read_csv(os.path.join(data, f), header=None, dtype=np.int32).values
                 for f in sorted(os.listdir(data))]
        arr = np.concatenate(parts, axis=0) if parts else np.zeros((0, 3), np.int32)
        return torch.from_numpy(np.ascontiguousarray(arr.astype(np.int32)))
    if isinstance(data, torch.Tensor):
        return data.detach().cpu()
    arr = np.asarray(data)
    if arr.dtype.kind not in "iu":
        arr = arr.astype(np.int64)
    if arr.dtype not in (np.int32, np.int64):
        arr = arr.astype(np.int64)
    return torch.from_numpy(np.ascontiguousarray(arr))


class DeviceBatcher:
    """Device-resident ``shuffle -> repeat -> batch`` stream.

    The triples stay resident on ``device``. Batch ``b`` is stream positions
    ``[b B, (b + 1) B)``; position ``p`` is row ``pi_e(p mod n)`` of epoch
    ``e = p div n``, so every batch has exactly ``batch_size`` rows and
    batches straddle epochs like ``repeat().batch()``. ``pi_e`` is a fresh
    permutation per epoch when shuffling (``reshuffle_each_iteration``): the
    stateless Philox-keyed Feistel permutation of ``kge_stream_desc``
    (``include/kge_hip.h``). On the GPU each epoch's permutation is
    materialised once (``kge_stream_permutation``, int32 [n]) and a batch is a
    gather through it (``kge_stream_batch_perm``); ``kge_stream_batch``
    computes the same rows per output row without the table (tiny sets whose
    batch spans more than two epochs). No host work per batch. On a
    CPU device the same rows come from the numpy restatement in
    ``_philox.stream_rows``. tf.data's buffered shuffle order itself is not
    reproducible (TF is not installed); the stream semantics are.
    """

    def __init__(self, data, batch_size, shuffle, seed=None, device=None, reuse_buffer=False, chunk=1):
        """``reuse_buffer``: every batch is written into the same device buffer
        (the caller consumes a batch before drawing the next -- the training
        loop; stream order makes the overwrite safe), saving an allocation
        per batch. ``chunk`` (with ``reuse_buffer``, shuffled, on the GPU):
        ``chunk`` consecutive batches are gathered by one launch into a ring
        and handed out as views of it, in order (the caller consumes them in
        stream order, as above); the rows are the same as batch by batch."""
        host = load_triples(data)
        if host.dtype not in (torch.int32, torch.int64):
            host = host.to(torch.int64)
        self.n = host.shape[0]
        if self.n == 0:
            raise ValueError("empty triple set")
        self.batch_size = int(batch_size)
        if self.batch_size <= 0:
            raise ValueError("batch_size must be > 0")
        self.shuffle = bool(shuffle)
        self.device = device if device is not None else torch.device("cpu")
        self.data = host.contiguous().to(self.device)
        self.seed = int(seed) if seed is not None else int.from_bytes(os.urandom(8), "little")
        self.seed &= (1 << 64) - 1
        self._pos = 0   # stream position of the next batch's first row
        self.reuse_buffer = bool(reuse_buffer)
        self._desc = None
        self._out = None
        self._perms = {}   # epoch -> its materialised permutation (device int32 [n])
        self._spare = []
        self._fast = None  # reused buffer: (e0, e1, entry, perm e0, perm e1, stream) of the last batch
        # ring of `chunk` batches filled by one gather (a window spans at most two epochs)
        self.chunk = int(chunk) if (self.reuse_buffer and self.shuffle and self.device.type == "cuda" and
                                    int(chunk) > 1 and int(chunk) * self.batch_size <= self.n) else 1
        self._ring = None
        self._ring_views = None
        self._slot = 0

    def __iter__(self):
        return self

    def rows(self, start, count):
        """Source row indices of stream positions [start, start + count) (host int64)."""
        from ._philox import stream_rows
        return stream_rows(self.n, self.seed, start, count, self.shuffle)

    def __next__(self):
        if self.chunk > 1:
            if self._ring is None or self._slot == self.chunk:
                self._fill_ring()
            v = self._ring_views[self._slot]
            self._slot += 1
            return v
        start, B = self._pos, self.batch_size
        f = self._fast
        if f is not None and start // self.n == f[0] and (start + B - 1) // self.n == f[1]:
            # the common case of a reused buffer: the same epoch pair as the last
            # batch -- one kge_stream_batch_perm call on the stream that batch used
            self._pos = start + B
            self._desc.start = start
            rc = f[2](self._dref, f[3], f[4], f[0], f[5])
            if rc:
                from . import _hip
                _hip.check(rc, "kge_stream_batch_perm")
            return self._out
        self._pos += B
        if self.data.is_cuda:
            import ctypes
            from . import _hip
            L = _hip.load()
            if self.reuse_buffer and self._out is not None:
                out = self._out
            else:
                out = torch.empty((B, 3), dtype=self.data.dtype, device=self.data.device)
                if self.reuse_buffer:
                    self._out = out
            d = self._desc
            if d is None:   # the descriptor is built once; a batch changes start and out
                d = _hip.kge_stream_desc()
                d.abi_version = _hip.ABI_VERSION
                d.idx_dtype = _hip.IDX_I64 if self.data.dtype == torch.int64 else _hip.IDX_I32
                d.triples = self.data.data_ptr()
                d.n_rows = self.n
                d.batch = B
                d.seed = self.seed
                d.shuffle = 1 if self.shuffle else 0
                self._desc = d
                self._dref = ctypes.byref(d)
            d.start = start
            d.out = out.data_ptr()
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.data.device).cuda_stream)
            if self.shuffle and B <= self.n and self.n <= 2 ** 31 - 1:
                # each epoch's permutation materialised once (kge_stream_permutation),
                # the batch gathered through it: the same rows as kge_stream_batch
                # without a per-batch cycle walk
                e0, e1 = start // self.n, (start + B - 1) // self.n
                perms = self._perms
                for e in list(perms):
                    if e < e0:   # (reused on this stream: stream order keeps it safe)
                        self._spare.append(perms.pop(e))
                for e in (e0, e1):
                    if e not in perms:
                        t = self._spare.pop() if self._spare else torch.empty(self.n, dtype=torch.int32,
                                                                                device=self.data.device)
                        _hip.check(L.kge_stream_permutation(self._dref, e, ctypes.c_void_p(t.data_ptr()), stream),
                                   "kge_stream_permutation")
                        perms[e] = t
                p0, p1 = ctypes.c_void_p(perms[e0].data_ptr()), ctypes.c_void_p(perms[e1].data_ptr())
                _hip.check(L.kge_stream_batch_perm(self._dref, p0, p1, e0, stream), "kge_stream_batch_perm")
                if self.reuse_buffer:   # (the permutation tensors stay in self._perms while e0 / e1 are current)
                    self._fast = (e0, e1, L.kge_stream_batch_perm, p0, p1, stream)
                return out
            _hip.check(L.kge_stream_batch(self._dref, stream), "kge_stream_batch")
            return out
        idx = torch.from_numpy(self.rows(start, B))
        return self.data.index_select(0, idx)


    def _fill_ring(self):
        """The next ``chunk`` batches, one kge_stream_batch_perm launch over
        stream positions [pos, pos + chunk B) into the ring (the same rows the
        batch-by-batch calls give: the window is one stretch of the stream)."""
        import ctypes
        from . import _hip
        L = _hip.load()
        G, B = self.chunk, self.batch_size
        if self._ring is None:
            self._ring = torch.empty((G * B, 3), dtype=self.data.dtype, device=self.data.device)
            self._ring_views = [self._ring[i * B:(i + 1) * B] for i in range(G)]
            d = _hip.kge_stream_desc()
            d.abi_version = _hip.ABI_VERSION
            d.idx_dtype = _hip.IDX_I64 if self.data.dtype == torch.int64 else _hip.IDX_I32
            d.triples = self.data.data_ptr()
            d.n_rows = self.n
            d.batch = G * B
            d.seed = self.seed
            d.shuffle = 1
            d.out = self._ring.data_ptr()
            self._ring_desc = d
            self._ring_dref = ctypes.byref(d)
        start = self._pos
        self._pos = start + G * B
        self._slot = 0
        d = self._ring_desc
        d.start = start
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.data.device).cuda_stream)
        e0, e1 = start // self.n, (start + G * B - 1) // self.n
        perms = self._perms
        for e in list(perms):
            if e < e0:   # (reused on this stream: stream order keeps it safe)
                self._spare.append(perms.pop(e))
        for e in (e0, e1):
            if e not in perms:
                t = self._spare.pop() if self._spare else torch.empty(self.n, dtype=torch.int32, device=self.data.device)
                _hip.check(L.kge_stream_permutation(self._ring_dref, e, ctypes.c_void_p(t.data_ptr()), stream),
                           "kge_stream_permutation")
                perms[e] = t
        _hip.check(L.kge_stream_batch_perm(self._ring_dref, ctypes.c_void_p(perms[e0].data_ptr()),
                                           ctypes.c_void_p(perms[e1].data_ptr()), e0, stream), "kge_stream_batch_perm")


def set_tf_iterator(data, batch_size, shuffle, buffer_size=None, seed=None, device=None, reuse_buffer=False, chunk=1):
    """Drop-in for ``set_tf_iterator`` (``data_utils.py:176-196``)."""
    if shuffle:
        assert buffer_size is not None, "buffer_size must be given when shuffle is True"
    return DeviceBatcher(data, batch_size, shuffle, seed=seed, device=device, reuse_buffer=reuse_buffer, chunk=chunk)
