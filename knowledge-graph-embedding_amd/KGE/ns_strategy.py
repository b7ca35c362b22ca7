"""Negative samplers (plugin surface of ``KGE/ns_strategy.py`` in the reference).

``__call__(X, negative_ratio, side) -> [n * negative_ratio]`` with X's dtype,
as in ``ns_strategy.py:39-64`` (uniform) and ``:94-132`` (typed). Both
samplers are counter-based: the object holds (seed, offset) and every call
consumes counter planes, so a run is reproducible from its seed (the
reference never seeds TF's RNG, so its draws are not).

CUDA tensors are sampled by ``kge_sample`` in ``libkge_hip.so``; the fused
training step draws the same ids in-kernel from the same planes. CPU tensors
are refused (RuntimeError) unless the host-development backend is selected
explicitly (``KGE_BACKEND=eager``), which samples on the host with the
identical spec (``_philox.py``): there is no silent CPU fallback.
"""

import os

import numpy as np
import torch

from . import _hip
from . import _philox


def _random_seed():
    return int.from_bytes(os.urandom(8), "little")


class NegativeSampler:
    """Base class (``ns_strategy.py:6-17``)."""

    def __init__(self):
        raise NotImplementedError("subclass of NegativeSampler should implement __init__() to init class")

    def __call__(self):
        raise NotImplementedError("subclass of NegativeSampler should implement __call__() to conduct negative sampling")


class _CounterSampler(NegativeSampler):
    def _init_rng(self, seed):
        self.seed = _random_seed() if seed is None else int(seed) & 0xFFFFFFFFFFFFFFFF
        self.offset = 0

    def reseed(self, seed):
        self._init_rng(seed)

    def take_planes(self, n):
        """Reserve ``n`` consecutive counter planes; returns the first."""
        o = self.offset
        self.offset += int(n)
        return o


class UniformStrategy(_CounterSampler):
    """Uniform entity draws from ``sample_pool`` (``ns_strategy.py:20-64``).

    Draws do not exclude the true entity and do not filter known positives,
    as in the reference.
    """

    def __init__(self, sample_pool, seed=None):
        pool = torch.as_tensor(np.asarray(sample_pool) if not isinstance(sample_pool, torch.Tensor)
                               else sample_pool).reshape(-1).to(torch.int64).cpu()
        self.sample_pool = pool
        self.n = int(pool.numel())
        self.identity = bool(self.n == 0 or torch.equal(pool, torch.arange(self.n)))
        self._dev_pool = {}
        self._init_rng(seed)

    def pool_for(self, device, dtype):
        """Device copy of a non-identity pool (None for range(E))."""
        if self.identity:
            return None
        key = (str(device), dtype)
        if key not in self._dev_pool:
            self._dev_pool[key] = self.sample_pool.to(device=device, dtype=dtype)
        return self._dev_pool[key]

    def sampler_desc(self, idx_dtype, device, plane):
        d = _hip.kge_sampler_desc()
        d.kind = _hip.SAMPLER_UNIFORM
        d.idx_dtype = idx_dtype
        d.seed = self.seed
        d.offset = plane
        d.n_entities = self.n
        pool = self.pool_for(device, torch.int64 if idx_dtype == _hip.IDX_I64 else torch.int32)
        d.pool = pool.data_ptr() if pool is not None else None
        return d

    def __call__(self, X, negative_ratio, side):
        X = torch.as_tensor(X)
        n = int(X.shape[0])
        plane = self.take_planes(1)
        if X.is_cuda:
            return _sample_cuda(self.sampler_desc(_idx_code(X), X.device, plane), X, negative_ratio, side)
        _host_allowed("UniformStrategy")
        idx = _philox.draw(self.seed, plane, np.arange(n * negative_ratio), X.dtype == torch.int64, self.n)
        out = self.sample_pool.numpy()[idx] if not self.identity else idx
        return torch.from_numpy(np.asarray(out)).to(X.dtype)


class TypedStrategy(_CounterSampler):
    """Same-type draws excluding the entity itself (``ns_strategy.py:67-132``,
    ``utils.py:11-16``). ``pool`` (a multiprocessing pool in the reference)
    is accepted and unused: sampling runs on the device.
    """

    def __init__(self, pool, metadata, seed=None):
        self.pool = pool
        self.metadata = metadata
        self._csr = None
        self._dev = {}
        self._init_rng(seed)

    def _build(self):
        if self._csr is not None:
            return self._csr
        md = self.metadata
        ind2type = list(md["ind2type"])
        E = len(ind2type)
        type2inds = md.get("type2inds")
        if type2inds is None:
            type2inds = {}
            for t in np.unique(ind2type):
                type2inds[t] = np.array([i for (i, ti) in enumerate(ind2type) if ti == t])
        types = list(type2inds.keys())
        tid = {t: k for k, t in enumerate(types)}
        offsets = [0]
        members = []
        pos_in_type = np.full(E, -1, dtype=np.int64)
        for t in types:
            inds = np.asarray(type2inds[t]).reshape(-1)
            for k, e in enumerate(inds):
                if 0 <= e < E and ind2type[e] == t and pos_in_type[e] < 0:
                    pos_in_type[e] = k
            members.extend(inds.tolist())
            offsets.append(len(members))
        ent_type = np.array([tid[t] for t in ind2type], dtype=np.int32)
        if (pos_in_type < 0).any():
            raise ValueError("TypedStrategy: every entity must appear in type2inds[ind2type[e]]")
        self._csr = {
            "ent_type": torch.from_numpy(ent_type),
            "type_offsets": torch.tensor(offsets, dtype=torch.int32),
            "type_members": torch.tensor(members, dtype=torch.int32),
            "pos_in_type": torch.from_numpy(pos_in_type.astype(np.int32)),
            "n_types": len(types),
            "E": E,
        }
        return self._csr

    def csr_on(self, device):
        csr = self._build()
        key = str(device)
        if key not in self._dev:
            self._dev[key] = {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in csr.items()}
        return self._dev[key]

    def sampler_desc(self, idx_dtype, device, plane):
        c = self.csr_on(device)
        d = _hip.kge_sampler_desc()
        d.kind = _hip.SAMPLER_TYPED
        d.idx_dtype = idx_dtype
        d.seed = self.seed
        d.offset = plane
        d.n_entities = c["E"]
        d.ent_type = c["ent_type"].data_ptr()
        d.type_offsets = c["type_offsets"].data_ptr()
        d.type_members = c["type_members"].data_ptr()
        d.pos_in_type = c["pos_in_type"].data_ptr()
        d.n_types = c["n_types"]
        return d

    def draw_host(self, ref, plane, negative_ratio, i64):
        """Host restatement of the device typed draw for reference entities ``ref``."""
        c = self._build()
        ref = np.asarray(ref, dtype=np.int64)
        n = np.arange(ref.shape[0] * negative_ratio)
        x = np.repeat(ref, negative_ratio)
        ty = c["ent_type"].numpy()[x]
        off = c["type_offsets"].numpy()
        beg, cnt = off[ty], off[ty + 1] - off[ty]
        if (cnt <= 1).any():
            raise ValueError("a typed-sampling pool is empty after removing the entity itself")
        k = _philox.draw(self.seed, plane, n, i64, (cnt - 1).astype(np.uint64))
        k = k + (k >= c["pos_in_type"].numpy()[x])
        return c["type_members"].numpy()[beg + k]

    def __call__(self, X, negative_ratio, side):
        X = torch.as_tensor(X)
        plane = self.take_planes(1)
        if X.is_cuda:
            return _sample_cuda(self.sampler_desc(_idx_code(X), X.device, plane), X, negative_ratio, side)
        _host_allowed("TypedStrategy")
        col = 0 if side == "h" else 2
        out = self.draw_host(X[:, col].numpy(), plane, negative_ratio, X.dtype == torch.int64)
        return torch.from_numpy(np.asarray(out)).to(X.dtype)


def _host_allowed(what):
    if os.environ.get("KGE_BACKEND", "fused").lower() != "eager":
        raise RuntimeError("%s: CPU tensors are sampled only with KGE_BACKEND=eager (host development); "
                           "move the triples to the GPU to use kge_sample" % what)


def _idx_code(X):
    if X.dtype == torch.int64:
        return _hip.IDX_I64
    if X.dtype == torch.int32:
        return _hip.IDX_I32
    raise ValueError("triples must be int32 or int64 (got %s)" % X.dtype)


def _sample_cuda(sdesc, X, negative_ratio, side):
    if side not in ("h", "t"):
        raise ValueError("side must be 'h' or 't'")
    X = X.contiguous()
    n = int(X.shape[0])
    out = torch.empty(n * negative_ratio, dtype=X.dtype, device=X.device)
    status = torch.zeros(1, dtype=torch.int32, device=X.device)
    d = _hip.kge_sample_desc()
    d.sampler = sdesc
    d.X = X.data_ptr()
    d.n = n
    d.side = _hip.SIDE_H if side == "h" else _hip.SIDE_T
    d.negative_ratio = int(negative_ratio)
    d.out = out.data_ptr()
    d.status = status.data_ptr()
    _hip.check(_hip.lib().kge_sample(d, _hip.stream_handle(X.device)), "kge_sample")
    _hip.check_device_status(status, "kge_sample")
    return out
