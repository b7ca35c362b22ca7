"""Host (numpy) implementation of the counter-based negative-draw and
input-stream specs.

Used only by the eager plugin path on CPU tensors; CUDA tensors are sampled
by ``kge_sample`` / the fused step in ``libkge_hip.so``. The spec (see
``include/kge_hip.h``): draw n of counter plane ``plane`` is Philox4x32-10
with key (seed lo, seed hi) and counter (block lo, block hi, plane lo,
plane hi), block = n // P, P = 4 (int32 ids) or 2 (int64 ids), mapped to
``bits % range`` like TF's ``UniformDistribution``.
"""

import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) for x in (c0, c1, c2, c3))
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & 0xFFFFFFFF
            k1 = (k1 + _W1) & 0xFFFFFFFF
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
    return c0, c1, c2, c3


def draw(seed, plane, n, i64, rng):
    """Uniform integers in [0, rng) for draw indices ``n`` (array) of ``plane``."""
    n = np.asarray(n, dtype=np.uint64)
    per = np.uint64(2 if i64 else 4)
    b = n // per
    q = (n % per).astype(np.int64)
    w = philox4x32_10(b & _MASK, b >> np.uint64(32), np.uint64(plane & 0xFFFFFFFF),
                      np.uint64((plane >> 32) & 0xFFFFFFFF), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    w = np.stack(w, axis=-1)
    if i64:
        lo = np.take_along_axis(w, (2 * q)[..., None], -1)[..., 0]
        hi = np.take_along_axis(w, (2 * q + 1)[..., None], -1)[..., 0]
        bits = lo | (hi << np.uint64(32))
        return (bits % np.asarray(rng, dtype=np.uint64)).astype(np.int64)
    bits = np.take_along_axis(w, q[..., None], -1)[..., 0]
    return (bits % np.asarray(rng, dtype=np.uint64)).astype(np.int64)


def _feistel_pass(x, h, seed, epoch):
    mask = np.uint64((1 << h) - 1)
    L, R = x >> np.uint64(h), x & mask
    for r in range(4):
        w = philox4x32_10(R, np.uint64(r), np.uint64(epoch & 0xFFFFFFFF), np.uint64((epoch >> 32) & 0xFFFFFFFF),
                          seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)[0]
        L, R = R, (L ^ w) & mask
    return (L << np.uint64(h)) | R


def stream_rows(n, seed, start, batch, shuffle):
    """Source rows of stream positions [start, start + batch) over n rows
    (``kge_stream_desc`` in include/kge_hip.h): epoch e = p // n, row
    pi_e(p % n), pi_e a cycle-walked 4-round Philox-keyed Feistel permutation
    (the identity when not shuffling)."""
    n = int(n)
    p = np.arange(int(start), int(start) + int(batch), dtype=np.uint64)
    k = p % np.uint64(n)
    if not shuffle or len(p) == 0:
        return k.astype(np.int64)
    w = 2
    while w < 64 and (1 << w) < n:
        w += 2
    h = w // 2
    e = p // np.uint64(n)
    out = np.empty_like(k)
    for ep in np.unique(e):
        sel = e == ep
        y = _feistel_pass(k[sel], h, int(seed), int(ep))
        bad = y >= np.uint64(n)
        while bad.any():
            y[bad] = _feistel_pass(y[bad], h, int(seed), int(ep))
            bad = y >= np.uint64(n)
        out[sel] = y
    return out.astype(np.int64)
