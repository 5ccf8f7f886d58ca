"""ORACLE — TEST INFRASTRUCTURE ONLY, NEVER A PRODUCT PATH.

numpy restatement of the InMemoryStorage index questions that zdl_store answers on the
device (zipkin_amd/csrc/zdl_store.hip), over per-span arrays in arrival order (low and high
trace id as u64, timestamp as i64, alive as bool). Used by tests/test_gpu_store.py to check
the device's eviction and selections position for position at sizes the pure-Python
InMemoryStorage oracle (dl_oracle.InMemoryStorage, pinned by the ITDependencies /
InMemoryStorageTest vectors) cannot reach; the two are cross-checked in
tests/test_oracle_cross.py.

Paths are relative to /root/reference/zipkin/src/main/java/zipkin2/.
"""
from __future__ import annotations

import numpy as np

SELECT_NEWEST, SELECT_ALL, SELECT_ALL_STRICT = 0, 1, 2


def evict(lo, ts, alive, to_recover):
    """storage/InMemoryStorage.java:184-211 evictToRecoverSpans / deleteOldestTrace: the last
    key of TIMESTAMP_DESCENDING is the smallest (timestamp, lowTraceId), and with it every span
    of that lowTraceId goes; repeated until to_recover spans are gone. Returns (alive after,
    evicted, exhausted); exhausted = the store ran empty first (TreeMap.lastKey throws
    NoSuchElementException after everything was evicted)."""
    alive = alive.copy()
    if to_recover <= 0:
        return alive, 0, False
    idx = np.nonzero(alive)[0]
    if len(idx) == 0:
        return alive, 0, True
    l, t = lo[idx], ts[idx]
    ulo, inv, counts = np.unique(l, return_inverse=True, return_counts=True)
    oldest = np.full(len(ulo), np.iinfo(np.int64).max, np.int64)
    np.minimum.at(oldest, inv.reshape(-1), t)
    tord = np.lexsort((ulo, oldest))  # (smallest timestamp, lowTraceId) ascending
    cum = np.cumsum(counts[tord])
    k = int(np.searchsorted(cum, to_recover))  # first trace whose cumulative count reaches it
    if k >= len(ulo):
        alive[idx] = False
        return alive, len(idx), True
    victims = ulo[tord[:k + 1]]
    dead = idx[np.isin(l, victims)]
    alive[dead] = False
    return alive, len(dead), False


def _storage_rank(l, t):
    """spansByTraceId (InMemoryStorage.java:448-454): inside a lowTraceId, its distinct
    (lowTraceId, timestamp) keys in first-seen order, each key's spans in arrival order. Per
    span: the arrival of its key's first span."""
    keys = np.stack([l, t.view(np.uint64)], axis=1)
    _, inv = np.unique(keys, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    first = np.full(inv.max() + 1, np.iinfo(np.int64).max, np.int64)
    np.minimum.at(first, inv, np.arange(len(l), dtype=np.int64))
    return first[inv]


def _offsets(new_trace):
    starts = np.nonzero(np.concatenate([[True], new_trace]))[0]
    return np.concatenate([starts, [len(new_trace) + 1]]).astype(np.uint64)


def select(lo, hi, ts, alive, mode):
    """The alive spans as (u32 positions in trace order, u64 CSR trace offsets):
    SELECT_NEWEST - getTraces(request) for getDependencies: TIMESTAMP_DESCENDING keys
      (timestamp, then lowTraceId, descending; :272-291, 356-366) meet a lowTraceId at its
      newest key;
    SELECT_ALL - getTraces() (:251-262): lowTraceIds ascending;
    SELECT_ALL_STRICT - the same split by full trace id in first-seen order (:241-249)."""
    idx = np.nonzero(alive)[0]
    if len(idx) == 0:
        return np.zeros(0, np.uint32), np.zeros(1, np.uint64)
    l, h, t = lo[idx], hi[idx], ts[idx]
    key_first = _storage_rank(l, t)
    arrival = np.arange(len(idx))
    if mode == SELECT_NEWEST:
        ulo, tinv = np.unique(l, return_inverse=True)
        newest = np.full(len(ulo), np.iinfo(np.int64).min, np.int64)
        np.maximum.at(newest, tinv.reshape(-1), t)
        newest = newest[tinv.reshape(-1)]
        order = np.lexsort((arrival, key_first, ~l, -newest))
        sel = idx[order]
        a = lo[sel]
        return sel.astype(np.uint32), _offsets(a[1:] != a[:-1])
    inner = np.lexsort((arrival, key_first, l))  # lowTraceId ascending, storage order inside
    if mode == SELECT_ALL:
        sel = idx[inner]
        a = lo[sel]
        return sel.astype(np.uint32), _offsets(a[1:] != a[:-1])
    rank = np.empty(len(idx), np.int64)
    rank[inner] = np.arange(len(idx))
    _, ginv = np.unique(np.stack([l, h], axis=1), axis=0, return_inverse=True)
    ginv = ginv.reshape(-1)
    gfirst = np.full(ginv.max() + 1, np.iinfo(np.int64).max, np.int64)
    np.minimum.at(gfirst, ginv, rank)
    sel = idx[np.lexsort((rank, gfirst[ginv], l))]
    a, b = lo[sel], hi[sel]
    return sel.astype(np.uint32), _offsets((a[1:] != a[:-1]) | (b[1:] != b[:-1]))
