"""Trace sharding across GPUs.

Traces are independent, so each rank links its own traces; the low 64 bits of
the trace id pick the rank, because getDependencies groups by lowTraceId
(InMemoryStorage.java:163, 330, 465-467): sharding on the full 128-bit id
would split mixed 64/128-bit traces. The only exchange is the combine of the
ranks' counts inside libzdl (DependencyLinker.merge semantics, :189-204;
zipkin_amd/csrc/zdl_xport.inc).
"""
from __future__ import annotations

import numpy as np

_M1, _M2, _G = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB), np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.asarray(x, np.uint64) + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def shard_of(trace_lo: np.ndarray, n_shards: int) -> np.ndarray:
    return (splitmix64(trace_lo) % np.uint64(n_shards)).astype(np.int64)


def partition_columns(cols, n_shards: int):
    """Splits CSR-grouped columns into n_shards Columns by trace: whole traces only,
    shard = splitmix64(trace_lo of the trace's first span) % n_shards, storage order kept."""
    from .columnar import Columns
    off = cols.offsets.astype(np.int64)
    sizes = np.diff(off)
    first = off[:-1]
    lo = cols.trace_lo[np.minimum(first, max(cols.n_spans - 1, 0))] if cols.n_spans else np.zeros(len(sizes), np.uint64)
    shard = shard_of(lo, n_shards)
    out = []
    span_shard = np.repeat(shard, sizes)
    for r in range(n_shards):
        tsel = shard == r
        ssel = span_shard == r
        pick = lambda a: np.ascontiguousarray(a[ssel])  # noqa: E731
        new_off = np.zeros(int(tsel.sum()) + 1, np.uint64)
        new_off[1:] = np.cumsum(sizes[tsel]).astype(np.uint64)
        out.append(Columns(pick(cols.trace_lo), pick(cols.id), pick(cols.parent_id), pick(cols.local_svc),
                           pick(cols.remote_svc), pick(cols.local_ip4), pick(cols.local_ip6),
                           pick(cols.port_flags), pick(cols.timestamp), new_off))
    return out
