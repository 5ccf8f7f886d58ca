"""Daily-bucketed dependency links on the MI355X engine.

Mirrors the aggregation the zipkin-dependencies job performs and the reference's
storage tests restate (``ITDependencies.aggregateLinks``,
zipkin/src/test/java/zipkin2/storage/ITDependencies.java:666-700): spans grouped by
low trace id in first-seen order (``GroupByTraceId.create(false)``,
storage/GroupByTraceId.java:41-54), each trace linked by the DependencyLinker of
its day (``flooredTraceTimestamp``, :680-690, over ``guessTimestamp``, :692-700),
and a map midnight -> ``DependencyLinker.link()`` in first-seen day order.

The day of a trace, the per-day (parent, child) counts and the insertion order are
computed on the device (``zdl_set_days`` / ``zdl_link_days``); the host packs the
columns with guessTimestamp in the timestamp column and chooses the day range.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

from . import _native as N
from .columnar import Dictionary, pack_traces
from .model import DependencyLink, Span

DAY_MS = 86_400_000


def guess_timestamp(s: Span) -> int:
    """ITDependencies.guessTimestamp: the span's timestamp, else the first annotation's."""
    if s.timestamp:
        return s.timestamp
    for ts, _ in s.annotations:
        if ts > 0:
            return ts
    return 0


def group_by_trace_id(spans: Sequence[Span]) -> List[List[Span]]:
    """GroupByTraceId.create(false): low 64-bit trace id, first-seen order."""
    groups: Dict[str, List[Span]] = {}
    for s in spans:
        groups.setdefault(s.trace_lo, []).append(s)
    return list(groups.values())


def _midnight(ms: int) -> int:
    return (ms // DAY_MS) * DAY_MS


def aggregate_links(spans: Sequence[Span], device: int = 0,
                    insertion_order: bool = True) -> Dict[int, List[DependencyLink]]:
    """midnight (epoch ms) -> that day's links, like ITDependencies.aggregateLinks."""
    traces = group_by_trace_id(spans)
    if not traces:
        return {}
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    cols.timestamp[:] = [guess_timestamp(s) for t in traces for s in t]
    nz = cols.timestamp[cols.timestamp != 0]
    if len(nz) == 0:
        raise ValueError("no span has a timestamp (flooredTraceTimestamp asserts one)")
    lo = _midnight(int(np.int64(nz.min()) // 1000))
    hi = _midnight(int(np.int64(nz.max()) // 1000))
    n_services = 48
    while n_services < len(svc):
        n_services *= 2
    ctx = N.Context(n_services, device, insertion_order=insertion_order)
    try:
        ctx.set_ranks(N.ZDL_DICT_SERVICE, svc.ranks())
        ctx.set_ranks(N.ZDL_DICT_IPV4, ip4.ranks())
        ctx.set_ranks(N.ZDL_DICT_IPV6, ip6.ranks())
        ctx.set_days(lo, (hi - lo) // DAY_MS + 1)
        ctx.put_spans(cols)
        days, day, p, c, n, e = ctx.link_days(N.ZDL_ORDER_INSERTION if insertion_order else N.ZDL_ORDER_SORTED)
    finally:
        ctx.close()
    out: Dict[int, List[DependencyLink]] = {int(d): [] for d in days}
    names = svc.strings
    for d, a, b, x, y in zip(day.tolist(), p.tolist(), c.tolist(), n.tolist(), e.tolist()):
        out[int(d)].append(DependencyLink.create(names[a], names[b], int(x), int(y)))
    return out
