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
from .linker import _capacity
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


def _java_div(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def trace_day(trace: Sequence[Span]) -> int:
    """The midnight a trace is bucketed under: ITDependencies.flooredTraceTimestamp (:680-690),
    which compares a span's micros with the current (millisecond) midnight. The host uses it
    only to route traces to a context whose day range holds them; the device computes the same
    day for every trace it links (and fails the put if a trace falls outside the range)."""
    m = (1 << 63) - 1
    for s in trace:
        ts = guess_timestamp(s)
        if ts != 0 and ts < m:
            m = _midnight(_java_div(ts, 1000))
    if m == (1 << 63) - 1:
        raise ValueError("a trace has no timestamp (flooredTraceTimestamp asserts one)")
    return m


# A context covers a contiguous range of at most 255 days (zdl_set_days) whose dense
# days x S x S count tables stay within this budget; days without traces between present
# ones are only skipped over when a range would exceed it.
TABLE_BUDGET_BYTES = 1 << 30


def _day_ranges(days: List[int], n_services: int) -> List[List[int]]:
    """The distinct days present, ascending, cut into ranges one context each can hold."""
    per_day = 16 * n_services * n_services  # call + err, u64 each
    max_days = max(1, min(255, TABLE_BUDGET_BYTES // per_day))
    out: List[List[int]] = []
    for d in sorted(set(days)):
        if out and (d - out[-1][0]) // DAY_MS < max_days:
            out[-1].append(d)
        else:
            out.append([d])
    return out


def aggregate_links(spans: Sequence[Span], device: int = 0,
                    insertion_order: bool = True) -> Dict[int, List[DependencyLink]]:
    """midnight (epoch ms) -> that day's links, like ITDependencies.aggregateLinks: the days in
    first-seen order, each day's links in its linker's order."""
    traces = group_by_trace_id(spans)
    if not traces:
        return {}
    days = [trace_day(t) for t in traces]
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    for t in traces:  # the service dictionary first: it sizes the contexts' tables
        for s in t:
            for e in (s.local_endpoint, s.remote_endpoint):
                if e is not None:
                    svc.id(e.service_name)
    cap = _capacity(max(len(svc), 1))
    per_day: Dict[int, List[DependencyLink]] = {}
    names = svc.strings
    for rng in _day_ranges(days, cap):
        lo, hi = rng[0], rng[-1]
        keep = set(rng)
        sel = [t for t, d in zip(traces, days) if d in keep]
        cols = pack_traces(sel, svc, ip4, ip6)
        cols.timestamp[:] = [guess_timestamp(s) for t in sel for s in t]
        ctx = N.Context(cap, device, insertion_order=insertion_order)
        try:
            ctx.set_ranks(N.ZDL_DICT_SERVICE, svc.ranks())
            ctx.set_ranks(N.ZDL_DICT_IPV4, ip4.ranks())
            ctx.set_ranks(N.ZDL_DICT_IPV6, ip6.ranks())
            ctx.set_days(lo, (hi - lo) // DAY_MS + 1)
            ctx.put_spans(cols)
            got_days, day, p, c, n, e = ctx.link_days(N.ZDL_ORDER_INSERTION if insertion_order
                                                      else N.ZDL_ORDER_SORTED)
        finally:
            ctx.close()
        for d in got_days:
            per_day.setdefault(int(d), [])
        for d, a, b, x, y in zip(day.tolist(), p.tolist(), c.tolist(), n.tolist(), e.tolist()):
            per_day[int(d)].append(DependencyLink.create(names[a], names[b], int(x), int(y)))
    out: Dict[int, List[DependencyLink]] = {}
    for d in days:  # first-seen day order (LinkedHashMap midnightToLinker)
        if d not in out:
            out[d] = per_day.get(d, [])
    return out
