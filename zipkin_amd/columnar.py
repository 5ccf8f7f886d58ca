"""Span -> columnar packing (the layout of zdl_span_cols, include/zdl.h).

What the Java facade would do before the JNI call: project each Span onto the
fields the linker reads (the same projection as mysql-v1's
DependencyLinkV2SpanIterator.java:88-159) and dictionary-encode strings.
Dictionaries hand out ids in first-seen order and keep rank tables in
java.lang.String.compareTo order (UTF-16 code units), which Trace.merge's
endpoint comparison needs (internal/Trace.java:105-116).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from ._native import (KIND_NULL, PF_ERROR, PF_KIND_SHIFT, PF_RIP4, PF_RIP6, PF_RPORT,
                      PF_SHARED_SHIFT)
from .model import Span, java_string_key

__all__ = ["Dictionary", "Columns", "pack_traces", "concat_columns"]


class Dictionary:
    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.strings: List[str] = []
        self._ranks: Optional[np.ndarray] = None

    def __len__(self):
        return len(self.strings)

    def id(self, s: Optional[str]) -> int:
        if s is None:
            return -1
        i = self.ids.get(s)
        if i is None:
            i = len(self.strings)
            self.ids[s] = i
            self.strings.append(s)
            self._ranks = None
        return i

    def lowered(self) -> list:
        """The strings lower-cased (DependencyLink.Builder's parent / child), cached."""
        lw = getattr(self, "_lowered", None)
        if lw is None or len(lw) != len(self.strings):
            lw = [x.lower() for x in self.strings]
            self._lowered = lw
        return lw

    def ranks(self) -> np.ndarray:
        if self._ranks is None or len(self._ranks) != len(self.strings):
            order = sorted(range(len(self.strings)), key=lambda i: java_string_key(self.strings[i]))
            r = np.empty(len(order), np.int32)
            r[np.asarray(order, dtype=np.int64)] = np.arange(len(order), dtype=np.int32)
            self._ranks = r
        return self._ranks


@dataclass
class Columns:
    trace_lo: np.ndarray   # u64
    id: np.ndarray         # u64
    parent_id: np.ndarray  # u64
    local_svc: np.ndarray  # i32
    remote_svc: np.ndarray
    local_ip4: np.ndarray
    local_ip6: np.ndarray
    port_flags: np.ndarray  # u32
    timestamp: np.ndarray   # i64
    offsets: np.ndarray     # u64, n_traces + 1

    @property
    def n_spans(self) -> int:
        return int(self.id.shape[0])

    @property
    def n_traces(self) -> int:
        return int(self.offsets.shape[0]) - 1


def port_flags_of(s: Span) -> int:
    pf = 0
    le, re = s.local_endpoint, s.remote_endpoint
    if le is not None:
        pf |= le.port & 0xFFFF
    pf |= (int(s.kind) if s.kind is not None else KIND_NULL) << PF_KIND_SHIFT
    pf |= (0 if s.shared is None else (2 if s.shared else 1)) << PF_SHARED_SHIFT
    if s.is_error:
        pf |= PF_ERROR
    if re is not None:
        if re.ipv4 is not None:
            pf |= PF_RIP4
        if re.ipv6 is not None:
            pf |= PF_RIP6
        if re.port:
            pf |= PF_RPORT
    return pf


def pack_traces(traces: Sequence[Sequence[Span]], svc: Dictionary, ip4: Dictionary,
                ip6: Dictionary) -> Columns:
    """The columns of `traces` (putTrace calls' spans, in call order). One pass of Python over the
    spans into lists, then one conversion per column (element-wise stores into numpy arrays cost
    more than the spans' own attribute reads)."""
    tl, ids, pids, ls, rs, l4, l6, pf, ts = [], [], [], [], [], [], [], [], []
    off = [0]
    sid, i4, i6 = svc.id, ip4.id, ip6.id
    for trace in traces:
        for s in trace:
            tl.append(int(s.trace_lo, 16))
            ids.append(int(s.id, 16))
            pids.append(int(s.parent_id, 16) if s.parent_id is not None else 0)
            le = s.local_endpoint
            if le is not None:
                ls.append(sid(le.service_name))
                l4.append(i4(le.ipv4))
                l6.append(i6(le.ipv6))
            else:
                ls.append(-1)
                l4.append(-1)
                l6.append(-1)
            re = s.remote_endpoint
            rs.append(sid(re.service_name) if re is not None else -1)
            pf.append(port_flags_of(s))
            ts.append(s.timestamp)
        off.append(len(ids))
    return Columns(np.array(tl, np.uint64), np.array(ids, np.uint64), np.array(pids, np.uint64),
                   np.array(ls, np.int32), np.array(rs, np.int32), np.array(l4, np.int32), np.array(l6, np.int32),
                   np.array(pf, np.uint32), np.array(ts, np.int64), np.array(off, np.uint64))


def concat_columns(parts: Iterable[Columns]) -> Columns:
    parts = list(parts)
    offs = [np.zeros(1, np.uint64)]
    base = 0
    for p in parts:
        offs.append(p.offsets[1:] + np.uint64(base))
        base += p.n_spans
    cat = lambda f: np.concatenate([getattr(p, f) for p in parts])  # noqa: E731
    return Columns(cat("trace_lo"), cat("id"), cat("parent_id"), cat("local_svc"), cat("remote_svc"),
                   cat("local_ip4"), cat("local_ip6"), cat("port_flags"), cat("timestamp"),
                   np.concatenate(offs))
