"""ORACLE — test infrastructure only. ctypes binding of the C++ restatement
(oracle/dl_ref.cpp -> oracle/liboracle.so). Imported by tests/, smoke() and
bench.py's cpu_baseline leg; never by zipkin_amd/."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


class OracleCols(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("id", "parent_id", "local_svc", "remote_svc", "local_ip4",
                                          "local_ip6", "port_flags", "timestamp")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.oracle_link.restype = vp
        L.oracle_link.argtypes = [C.POINTER(OracleCols), C.c_uint64, vp, C.c_uint64, vp, C.c_uint32, vp,
                                  C.c_uint32, vp, C.c_uint32, C.c_int, C.c_int64, C.c_int64, C.c_int]
        L.oracle_status.argtypes = [vp]
        L.oracle_count.argtypes = [vp]
        L.oracle_count.restype = C.c_uint64
        L.oracle_copy.argtypes = [vp, vp, vp, vp, vp]
        L.oracle_free.argtypes = [vp]
        _lib = L
    return _lib


def link(cols, svc_rank=None, ip4_rank=None, ip6_rank=None, window=None, threads=1):
    """Runs the restatement over columnar.Columns. Returns (status, p, c, call, err) in the
    reference's insertion order. window = (end_ts_ms, lookback_ms) or None."""
    L = lib()
    p = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    oc = OracleCols(p(cols.id), p(cols.parent_id), p(cols.local_svc), p(cols.remote_svc), p(cols.local_ip4),
                    p(cols.local_ip6), p(cols.port_flags), p(cols.timestamp))
    ranks = [np.ascontiguousarray(r, np.int32) if r is not None else None for r in (svc_rank, ip4_rank, ip6_rank)]
    lo = hi = 0
    if window is not None:
        end, lb = window
        lo, hi = (end - lb) * 1000, end * 1000
    h = L.oracle_link(C.byref(oc), cols.n_spans, cols.offsets.ctypes.data, cols.n_traces,
                      p(ranks[0]), len(ranks[0]) if ranks[0] is not None else 0,
                      p(ranks[1]), len(ranks[1]) if ranks[1] is not None else 0,
                      p(ranks[2]), len(ranks[2]) if ranks[2] is not None else 0,
                      1 if window is not None else 0, lo, hi, threads)
    try:
        st = L.oracle_status(h)
        n = L.oracle_count(h)
        out = (np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.int64), np.empty(n, np.int64))
        L.oracle_copy(h, *(a.ctypes.data for a in out))
    finally:
        L.oracle_free(h)
    return (st,) + out
