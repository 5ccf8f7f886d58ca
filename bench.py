"""Benchmark: spans/sec linked to DependencyLinks on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch already resident in HBM:
reset the S x S counts, zdl_put_spans_device (k_link, k_tail), for N > 1 one RCCL
all-reduce of the count tables, then zdl_link (ordered compaction into mapped pinned
memory, one sync) -> the DependencyLink list. At N = 1 two steps are in flight (two
contexts, two streams: step k+1 is launched before step k's links are read, so host work
overlaps device work); `config.ms_per_step_serial` is the same step run one at a time.

N = 1 runs C2 (10M spans / 1M traces / 50 services), BASELINE.json configs[1]. N > 1 is
weak scaling on C3's shape (500 services): every rank links its own C3 per-GPU shard
(12.5M traces = 125M spans, the 1B / 8 split) of traces picked by splitmix64(trace_lo) % N,
and the ranks sum their tables once (RCCL over xGMI). `--config c3` runs that shard at N = 1.

Roofline accounting follows SURVEY.md §8(d) / BASELINE.md: algorithmic bytes
W = 44 B/span (trace_lo, id, parent_id, 4 dictionary ids, port_flags) + 8 B/trace (CSR
offset). `roofline` prices the dominant kernel (k_link, HIP events on the context stream)
with W; `config.step_roofline_frac` prices the whole device step (reset, kernels, combine,
link) with W; `config.k_link_read_frac` uses the 36 B/span k_link actually reads (the CSR
grouping replaces trace_lo).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "spans/sec linked to DependencyLinks at 1/2/4/8 MI355X; % of HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_SPAN = 44            # trace_lo 8 + id 8 + parent_id 8 + 4 x i32 ids + port_flags 4
READ_BYTES_PER_SPAN = 36       # what k_link reads: the CSR grouping stands in for trace_lo
BYTES_PER_TRACE = 8            # CSR offset (k_link plans its windows from them)
C3_TRACES_PER_GPU = 12_500_000  # C3's 100M traces over 8 GPUs


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# k_proto3_spans' compulsory traffic beyond the message bytes: span start (8) + length (4) read,
# columns written (trace_lo, id, parent_id 8 each; 4 ids and port_flags 4 each; timestamp 8),
# the per-span miss byte
P3_BYTES_PER_SPAN = 12 + 52 + 1


def proto3_leg(cols, w, S, device, doff, links, reps=5):
    """Decode the batch's proto3 encoding on the device, then link the decoded columns with the
    batch's trace offsets (the encoding keeps the span order): the links must equal the columnar
    path's `links` by service name. Kernel time from HIP events around k_proto3_spans; the call
    time includes the host's top-level scan, the PCIe upload and the trace-id/timestamp download."""
    from zipkin_amd import synth
    from zipkin_amd.columnar import Dictionary
    from zipkin_amd import _native as N
    from zipkin_amd.proto3 import Proto3Decoder
    names = synth.service_names(w)
    data = synth.encode_proto3(cols, names).tobytes()
    dicts = (Dictionary(), Dictionary(), Dictionary())
    dec = Proto3Decoder(*dicts, device=device)
    b = dec.decode(data)  # first pass binds the names
    ks, cs = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        b = dec.decode(data)
        cs.append(time.perf_counter() - t0)
        ks.append(dec._dec.kernel_ms())
    km, cm = float(np.median(ks)), float(np.median(cs)) * 1e3
    svc = dicts[0]
    ctx = N.Context(max(len(svc), 1), device=device)
    dptr = {k: getattr(b.dev, k) for k in ("id", "parent_id", "local_svc", "remote_svc", "local_ip4",
                                            "local_ip6", "port_flags")}
    ctx.put_spans_device(dptr, b.n_spans, doff.data_ptr(), cols.n_traces)
    gp, gc, gn, ge = ctx.link()
    ctx.close()
    got = sorted(zip((svc.strings[i] for i in gp.tolist()), (svc.strings[i] for i in gc.tolist()),
                     gn.tolist(), ge.tolist()))
    p, c, n, e = links
    exp = sorted(zip((names[i] for i in p.tolist()), (names[i] for i in c.tolist()), n.tolist(), e.tolist()))
    dec.close()
    algo = len(data) + b.n_spans * P3_BYTES_PER_SPAN
    return {"bytes": len(data), "spans": b.n_spans, "kernel_ms": km, "call_ms": cm,
            "spans_per_s": b.n_spans / (km * 1e-3), "kernel_gbs": algo / (km * 1e-3) / 1e9,
            "kernel_roofline_frac": algo / (km * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "algorithmic_bytes": algo, "call_spans_per_s": b.n_spans / (cm * 1e-3),
            "parity": "same links" if got == exp else "MISMATCH"}


def json_v2_leg(cols, w, device, doff, links, reps=3):
    """Decode the batch's JSON v2 encoding (V2SpanWriter member order, synth.encode_json_v2) on the
    device, then link the decoded columns with the batch's trace offsets: the links must equal the
    columnar path's `links` by service name. Device time = the structure passes (block functions,
    scans, object starts) + k_js_fast / k_js_spans_list, by HIP events; the call time adds the PCIe upload and the
    trace-id/timestamp download. Compulsory traffic: the bytes once + 52 B/span of columns.
    `exact_spans`: spans the exact reader took instead of the fast path (0 for the writer's shape)."""
    from zipkin_amd import synth
    from zipkin_amd.columnar import Dictionary
    from zipkin_amd import _native as N
    from zipkin_amd.jsonv2 import JsonV2Decoder
    names = synth.service_names(w)
    data = synth.encode_json_v2(cols, names).tobytes()
    dicts = (Dictionary(), Dictionary(), Dictionary())
    dec = JsonV2Decoder(*dicts, device=device)
    b = dec.decode(data)  # first pass binds the names
    ks, ss, cs = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        b = dec.decode(data)
        cs.append(time.perf_counter() - t0)
        ks.append(dec.kernel_ms())
        ss.append(dec.struct_ms())
    km, sm, cm = float(np.median(ks)), float(np.median(ss)), float(np.median(cs)) * 1e3
    n_exact = dec.exact_spans()
    svc = dicts[0]
    ctx = N.Context(max(len(svc), 1), device=device)
    dptr = {k: getattr(b.dev, k) for k in ("id", "parent_id", "local_svc", "remote_svc", "local_ip4",
                                            "local_ip6", "port_flags")}
    ctx.put_spans_device(dptr, b.n_spans, doff.data_ptr(), cols.n_traces)
    gp, gc, gn, ge = ctx.link()
    ctx.close()
    got = sorted(zip((svc.strings[i] for i in gp.tolist()), (svc.strings[i] for i in gc.tolist()),
                     gn.tolist(), ge.tolist()))
    p, c, n, e = links
    exp = sorted(zip((names[i] for i in p.tolist()), (names[i] for i in c.tolist()), n.tolist(), e.tolist()))
    dec.close()
    dev_ms = km + sm
    algo = len(data) + b.n_spans * 52
    return {"bytes": len(data), "spans": b.n_spans, "structure_ms": sm, "spans_kernel_ms": km, "device_ms": dev_ms,
            "call_ms": cm, "spans_per_s": b.n_spans / (dev_ms * 1e-3), "device_gbs": algo / (dev_ms * 1e-3) / 1e9,
            "roofline_frac": algo / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": algo,
            "call_spans_per_s": b.n_spans / (cm * 1e-3), "exact_spans": n_exact,
            "parity": "same links" if got == exp else "MISMATCH"}


def store_leg(cols, S, device, links, names, reps=5):
    """InMemoryStorage.getDependencies(endTs, lookback) over the batch resident in a zdl_store
    (IMS:323-332). accept appends the columns to HBM and merges the batch into the
    store's resident trace index (zdl_store_index.h: radix sorts of the batch + merges, the
    reference's TreeMap inserts at accept); a query filters the alive spans of that index,
    orders the traces newest first (one sort of a key per trace), gathers and links them under
    the window (zdl_put_selection); nothing crosses PCIe but counts and the links. Timed two
    ways: the raw context (sorted output) and the InMemoryStorage facade exactly as shipped
    (insertion-order DependencyLinker context sized by _capacity for a window, service ranks,
    DependencyLink objects out), with the facade's store holding the same columns. The window
    covers the batch, so the links must equal the columnar path's."""
    from zipkin_amd import _native as N
    from zipkin_amd.storage import InMemoryStorage
    st = N.Store(device)
    t0 = time.perf_counter()
    st.append(cols)
    accept_ms = (time.perf_counter() - t0) * 1e3
    # a collector appends batch after batch into a store that has its capacity: the same append
    # after zdl_store_clear (HBM columns and index buffers kept) - PCIe copies + the index merge
    warm = []
    for _ in range(3):
        st.clear()
        t0 = time.perf_counter()
        st.append(cols)
        warm.append((time.perf_counter() - t0) * 1e3)
    accept_warm_ms = float(np.median(warm))
    ctx = N.Context(S, device=device)
    end_ms = int(cols.timestamp.max()) // 1000 + 1
    lookback = end_ms - int(cols.timestamp.min()) // 1000 + 1
    ctx.set_window(end_ms, lookback)

    def query():
        ctx.reset()
        st.select(N.ZDL_SELECT_NEWEST)
        ctx.put_selection(st)
        return ctx.link()

    got = query()
    qs, ss = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        query()
        qs.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        st.select(N.ZDL_SELECT_NEWEST)
        ss.append(time.perf_counter() - t0)
    ctx.close()
    st.close()
    same = all(np.array_equal(a, b) for a, b in zip(got, links))
    # the facade as shipped: its own store (the same columns appended), its dictionary
    ims = InMemoryStorage(max_span_count=max(cols.n_spans, 500000), device=device)
    for nm in names:
        ims._linker.svc.id(nm)
    ims._st().append(cols)
    fl = ims.get_dependencies(end_ms, lookback).execute()
    fs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ims.get_dependencies(end_ms, lookback).execute()
        fs.append(time.perf_counter() - t0)
    ims.close()
    p, c, n, e = links
    exp = sorted(zip((names[i] for i in p.tolist()), (names[i] for i in c.tolist()), n.tolist(), e.tolist()))
    fsame = sorted((l.parent, l.child, l.call_count, l.error_count) for l in fl) == exp
    qm, sm, fm = float(np.median(qs)) * 1e3, float(np.median(ss)) * 1e3, float(np.median(fs)) * 1e3
    return {"spans": cols.n_spans, "accept_ms": accept_ms, "accept_warm_ms": accept_warm_ms, "get_dependencies_ms": qm, "select_ms": sm,
            "facade_get_dependencies_ms": fm, "spans_per_s": cols.n_spans / (qm * 1e-3),
            "note": "accept: host columns -> HBM + resident index merge; query: wall clock of select + gather + "
                    "link + link() download, store resident in HBM; facade: InMemoryStorage.get_dependencies"
                    "(endTs, lookback).execute() as shipped (insertion order, DependencyLink objects)",
            "parity": "same links" if same and fsame else "MISMATCH"}


def mysql_rows_leg(cols, S, device, max_spans=2_000_000, reps=3):
    """The first traces of the batch (<= max_spans spans) as mysql-v1 cursor rows (one row per
    annotation a span would carry in v1: sr/ca for servers, cs/sa for clients, lc for local spans,
    an error tag row) through zdl_put_mysql_rows + link: rows/s with the rows in host memory
    (as a JDBC cursor delivers them), i.e. PCIe-inclusive. Timing only (parity: tests/)."""
    from zipkin_amd import _native as N
    k = int(np.searchsorted(cols.offsets, max_spans, side="right")) - 1
    m = int(cols.offsets[k])
    kind = (cols.port_flags[:m] >> 16) & 7
    err = (cols.port_flags[:m] >> 21) & 1
    loc, rem = cols.local_svc[:m], cols.remote_svc[:m]
    key = np.zeros((m, 3), np.uint8)
    svc = np.full((m, 3), -1, np.int32)
    key[:, 0] = np.where(kind == 1, N.ZDL_AKEY_SR, np.where(kind == 0, N.ZDL_AKEY_CS, N.ZDL_AKEY_LC))
    svc[:, 0] = loc
    key[:, 1] = np.where(kind == 1, N.ZDL_AKEY_CA, np.where(kind == 0, N.ZDL_AKEY_SA, 0))
    svc[:, 1] = np.where(key[:, 1] > 0, rem, -1)
    key[:, 2] = np.where(err > 0, N.ZDL_AKEY_ERROR, 0)
    svc[:, 2] = np.where(err > 0, loc, -1)
    keep = ((key > 0) & (svc >= 0)).reshape(-1)
    keep.reshape(m, 3)[:, 0] = True  # every span has its row (the left join)
    span = np.repeat(np.arange(m), 3)[keep]
    a = N.MysqlRows.arrays(np.zeros(len(span), np.uint64), cols.trace_lo[span], cols.parent_id[span],
                           cols.id[span], key.reshape(-1)[keep], np.full(len(span), 6, np.int32),
                           svc.reshape(-1)[keep])
    lower = np.arange(S, dtype=np.int32)
    ctx = N.Context(S, device=device)
    ctx.put_mysql_rows(a, lower)  # warm
    ts = []
    for _ in range(reps):
        ctx.reset()
        t0 = time.perf_counter()
        ctx.put_mysql_rows(a, lower)
        ctx.link()
        ts.append(time.perf_counter() - t0)
    ctx.close()
    t = float(np.median(ts))
    return {"rows": int(len(span)), "spans": m, "traces": k, "ms": t * 1e3, "rows_per_s": len(span) / t,
            "spans_per_s": m / t, "note": "rows host-resident (PCIe-inclusive), timing only"}


def put_trace_leg(cols, S, device, links, reps=3):
    """DependencyLinker.putTrace called once per trace, as the reference's callers loop
    (InMemoryStorage.java:340, AggregateDependencies.java:81): libzdl_synth's native driver
    calls zdl_put_trace for each of the batch's traces in order (what a JNI shim does after
    packing a trace), then zdl_link. The traces are staged into pinned CSR batches and put one
    launch per batch. PCIe-inclusive (host columns in), timed wall clock; the
    links must equal the columnar path's. Compare with cpu_baseline.single_thread (one
    DependencyLinker restated in C++ over the same batch)."""
    from zipkin_amd import _native as N
    from zipkin_amd import synth
    ctx = N.Context(S, device=device)
    ts = []
    out = None
    for k in range(reps + 1):
        ctx.reset()
        t0 = time.perf_counter()
        synth.put_trace_loop(ctx, cols)
        out = ctx.link()
        ts.append(time.perf_counter() - t0)
    ctx.close()
    t = float(np.median(ts[1:]))
    return {"traces": cols.n_traces, "spans": cols.n_spans, "calls": cols.n_traces, "ms": t * 1e3,
            "spans_per_s": cols.n_spans / t, "us_per_call": t / cols.n_traces * 1e6,
            "parity": "same links" if _same_links(out, links) else "MISMATCH",
            "note": "one zdl_put_trace per trace from native code (the JNI caller's loop) + zdl_link; host "
                    "columns, PCIe-inclusive; staged in pinned batches of 2^20 spans"}


def put_trace_c4_leg(device, traces=1_000_000, reps=3):
    """The same per-trace call pattern over C4 (messaging-heavy, 5 % of spans split into merge
    fragments, duplicate ids, missing brokers): every trace through one zdl_put_trace. A trace
    goes alone and synchronously only when its Trace.merge could throw (an (id, shared) group
    holding a null and an incomplete endpoint, zdl_stage.inc); C4's splits never can, so every
    trace is staged. Beside it: one DependencyLinker restated in C++ over the same batch on one
    thread (the reference's single-linker loop), and the links compared."""
    from oracle import ref
    from zipkin_amd import _native as N
    from zipkin_amd import synth
    w = synth.C4.scaled(traces)
    cols = synth.generate(w)
    # traces holding a merge run candidate: two spans with one (id, shared)
    sh = ((cols.port_flags >> np.uint32(19)) & np.uint32(3)) == 2
    tix = np.repeat(np.arange(cols.n_traces), np.diff(cols.offsets.astype(np.int64)))
    key = np.stack([tix, cols.id.view(np.int64), sh.astype(np.int64)])
    o = np.lexsort(key[::-1])
    dup = np.all(key[:, o][:, 1:] == key[:, o][:, :-1], axis=0)
    merge_traces = int(np.unique(key[0, o][1:][dup]).size)
    ctx = N.Context(w.total_services, device=device)
    ts = []
    out = None
    for _ in range(reps + 1):
        ctx.reset()
        t0 = time.perf_counter()
        synth.put_trace_loop(ctx, cols)
        out = ctx.link()
        ts.append(time.perf_counter() - t0)
    ctx.close()
    t = float(np.median(ts[1:]))
    t1 = time.perf_counter()
    st, op, oc, on, oe = ref.link(cols, threads=1)
    t_one = time.perf_counter() - t1
    same = st == 0 and _same_links(out, (op, oc, on, oe))
    return {"workload": w.name, "traces": cols.n_traces, "spans": cols.n_spans, "merge_run_traces": merge_traces,
            "ms": t * 1e3, "spans_per_s": cols.n_spans / t, "us_per_call": t / cols.n_traces * 1e6,
            "cpu_single_thread_ms": t_one * 1e3, "cpu_single_thread_spans_per_s": cols.n_spans / t_one,
            "speedup_vs_single_thread": t_one / t,
            "parity": "bit-exact vs C++ restatement" if same else "MISMATCH",
            "note": "one zdl_put_trace per trace from native code + zdl_link, host columns, PCIe-inclusive; "
                    "the CPU figure is one linker on one thread over the same traces"}


def facade_put_trace_leg(device, traces=20_000):
    """The shipped Python facade's call pattern: zipkin_amd.linker.DependencyLinker.put_trace once
    per trace, each a list of zipkin2 Span objects (C2's first `traces` traces converted, not
    timed), then link() (insertion order, DependencyLink objects). The time is Python's: every
    span's fields are read and packed into columns on the host before the engine sees them (the
    JNI caller passes columns; put_trace_loop times that path). Links compared by service name with
    the C++ restatement over the same traces."""
    from oracle import ref
    from zipkin_amd import synth
    from zipkin_amd.linker import DependencyLinker
    w = synth.C2.scaled(traces)
    cols = synth.generate(w)
    trs = synth.spans_of(cols, w, traces)
    lk = DependencyLinker(device=device)
    warm = 200  # (the engine context and the dictionaries exist before the timed calls)
    for tr in trs[:warm]:
        lk.put_trace(tr)
    lk.link()
    t0 = time.perf_counter()
    for tr in trs[warm:]:
        lk.put_trace(tr)
    links = lk.link()
    t = time.perf_counter() - t0
    timed = len(trs) - warm
    names = synth.service_names(w)
    st, p, c, n, e = ref.link(cols, threads=4)
    exp = sorted(zip([names[i] for i in p], [names[i] for i in c], n.tolist(), e.tolist()))
    got = sorted((l.parent, l.child, l.call_count, l.error_count) for l in links)
    timed_spans = int(cols.offsets[-1] - cols.offsets[warm])
    return {"traces": timed, "spans": timed_spans, "ms": t * 1e3, "us_per_call": t / timed * 1e6,
            "spans_per_s": timed_spans / t, "parity": "same links" if st == 0 and got == exp else "MISMATCH",
            "note": "DependencyLinker.put_trace per trace from Python (Span objects, host packing in Python) + "
                    "link(); C2's first traces; the Python work dominates - the native per-trace path is "
                    "put_trace_loop"}


def _sorted_links(p, c, n, e):
    o = np.lexsort((c, p))
    return p[o], c[o], n[o], e[o]


def _same_links(a, b):
    a, b = _sorted_links(*a), _sorted_links(*b)
    return len(a[0]) == len(b[0]) and all(np.array_equal(x, y) for x, y in zip(a, b))


def _small_bytes(sizes, n_traces):
    """k_link's algorithmic bytes: 44 B per span of the traces it links (<= 64 spans) + the
    8-B offset of every trace (it plans its windows from all of them)."""
    return BYTES_PER_SPAN * int(sizes[sizes <= 64].sum()) + BYTES_PER_TRACE * (n_traces + 1)


def c5_leg(device, steps=48, parity=True, threads=16, host_threads=2, warm_ms=200.0):
    """BASELINE.json configs[4] (C5: 10 000 services, Zipf(1.1), depth 64, fan-out <= 1000,
    Pareto(1.2) trace sizes clipped to [1, 200 000]: 81.1M spans / 16M traces) on one GPU, a
    sparse context (the link list sorted by cell, no S x S table). One step = reset, put of the
    HBM-resident batch (k_link, k_mid, the giant tier, k_tail, the log's sort/merge), link() into
    pinned host columns (4.5M links, 107 MB over PCIe). Per phase: HIP events (ZDL_FLAG_TIMING_ALL,
    the last step), priced at 44 B per span of the traces that phase links."""
    import torch
    from zipkin_amd import _native as N
    from zipkin_amd import synth
    w = synth.C5
    t0 = time.time()
    cols = synth.generate(w)
    log(f"c5: generated {cols.n_spans} spans / {cols.n_traces} traces in {time.time() - t0:.1f}s")
    S = w.total_services
    sizes = np.diff(cols.offsets.astype(np.int64))
    dev = torch.device("cuda", device)
    names = ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags")
    dc = {k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
        np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev) for k in names}
    doff = torch.from_numpy(cols.offsets.view(np.int64)).to(dev)
    # each context reads its own copy of the batch (2.9 GB each)
    dc2 = {k: v.clone() for k, v in dc.items()}
    doff2 = doff.clone()
    bufs = [({k: v.data_ptr() for k, v in dc.items()}, doff), ({k: v.data_ptr() for k, v in dc2.items()}, doff2)]
    # two contexts, two steps in flight: step k's link list crosses PCIe (zdl_link_start) while
    # step k + 1's put runs; every step resets, links every span and reads every link back
    ctxs = [N.Context(S, device=device, timing_all=True) for _ in range(2)]

    def put(c):
        bp, bo = bufs[0 if c is ctxs[0] else 1]
        c.reset()
        c.put_spans_device(bp, cols.n_spans, bo.data_ptr(), cols.n_traces)
        c.link_start()

    for c in ctxs:  # warm (allocations)
        put(c)
        c.link_finish(copy=False)
    torch.cuda.synchronize(dev)
    # one host thread per context (ctypes drops the GIL in every libzdl call): a context's host
    # waits (the giant tier reads two counts back) do not hold up the other context's launches
    import threading
    outs = [None, None]
    errs = []

    def worker(j, n):
        try:
            for _ in range(j, n, 2):
                put(ctxs[j])
                outs[j] = ctxs[j].link_finish(copy=False)
        except Exception as e:  # surfaced after the join
            errs.append(e)

    def run(n):
        if host_threads == 2:
            th = [threading.Thread(target=worker, args=(j, n)) for j in range(2)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        else:  # one host thread alternating the contexts (A/B)
            for k in range(n):
                put(ctxs[k % 2])
                if k:
                    outs[(k - 1) % 2] = ctxs[(k - 1) % 2].link_finish(copy=False)
            outs[(n - 1) % 2] = ctxs[(n - 1) % 2].link_finish(copy=False)
        if errs:
            raise errs[0]
    t_w = time.perf_counter()
    while (time.perf_counter() - t_w) * 1e3 < warm_ms:  # warm-up: the generation left the GPU idle
        run(8)
    t1 = time.perf_counter()
    run(steps)
    ms = (time.perf_counter() - t1) / steps * 1e3
    if errs:
        raise errs[0]
    out = tuple(a.copy() for a in outs[(steps - 1) % 2])
    # the phases of one step run alone (HIP events)
    c = ctxs[0]
    put(c)
    c.link_finish(copy=False)
    t2 = time.perf_counter()
    put(c)
    c.link_finish(copy=False)
    serial_ms = (time.perf_counter() - t2) * 1e3
    k = c.kernel_times()
    ph = [{"k_link": k.tiles_ms, "k_mid": k.mid_ms, "giant_tier": k.giant_ms, "k_tail": k.big_ms,
           "sparse_merge": k.sparse_ms, "link_compact": k.compact_ms}]
    sparse_entries = int(k.sparse_entries)
    for c in ctxs:
        c.close()
    del dc, doff, dc2, doff2, bufs
    gmin = int(os.environ.get("ZDL_GIANT_MIN", "2048")) or None
    gmin = max(gmin, 192) if gmin else None
    big = sizes > 192
    giant = (sizes > gmin) & (sizes <= (1 << 20)) if gmin else np.zeros_like(big)
    spans = {"k_link": int(sizes[sizes <= 64].sum()), "k_mid": int(sizes[(sizes > 64) & ~big].sum()),
             "giant_tier": int(sizes[giant].sum()), "k_tail": int(sizes[big & ~giant].sum())}
    algo = {k: BYTES_PER_SPAN * v for k, v in spans.items()}
    algo["k_link"] = _small_bytes(sizes, cols.n_traces)
    last = ph[-1]
    kern = {}
    for k in ("k_link", "k_mid", "giant_tier", "k_tail"):
        t = last[k]
        gbs = algo[k] / (t * 1e-3) / 1e9 if t and t > 0 else None
        kern[k] = {"ms": t, "spans": spans[k], "algorithmic_bytes": algo[k], "achieved_gbs": gbs,
                   "frac": gbs / HBM_PEAK_GBS if gbs else None}
    for k in ("sparse_merge", "link_compact"):
        kern[k] = {"ms": last[k]}
    # the merge: the put's link log (sparse_entries, 4 B each) read once and the summed list
    # (cell, call, error: 4 + 8 + 8 B a link) written once
    sm = last["sparse_merge"]
    sm_bytes = 4 * sparse_entries + 20 * int(len(out[0]))
    sm_gbs = sm_bytes / (sm * 1e-3) / 1e9 if sm and sm > 0 else None
    kern["sparse_merge"].update({"entries": sparse_entries, "algorithmic_bytes": sm_bytes, "achieved_gbs": sm_gbs,
                                 "frac": sm_gbs / HBM_PEAK_GBS if sm_gbs else None})
    res = {"workload": w.name, "spans": cols.n_spans, "traces": cols.n_traces, "services": S,
           "ms_per_step": ms, "spans_per_s": cols.n_spans / (ms * 1e-3), "inflight": 2, "host_threads": host_threads,
           "ms_per_step_serial": serial_ms,
           "step_roofline_frac": (BYTES_PER_SPAN * cols.n_spans + BYTES_PER_TRACE * (cols.n_traces + 1))
           / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "steps": steps, "giant_min": gmin, "links": int(len(out[0])), "phases": kern,
           "note": "phase times: HIP events of one step run alone (the giant tier's include its two host syncs); "
                   "step: wall clock of reset + put + link into pinned host columns, two contexts in flight "
                   "(host_threads 1: one thread alternating them, zdl_link_start / zdl_link_finish; 2: a thread "
                   "each), a step's link list crossing PCIe while the other context's put runs",
           "parity": None}
    if parity:
        from oracle import ref
        t1 = time.perf_counter()
        st, op, oc, on, oe = ref.link(cols, threads=threads)
        res["parity"] = "bit-exact" if st == 0 and _same_links(out, (op, oc, on, oe)) else "MISMATCH"
        res["oracle_s"] = time.perf_counter() - t1
    return res


def pmc_probe(config, traces, puts=4):
    """The dominant kernel alone for the PMC passes (run under rocprofv3 by pmc_traffic): the
    same batch as the measured step, `puts` puts on a sorted context."""
    import torch
    from zipkin_amd import _native as N
    from zipkin_amd import synth
    w = synth.CONFIGS[config]
    if config == "c3":
        w = w.scaled(C3_TRACES_PER_GPU)
    if traces:
        w = w.scaled(traces)
    cols = synth.generate(w)
    names = ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags")
    dev = torch.device("cuda", 0)
    dc = {k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
        np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev) for k in names}
    doff = torch.from_numpy(cols.offsets.view(np.int64)).to(dev)
    ctx = N.Context(w.total_services, device=0)
    for _ in range(puts):
        ctx.reset()
        ctx.put_spans_device({k: v.data_ptr() for k, v in dc.items()}, cols.n_spans, doff.data_ptr(), cols.n_traces)
        ctx.link()
    ctx.close()
    print(json.dumps({"n_spans": cols.n_spans, "puts": puts}))
    return 0


def pmc_traffic(config, traces, kernel="k_link<", timeout=150):
    """roofline.traffic measured for the build that just ran: two rocprofv3 passes over
    `bench.py --pmc-probe` in child processes (FETCH_SIZE, then WRITE_SIZE: one counter block
    each), averaged over the probe's launches of the dominant kernel. HBM bytes per launch =
    2 x FETCH_SIZE + WRITE_SIZE in KiB (the gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md
    §HBM; calibrated for k_link's 4/8-B lanes, profiles/*_fetch_calibration.json). None if
    rocprofv3 is missing or a pass fails."""
    import csv
    import shutil
    import signal
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, None
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="zdl_pmc_")
        cmd = [prof, "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-probe", "--config", config]
        if traces:
            cmd += ["--traces", str(traces)]
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, start_new_session=True)
        try:
            rc = p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            log(f"pmc {counter}: timed out")
            return None, None
        rows = []
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    rows += [r for r in csv.DictReader(open(os.path.join(root, f)))
                             if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
        shutil.rmtree(d, ignore_errors=True)
        if rc != 0 or not rows:
            log(f"pmc {counter}: rc {rc}, {len(rows)} rows")
            return None, None
        vals[counter] = sum(float(r["Counter_Value"]) for r in rows) / len(rows) * 1024
    hbm = 2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]
    return hbm, {"fetch_size_bytes": vals["FETCH_SIZE"], "write_size_bytes": vals["WRITE_SIZE"],
                 "how": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --pmc-probe (this build, "
                        "same batch), 2 x FETCH_SIZE + WRITE_SIZE per k_link launch"}


def cpu_info():
    """The host cores this process may run on: affinity mask, capped by a cgroup CPU quota
    (the GPU box shares its host: nproc shows the whole machine), plus the CPU model."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    env = os.environ.get("OMP_NUM_THREADS")
    why = f"affinity {aff} of nproc {nproc}" + (f", cgroup quota {quota:g} CPUs" if quota else ", no cgroup quota")
    if env and env.isdigit() and int(env) < usable:
        usable = int(env)
        why += f", OMP_NUM_THREADS={env} (the box's CPU share)"
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": nproc, "affinity": aff, "quota": quota, "usable": usable, "model": model, "why": why}


def c3_job_leg(device, ranks=8, traces_per_rank=C3_TRACES_PER_GPU, steps=5, parity=True, threads=16, warm_ms=200.0):
    """BASELINE.json configs[2] as stated - 1B synthetic spans / 100M traces / 500 services sharded
    by splitmix64(trace_lo) over 8 ranks, the ranks' counts combined (DependencyLinker.merge's sum,
    DependencyLinker.java:189-204) - on ONE MI355X: the 8 ranks are contexts of this process joined
    by zdl_comm_init_local (zipkin_amd/csrc/zdl_xport.inc), so every rank's put, its LOG reduce and
    the job's sum all-reduce run the code of an 8-GPU job; only the combine's bytes move by device
    copies instead of xGMI.

    1. the whole batch is generated in host memory, and split into the 8 shards by the device
       group's host split (zdl_shard.h, timed: `host_split`, SURVEY §8(e)'s named scaling risk);
    2. each shard goes to HBM, and the C++ restatement links it on the host (parity, summed);
    3. `ms_per_job_step`: the 8 ranks' reset + put + link on 8 host threads, median of `steps`;
    4. `phased`: the same with a barrier between the puts and the links, so the link phase
       (the local sum all-reduce + compaction + read-back) is timed apart from the puts; and one
       rank's shard linked on a context outside the world, for the link without a combine."""
    import threading

    import torch
    from zipkin_amd import _native as N
    from zipkin_amd import synth
    w = synth.C3.scaled(ranks * traces_per_rank)
    S = w.total_services
    t0 = time.perf_counter()
    full = synth.generate(w, threads=threads)
    gen_s = time.perf_counter() - t0
    n_spans, n_traces = full.n_spans, full.n_traces
    shards, split_s = synth.shard_host(full, ranks, threads=threads, timestamps=False)
    split_bytes = 2 * (BYTES_PER_SPAN * n_spans + BYTES_PER_TRACE * (n_traces + 1))
    host_split = {"seconds": split_s, "spans": n_spans, "shards": ranks, "threads": threads,
                  "spans_per_s": n_spans / split_s, "host_gbs": split_bytes / split_s / 1e9,
                  "note": "zdl_shard.h plan + scatter (what zdl_put_spans on a device group runs on the host before "
                          "its uploads): 44 B/span + 8 B/trace read and written; host memory bandwidth bound"}
    del full
    log(f"c3 job: generated {n_spans} spans in {gen_s:.1f}s; host split into {ranks} shards {split_s:.2f}s "
        f"({n_spans / split_s:.3e} spans/s on {threads} threads)")
    dev = torch.device("cuda", device)
    names = ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags")
    dcols, doffs, meta = [], [], []
    call = np.zeros(S * S, np.int64)
    err = np.zeros(S * S, np.int64)
    oracle_s = 0.0
    for r in range(ranks):
        cols = shards[r]
        dcols.append({k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
            np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev) for k in names})
        doffs.append(torch.from_numpy(cols.offsets.view(np.int64)).to(dev))
        meta.append((cols.n_spans, cols.n_traces))
        if parity:
            from oracle import ref
            t1 = time.perf_counter()
            st, op, oc, on, oe = ref.link(cols, threads=threads)
            oracle_s += time.perf_counter() - t1
            assert st == 0, st
            np.add.at(call, op.astype(np.int64) * S + oc, on)
            np.add.at(err, op.astype(np.int64) * S + oc, oe)
        shards[r] = None
    torch.cuda.synchronize(dev)
    ctxs = [N.Context(S, device=device) for _ in range(ranks)]
    N.Context.comm_init_local(ctxs)

    def put(r):
        p = {k: v.data_ptr() for k, v in dcols[r].items()}
        ctxs[r].reset()
        ctxs[r].put_spans_device(p, meta[r][0], doffs[r].data_ptr(), meta[r][1])

    out = [None] * ranks
    bar = threading.Barrier(ranks)
    marks = [[0.0, 0.0, 0.0] for _ in range(ranks)]

    def step(phased):
        errs = []

        def run(r):
            try:
                put(r)
                if phased:
                    ctxs[r].sync()
                    marks[r][0] = time.perf_counter()
                    bar.wait()
                    marks[r][1] = time.perf_counter()
                out[r] = ctxs[r].link()
                marks[r][2] = time.perf_counter()
            except Exception as ex:  # noqa: BLE001
                errs.append((r, repr(ex)))
                bar.abort()

        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        th = [threading.Thread(target=run, args=(r,)) for r in range(ranks)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise RuntimeError(f"c3 job: rank failure {errs}")
        t2 = time.perf_counter()
        if not phased:
            return (t2 - t1) * 1e3, None, None
        puts = max(m[0] for m in marks) - t1
        links = max(m[2] for m in marks) - max(m[1] for m in marks)
        return (t2 - t1) * 1e3, puts * 1e3, links * 1e3

    t_w = time.perf_counter()
    while True:  # warm-up: at least one step and warm_ms of load (the generation left the GPU idle)
        step(False)
        if (time.perf_counter() - t_w) * 1e3 >= warm_ms:
            break
    job = [step(False)[0] for _ in range(steps)]
    ph = [step(True) for _ in range(steps)]
    ranks_agree = all(all(np.array_equal(a, b) for a, b in zip(out[0], out[r])) for r in range(ranks))
    for c in ctxs:
        c.close()
    # the link of one rank's shard without a combine: a context outside the world
    solo = N.Context(S, device=device)
    sl = []
    for _ in range(steps + 1):
        p = {k: v.data_ptr() for k, v in dcols[0].items()}
        solo.reset()
        solo.put_spans_device(p, meta[0][0], doffs[0].data_ptr(), meta[0][1])
        solo.sync()
        t1 = time.perf_counter()
        solo.link()
        sl.append((time.perf_counter() - t1) * 1e3)
    solo.close()
    del dcols, doffs
    torch.cuda.empty_cache()
    ms = float(np.median(job))
    link_phase = float(np.median([x[2] for x in ph]))
    solo_link = float(np.median(sl[1:]))
    res = {"workload": "c3_1B_spans_100M_traces_500_services as BASELINE.json states it: an 8-rank job on one "
                       "MI355X (zdl_comm_init_local; the ranks' bytes move by device copies, not xGMI)",
           "ranks": ranks, "spans": n_spans, "traces": n_traces, "services": S, "steps": steps,
           "ms_per_job_step": ms, "spans_per_s": n_spans / (ms * 1e-3),
           "step_roofline_frac": (BYTES_PER_SPAN * n_spans + BYTES_PER_TRACE * (n_traces + ranks)) / (ms * 1e-3) / 1e9
           / HBM_PEAK_GBS,
           "phased": {"ms_per_job_step": float(np.median([x[0] for x in ph])),
                      "puts_ms": float(np.median([x[1] for x in ph])),
                      "link_phase_ms": link_phase, "solo_link_ms": solo_link,
                      "combine_ms": max(link_phase - solo_link, 0.0),
                      "note": "puts: step start to the last rank's put done (8 ranks' k_link + LOG reduce on one GPU); "
                              "link phase: every rank's zdl_link after a barrier (the local sum all-reduce of the "
                              "500 x 500 tables + compaction + read-back), max over ranks; combine = link phase - "
                              "the same link on a context outside the world"},
           "host_split": host_split, "generate_s": gen_s, "links": int(len(out[0][0])), "ranks_agree": ranks_agree}
    if parity:
        nz = np.nonzero(call)[0]
        exp = sorted(zip((nz // S).tolist(), (nz % S).tolist(), call[nz].tolist(), err[nz].tolist()))
        got = sorted(zip(*(a.tolist() for a in out[0])))
        res["parity"] = "bit-exact vs the C++ restatement over every span" if got == exp and ranks_agree else "MISMATCH"
        res["oracle_s"] = oracle_s
        res["calls"] = int(call.sum())
    return res


def h2d_leg(cols, S, device, reps=3):
    """Host-buffer side of the path (not `value`): the batch's 44 B/span columns + offsets
    copied from pinned host memory (the PCIe rate a JNI caller with pinned buffers gets), and
    a whole zdl_put_spans + zdl_link from pageable numpy columns (pack excluded)."""
    import torch
    from zipkin_amd import _native as N
    names = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags")
    host = [torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
        np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).pin_memory() for k in names]
    host.append(torch.from_numpy(cols.offsets.view(np.int64)).pin_memory())
    dev = torch.device("cuda", device)
    outs = [torch.empty_like(h, device=dev) for h in host]
    nbytes = sum(h.numel() * h.element_size() for h in host)
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for h, o in zip(host, outs):
            o.copy_(h, non_blocking=True)
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    h2d = float(np.median(ts[1:]))
    ctx = N.Context(S, device=device)
    es = []
    for _ in range(reps + 1):
        ctx.reset()
        t0 = time.perf_counter()
        ctx.put_spans(cols)
        ctx.link()
        es.append(time.perf_counter() - t0)
    ctx.close()
    e2e = float(np.median(es[1:]))
    del outs, host
    return {"bytes": nbytes, "h2d_ms": h2d * 1e3, "h2d_gbs": nbytes / h2d / 1e9, "e2e_ms": e2e * 1e3,
            "e2e_spans_per_s": cols.n_spans / e2e,
            "note": "h2d: pinned host -> HBM copy of the 44 B/span columns; e2e: zdl_put_spans (pageable host "
                    "columns, staged copies) + zdl_link, PCIe-inclusive"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200,
                    help="timed steps (the pipeline of two steps in flight fills and drains once per leg: ~5 %% of 20 steps)")
    ap.add_argument("--warmup", type=int, default=20, help="untimed steps before the timed ones")
    ap.add_argument("--warm-ms", type=float, default=200.0,
                    help="after the --warmup steps, more untimed steps until the warm-up has lasted this long "
                         "(the GPU's clocks ramp over the first ~50 ms of load: profiles/r06i_warm_probe.txt)")
    ap.add_argument("--config", default=None, help="default: c2 at N = 1, c3 (per-GPU shard) at N > 1")
    ap.add_argument("--traces", type=int, default=0, help="override traces per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-h2d", action="store_true", help="skip the host-buffer (PCIe-inclusive) leg")
    ap.add_argument("--no-proto3", action="store_true", help="skip the proto3 ingest side leg")
    ap.add_argument("--no-mysql-rows", action="store_true", help="skip the mysql-v1 rows side leg")
    ap.add_argument("--no-json", action="store_true", help="skip the JSON v2 ingest side leg")
    ap.add_argument("--no-store", action="store_true", help="skip the resident-store getDependencies side leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (high-cardinality) side leg")
    ap.add_argument("--no-put-trace", action="store_true", help="skip the per-trace putTrace loop side leg")
    ap.add_argument("--no-c3-job", action="store_true",
                    help="skip the 1B-span C3 job side leg (8 ranks as a local world on this GPU)")
    ap.add_argument("--c3-job-traces", type=int, default=C3_TRACES_PER_GPU, help=argparse.SUPPRESS)
    ap.add_argument("--c5-host-threads", type=int, default=2, choices=(1, 2),
                    help="C5 leg: one host thread per context (2) or one alternating both (1)")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 FETCH_SIZE / WRITE_SIZE passes behind roofline.traffic")
    ap.add_argument("--pmc-probe", action="store_true", help=argparse.SUPPRESS)  # child of pmc_traffic
    ap.add_argument("--timing-stride", type=int, default=8,
                    help="k_link HIP events around every n-th put of a context (roofline.achieved)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="steps in flight (contexts used round-robin): default 2")
    ap.add_argument("--no-insertion-order", action="store_true",
                    help="skip the side measurement of the insertion-order mode (N = 1 only)")
    args = ap.parse_args()

    if args.pmc_probe:
        return pmc_probe(args.config or "c2", args.traces)

    import torch

    from zipkin_amd import _native as N
    from zipkin_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dist = None
    if world > 1:
        # a CPU (gloo) group for the bootstrap only: the RCCL unique id broadcast, barriers and
        # the max-over-ranks timing. The one communicator on the GPUs is libzdl's own (zdl_comm_init).
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("gloo", init_method="env://")
    dev = torch.device("cuda", local)

    config = args.config or ("c2" if world == 1 else "c3")
    w = synth.CONFIGS[config]
    if config == "c3":  # weak scaling: one C3 per-GPU shard per rank
        w = w.scaled(C3_TRACES_PER_GPU)
    if args.traces:
        w = w.scaled(args.traces)
    if world > 1:
        w = w.sharded(rank, world)
    t0 = time.time()
    cols = synth.generate(w)
    log(f"[rank {rank}] generated {cols.n_spans} spans / {cols.n_traces} traces in {time.time() - t0:.1f}s")
    S = w.total_services

    names = ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags", "timestamp")
    dcols = {k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
        np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev) for k in names}
    doff = torch.from_numpy(cols.offsets.view(np.int64)).to(dev)
    ptrs = {k: v.data_ptr() for k, v in dcols.items()}
    ptrs["timestamp"] = None
    inflight = args.inflight or 2
    # every in-flight context links its OWN copy of the batch (C2: 448 MB each), so a second
    # reader of the same bytes cannot be served from the 256 MiB Infinity Cache; the
    # shared-input step is measured beside it (config.ms_per_step_shared_input)
    batches = [(ptrs, doff)]
    keep = [dcols]
    for _ in range(inflight - 1):
        dc2 = {k: v.clone() for k, v in dcols.items()}
        keep.append(dc2)
        p2 = {k: v.data_ptr() for k, v in dc2.items()}
        p2["timestamp"] = None
        batches.append((p2, doff.clone()))
        keep.append(batches[-1][1])
    torch.cuda.synchronize(dev)

    # Steps in flight: with 2, step k+1's reset and put (another context, its own stream) are
    # enqueued before step k's links are read, so the host's work of reading one step's links
    # and launching the next overlaps the GPU's work instead of idling it (~25 us a step at C2).
    # Every step still resets, links every span and reads every link back. HIP events time
    # k_link on every timing_stride-th put (each event pair costs the step a few microseconds).
    ctxs = [N.Context(S, device=local, timing=True, timing_stride=args.timing_stride)
            for _ in range(inflight)]
    ctx = ctxs[0]
    combine = "none"
    if world > 1:
        # Every in-flight context joins its own RCCL communicator (zdl_comm_init): zdl_link sums
        # every rank's tables with ncclAllReduce over xGMI inside the library, as a JVM caller
        # would get it. The contexts' links are read one at a time in the same order on every
        # rank (link() returns after its all-reduce), so the communicators' collectives never
        # overlap. There is no other combine path: a rank that cannot join fails the run.
        uids = [[N.Context.comm_unique_id() for _ in range(inflight)] if rank == 0 else None]
        dist.broadcast_object_list(uids, src=0)
        try:
            for c, uid in zip(ctxs, uids[0]):
                c.comm_init(uid, rank, world)
        except N.ZdlError as ex:
            log(f"[rank {rank}] zdl_comm_init failed: {ex}")
            sys.exit(1)
        combine = f"libzdl RCCL all-reduce (zdl_comm_init, one communicator per in-flight context x{inflight})"

    def launch(c, j=0):
        bp, bo = batches[j]
        c.reset()
        c.put_spans_device(bp, cols.n_spans, bo.data_ptr(), cols.n_traces)

    def run(k_steps, shared=False):
        """k_steps steps: every step's put is launched, every step's links are read. Context j
        reads batch copy j (shared: every context reads copy 0)."""
        res = None
        for k in range(k_steps):
            launch(ctxs[k % inflight], 0 if shared else k % inflight)
            if k >= inflight - 1:
                res = ctxs[(k - inflight + 1) % inflight].link(copy=False)
        for k in range(max(k_steps - inflight + 1, 0), k_steps):
            res = ctxs[k % inflight].link(copy=False)
        return tuple(a.copy() for a in res)  # views of the context's output columns until its next link

    def sync_all():
        for c in ctxs:
            c.sync()
        torch.cuda.synchronize(dev)

    # Warm-up: --warmup steps, then more in chunks until --warm-ms have passed (every rank runs the
    # same number: with RCCL each link() is a collective). A run's first ~50 ms of steps are up to
    # 20 % slower than the steady state whatever the step count (profiles/r06i_warm_probe.txt).
    t_warm = time.perf_counter()
    run(args.warmup)
    warm_steps = args.warmup
    chunk = max(inflight * 4, 8)
    while True:
        sync_all()
        more = torch.tensor([1 if (time.perf_counter() - t_warm) * 1e3 < args.warm_ms else 0])
        if dist:
            dist.all_reduce(more, op=dist.ReduceOp.MAX)
        if not int(more):
            break
        run(chunk)
        warm_steps += chunk
    warm_ms = (time.perf_counter() - t_warm) * 1e3
    for c in ctxs:
        c.kernel_times()  # drops the warmup puts from the k_link event rings
    if dist:
        dist.barrier()
    sync_all()
    t_start = time.perf_counter()
    out = run(args.steps)
    sync_all()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    # HIP events around every timed put's k_link (a ring per context), averaged once here:
    # with steps in flight two launches overlap, so this is NOT a kernel duration (reported as
    # kernel_ms.k_link_inflight_events, never priced)
    kts = [float(c.kernel_times().tiles_ms) for c in ctxs]
    kts = [x for x in kts if x > 0] or [float("nan")]
    tiles_inflight = float(np.mean(kts))
    shared_ms = None
    legs = None
    if inflight > 1:
        # the same in-flight steps with every context reading ONE copy of the batch, interleaved
        # with more distinct-copy legs (shared, distinct, shared, distinct after the headline
        # leg): a difference that follows the input and not the position is the input's
        legs = []
        for shared in (True, False, True, False):
            sync_all()
            t1 = time.perf_counter()
            run(args.steps, shared=shared)
            sync_all()
            legs.append({"input": "shared" if shared else "distinct",
                         "ms_per_step": (time.perf_counter() - t1) / args.steps * 1e3})
        shared_ms = float(np.median([g["ms_per_step"] for g in legs if g["input"] == "shared"]))
    # The step's contexts are done: close them before the serial leg and the side legs. Each
    # context owns a HIP stream, and with GPU_MAX_HW_QUEUES=4 (the box's setting) streams beyond
    # four share hardware queues - the C5 leg's two contexts then ran one after the other (7.7 ms
    # a step instead of 6.1 with its two streams on queues of their own).
    for c in ctxs:
        c.close()
    # The serial leg: the same step one at a time on a context timing EVERY k_link (HIP events
    # on its stream, nothing else on the GPU) - this k_link duration prices `roofline`
    sctx = N.Context(S, device=local, timing=True, timing_stride=1) if world == 1 else None
    serial_ms = None
    tiles = tiles_inflight
    if sctx is not None:
        ns = max(min(args.steps, 20), 3)
        # its own warm-up: the contexts' close and this one's setup leave the GPU idle for a few
        # ms, after which k_link runs ~5 % slower until the load has lasted ~50 ms again
        t_sw = time.perf_counter()
        while True:
            launch(sctx)
            sctx.link()
            if (time.perf_counter() - t_sw) * 1e3 >= args.warm_ms / 2:
                break
        sctx.sync()
        sctx.kernel_times()
        t1 = time.perf_counter()
        for _ in range(ns):
            launch(sctx)
            sctx.link(copy=False)
        sctx.sync()
        serial_ms = (time.perf_counter() - t1) / ns * 1e3
        tiles = float(sctx.kernel_times().tiles_ms)
        sctx.close()
    log_reduce = None
    if world == 1 and config == "c3":
        # LOG mode's reduce of k_link's emit log (zdl_log.inc), one put alone with HIP events
        # around every phase (ZDL_FLAG_TIMING_ALL): priced on its input, 4 B an entry read once
        pctx = N.Context(S, device=local, timing_all=True)
        for _ in range(2):
            launch(pctx)
            pctx.link(copy=False)
        pctx.sync()
        kt = pctx.kernel_times()
        pctx.close()
        ent = int(kt.log_entries)
        rms = float(kt.reduce_ms)
        gbs = 4 * ent / (rms * 1e-3) / 1e9 if rms > 0 else None
        log_reduce = {"ms": rms, "entries": ent, "algorithmic_bytes": 4 * ent,
                      "moved_bytes_model": 4 * ent,
                      "achieved_gbs": gbs, "frac": gbs / HBM_PEAK_GBS if gbs else None,
                      "k_link_ms_same_put": float(kt.tiles_ms),
                      "note": "k_hist3 of one put (HIP events): the block pool read once (4 B/entry); k_link's "
                              "workgroups moved the log into the pool by partition at their ends (8 B/entry, "
                              "inside k_link's time)"}
    ctxs = []
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tot = torch.tensor([cols.n_spans], dtype=torch.int64)
        dist.all_reduce(tot)
        total_spans = int(tot.item())
    else:
        total_spans = cols.n_spans

    p, c, n, e = out
    # side measurement (not `value`): the same batch on an insertion-order context, whose
    # link() is DependencyLinker.link()'s list order (k_link plans, k_tail links exactly)
    ins = None
    ins_out = None
    side = world == 1 and config == "c2"  # the side legs run on C2 only
    if side and not args.no_insertion_order:
        # the DependencyLinker facade's engine configuration: its table capacity for S services
        # (_capacity: the dense LDS table up to 67) on an insertion-order context, service ranks set;
        # two contexts in flight as in the headline (a caller linking consecutive batches), and
        # the same steps one at a time on one context (as the Python facade drives it)
        from zipkin_amd.linker import _capacity
        names_w = synth.service_names(w)
        rk = np.empty(S, np.int32)
        rk[np.argsort(np.array(names_w, dtype=object), kind="stable")] = np.arange(S, dtype=np.int32)
        ictxs = [N.Context(_capacity(S), device=local, insertion_order=True) for _ in range(2)]
        for ic in ictxs:
            ic.set_ranks(N.ZDL_DICT_SERVICE, rk)

        def iput(ic, j):
            bp, bo = batches[j] if j < len(batches) else batches[0]
            ic.reset()
            ic.put_spans_device(bp, cols.n_spans, bo.data_ptr(), cols.n_traces)

        def irun(k_steps, inflight_i):
            res = None
            for k in range(k_steps):
                iput(ictxs[k % inflight_i], k % inflight_i)
                if k >= inflight_i - 1:
                    res = ictxs[(k - inflight_i + 1) % inflight_i].link(N.ZDL_ORDER_INSERTION)
            for k in range(max(k_steps - inflight_i + 1, 0), k_steps):
                res = ictxs[k % inflight_i].link(N.ZDL_ORDER_INSERTION)
            return res

        t_w = time.perf_counter()
        while True:  # warm-up (the contexts' setup left the GPU idle for a few ms)
            irun(8, 2)
            if (time.perf_counter() - t_w) * 1e3 >= args.warm_ms / 2:
                break
        for ic in ictxs:
            ic.sync()
        ik = max(args.steps, 10)
        t1 = time.perf_counter()
        ins_out = irun(ik, 2)
        for ic in ictxs:
            ic.sync()
        it = (time.perf_counter() - t1) / ik
        t1 = time.perf_counter()
        irun(ik, 1)
        ictxs[0].sync()
        it1 = (time.perf_counter() - t1) / ik
        for ic in ictxs:
            ic.close()
        ins = {"ms_per_step": it * 1e3, "spans_per_s": cols.n_spans / it, "steps": ik, "inflight": 2,
               "ms_per_step_serial": it1 * 1e3, "parity": None,
               "capacity": _capacity(S), "note": "DependencyLinker facade's context: _capacity(S) services, "
                                                 "insertion order, service ranks; reset + put + link(ZDL_ORDER_"
                                                 "INSERTION) per step, two contexts in flight like the headline "
                                                 "(serial: one context, one step at a time)"}
    del keep, batches[1:]  # (the insertion-order leg's second context read its own copy, as the headline's)
    # side measurement (not `value`): the same batch as a proto3 ListOfSpans decoded on the device
    # (zdl_decode_proto3) and linked from the decoded HBM columns
    p3 = None
    if side and not args.no_proto3:
        p3 = proto3_leg(cols, w, S, local, doff, (p, c, n, e))
        log(f"proto3 ingest: kernel {p3['kernel_ms']:.3f} ms ({p3['kernel_gbs']:.0f} GB/s), "
            f"call {p3['call_ms']:.1f} ms, links {p3['parity']}")
    jleg = None
    if side and not args.no_json:
        jleg = json_v2_leg(cols, w, local, doff, (p, c, n, e))
        log(f"json v2 ingest: {jleg['bytes'] / 1e9:.2f} GB, device {jleg['device_ms']:.2f} ms "
            f"(structure {jleg['structure_ms']:.2f}, spans {jleg['spans_kernel_ms']:.2f}), "
            f"call {jleg['call_ms']:.1f} ms, links {jleg['parity']}")
    sleg = None
    if side and not args.no_store:
        sleg = store_leg(cols, S, local, (p, c, n, e), synth.service_names(w))
        log(f"store getDependencies: {sleg['get_dependencies_ms']:.2f} ms (select {sleg['select_ms']:.2f} ms), "
            f"facade {sleg['facade_get_dependencies_ms']:.2f} ms, accept {sleg['accept_ms']:.1f} ms (warm {sleg['accept_warm_ms']:.1f}), "
            f"links {sleg['parity']}")
    rows_leg = None
    if side and not args.no_mysql_rows:
        rows_leg = mysql_rows_leg(cols, S, local)
        log(f"mysql rows: {rows_leg['rows']} rows in {rows_leg['ms']:.1f} ms ({rows_leg['rows_per_s']:.3e} rows/s)")
    h2d = None
    if side and not args.no_h2d:
        h2d = h2d_leg(cols, S, local)
        log(f"host buffers: H2D {h2d['h2d_ms']:.2f} ms ({h2d['h2d_gbs']:.1f} GB/s pinned), put+link from pageable "
            f"host columns {h2d['e2e_ms']:.2f} ms")
    ptl = None
    if side and not args.no_put_trace:
        ptl = put_trace_leg(cols, S, local, (p, c, n, e))
        log(f"putTrace loop: {ptl['ms']:.1f} ms for {ptl['calls']} calls ({ptl['spans_per_s']:.3e} spans/s, "
            f"{ptl['us_per_call']:.3f} us/call), links {ptl['parity']}")
    ptc4 = None
    if side and not args.no_put_trace:
        ptc4 = put_trace_c4_leg(local)
        log(f"putTrace loop c4: {ptc4['ms']:.1f} ms for {ptc4['traces']} calls ({ptc4['merge_run_traces']} with merge "
            f"runs), {ptc4['us_per_call']:.3f} us/call; one C++ linker on 1 thread {ptc4['cpu_single_thread_ms']:.0f} "
            f"ms ({ptc4['speedup_vs_single_thread']:.1f}x), links {ptc4['parity']}")
    fpt = None
    if side and not args.no_put_trace:
        fpt = facade_put_trace_leg(local)
        log(f"putTrace from the Python facade: {fpt['ms']:.0f} ms for {fpt['traces']} calls "
            f"({fpt['us_per_call']:.1f} us/call, {fpt['spans_per_s']:.3e} spans/s), links {fpt['parity']}")
    c5 = None
    if side and not args.no_c5:
        c5 = c5_leg(local, parity=not args.no_parity, threads=cpu_info()["usable"], host_threads=args.c5_host_threads,
                    warm_ms=args.warm_ms)
        log(f"c5: {c5['ms_per_step']:.2f} ms/step ({c5['spans_per_s']:.3e} spans/s), links {c5['parity']}, "
            + ", ".join(f"{k} {v['ms']:.3f} ms" for k, v in c5["phases"].items() if v["ms"] is not None))
    c3job = None
    if side and not args.no_c3_job:
        c3job = c3_job_leg(local, traces_per_rank=args.c3_job_traces, parity=not args.no_parity,
                           threads=cpu_info()["usable"], warm_ms=args.warm_ms)
        log(f"c3 job (1B spans, 8 ranks on one GPU): {c3job['ms_per_job_step']:.2f} ms/job step "
            f"({c3job['spans_per_s']:.3e} spans/s), puts {c3job['phased']['puts_ms']:.2f} ms, link phase "
            f"{c3job['phased']['link_phase_ms']:.2f} ms (combine {c3job['phased']['combine_ms']:.2f} ms), "
            f"links {c3job.get('parity')}")
    parity = None
    cpu = None
    if rank == 0 and world == 1 and not args.no_parity:
        from oracle import ref
        ci = cpu_info()
        threads = ci["usable"]
        t1 = time.perf_counter()
        st, op, oc, on, oe = ref.link(cols, threads=threads)
        t_multi = time.perf_counter() - t1
        got = sorted(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))
        exp = sorted(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))
        parity = "bit-exact" if (st == 0 and got == exp) else "MISMATCH"
        if ins is not None:
            ip, ic, inn, ie = ins_out
            iseq = list(zip(ip.tolist(), ic.tolist(), inn.tolist(), ie.tolist()))
            oseq = list(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))
            ins["parity"] = "exact order" if (st == 0 and iseq == oseq) else "MISMATCH"
            log(f"insertion order: {ins['ms_per_step']:.3f} ms/step in flight ({ins['ms_per_step_serial']:.3f} serial), "
                f"{ins['parity']}")
        log(f"parity vs C++ restatement ({threads} threads, {t_multi:.2f}s): {parity}, {len(got)} links")
        if not args.no_cpu_baseline:
            # the whole batch on one thread = one DependencyLinker over every trace
            t1 = time.perf_counter()
            ref.link(cols, threads=1)
            t_one = time.perf_counter() - t1
            cpu = {"value": cols.n_spans / t_multi, "unit": "spans/s", "cores": threads, "kind": "port",
                   "sample": f"the whole {w.name} batch ({cols.n_spans} spans), trace-sharded C++ restatement "
                             f"of DependencyLinker (one linker per thread + DependencyLinker.merge) on {threads} "
                             f"threads = every core this process may use ({ci['why']})",
                   "cpu": ci, "seconds": t_multi,
                   "single_thread": {"value": cols.n_spans / t_one, "cores": 1, "seconds": t_one,
                                     "sample": "the same batch through one linker, 1 thread"}}
            log(f"cpu baseline: {cols.n_spans / t_one:.3e} spans/s on 1 thread; {cols.n_spans / t_multi:.3e} on "
                f"{threads} ({ci['model']})")

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        # every span once (44 B) and every trace offset once
        bytes_launch = BYTES_PER_SPAN * cols.n_spans + BYTES_PER_TRACE * (cols.n_traces + 1)
        # k_link is priced with the spans it links (traces of <= 64 spans: all of C2's and C3's)
        sizes = np.diff(cols.offsets.astype(np.int64))
        klink_bytes = _small_bytes(sizes, cols.n_traces)
        small = int(sizes[sizes <= 64].sum())
        read_launch = READ_BYTES_PER_SPAN * small + BYTES_PER_TRACE * (cols.n_traces + 1)
        achieved = klink_bytes / (tiles * 1e-3) / 1e9
        traffic = None
        traffic_src = None
        if world == 1 and not args.no_traffic:  # PMC passes of this very build, in child processes
            traffic, traffic_src = pmc_traffic(config, args.traces)
        line = {
            "metric": METRIC,
            "value": total_spans / elapsed * args.steps,
            "unit": "spans/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": w.name, "spans_per_gpu": cols.n_spans, "traces_per_gpu": cols.n_traces,
                       "services": S, "parallelism": f"trace-shard x{world}", "combine": combine,
                       "inflight": inflight, "warm_up": {"steps": warm_steps, "ms": warm_ms},
                       "ms_per_step_serial": serial_ms,
                       "ms_per_step_shared_input": shared_ms,
                       "interleaved_legs": legs,
                       "step_roofline_frac_serial": (bytes_launch / (serial_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                                     if serial_ms else None),
                       "kernel_ms": {"k_link": tiles,
                                     "k_link_source": "HIP events around every k_link of the serial leg (one "
                                                      "step at a time, nothing else on the GPU)" if world == 1
                                     else "HIP events around every 8th k_link (one step in flight)",
                                     "k_link_inflight_events": tiles_inflight},
                       "step_roofline_frac": bytes_launch / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                       "k_link_read_frac": read_launch / (tiles * 1e-3) / 1e9 / HBM_PEAK_GBS,
                       "log_reduce": log_reduce,
                       "parity": parity, "links": int(len(p)), "insertion_order": ins, "host_buffers": h2d,
                       "proto3_ingest": p3, "json_v2_ingest": jleg, "store_get_dependencies": sleg,
                       "mysql_rows": rows_leg, "put_trace_loop": ptl, "put_trace_loop_c4": ptc4, "facade_put_trace_python": fpt,
                       "c5": c5, "c3_job": c3job},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_link", "algorithmic_bytes_per_launch": klink_bytes,
                         "bytes_per_span": BYTES_PER_SPAN, "bytes_per_trace": BYTES_PER_TRACE},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
