"""A job's combines with W > 1 ranks, executed on the box's one GPU (zdl_comm_init_local,
zipkin_amd/csrc/zdl_xport.inc): W contexts of this process are ranks 0..W-1, each links its
splitmix64(trace_lo) shard (shard.partition_columns), and every rank's zdl_link
runs on its own thread, as the processes of an RCCL job call it. Everything above the transport
runs as in an RCCL job - the dense tables' sum all-reduce, the insertion-order MIN of rank-tagged
first ranks, the sparse reduce-scatter by cell range (samples, splitters, W x W slice lengths,
the all-to-all, the per-range sums, the all-gather of the ranges); only the bytes move by device
copies instead of xGMI. Every rank must return the links of the whole batch:

* sorted output: the C++ restatement over every trace (DependencyLinker.merge's sums,
  DependencyLinker.java:189-204);
* insertion order: DependencyLinker.merge (the oracle's) over the ranks' own link() lists -
  the restatement over each shard - concatenated in rank order.
"""
import threading
from collections import namedtuple

import numpy as np
import pytest

from oracle import dl_oracle as O
from oracle import ref
from zipkin_amd import _native as N
from zipkin_amd import shard, synth
from zipkin_amd.columnar import Columns, concat_columns

pytestmark = pytest.mark.gpu

Link = namedtuple("Link", "parent child call_count error_count")


def _tuples(p, c, n, e):
    return list(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))


def _oracle(cols, threads=16):
    st, p, c, n, e = ref.link(cols, threads=threads)
    assert st == 0
    return _tuples(p, c, n, e)


def _empty():
    z = lambda t: np.zeros(0, t)  # noqa: E731
    return Columns(z(np.uint64), z(np.uint64), z(np.uint64), z(np.int32), z(np.int32), z(np.int32), z(np.int32),
                   z(np.uint32), z(np.int64), np.zeros(1, np.uint64))


def _concurrently(ctxs, fn):
    """fn(k, ctx) on one thread per rank, all at once (the ranks of a job); returns the results."""
    out = [None] * len(ctxs)
    errs = []

    def run(k):
        try:
            out[k] = fn(k, ctxs[k])
        except Exception as ex:  # noqa: BLE001 - reported below with the rank
            errs.append((k, repr(ex)))

    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(ctxs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a rank is still running"
    assert not errs, errs
    return out


def _job(parts, S, puts=1, **kw):
    ctxs = [N.Context(S, **kw) for _ in parts]
    N.Context.comm_init_local(ctxs)
    for c, p in zip(ctxs, parts):
        for _ in range(puts):
            c.put_spans(p)
    return ctxs


def _close(ctxs):
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("W", [2, 3, 8])
@pytest.mark.parametrize("config", ["c2", "c3"])
def test_dense_tables_summed_over_ranks(W, config):
    """C2's dense LDS table (50 services) and C3's LOG-mode tables (500 services): the sum
    all-reduce (comm_sum_tables) gives every rank the whole batch's links; a second link of the
    same job and a reset + put reuse the collectives."""
    w = synth.CONFIGS[config].scaled(60_000)
    cols = synth.generate(w)
    parts = shard.partition_columns(cols, W)
    assert all(p.n_spans > 0 for p in parts)
    ctxs = _job(parts, w.total_services)
    try:
        got = _concurrently(ctxs, lambda k, c: sorted(_tuples(*c.link())))
        again = _concurrently(ctxs, lambda k, c: sorted(_tuples(*c.link())))

        def reput(k, c):
            c.reset()
            c.put_spans(parts[k])
            c.put_spans(parts[k])
            return sorted(_tuples(*c.link()))
        twice = _concurrently(ctxs, reput)
    finally:
        _close(ctxs)
    exp = sorted(_oracle(cols))
    assert len(exp) > 100
    for k in range(W):
        assert got[k] == exp and again[k] == exp
        assert twice[k] == [(a, b, 2 * n, 2 * e) for a, b, n, e in exp]


def _merge_in_rank_order(parts):
    """DependencyLinker.merge (oracle) over each shard's link() list (the restatement's
    insertion order), concatenated in rank order."""
    links = []
    for p in parts:  # the oracle's merge keys links by service name: ids as names, and back
        if p.n_spans:
            links += [Link(f"s{a}", f"s{b}", n, e) for a, b, n, e in _oracle(p)]
    return [(int(l.parent[1:]), int(l.child[1:]), l.call_count, l.error_count)
            for l in O.DependencyLinker.merge(links)]


@pytest.mark.parametrize("W", [2, 3, 8])
@pytest.mark.parametrize("config", ["c2", "c4"])
def test_insertion_order_across_ranks(W, config):
    """comm_sum_ord: the sums, and the MIN of the rank-tagged first-seen ranks, give every rank
    DependencyLinker.merge's order over the ranks' lists in rank order - exactly."""
    w = synth.CONFIGS[config].scaled(30_000)
    cols = synth.generate(w)
    parts = shard.partition_columns(cols, W)
    ctxs = _job(parts, w.total_services, insertion_order=True)
    try:
        got = _concurrently(ctxs, lambda k, c: _tuples(*c.link(N.ZDL_ORDER_INSERTION)))
    finally:
        _close(ctxs)
    exp = _merge_in_rank_order(parts)
    assert len(exp) > 100
    for k in range(W):
        assert got[k] == exp


@pytest.mark.parametrize("W", [3, 8])
def test_insertion_order_local_order_tags(W, monkeypatch):
    """The combine's second tagging (beyond 64 ranks: each rank's first ranks replaced by their
    order among its own pairs, rank << 32 | index), forced at a small world: the same order."""
    monkeypatch.setenv("ZDL_ORD_LOCAL_ORDER", "1")
    w = synth.C4.scaled(20_000)
    cols = synth.generate(w)
    parts = [_empty()] + shard.partition_columns(cols, W - 1)
    ctxs = _job(parts, w.total_services, insertion_order=True, puts=2)
    try:
        got = _concurrently(ctxs, lambda k, c: _tuples(*c.link(N.ZDL_ORDER_INSERTION)))
    finally:
        _close(ctxs)
    exp = _merge_in_rank_order(parts)
    assert len(exp) > 100
    for k in range(W):
        assert [(a, b, n // 2, e // 2) for a, b, n, e in got[k]] == exp


def test_insertion_order_beyond_64_ranks():
    """66 ranks (the rank tag's 6 bits no longer suffice): the local-order tags, exact order."""
    W = 66
    w = synth.C2.scaled(6_600)
    cols = synth.generate(w)
    parts = shard.partition_columns(cols, W)
    ctxs = _job(parts, w.total_services, insertion_order=True)
    try:
        got = _concurrently(ctxs, lambda k, c: _tuples(*c.link(N.ZDL_ORDER_INSERTION)))
    finally:
        _close(ctxs)
    exp = _merge_in_rank_order(parts)
    assert len(exp) > 100
    for k in (0, 1, 33, W - 1):
        assert got[k] == exp


def test_insertion_order_empty_first_rank():
    """Rank 0 holds nothing: its tags never win the MIN; the order starts at rank 1's list."""
    w = synth.C4.scaled(20_000)
    cols = synth.generate(w)
    parts = [_empty()] + shard.partition_columns(cols, 2)
    ctxs = _job(parts, w.total_services, insertion_order=True)
    try:
        got = _concurrently(ctxs, lambda k, c: _tuples(*c.link(N.ZDL_ORDER_INSERTION)))
    finally:
        _close(ctxs)
    exp = _merge_in_rank_order(parts)
    for k in range(3):
        assert got[k] == exp


def _c5_like(traces):
    return synth.Workload("c5_like_10k", 0x5EED0078, traces, 10_000, max_depth=32, size_dist=1, pareto_alpha=1.3,
                          max_size=3000, max_fanout=200, zipf_s=1.1)


@pytest.mark.parametrize("W,empty_at", [(2, None), (3, 1), (8, None), (8, 0), (8, 7)])
def test_sparse_lists_reduce_scattered(W, empty_at):
    """Above 1024 services every rank keeps a sorted list; comm_sum_sparse samples the lists,
    picks cell-range bounds, sends every slice to its range's rank, sums each range there and
    all-gathers the ranges: every rank holds the job's list (sorted, each pair once). With an
    empty rank (its list has no entries and no samples), first, in the middle or last."""
    w = _c5_like(40_000)
    cols = synth.generate(w)
    if empty_at is None:
        parts = shard.partition_columns(cols, W)
    else:
        parts = shard.partition_columns(cols, W - 1)
        parts.insert(empty_at, _empty())
    ctxs = _job(parts, w.total_services)
    try:
        got = _concurrently(ctxs, lambda k, c: sorted(_tuples(*c.link())))

        def reput(k, c):
            c.put_spans(parts[k])  # accumulates: every pair twice
            return sorted(_tuples(*c.link()))
        twice = _concurrently(ctxs, reput)
    finally:
        _close(ctxs)
    exp = sorted(_oracle(cols))
    assert len(exp) > 10_000
    for k in range(W):
        assert got[k] == exp
        assert twice[k] == [(a, b, 2 * n, 2 * e) for a, b, n, e in exp]


def test_sparse_forced_small_dictionary_and_hot_cells(monkeypatch):
    """ZDL_SPARSE=1 at C2's 50 services: 2 500 cells, Zipf-hot; many sampled cells are equal,
    so several range bounds coincide and some ranks own empty ranges."""
    monkeypatch.setenv("ZDL_SPARSE", "1")
    w = synth.C2.scaled(40_000)
    cols = synth.generate(w)
    parts = shard.partition_columns(cols, 8)
    ctxs = _job(parts, w.total_services, puts=3)
    try:
        got = _concurrently(ctxs, lambda k, c: sorted(_tuples(*c.link())))
    finally:
        _close(ctxs)
    exp = sorted(_oracle(cols))
    for k in range(8):
        assert got[k] == [(a, b, 3 * n, 3 * e) for a, b, n, e in exp]


def test_sparse_job_of_empty_ranks():
    """No rank holds a link: the combine moves nothing and every rank returns an empty list."""
    ctxs = _job([_empty(), _empty(), _empty()], 10_000)
    try:
        got = _concurrently(ctxs, lambda k, c: _tuples(*c.link()))
    finally:
        _close(ctxs)
    assert got == [[], [], []]


def test_table_export_sums_over_ranks():
    """zdl_table_export of every rank (concurrently) returns the job's S x S tables."""
    import torch
    w = synth.C4.scaled(40_000)
    cols = synth.generate(w)
    S = w.total_services
    parts = shard.partition_columns(cols, 3)
    ctxs = _job(parts, S)
    dev = torch.device("cuda", 0)
    bufs = [(torch.zeros(S * S, dtype=torch.int64, device=dev), torch.zeros(S * S, dtype=torch.int64, device=dev))
            for _ in ctxs]
    try:
        def export(k, c):
            c.table_export(bufs[k][0].data_ptr(), bufs[k][1].data_ptr())
            c.sync()
        _concurrently(ctxs, export)
    finally:
        _close(ctxs)
    torch.cuda.synchronize(dev)
    exp = sorted(_oracle(cols))
    for tc, te in bufs:
        c, e = tc.cpu().numpy(), te.cpu().numpy()
        nz = np.nonzero(c)[0]
        assert sorted((int(i) // S, int(i) % S, int(c[i]), int(e[i])) for i in nz) == exp


def test_local_world_refusals():
    """Ranks must share one service count; a context joins one job only."""
    a, b = N.Context(50), N.Context(60)
    with pytest.raises(N.ZdlError):
        N.Context.comm_init_local([a, b])
    c = N.Context(50)
    N.Context.comm_init_local([a, c])
    with pytest.raises(N.ZdlError):
        N.Context.comm_init_local([a, b])
    for x in (a, b, c):
        x.close()


def test_job_matches_one_context_over_concatenated_shards():
    """The C3 shape at W = 4 against ONE context fed the shards one after another: the job's sum
    is the single linker's table (the data path has no collective; only the counts combine)."""
    w = synth.C3.scaled(100_000)
    cols = synth.generate(w)
    parts = shard.partition_columns(cols, 4)
    ctxs = _job(parts, w.total_services)
    try:
        got = _concurrently(ctxs, lambda k, c: sorted(_tuples(*c.link())))
    finally:
        _close(ctxs)
    one = N.Context(w.total_services)
    one.put_spans(concat_columns(parts))
    exp = sorted(_tuples(*one.link()))
    one.close()
    for k in range(4):
        assert got[k] == exp
