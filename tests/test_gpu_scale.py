"""Every BASELINE config on the engine at its defining scale, against the C++ restatement
(oracle/dl_ref.cpp), bit-exact on every (parent, child, callCount, errorCount):

* C3: a per-GPU shard shape (500 services, C2 shape, 1M traces = 10M spans) through the
  raw context (sorted output) and through the facade's table capacity on an
  insertion-order context (DependencyLinker.link()'s exact list order);
* C5: the Pareto body plus unclipped giant traces of 60k-190k spans (depth 64,
  fan-out <= 1000), which take k_tail's big-trace path;
* the multi-GPU combine on one device: contexts over disjoint splitmix64(trace_lo) shards,
  zdl_table_export -> sum -> zdl_table_import -> zdl_link equals one context over
  everything (DependencyLinker.merge semantics, DependencyLinker.java:189-204).
"""
import numpy as np
import pytest

from oracle import ref
from zipkin_amd import _native as N
from zipkin_amd import shard, synth
from zipkin_amd.columnar import concat_columns
from zipkin_amd.linker import _capacity

pytestmark = pytest.mark.gpu


def _tuples(p, c, n, e):
    return list(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))


def _oracle(cols, threads=16):
    st, p, c, n, e = ref.link(cols, threads=threads)
    assert st == 0
    return _tuples(p, c, n, e)


def test_c3_shard_sorted_vs_cpp():
    w = synth.C3.scaled(1_000_000)
    cols = synth.generate(w)
    assert cols.n_spans > 9_000_000
    ctx = N.Context(w.total_services)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.close()
    exp = sorted(_oracle(cols))
    assert len(exp) > 100_000
    assert got == exp


def test_c3_shard_facade_capacity_insertion_order_vs_cpp():
    """The DependencyLinker facade's context for 500 services (capacity 768) on the
    insertion-order path: the reference's list order, exactly."""
    w = synth.C3.scaled(1_000_000)
    cols = synth.generate(w)
    cap = _capacity(w.total_services)
    assert cap > w.total_services
    ctx = N.Context(cap, insertion_order=True)
    ctx.put_spans(cols)
    got = _tuples(*ctx.link(N.ZDL_ORDER_INSERTION))
    ctx.close()
    assert got == _oracle(cols)


def _c5_with_giants():
    body = synth.generate(synth.C5.scaled(300_000))
    giants = []
    for k, size in enumerate((60_000, 120_000, 190_000)):
        g = synth.Workload(f"c5_giant_{k}", 0x5EED0050 + k, 1, 10_000, max_depth=64, size_dist=2,
                           max_size=size, max_fanout=1000, zipf_s=1.1)
        giants.append(synth.generate(g))
    # giants first, in the middle and last: each sits in a different wave's chunk
    h = body.n_traces // 2
    first = _slice_traces(body, 0, h)
    second = _slice_traces(body, h, body.n_traces)
    return concat_columns([giants[0], first, giants[1], second, giants[2]])


def _slice_traces(cols, t0, t1):
    from zipkin_amd.columnar import Columns
    a, b = int(cols.offsets[t0]), int(cols.offsets[t1])
    f = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
         "timestamp")
    return Columns(*(np.ascontiguousarray(getattr(cols, n)[a:b]) for n in f),
                   np.ascontiguousarray(cols.offsets[t0:t1 + 1] - np.uint64(a)))


def test_c5_unclipped_giant_traces_vs_cpp():
    cols = _c5_with_giants()
    sizes = np.diff(cols.offsets.astype(np.int64))
    assert (sizes >= 50_000).sum() >= 3 and sizes.max() <= 200_000
    ctx = N.Context(10_000)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.close()
    assert got == sorted(_oracle(cols))


@pytest.mark.parametrize("config", ["c4", "c3"])
def test_two_shard_table_combine_on_one_device(config):
    """bench.py's multi-GPU step on one device: per-shard contexts, their S x S tables
    exported, summed (what the RCCL all-reduce does across ranks), imported, linked."""
    import torch
    w = synth.CONFIGS[config].scaled(200_000)
    cols = synth.generate(w)
    S = w.total_services
    parts = shard.partition_columns(cols, 2)
    assert all(p.n_spans > 0 for p in parts)
    dev = torch.device("cuda", 0)
    tables = []
    for p in parts:
        ctx = N.Context(S)
        ctx.put_spans(p)
        tc = torch.zeros(S * S, dtype=torch.int64, device=dev)
        te = torch.zeros(S * S, dtype=torch.int64, device=dev)
        ctx.table_export(tc.data_ptr(), te.data_ptr())
        ctx.sync()
        ctx.close()
        tables.append((tc, te))
    call = tables[0][0] + tables[1][0]
    err = tables[0][1] + tables[1][1]
    torch.cuda.synchronize(dev)
    ctx = N.Context(S)
    ctx.table_import(call.data_ptr(), err.data_ptr())
    got = sorted(_tuples(*ctx.link()))
    ctx.close()
    one = N.Context(S)
    one.put_spans(cols)
    whole = sorted(_tuples(*one.link()))
    one.close()
    assert got == whole
    assert got == sorted(_oracle(cols))


@pytest.mark.parametrize("n_services", [67, 68, 90, 500, 1024, 1025])
@pytest.mark.parametrize("mode", ["auto", "hash"])
def test_table_modes_vs_cpp(n_services, mode, monkeypatch):
    """Dense LDS cells (S <= 67), the emit log (68 <= S <= 1024; 90: also k_tail's mapped
    ordered output) and the LDS hash with HBM spill (S > 1024, or forced by ZDL_TM=hash)
    count the same links."""
    import random
    from tests.stress import random_trace
    from zipkin_amd.columnar import Dictionary, pack_traces
    if mode == "hash":
        monkeypatch.setenv("ZDL_TM", "hash")
    r = random.Random(n_services)
    traces = [random_trace(r, n=r.randint(1, 30), allow_npe=False)
              for _ in range(3000)]
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    # spread the ids over the whole table: every partition of the log gets entries
    perm = np.random.default_rng(n_services).permutation(n_services)[:len(svc)].astype(np.int32)
    for f in ("local_svc", "remote_svc"):
        a = getattr(cols, f)
        setattr(cols, f, np.where(a >= 0, perm[np.maximum(a, 0)], -1).astype(np.int32))
    rank = np.empty(n_services, np.int32)
    rank[:] = np.arange(n_services) + len(svc)
    rank[perm] = svc.ranks()
    ctx = N.Context(n_services)
    ctx.set_ranks(N.ZDL_DICT_SERVICE, rank)
    ctx.set_ranks(N.ZDL_DICT_IPV4, ip4.ranks())
    ctx.set_ranks(N.ZDL_DICT_IPV6, ip6.ranks())
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.close()
    st, p, c, n, e = ref.link(cols, rank, ip4.ranks(), ip6.ranks(), threads=8)
    assert st == 0
    assert got == sorted(_tuples(p, c, n, e))


def test_c3_window_vs_cpp():
    """The time window (QueryRequest.test) on the LOG-mode path."""
    w = synth.C3.scaled(300_000)
    cols = synth.generate(w)
    base_ms = w.base_ts_us // 1000
    window = (base_ms + 200_000, 100_000)
    ctx = N.Context(w.total_services)
    ctx.set_window(*window)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.close()
    st, p, c, n, e = ref.link(cols, window=window, threads=16)
    assert st == 0 and len(p) > 1000
    assert got == sorted(_tuples(p, c, n, e))


def test_c3_repeated_puts_accumulate():
    """Several puts into one LOG-mode context add up (and reset clears)."""
    w = synth.C3.scaled(200_000)
    cols = synth.generate(w)
    ctx = N.Context(w.total_services)
    ctx.put_spans(cols)
    one = sorted(_tuples(*ctx.link()))
    ctx.put_spans(cols)
    ctx.put_spans(cols)
    three = sorted(_tuples(*ctx.link()))
    assert [(a, b, 3 * x, 3 * y) for a, b, x, y in one] == three
    ctx.reset()
    assert len(ctx.link()[0]) == 0
    ctx.close()
    assert one == sorted(_oracle(cols))


@pytest.mark.parametrize("config", ["c2", "c3"])
def test_device_group_of_one_equals_single_context(config):
    """The device-group path (zdl_config.device_ids: host sharding by splitmix64(trace_lo),
    per-device contexts, ncclReduce of the tables, compaction of the sum) on the one device
    the box has, against a plain context and the C++ restatement."""
    w = synth.CONFIGS[config].scaled(200_000)
    cols = synth.generate(w)
    g = N.Context(w.total_services, device_ids=[0])
    assert g.device_count() == 1
    g.put_spans(cols)
    g.put_spans(cols)  # accumulates like repeated putTrace
    got = sorted(_tuples(*g.link()))
    g.close()
    exp = sorted(_oracle(cols))
    assert got == [(a, b, 2 * n, 2 * e) for a, b, n, e in exp]


def test_device_group_ungrouped_and_export():
    import torch
    w = synth.C4.scaled(100_000)
    cols = synth.generate(w)
    S = w.total_services
    g = N.Context(S, device_ids=[0])
    g.put_spans_ungrouped(cols)
    dev = torch.device("cuda", 0)
    tc = torch.zeros(S * S, dtype=torch.int64, device=dev)
    te = torch.zeros(S * S, dtype=torch.int64, device=dev)
    g.table_export(tc.data_ptr(), te.data_ptr())
    g.sync()
    torch.cuda.synchronize(dev)
    got = sorted(_tuples(*g.link()))
    g.close()
    exp = sorted(_oracle(cols))
    assert got == exp
    c, e = tc.cpu().numpy(), te.cpu().numpy()
    nz = np.nonzero(c)[0]
    assert sorted((int(i) // S, int(i) % S, int(c[i]), int(e[i])) for i in nz) == exp


@pytest.mark.parametrize("config", ["c2", "c3"])
def test_comm_job_of_one_rank(config):
    """zdl_comm_init with world 1: zdl_link goes through the ncclAllReduce path bench.py
    uses at N > 1 (one process per GPU)."""
    w = synth.CONFIGS[config].scaled(100_000)
    cols = synth.generate(w)
    ctx = N.Context(w.total_services)
    ctx.comm_init(N.Context.comm_unique_id(), 0, 1)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.reset()
    ctx.put_spans(cols)
    again = sorted(_tuples(*ctx.link()))
    ctx.close()
    assert got == again == sorted(_oracle(cols))


def _c5_like(traces=100_000):
    return synth.Workload("c5_like_10k", 0x5EED0078, traces, 10_000, max_depth=32, size_dist=1, pareto_alpha=1.3,
                          max_size=3000, max_fanout=200, zipf_s=1.1)


@pytest.mark.parametrize("forced", [False, True])
def test_device_group_sparse_lists_combined(forced, monkeypatch):
    """Device groups above 1024 services keep a sparse list per device; zdl_link sends every
    device's list to the first (ncclSend/ncclRecv) and sums them per cell there (sparse_add:
    DependencyLinker.merge). On the box's one device, and forced (ZDL_SPARSE=1) at C4's size."""
    if forced:
        monkeypatch.setenv("ZDL_SPARSE", "1")
    w = synth.C4.scaled(100_000) if forced else _c5_like()
    cols = synth.generate(w)
    g = N.Context(w.total_services, device_ids=[0])
    g.put_spans(cols)
    g.put_spans(cols)
    got = sorted(_tuples(*g.link()))
    g.reset()
    g.put_spans(cols)
    once = sorted(_tuples(*g.link()))
    g.close()
    exp = sorted(_oracle(cols))
    assert once == exp
    assert got == [(a, b, 2 * n, 2 * e) for a, b, n, e in exp]


def test_comm_job_of_one_rank_sparse():
    """A sparse context joined to a one-rank job: zdl_link exchanges list lengths
    (ncclAllGather) and lists (ncclSend/ncclRecv) and sums them (comm_sum_sparse)."""
    w = _c5_like()
    cols = synth.generate(w)
    ctx = N.Context(w.total_services)
    ctx.comm_init(N.Context.comm_unique_id(), 0, 1)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.put_spans(cols)
    twice = sorted(_tuples(*ctx.link()))
    ctx.close()
    exp = sorted(_oracle(cols))
    assert got == exp
    assert twice == [(a, b, 2 * n, 2 * e) for a, b, n, e in exp]


@pytest.mark.parametrize("exact", [False, True])
def test_c5_body_big_trace_paths_vs_cpp(exact, monkeypatch):
    """Traces above 64 spans: the sort-free path for simple ids (big_simple, LDS-resident up
    to ~1600 spans, HBM scratch beyond) and the exact sorting path (ZDL_BIG_EXACT=1) both
    equal the C++ restatement on C5's Pareto body (depth 64, fan-out <= 1000)."""
    if exact:
        monkeypatch.setenv("ZDL_BIG_EXACT", "1")
    cols = synth.generate(synth.C5.scaled(200_000))
    sizes = np.diff(cols.offsets.astype(np.int64))
    assert (sizes > 64).sum() > 500 and (sizes > 2000).sum() > 5
    ctx = N.Context(10_000)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.close()
    assert got == sorted(_oracle(cols))


@pytest.mark.parametrize("config", ["c2", "c4"])
def test_sparse_context_forced_small(config, monkeypatch):
    """ZDL_SPARSE=1: the sorted-list table (zdl_sparse.h) at a small dictionary, against the
    dense context and the restatement, over three puts (merge of lists) and a reset."""
    monkeypatch.setenv("ZDL_SPARSE", "1")
    w = synth.CONFIGS[config].scaled(100_000)
    cols = synth.generate(w)
    ctx = N.Context(w.total_services)
    ctx.put_spans(cols)
    one = sorted(_tuples(*ctx.link()))
    ctx.put_spans(cols)
    ctx.put_spans(cols)
    three = sorted(_tuples(*ctx.link()))
    ctx.reset()
    assert len(ctx.link()[0]) == 0
    ctx.put_spans(cols)
    again = sorted(_tuples(*ctx.link()))
    ctx.close()
    exp = sorted(_oracle(cols))
    assert one == exp == again
    assert three == [(a, b, 3 * n, 3 * e) for a, b, n, e in exp]


def test_sparse_vs_dense_table_large_dictionary():
    """2000 services: sparse by default, the S x S table with ZDL_FLAG_DENSE_TABLE; with a
    service rank table (sorted output by name order), a time window and add_links."""
    w = synth.Workload("c5_like_2000", 0x5EED0077, 200_000, 2000, max_depth=32, size_dist=1, pareto_alpha=1.3,
                       max_size=5000, max_fanout=200, zipf_s=1.1)
    cols = synth.generate(w)
    rank = np.random.default_rng(5).permutation(2000).astype(np.int32)
    base_ms = w.base_ts_us // 1000
    out = []
    for dense in (False, True):
        ctx = N.Context(2000, dense_table=dense)
        ctx.set_ranks(N.ZDL_DICT_SERVICE, rank)
        ctx.put_spans(cols)
        full = _tuples(*ctx.link())
        ctx.add_links(np.array([3, 3, 1999], np.int32), np.array([4, 4, 0], np.int32), np.array([5, 1, 2], np.int64),
                      np.array([1, 0, 2], np.int64))
        added = _tuples(*ctx.link())
        ctx.reset()
        ctx.set_window(base_ms + 120_000, 60_000)
        ctx.put_spans(cols)
        windowed = _tuples(*ctx.link())
        ctx.close()
        out.append((full, added, windowed))
    assert out[0] == out[1]  # the same links in the same (rank) order
    full, added, windowed = out[0]
    assert sorted(full) == sorted(_oracle(cols))
    assert [(rank[p], rank[c]) for p, c, _, _ in full] == sorted((rank[p], rank[c]) for p, c, _, _ in full)
    st, p, c, n, e = ref.link(cols, window=(base_ms + 120_000, 60_000), threads=16)
    assert st == 0 and sorted(windowed) == sorted(_tuples(p, c, n, e))
    d = {(a, b): (x, y) for a, b, x, y in full}
    for a, b, x, y in ((3, 4, 6, 1), (1999, 0, 2, 2)):
        x0, y0 = d.get((a, b), (0, 0))
        assert (a, b, x0 + x, y0 + y) in added


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("wave", [True, False])
def test_mid_size_messy_traces_vs_cpp(sparse, wave, monkeypatch):
    """Traces of 65..400 spans with C4's faults (split spans, duplicate ids, missing brokers,
    extra roots): k_tail's wave_big (<= 208 spans, one wave each; a trace whose ids are not
    simple is retried on the exact path by the last workgroup) and the workgroup paths
    (ZDL_WAVE_BIG=0), dense and sparse tables, with and without a time window."""
    if sparse:
        monkeypatch.setenv("ZDL_SPARSE", "1")
    if not wave:
        monkeypatch.setenv("ZDL_WAVE_BIG", "0")
    w = synth.Workload("mid_messy", 0x5EED0078, 80_000, 50, n_brokers=4, max_depth=16, size_dist=1,
                       pareto_alpha=0.7, max_size=400, max_fanout=40, p_error=0.05, p_messaging=0.3,
                       p_missing_broker=0.1, p_delete=0.05, p_extra_root=0.03, p_uninstrumented=0.1,
                       p_drop_shared_parent=0.1, p_split=0.05)
    cols = synth.generate(w)
    sizes = np.diff(cols.offsets.astype(np.int64))
    assert ((sizes > 64) & (sizes <= 208)).sum() > 1000 and (sizes > 208).sum() > 100
    base_ms = w.base_ts_us // 1000
    ctx = N.Context(w.total_services)
    ctx.put_spans(cols)
    got = sorted(_tuples(*ctx.link()))
    ctx.reset()
    ctx.set_window(base_ms + 60_000, 30_000)  # traces start 1 ms apart: about the middle third
    ctx.put_spans(cols)
    windowed = sorted(_tuples(*ctx.link()))
    ctx.close()
    assert got == sorted(_oracle(cols))
    st, p, c, n, e = ref.link(cols, window=(base_ms + 60_000, 30_000), threads=16)
    assert st == 0 and len(p) > 100 and windowed == sorted(_tuples(p, c, n, e))


@pytest.mark.parametrize("config", ["c2", "c4"])
def test_comm_job_of_one_rank_insertion_order(config):
    """An insertion-order context joined to a one-rank job: zdl_link(ZDL_ORDER_INSERTION) sums
    the tables and MIN-reduces the rank-tagged first-seen ranks (comm_sum_ord, zdl_xplan.h);
    with one rank that is the single context's exact list order, the C++ restatement's."""
    w = synth.CONFIGS[config].scaled(50_000)
    cols = synth.generate(w)
    S = w.total_services
    ctx = N.Context(S, insertion_order=True)
    ctx.comm_init(N.Context.comm_unique_id(), 0, 1)
    ctx.put_spans(cols)
    got = list(_tuples(*ctx.link(N.ZDL_ORDER_INSERTION)))
    ctx.put_spans(cols)
    twice = list(_tuples(*ctx.link(N.ZDL_ORDER_INSERTION)))
    ctx.close()
    exp = list(_oracle(cols))
    assert got == exp
    assert twice == [(a, b, 2 * n, 2 * e) for a, b, n, e in exp]
