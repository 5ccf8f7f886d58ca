"""Parity of the HIP engine (through the C ABI) with the oracle.

* the reference's own test vectors (tests/golden/) through the DependencyLinker and
  InMemoryStorage facades;
* random corner-case traces vs the Python oracle, including the Q1 NPE;
* synthetic BASELINE workloads (C2, C4, C5-shaped, windowed) vs the C++ restatement,
  bit-exact on every (parent, child, callCount, errorCount).

The DependencyLinker facade runs on an insertion-order context, so the golden cases
apply the reference's own assertion (containsExactly or containsOnly); the raw-context
workload tests use the streaming path (sorted output) and compare as sets; the exact
insertion order of those workloads is tests/test_gpu_insertion_order.py's.
DependencyLinker.merge keeps first-seen order and is compared exactly.
"""
import random

import numpy as np
import pytest

from oracle import dl_oracle as O
from oracle import ref
from tests.golden_io import check_links, links, load, spans
from tests.stress import random_trace
from zipkin_amd import _native as N
from zipkin_amd import synth
from zipkin_amd.columnar import Dictionary, pack_traces
from zipkin_amd.linker import DependencyLinker
from zipkin_amd.storage import InMemoryStorage

pytestmark = pytest.mark.gpu

DL = load("dependency_linker.json")
ST = load("storage_dependencies.json")


def as_set(ls):
    return sorted((l.parent, l.child, l.call_count, l.error_count) for l in ls)


# The engine paths the reference's vectors run through: the facade's default (insertion order,
# k_link mode 4 + k_tail's exact path), the benchmarked streaming path (sorted output: k_link
# mode 0 on the dense LDS table), and the table modes forced at the golden cases' small
# dictionaries - LOG (ZDL_TM=log: k_link's emit log + k_scatter / k_hist), sorted and ranked,
# and the sparse list (ZDL_SPARSE=1: TM_SORT + the log's sort/merge, sorted output only).
PATHS = {"insertion": (True, {}), "sorted": (False, {}), "sorted_log": (False, {"ZDL_TM": "log"}),
         "insertion_log": (True, {"ZDL_TM": "log"}), "sorted_sparse": (False, {"ZDL_SPARSE": "1"})}


def _path(name, monkeypatch):
    ins, env = PATHS[name]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    return ins


@pytest.mark.parametrize("case", [c for c in DL["cases"] if c["mode"] == "log"], ids=lambda c: c["name"])
def test_golden_dependency_linker_log(case):
    """The cases that assert FINE log text only: the device's reason codes rendered."""
    from tests.test_gpu_finelog import _device_log
    msgs, _ = _device_log([spans(t) for t in case["traces"]], name=case["name"])
    assert all(m in msgs for m in case["log_contains"])


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("case", [c for c in DL["cases"] if c["mode"] != "log"], ids=lambda c: c["name"])
def test_golden_dependency_linker(case, path, monkeypatch):
    ins = _path(path, monkeypatch)
    linker = DependencyLinker(insertion_order=ins)
    for t in case["traces"]:
        linker.put_trace(spans(t))
    # containsExactly needs the reference's list order: sorted paths are compared as sets
    check_links(linker.link(), case["expect"], case["mode"] if ins else "only")
    linker.close()


@pytest.mark.parametrize("path", ["insertion", "insertion_log"])
@pytest.mark.parametrize("case", [c for c in DL["cases"] if c["mode"] == "exact"],
                         ids=lambda c: c["name"])
def test_golden_response_bytes(case, path, monkeypatch):
    """The JSON_V1 bytes of the device's links equal those of the expected links, in order."""
    from zipkin_amd.codec import encode_links
    _path(path, monkeypatch)
    linker = DependencyLinker()
    for t in case["traces"]:
        linker.put_trace(spans(t))
    assert encode_links(linker.link()) == encode_links(links(case["expect"]))
    linker.close()


@pytest.mark.parametrize("path", ["sorted", "sorted_log", "sorted_sparse"])
@pytest.mark.parametrize("case", [c for c in DL["cases"] if c["mode"] != "log"], ids=lambda c: c["name"])
def test_golden_response_bytes_sorted(case, path, monkeypatch):
    """The sorted paths' JSON_V1 bytes equal the expected links' bytes in (parent, child) order."""
    from zipkin_amd.codec import encode_links
    _path(path, monkeypatch)
    linker = DependencyLinker(insertion_order=False)
    for t in case["traces"]:
        linker.put_trace(spans(t))
    got = linker.link()
    linker.close()
    if isinstance(case["expect"], dict):
        return
    exp = sorted(links(case["expect"]), key=lambda l: (l.parent, l.child))
    assert encode_links(got) == encode_links(exp)


@pytest.mark.parametrize("case", DL["merge_cases"], ids=lambda c: c["name"])
def test_golden_merge_exact_order(case):
    check_links(DependencyLinker.merge(links(case["links"])), case["expect"], case["mode"])


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("case", ST["cases"], ids=lambda c: c["name"])
def test_golden_storage(case, path, monkeypatch):
    store = InMemoryStorage(strict_trace_id=True, insertion_order=_path(path, monkeypatch))
    for b in case["batches"]:
        store.accept(spans(b)).execute()
    for q in case["queries"]:
        check_links(store.get_dependencies(q["endTs"], q["lookback"]).execute(), q["expect"], "only")


def test_linker_reusable_and_call_single_use():
    t = spans(DL["cases"][1]["traces"][0])
    linker = DependencyLinker().put_trace(t)
    assert as_set(linker.link()) == as_set(linker.link())
    linker.put_trace(t)
    assert {l.call_count for l in linker.link()} == {2}
    store = InMemoryStorage()
    call = store.get_dependencies(1, 1)
    call.execute()
    with pytest.raises(Exception, match="Already Executed"):
        call.execute()


@pytest.mark.parametrize("seed", range(300))
def test_random_traces_vs_python_oracle(seed):
    r = random.Random(1000 + seed)
    traces = [random_trace(r) for _ in range(r.randint(1, 5))]
    ol = O.DependencyLinker()
    try:
        for t in traces:
            ol.put_trace(t)
        expect = as_set(ol.link())
    except O.ReferenceNPE:
        expect = "NPE"
    gl = DependencyLinker()
    if expect == "NPE":
        with pytest.raises(N.ReferenceNullPointerException):
            gl.put_traces(traces)
    else:
        gl.put_traces(traces)
        assert as_set(gl.link()) == expect
    gl.close()


def _engine_vs_cpp(cols, n_services, window=None, svc_rank=None, ip4_rank=None, ip6_rank=None):
    ctx = N.Context(n_services)
    if svc_rank is not None:
        ctx.set_ranks(N.ZDL_DICT_SERVICE, svc_rank)
    if ip4_rank is not None:
        ctx.set_ranks(N.ZDL_DICT_IPV4, ip4_rank)
    if ip6_rank is not None:
        ctx.set_ranks(N.ZDL_DICT_IPV6, ip6_rank)
    if window is not None:
        ctx.set_window(*window)
    ctx.put_spans(cols)
    p, c, n, e = ctx.link()
    ctx.close()
    st, op, oc, on, oe = ref.link(cols, svc_rank, ip4_rank, ip6_rank, window=window, threads=8)
    assert st == 0
    got = sorted(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))
    exp = sorted(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))
    assert got == exp
    return got


def test_random_no_npe_batch_vs_cpp_oracle():
    r = random.Random(99)
    traces = [random_trace(r, n=r.randint(1, 40), allow_npe=False) for _ in range(3000)]
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    _engine_vs_cpp(cols, 64, svc_rank=svc.ranks(), ip4_rank=ip4.ranks(), ip6_rank=ip6.ranks())


def test_big_traces_vs_cpp_oracle():
    """Traces longer than the tile kernel's SMALL_MAX take the big-trace kernel."""
    r = random.Random(5)
    traces = [random_trace(r, n=r.choice([129, 300, 1000, 4097]), allow_npe=False, id_pool=r.choice([50, 2000]))
              for _ in range(12)]
    traces += [random_trace(r, n=r.randint(1, 20), allow_npe=False) for _ in range(200)]
    r.shuffle(traces)
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    _engine_vs_cpp(cols, 64, svc_rank=svc.ranks(), ip4_rank=ip4.ranks(), ip6_rank=ip6.ranks())


@pytest.mark.parametrize("n_services", [64, 65, 300])
def test_dense_and_hash_tables_agree(n_services):
    r = random.Random(3)
    traces = [random_trace(r, n=r.randint(1, 30), allow_npe=False) for _ in range(2000)]
    svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
    cols = pack_traces(traces, svc, ip4, ip6)
    _engine_vs_cpp(cols, n_services, svc_rank=svc.ranks(), ip4_rank=ip4.ranks(), ip6_rank=ip6.ranks())


def test_c2_synthetic_vs_cpp_oracle():
    w = synth.C2.scaled(200_000)
    links = _engine_vs_cpp(synth.generate(w), w.total_services)
    assert len(links) > 100


def test_c4_messaging_stress_vs_cpp_oracle():
    w = synth.C4.scaled(200_000)
    _engine_vs_cpp(synth.generate(w), w.total_services)


def test_c5_high_cardinality_vs_cpp_oracle():
    w = synth.C5.scaled(20_000)
    w = synth.Workload(**{**w.__dict__, "max_size": 20_000})
    _engine_vs_cpp(synth.generate(w), w.total_services)


def test_window_vs_cpp_oracle():
    w = synth.C2.scaled(100_000)
    cols = synth.generate(w)
    base_ms = w.base_ts_us // 1000
    # traces start at base + t ms; keep roughly the middle third
    _engine_vs_cpp(cols, w.total_services, window=(base_ms + 66_000, 33_000))


def test_accumulates_across_puts_and_reset():
    w = synth.C2.scaled(50_000)
    cols = synth.generate(w)
    ctx = N.Context(w.total_services)
    ctx.put_spans(cols)
    p1, c1, n1, e1 = ctx.link()
    ctx.put_spans(cols)
    p2, c2, n2, e2 = ctx.link()
    assert np.array_equal(p1, p2) and np.array_equal(n2, 2 * n1) and np.array_equal(e2, 2 * e1)
    ctx.reset()
    assert len(ctx.link()[0]) == 0
    ctx.close()


def test_bad_service_id_is_einval():
    w = synth.C2.scaled(1000)
    cols = synth.generate(w)
    ctx = N.Context(10)  # ids up to 49 present
    with pytest.raises(N.ZdlError):
        ctx.put_spans(cols)
    ctx.close()


def _sorted_links(ctx):
    p, c, n, e = ctx.link()
    return sorted(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))


def _interleave_keep_order(owner, rng):
    # draw a random sequence of trace labels with each trace's multiplicity, then give the
    # k-th occurrence of trace t the k-th span of t
    labels = rng.permutation(owner)
    first = np.zeros(owner.max() + 2, np.int64)
    np.add.at(first, owner + 1, 1)
    start = np.cumsum(first)[:-1]
    k = np.zeros(len(owner), np.int64)
    seen = np.zeros(owner.max() + 1, np.int64)
    for i, t in enumerate(labels):
        k[i] = start[t] + seen[t]
        seen[t] += 1
    return k


def _take(cols, idx):
    from zipkin_amd.columnar import Columns
    f = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
         "timestamp")
    return Columns(*(np.ascontiguousarray(getattr(cols, n)[idx]) for n in f), cols.offsets)


@pytest.mark.parametrize("use_ord", [False, True])
def test_ungrouped_input_grouped_on_device(use_ord):
    """trace_offsets == NULL: the device groups by trace_lo (InMemoryStorage.java:448-467)."""
    w = synth.C2.scaled(20_000)
    cols = synth.generate(w)
    rng = np.random.default_rng(7)
    ctx = N.Context(w.total_services)
    ctx.put_spans(cols)
    exp = _sorted_links(ctx)
    ctx.reset()
    if use_ord:  # any span order; ord = the position within the trace's storage order
        idx = rng.permutation(cols.n_spans)
        ctx.put_spans_ungrouped(_take(cols, idx), ord=idx.astype(np.uint32))
    else:  # traces interleaved, each trace's spans still in storage order
        ctx.put_spans_ungrouped(_take(cols, _interleave_keep_order(
            np.repeat(np.arange(cols.n_traces), np.diff(cols.offsets.astype(np.int64))), rng)))
    assert _sorted_links(ctx) == exp
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("tm,window", [(1, 0), (1, 1), (2, 0), (2, 1), (3, 0), (0, 0)])
def test_k_link_two_workgroups_per_cu(tm, window):
    """k_link's design point: two 16-wave workgroups per CU (8 waves a SIMD), each with exactly
    80 KB of LDS in the dense mode. A few bytes of static __shared__ in k_link (or in anything it
    calls) halve that silently - it cost C2's k_link 127 -> 165 us once (profiles/r03f_*)."""
    from zipkin_amd import _native as N
    assert N.lib().zdl_link_occupancy(0, tm, window) == 2
