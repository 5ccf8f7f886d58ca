"""Synthetic workload generator: deterministic, thread-count invariant, shaped as
SURVEY.md §8(d) says."""
import numpy as np

from zipkin_amd import synth


def cols_equal(a, b):
    for f in ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6",
              "port_flags", "timestamp", "offsets"):
        if not np.array_equal(getattr(a, f), getattr(b, f)):
            return False
    return True


def test_deterministic_and_thread_invariant():
    w = synth.C2.scaled(5000)
    assert cols_equal(synth.generate(w, threads=1), synth.generate(w, threads=7))


def test_c2_shape():
    w = synth.C2.scaled(20000)
    c = synth.generate(w)
    sizes = np.diff(c.offsets.astype(np.int64))
    assert 9.5 < sizes.mean() < 10.5  # 1 + Poisson(9)
    assert c.local_svc.max() < 50 and c.remote_svc.max() < 50
    assert (c.id != 0).all()
    # every span of a trace shares its trace_lo
    t = np.repeat(np.arange(len(sizes)), sizes)
    first = c.trace_lo[c.offsets[:-1].astype(np.int64)]
    assert (c.trace_lo == first[t]).all()


def test_sharding_by_trace_lo():
    w = synth.C2.scaled(2000).sharded(1, 4)
    c = synth.generate(w)
    from zipkin_amd.shard import shard_of
    assert (shard_of(c.trace_lo, 4) == 1).all()


def test_c4_has_messaging_and_fragments():
    c = synth.generate(synth.C4.scaled(20000))
    kinds = (c.port_flags >> 16) & 7
    assert (kinds == 2).any() and (kinds == 3).any()
    assert (c.remote_svc >= 50).any()  # brokers


def test_spans_of_round_trip():
    """synth.spans_of (the facade leg's Span objects) packs back to columns that link to the same
    links by service name - C2 and C4 (messaging, fragments, errors) - as the original columns."""
    from oracle import ref
    from zipkin_amd.columnar import Dictionary, pack_traces
    for w in (synth.C2.scaled(2000), synth.C4.scaled(2000)):
        cols = synth.generate(w)
        traces = synth.spans_of(cols, w, cols.n_traces)
        svc, ip4, ip6 = Dictionary(), Dictionary(), Dictionary()
        back = pack_traces(traces, svc, ip4, ip6)
        assert back.n_spans == cols.n_spans
        names = synth.service_names(w)
        st, p, c, n, e = ref.link(cols, threads=2)
        assert st == 0
        exp = sorted(zip([names[i] for i in p], [names[i] for i in c], n.tolist(), e.tolist()))
        st, p, c, n, e = ref.link(back, threads=2)
        assert st == 0
        got = sorted(zip([svc.strings[i] for i in p], [svc.strings[i] for i in c], n.tolist(), e.tolist()))
        assert got == exp and len(exp) > 10
