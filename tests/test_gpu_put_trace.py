"""putTrace called trace by trace (zdl_put_trace): the staged batches give
the reference's links in the reference's order, an NPE (quirk Q1) is raised by the very call
whose trace throws, and the linker keeps working afterwards, as the Java object does
(DependencyLinker.java:53-186; Trace.java:52-68). Small staging slots (ZDL_STAGE_SPANS) make
every test cross many flushes."""
import random

import numpy as np
import pytest

from oracle import dl_oracle as O
from oracle import ref
from tests.stress import random_trace
from zipkin_amd import _native as N
from zipkin_amd import synth
from zipkin_amd.linker import DependencyLinker

pytestmark = pytest.mark.gpu


def _as_list(ls):
    return [(l.parent, l.child, l.call_count, l.error_count) for l in ls]


@pytest.fixture(params=["7", "64", "100000"])
def stage(request, monkeypatch):
    monkeypatch.setenv("ZDL_STAGE_SPANS", request.param)
    return int(request.param)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("order", [True, False])
def test_put_trace_loop_matches_oracle(stage, seed, order):
    r = random.Random(500 + seed)
    traces = [random_trace(r, n=r.randint(1, 30), allow_npe=False) for _ in range(300)]
    traces += [random_trace(r, n=r.choice([65, 200]), allow_npe=False, id_pool=300) for _ in range(3)]
    r.shuffle(traces)
    ol = O.DependencyLinker()
    gl = DependencyLinker(insertion_order=order)
    for t in traces:
        ol.put_trace(t)
        gl.put_trace(t)
    want = _as_list(ol.link())
    got = _as_list(gl.link())
    assert got == want if order else sorted(got) == sorted(want)
    # link() leaves the linker usable: more traces, then the merged result
    more = [random_trace(r, n=r.randint(1, 20), allow_npe=False) for _ in range(50)]
    for t in more:
        ol.put_trace(t)
        gl.put_trace(t)
    got, want = _as_list(gl.link()), _as_list(ol.link())
    assert got == want if order else sorted(got) == sorted(want)
    gl.close()


@pytest.mark.parametrize("seed", range(8))
def test_npe_raised_by_its_own_put_trace(stage, seed):
    """Traces that make Trace.merge throw are mixed in; each raises from its own putTrace, adds
    nothing, and the traces around it are linked exactly as the reference links them when the
    caller catches the exception and goes on."""
    r = random.Random(900 + seed)
    ol = O.DependencyLinker()
    gl = DependencyLinker()
    npes = 0
    for _ in range(400):
        t = random_trace(r, n=r.randint(1, 10))
        try:
            ol.put_trace(t)
            raised = False
        except O.ReferenceNPE:
            raised = True
        if raised:
            npes += 1
            with pytest.raises(N.ReferenceNullPointerException):
                gl.put_trace(t)
        else:
            gl.put_trace(t)
    assert npes > 0
    assert _as_list(gl.link()) == _as_list(ol.link())
    gl.close()


def test_reset_drops_staged_traces(stage):
    r = random.Random(3)
    a = [random_trace(r, n=5, allow_npe=False) for _ in range(20)]
    b = [random_trace(r, n=5, allow_npe=False) for _ in range(20)]
    gl = DependencyLinker()
    for t in a:
        gl.put_trace(t)
    gl._ctx.reset()
    for t in b:
        gl.put_trace(t)
    ol = O.DependencyLinker()
    for t in b:
        ol.put_trace(t)
    assert _as_list(gl.link()) == _as_list(ol.link())
    gl.close()


def test_native_put_trace_loop_c2_vs_cpp():
    """The JNI-style caller loop (one zdl_put_trace per trace, libzdl_synth's driver) over a
    C2-shaped batch: the links equal the C++ restatement's over the same traces."""
    w = synth.C2.scaled(50_000)
    cols = synth.generate(w)
    ctx = N.Context(w.total_services, device=0)
    synth.put_trace_loop(ctx, cols)
    p, c, n, e = ctx.link()
    ctx.close()
    st, op, oc, on, oe = ref.link(cols, threads=8)
    assert st == 0
    got = sorted(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))
    assert got == sorted(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("cap", ["300", "2000"])
def test_lone_put_after_staged_big_traces_sorted(monkeypatch, seed, cap):
    """Sorted order (the lazy k_mid / k_tail path): staged batches holding traces of 65-200
    spans leave k_mid / k_tail deferred; a trace put alone right after (its merge may throw,
    or it is longer than the staging slot) must not regrow or refill the columns those
    deferred kernels read. Links equal the oracle's."""
    monkeypatch.setenv("ZDL_STAGE_SPANS", cap)
    r = random.Random(1300 + seed)
    ol = O.DependencyLinker()
    gl = DependencyLinker(insertion_order=False)
    npes = 0
    for i in range(120):
        x = r.random()
        if x < 0.3:
            t = random_trace(r, n=r.randint(65, 200), allow_npe=False, id_pool=400)
        elif x < 0.45:
            t = random_trace(r, n=r.randint(2, 10))  # allow_npe: may go alone and may throw
        elif x < 0.5:
            t = random_trace(r, n=int(cap) + r.randint(1, 300), allow_npe=False, id_pool=4000)
        else:
            t = random_trace(r, n=r.randint(1, 30), allow_npe=False)
        try:
            ol.put_trace(t)
            raised = False
        except O.ReferenceNPE:
            raised = True
        if raised:
            npes += 1
            with pytest.raises(N.ReferenceNullPointerException):
                gl.put_trace(t)
        else:
            gl.put_trace(t)
    assert sorted(_as_list(gl.link())) == sorted(_as_list(ol.link()))
    gl.close()


@pytest.mark.parametrize("seed", range(4))
def test_merge_runs_are_staged_and_linked(stage, seed):
    """Traces with merge runs whose Trace.merge cannot throw (every non-null endpoint complete)
    are staged like any other; the links (and insertion order) equal the oracle's."""
    r = random.Random(1700 + seed)
    traces = [random_trace(r, n=r.randint(2, 40), allow_npe=False, id_pool=3) for _ in range(200)]
    ol = O.DependencyLinker()
    gl = DependencyLinker()
    for t in traces:
        ol.put_trace(t)
        gl.put_trace(t)
    assert _as_list(gl.link()) == _as_list(ol.link())
    gl.close()
