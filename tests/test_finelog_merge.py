"""The FINE log quotes the span Trace.merge leaves (DependencyLinker.java:66, 158 print the
merged Span): zipkin_amd.linker._merged_spans replays Trace.merge's merge loop
(Trace.java:42-84) over the fragments in the device's sort order. Checked here on CPU against
the oracle's Trace.merge restatement (oracle/dl_oracle.py trace_merge_sources, pinned by
TraceTest's vectors) on random corner-case traces: fragments, shared spans without parent ids,
mixed trace-id widths."""
import functools
import random

import pytest

from oracle import dl_oracle as O
from tests.stress import random_trace
from zipkin_amd.linker import _merged_spans


def _positions(tr):
    order = sorted(range(len(tr)), key=functools.cmp_to_key(lambda a, b: O.cleanup_compare(tr[a], tr[b])))
    pos = [0] * len(tr)
    for k, i in enumerate(order):
        pos[i] = k
    tid = tr[0].trace_id  # Trace.java:34-38
    for k in range(1, len(tr)):
        if len(tid) != 32:
            tid = tr[order[k]].trace_id
    return pos, tid


@pytest.mark.parametrize("chunk", range(8))
def test_merged_spans_equal_trace_merge(chunk):
    checked = 0
    for seed in range(chunk * 400, (chunk + 1) * 400):
        r = random.Random(seed)
        tr = list(random_trace(r, n=r.randint(1, 30), allow_npe=False, id_pool=r.choice([3, 6, 20])))
        out, src = O.trace_merge_sources(tr)
        pos, tid = _positions(tr)
        assert _merged_spans(tr, pos, tid) == {s[0]: o for o, s in zip(out, src)}, seed
        checked += len(tr) != len(out)
    assert checked > 20  # traces with merged fragments were among them
