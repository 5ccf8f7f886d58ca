"""The reference's UI test traces (zipkin-ui/testdata/*.json, copied by
tests/golden/make_ui_fixtures.py): real multi-service traces with messaging, shared spans
and clock skew. Their links are oracle-derived (the reference asserts none for these
files), so the CPU test only checks the fixture still matches the oracle; the GPU tests put
them through the engine's facades and compare links (exact list order) and trees."""
import pytest

from oracle import dl_oracle as O
from tests.golden_io import load, spans

UI = load("ui_testdata.json")


def _links(ls):
    return [{"parent": l.parent, "child": l.child, "callCount": l.call_count, "errorCount": l.error_count}
            for l in ls]


@pytest.mark.parametrize("case", UI["cases"], ids=lambda c: c["name"])
def test_fixture_matches_oracle(case):
    linker = O.DependencyLinker()
    for trace in O.group_by_trace_id(spans(case["spans"])):
        linker.put_trace(trace)
    assert _links(linker.link()) == case["expect_oracle"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", UI["cases"], ids=lambda c: c["name"])
def test_engine_facades(case):
    from zipkin_amd.linker import DependencyLinker
    from zipkin_amd.storage import InMemoryStorage
    traces = O.group_by_trace_id(spans(case["spans"]))
    linker = DependencyLinker()
    for t in traces:
        linker.put_trace(t)
    assert _links(linker.link()) == case["expect_oracle"]
    linker.close()
    store = InMemoryStorage(strict_trace_id=False)
    store.accept(spans(case["spans"])).execute()
    ref = O.InMemoryStorage(strict_trace_id=False)
    ref.accept(spans(case["spans"]))
    assert _links(store.get_dependencies()) == _links(ref.get_dependencies_all())
    store.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", UI["cases"], ids=lambda c: c["name"])
def test_engine_trees(case):
    from tests.test_gpu_tree import _gpu_heads
    traces = O.group_by_trace_id(spans(case["spans"]))
    for t, got in zip(traces, _gpu_heads(traces)):
        assert got == O.tree_heads(t)
