"""Loads the transcribed reference fixtures (tests/golden/*.json)."""
import json
import os

from zipkin_amd.codec import link_from_json, span_from_json

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def spans(lst):
    return [span_from_json(d) for d in lst]


def links(lst):
    return [link_from_json(d) for d in lst]


def check_links(actual, case_expect, mode):
    """Applies the reference assertion: 'exact' = containsExactly, 'only' = containsOnly,
    dict = {'size': n, 'all_call_count': c} (ITDependencies.manyLinks)."""
    if isinstance(case_expect, dict):
        assert len(actual) == case_expect["size"]
        assert all(l.call_count == case_expect["all_call_count"] for l in actual)
        return
    exp = links(case_expect)
    if mode == "exact":
        assert list(actual) == exp
    else:
        assert sorted(actual, key=_k) == sorted(exp, key=_k), (actual, exp)
        assert len(set(actual)) == len(actual)


def _k(l):
    return (l.parent, l.child, l.call_count, l.error_count)
