"""Copies the seven real traces of the reference's UI test data
(/root/reference/zipkin-ui/testdata/*.json, JSON v2 span lists) into
tests/golden/ui_testdata.json as extra inputs, with the links of each trace as the
oracle (oracle/dl_oracle.py, pinned by the reference's own test vectors) computes them.

The spans are data, copied field by field as the decoder reads them; the expected links
are ORACLE-DERIVED, NOT REFERENCE-PINNED: the reference asserts no links for these files.
Runs in this container only (/root/reference does not travel to the GPU box):

    python tests/golden/make_ui_fixtures.py
"""
from __future__ import annotations

import glob
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

from oracle import dl_oracle as O  # noqa: E402
from zipkin_amd.codec import span_from_json, span_to_json  # noqa: E402

SRC = "/root/reference/zipkin-ui/testdata"


def main():
    cases = []
    for path in sorted(glob.glob(os.path.join(SRC, "*.json"))):
        raw = json.load(open(path))
        spans = [span_from_json(d) for d in raw]
        linker = O.DependencyLinker()
        # one putTrace per low trace id, first-seen order (InMemoryStorage groups the same way)
        for trace in O.group_by_trace_id(spans):
            linker.put_trace(trace)
        links = [{"parent": l.parent, "child": l.child, "callCount": l.call_count, "errorCount": l.error_count}
                 for l in linker.link()]
        cases.append({"name": os.path.basename(path)[:-5], "ref": "zipkin-ui/testdata/" + os.path.basename(path),
                      "spans": [span_to_json(s) for s in spans], "expect_oracle": links})
    out = {"source": "zipkin-ui/testdata/*.json (data); expectations oracle-derived, not reference-pinned",
           "cases": cases}
    with open(os.path.join(ROOT, "tests", "golden", "ui_testdata.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
