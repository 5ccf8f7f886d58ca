"""Times the device store index at C2 scale: eviction, the three selections, and a
getDependencies-style select + gather + link, over a 10M-span resident store."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zipkin_amd import _native as N  # noqa: E402
from zipkin_amd import synth  # noqa: E402

w = synth.C2
cols = synth.generate(w)
st = N.Store(0)
st.append(cols)
out = {"n_spans": cols.n_spans}


def t(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - a)
    return round(1e3 * min(ts), 3)


for name, mode in (("select_newest_ms", 0), ("select_all_ms", 1), ("select_all_strict_ms", 2)):
    out[name] = t(lambda: st.select(mode))
ctx = N.Context(w.total_services)


def query():
    ctx.reset()
    st.select(0)
    ctx.put_selection(st)
    ctx.link()


out["get_dependencies_ms"] = t(query)
a = time.perf_counter()
ev = st.evict(100_000)
out["evict_100k_ms"] = round(1e3 * (time.perf_counter() - a), 3)
out["evicted"] = ev
a = time.perf_counter()
st.compact_evicted()
out["compact_ms"] = round(1e3 * (time.perf_counter() - a), 3)
print(json.dumps(out), flush=True)
