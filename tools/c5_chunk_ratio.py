"""How much would pre-aggregating C5's sparse link log per k_link workgroup buy?

On the CPU: C5's generator scaled to --traces, its traces of at most 64 spans (the ones k_link
links and logs) cut into consecutive chunks of --chunk traces (a k_link workgroup's share at the
full size: 16M traces over 512 workgroups = 31 250), each chunk linked by the C++ restatement.
Per chunk: log entries (the sum of call counts = one entry per addLink) against distinct cells,
and the entries an LDS table of the chunk's H hottest cells would absorb.

    python tools/c5_chunk_ratio.py [--traces 2000000] [--chunk 31250]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--traces", type=int, default=2_000_000)
    ap.add_argument("--chunk", type=int, default=31_250)
    a = ap.parse_args()
    from oracle import ref
    from zipkin_amd import synth
    from zipkin_amd.columnar import Columns

    cols = synth.generate(synth.C5.scaled(a.traces))
    off = cols.offsets.astype(np.int64)
    n = np.diff(off)
    small = np.nonzero(n <= 64)[0]
    print(f"C5 scaled to {cols.n_traces} traces / {cols.n_spans} spans; {len(small)} traces of <= 64 spans "
          f"({int(n[small].sum())} spans)")
    ent_tot = dis_tot = 0
    hot = {256: 0, 1024: 0, 4096: 0}
    rows = []
    for c0 in range(0, len(small), a.chunk):
        t = small[c0:c0 + a.chunk]
        idx = np.concatenate([np.arange(off[i], off[i + 1]) for i in t])
        sub = Columns(*(getattr(cols, f)[idx] for f in ("trace_lo", "id", "parent_id", "local_svc", "remote_svc",
                                                         "local_ip4", "local_ip6", "port_flags", "timestamp")),
                      offsets=np.concatenate([[0], np.cumsum(n[t])]).astype(np.uint64))
        st, p, c, call, err = ref.link(sub, threads=8)
        ent = int(call.sum())
        ent_tot += ent
        dis_tot += len(call)
        srt = np.sort(call)[::-1]
        for h in hot:
            hot[h] += int(srt[:h].sum())
        rows.append((ent, len(call)))
    r = np.array(rows, dtype=np.float64)
    print(f"chunks of {a.chunk} small traces: {len(rows)}; entries per chunk {r[:, 0].mean():.0f}, distinct cells "
          f"{r[:, 1].mean():.0f}: entries / distinct = {ent_tot / dis_tot:.2f}")
    for h, v in hot.items():
        print(f"  an LDS table of each chunk's {h} hottest cells would absorb {v / ent_tot:.1%} of the entries")


if __name__ == "__main__":
    main()
