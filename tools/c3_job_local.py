"""C3 as BASELINE.json states it - 1B synthetic spans / 100M traces / 500 services, sharded by
splitmix64(trace_lo) over 8 ranks, the ranks' counts combined - executed on ONE MI355X: the 8
ranks are contexts of this process joined by zdl_comm_init_local (zipkin_amd/csrc/zdl_xport.inc),
so every rank's put, the LOG-mode reduce and the job's sum all-reduce run as in an 8-GPU job,
only the combine's bytes move by device copies instead of xGMI. Each rank's shard is the one
bench.py --gpus 8 generates for that rank (synth C3, 12.5M traces a rank).

Checks every rank's link() against the C++ restatement of DependencyLinker over all 1B spans
(oracle/dl_ref.cpp, run per shard on the host and summed: DependencyLinker.merge's sum,
DependencyLinker.java:189-204) and reports the job's step time on the one GPU.
   python tools/c3_job_local.py [--ranks 8] [--traces-per-rank 12500000] [--steps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def log(*a):
    print(*a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--traces-per-rank", type=int, default=12_500_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-oracle", action="store_true")
    args = ap.parse_args()
    import torch

    from zipkin_amd import _native as N
    from zipkin_amd import synth

    W = args.ranks
    dev = torch.device("cuda", 0)
    w0 = synth.C3.scaled(args.traces_per_rank)
    S = w0.total_services
    names = ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags", "timestamp")
    shards, dcols, doffs = [], [], []
    t0 = time.time()
    n_spans = 0
    for r in range(W):
        cols = synth.generate(w0.sharded(r, W))
        n_spans += cols.n_spans
        dcols.append({k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
            np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev) for k in names})
        doffs.append(torch.from_numpy(cols.offsets.view(np.int64)).to(dev))
        shards.append(cols if not args.no_oracle else (cols.n_spans, cols.n_traces))
        log(f"rank {r}: {cols.n_spans} spans / {cols.n_traces} traces ({time.time() - t0:.1f}s)")
    torch.cuda.synchronize(dev)
    ctxs = [N.Context(S, device=0) for _ in range(W)]
    N.Context.comm_init_local(ctxs)

    def meta(r):
        s = shards[r]
        return (s.n_spans, s.n_traces) if not args.no_oracle else s

    def put_and_link(r, c):
        p = {k: v.data_ptr() for k, v in dcols[r].items()}
        p["timestamp"] = None
        ns, nt = meta(r)
        c.reset()
        c.put_spans_device(p, ns, doffs[r].data_ptr(), nt)
        return c.link()

    out = [None] * W
    times = []
    for step in range(args.steps + 1):
        errs = []

        def run(r):
            try:
                out[r] = put_and_link(r, ctxs[r])
            except Exception as ex:  # noqa: BLE001
                errs.append((r, repr(ex)))

        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        ts = [threading.Thread(target=run, args=(r,)) for r in range(W)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise SystemExit(f"rank failure: {errs}")
        dt = time.perf_counter() - t1
        if step:
            times.append(dt)
        log(f"step {step}: {dt * 1e3:.1f} ms ({len(out[0][0])} links on every rank)")
    for c in ctxs:
        c.close()
    ms = float(np.median(times)) * 1e3
    res = {"workload": "c3 as BASELINE.json states it, 8-rank job on one MI355X (zdl_comm_init_local)",
           "ranks": W, "spans": n_spans, "traces": W * args.traces_per_rank, "services": S,
           "ms_per_job_step": ms, "spans_per_s_one_gpu": n_spans / (ms * 1e-3), "steps": args.steps,
           "links": int(len(out[0][0])),
           "ranks_agree": all(all(np.array_equal(a, b) for a, b in zip(out[0], out[r])) for r in range(W))}
    if not args.no_oracle:
        from oracle import ref
        t1 = time.time()
        call = np.zeros(S * S, np.int64)
        err = np.zeros(S * S, np.int64)
        for r, cols in enumerate(shards):
            st, p, c, n, e = ref.link(cols, threads=16)
            assert st == 0
            np.add.at(call, p.astype(np.int64) * S + c, n)
            np.add.at(err, p.astype(np.int64) * S + c, e)
        nz = np.nonzero(call)[0]
        exp = sorted(zip((nz // S).tolist(), (nz % S).tolist(), call[nz].tolist(), err[nz].tolist()))
        got = sorted(zip(*(a.tolist() for a in out[0])))
        res["parity"] = "bit-exact vs the C++ restatement over every span" if got == exp else "MISMATCH"
        res["oracle_s"] = time.time() - t1
        res["calls"] = int(call.sum())
    log(json.dumps(res))


if __name__ == "__main__":
    main()
