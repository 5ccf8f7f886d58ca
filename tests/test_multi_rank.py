"""The sharding the multi-GPU path relies on, checked on CPU with world-size-2 gloo processes.

Traces shard by splitmix64 of the low 64 bits of the trace id (shard.partition_columns, the
same rule as zdl_shard_of and bench.py's per-rank generator), so no trace crosses ranks, and
the job's result is DependencyLinker.merge over the ranks' lists (DependencyLinker.java:189-204).
Here each gloo rank runs the oracle over its own shard and the ranks exchange their lists
(all_gather_object): the merged sums equal one linker over every trace. This checks the
sharding rule and the merge semantics only - the oracle stands in for each rank's linker. The
engine's own combines (libzdl: the sum / MIN all-reduces and the sparse reduce-scatter) run
with W = 2, 3 and 8 ranks on one GPU in tests/test_gpu_local_world.py."""
import os
import socket
from collections import namedtuple

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import dl_oracle as O
from oracle import ref
from zipkin_amd import shard, synth

Link = namedtuple("Link", "parent child call_count error_count")


def _links(cols):
    st, p, c, n, e = ref.link(cols, threads=2)
    assert st == 0
    return list(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = synth.C4.scaled(4000)
    cols = synth.generate(w, threads=2)
    mine = shard.partition_columns(cols, world)[rank]
    # every trace of this rank's shard hashes to this rank (no trace crosses ranks)
    lo = mine.trace_lo[mine.offsets[:-1].astype(np.int64)] if mine.n_traces else np.zeros(0, np.uint64)
    assert (shard.shard_of(lo, world) == rank).all()
    lists = [None] * world
    dist.all_gather_object(lists, _links(mine) if mine.n_spans else [])
    if rank == 0:
        out.put(lists)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shards_merge_to_the_whole():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    lists = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = synth.C4.scaled(4000)
    full = synth.generate(w, threads=2)
    # the oracle's merge keys links by service name: ids as names, and back
    merged = O.DependencyLinker.merge([Link(f"s{a}", f"s{b}", n, e) for lst in lists for a, b, n, e in lst])
    got = sorted((int(l.parent[1:]), int(l.child[1:]), l.call_count, l.error_count) for l in merged)
    assert got == sorted(_links(full))
    assert sum(len(lst) for lst in lists) > len(got)  # both ranks saw some of the same pairs


def test_partition_keeps_mixed_width_trace_ids_together():
    """Spans of one trace that carry 128-bit and 64-bit trace ids share trace_lo, so
    they land on one rank (ITDependencies.getDependencies_strictTraceId)."""
    from zipkin_amd.columnar import Dictionary, pack_traces
    from zipkin_amd.model import Kind, Span, Endpoint
    t = [Span.create("7180c278b62e8f6a216a2aea45d08fc9", "1", None, Kind.SERVER,
                     local_endpoint=Endpoint.create("frontend")),
         Span.create("216a2aea45d08fc9", "2", "1", Kind.SERVER, shared=True,
                     local_endpoint=Endpoint.create("backend")),
         Span.create("7180c278b62e8f6a216a2aea45d08fc9", "2", "1", Kind.CLIENT,
                     local_endpoint=Endpoint.create("frontend"))]
    cols = pack_traces([t], Dictionary(), Dictionary(), Dictionary())
    parts = shard.partition_columns(cols, 4)
    assert sorted(p.n_spans for p in parts) == [0, 0, 0, 3]


def _same_columns(a, b):
    for k in ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
              "timestamp"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    # partition_columns keeps empty traces (the host split drops them: they link nothing)
    assert np.array_equal(a.offsets, np.unique(b.offsets))


def test_host_split_equals_partition_columns():
    """A device group's host split (zdl_shard.h, run by libzdl's group_put; here through
    libzdl_synth) gives every shard exactly shard.partition_columns' traces, in storage order,
    with the same CSR offsets - at 1, 2, 3, 8 and 64 shards, on 1 and 4 threads, with empty
    traces (which go nowhere) mixed in."""
    from zipkin_amd.columnar import Columns
    cols = synth.generate(synth.C4.scaled(6000), threads=2)
    sizes = np.diff(cols.offsets.astype(np.int64))
    # empty traces inserted every 97th trace
    new_sizes = np.insert(sizes, np.arange(0, len(sizes), 97), 0)
    off = np.zeros(len(new_sizes) + 1, np.uint64)
    off[1:] = np.cumsum(new_sizes)
    holey = Columns(cols.trace_lo, cols.id, cols.parent_id, cols.local_svc, cols.remote_svc, cols.local_ip4,
                    cols.local_ip6, cols.port_flags, cols.timestamp, off)
    for c in (cols, holey):
        for n in (1, 2, 3, 8, 64):
            want = shard.partition_columns(c, n)
            for th in (1, 4):
                got, sec = synth.shard_host(c, n, threads=th)
                assert sec >= 0 and len(got) == n
                for g, w in zip(got, want):
                    _same_columns(g, w)


def test_host_split_ungrouped_keeps_input_order():
    """Ungrouped input (no offsets): every span by its own trace_lo, input order kept."""
    cols = synth.generate(synth.C2.scaled(3000), threads=2)
    perm = np.random.default_rng(5).permutation(cols.n_spans)
    from zipkin_amd.columnar import Columns
    sh = Columns(*(getattr(cols, k)[perm] for k in ("trace_lo", "id", "parent_id", "local_svc", "remote_svc",
                                                    "local_ip4", "local_ip6", "port_flags", "timestamp")),
                 np.zeros(1, np.uint64))
    got, _ = synth.shard_host(sh, 5, threads=3, grouped=False)
    d = shard.shard_of(sh.trace_lo, 5)
    for r in range(5):
        assert np.array_equal(got[r].id, sh.id[d == r])
        assert np.array_equal(got[r].trace_lo, sh.trace_lo[d == r])
        assert np.array_equal(got[r].port_flags, sh.port_flags[d == r])
