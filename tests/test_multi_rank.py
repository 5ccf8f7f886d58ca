"""Multi-process path on CPU (gloo, world_size 2): traces sharded by the low 64 bits
of the trace id, each rank links its shard, one all-reduce of the S x S tables
(zipkin_amd.shard.combine_tables, the same call bench.py makes over RCCL) equals
linking everything at once. The per-rank linking uses the C++ restatement here
(no GPU in this container); on the GPU box the engine fills the table."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref
from zipkin_amd import shard, synth


def _table(cols, S):
    st, p, c, n, e = ref.link(cols, threads=2)
    assert st == 0
    call = torch.zeros(S * S, dtype=torch.int64)
    err = torch.zeros(S * S, dtype=torch.int64)
    idx = torch.from_numpy(p.astype(np.int64) * S + c)
    call[idx] = torch.from_numpy(n)
    err[idx] = torch.from_numpy(e)
    return call, err


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = synth.C4.scaled(4000)
    cols = synth.generate(w, threads=2)
    mine = shard.partition_columns(cols, world)[rank]
    call, err = _table(mine, w.total_services)
    shard.combine_tables(call, err)
    if rank == 0:
        out.put((call.numpy().copy(), err.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shard_and_combine_equals_single():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, PORT, q)) for r in range(2)]
    for p in procs:
        p.start()
    call, err = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = synth.C4.scaled(4000)
    full = synth.generate(w, threads=2)
    c1, e1 = _table(full, w.total_services)
    assert np.array_equal(call, c1.numpy()) and np.array_equal(err, e1.numpy())


PORT = _free_port()


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
