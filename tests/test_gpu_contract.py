"""API contracts of the C ABI that the kernels' results do not show: nothing may use
a context between zdl_link_start and zdl_link_finish, and a decoded batch's host views are
refused once its decoder has decoded another batch."""
import numpy as np
import pytest

from oracle import proto3_oracle as P
from zipkin_amd import _native as N
from zipkin_amd import synth
from zipkin_amd.columnar import Dictionary
from zipkin_amd.model import Span
from zipkin_amd.proto3 import Proto3Decoder

pytestmark = pytest.mark.gpu


def test_started_link_locks_the_context():
    w = synth.C2.scaled(2000)
    cols = synth.generate(w)
    ctx = N.Context(w.total_services, device=0)
    ctx.put_spans(cols)
    want = ctx.link()
    ctx.reset()
    ctx.put_spans(cols)
    ctx.link_start()
    for call in (lambda: ctx.put_spans(cols), ctx.reset, lambda: ctx.link(),
                 lambda: ctx.add_links(want[0][:1], want[1][:1], [1], [0])):
        with pytest.raises(N.ZdlError) as e:
            call()
        assert e.value.code == N.ZDL_EINVAL and "started link" in str(e.value)
    got = ctx.link_finish()
    assert all(np.array_equal(a, b) for a, b in zip(got, want))
    ctx.reset()  # usable again
    ctx.put_spans(cols)
    assert all(np.array_equal(a, b) for a, b in zip(ctx.link(), want))
    ctx.close()


def test_decoded_batch_views_expire_with_the_next_decode():
    dec = Proto3Decoder(Dictionary(), Dictionary(), Dictionary())
    a = dec.decode(P.write_list([Span.create("a1", "1"), Span.create("a2", "2")]))
    assert a.trace_lo.tolist() == [0xA1, 0xA2]
    b = dec.decode(P.write_list([Span.create("b1", "1")]))
    with pytest.raises(RuntimeError, match="next decode"):
        a.trace_lo
    assert b.trace_lo.tolist() == [0xB1]
    dec.close()
