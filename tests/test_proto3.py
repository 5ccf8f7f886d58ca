"""Proto3 ingest: the oracle restatement pinned by the reference's own proto3
vectors (CPU), and the device decoder zdl_decode_proto3 checked exactly against it (GPU):
same columns, same dictionary ids, same errors, and storage queries fed by accept_proto3
answering like accept(decodeList(bytes)).

Reference vectors transcribed: Proto3ZipkinFieldsTest (span_write_writesIds bytes,
span_write_kind index 22/23, span_write_debug / span_write_shared trailing bytes,
span_read_kind_tolerant, the span_read_* round trips), SpanBytesDecoderTest PROTO3 cases
(falseOnEmpty_inputSpans, niceErrorOnMalformed_inputSpans "Truncated: length 101 > bytes
remaining 3", traceRoundTrip / spansRoundTrip over the golden traces). Non-ASCII service names
(Java toLowerCase vs Python lower) and the lenient cross-message reads are parity-unpinned.
"""
import random
import struct

import numpy as np
import pytest

from golden_io import load, spans
from oracle import proto3_oracle as P
from zipkin_amd.columnar import Dictionary, pack_traces
from zipkin_amd.model import Endpoint, Kind, Span

DL = load("dependency_linker.json")
ST = load("storage_dependencies.json")
GOLDEN_SPANS = [s for c in DL["cases"] for t in c["traces"] for s in spans(t)]


def base():
    return Span.create("1", "2")


# ---------------- oracle vs the reference's vectors (CPU) ----------------

def test_write_ids_bytes():  # Proto3ZipkinFieldsTest.span_write_writesIds
    b = P.write_list([base()])
    assert list(b[:22]) == [0b00001010, 20, 0b00001010, 8, 0, 0, 0, 0, 0, 0, 0, 1,
                            0b00011010, 8, 0, 0, 0, 0, 0, 0, 0, 2]
    assert len(b) == 22


def test_write_kind_and_flags():  # span_write_kind / span_write_debug / span_write_shared
    b = P.write_list([base().to_builder(kind=Kind.PRODUCER)])
    assert b[22] == 0b0100000 and b[23] == 3
    b = P.write_list([base().to_builder(debug=True)])
    assert list(b[-2:]) == [0b01100000, 1]
    b = P.write_list([base().to_builder(shared=True)])
    assert list(b[-2:]) == [0b01101000, 1]


def test_write_omits_empty_endpoints():
    assert len(P.write_list([base().to_builder(local_endpoint=Endpoint(), remote_endpoint=Endpoint())])) == 22


def test_read_kind_tolerant():  # span_read_kind_tolerant
    b = bytearray(P.write_list([base().to_builder(kind=Kind.CONSUMER)]))
    b[1] += 0  # length unchanged
    b[23] = 5  # undefined kind: skipped
    assert P.read_list(bytes(b)) == ([base()], False)
    b[23] = 0
    assert P.read_list(bytes(b)) == ([base()], False)


@pytest.mark.parametrize("span", [
    base().to_builder(parent_id="1"), base().to_builder(name="romeo"), base().to_builder(kind=Kind.CONSUMER),
    base().to_builder(timestamp=1472470996199000, duration=134),
    base().to_builder(local_endpoint=Endpoint.create("frontend", "172.17.0.13"),
                      remote_endpoint=Endpoint.create("backend", "192.168.99.101", 9000)),
    base().to_builder(annotations=((1472470996199000, "parked on sidewalk"),)),
    base().to_builder(tags={"foo": "bar"}), base().to_builder(tags={"empty": ""}),
    base().to_builder(shared=True), base().to_builder(debug=True),
    base().to_builder(local_endpoint=Endpoint.create("x", "2001:db8::c001", 80)),
], ids=lambda s: "span")
def test_read_round_trip(span):  # span_read_* (assertRoundTrip)
    assert P.read_list(P.write_list([span])) == ([span], False)


def test_trace_round_trip_golden():  # traceRoundTrip_PROTO3 / spansRoundTrip_PROTO3
    assert P.read_list(P.write_list(GOLDEN_SPANS)) == (GOLDEN_SPANS, False)


def test_empty_and_malformed():  # falseOnEmpty_inputSpans / niceErrorOnMalformed_inputSpans
    assert P.read_list(b"") == ([], False)
    with pytest.raises(P.IllegalArgument, match="Truncated: length 101 > bytes remaining 3"):
        P.read_list(b"hello")
    assert P.read_list(P.write_list([base()]) + b"\x0a\x00" + P.write_list([base()])) == ([], False)


def test_ipv6_text_and_embedded_ipv4():
    assert P.write_ipv6(bytes.fromhex("20010db8000000000000000000000000")) == "2001:db8::"
    assert P.write_ipv6(bytes(16)) == "::"
    assert P.parse_ip_bytes(bytes(12) + bytes([1, 2, 3, 4]))[0] == "1.2.3.4"   # IPv4-compatible
    assert P.parse_ip_bytes(bytes(15) + b"\x01")[1] == "::1"                   # localhost stays v6
    mapped = bytes(10) + b"\xff\xff" + bytes([1, 2, 3, 4])                       # flag != -1: stays v6
    assert P.parse_ip_bytes(mapped)[1] == "::ffff:102:304"


# ---------------- generators ----------------

SVC = ["frontend", "Backend", "DB", "kafka", "web", "app", "MySQL", "cache", "a", "zz-top"]


def rand_endpoint(r):
    if r.random() < 0.15:
        return None
    svc = r.choice(SVC) if r.random() < 0.8 else None
    ip = None
    x = r.random()
    if x < 0.3:
        ip = f"10.0.{r.randrange(3)}.{r.randrange(4)}"
    elif x < 0.45:
        ip = r.choice(["2001:db8::c001", "fe80::1", "::1", "2001:db8:0:0:1::"])
    port = r.choice([0, 0, 80, 8080, 9411])
    e = Endpoint.create(svc, ip, port)
    return None if e.is_empty() else e


def rand_span(r, trace_id):
    sid = r.randrange(1, 1 << 64) if r.random() < 0.9 else r.randrange(1, 300)
    pid = r.choice([None, r.randrange(1, 1 << 64), r.randrange(1, 300)])
    tags = {}
    if r.random() < 0.2:
        tags["error"] = r.choice(["", "500"])
    if r.random() < 0.3:
        tags["http.path"] = "/api"
    return Span.create(trace_id, sid, pid, r.choice([None, Kind.CLIENT, Kind.SERVER, Kind.PRODUCER, Kind.CONSUMER]),
                       name=r.choice([None, "get", "Post"]),
                       timestamp=r.choice([0, 1472470996199000 + r.randrange(10 ** 6)]),
                       duration=r.choice([0, 134, 1 << 40]),
                       local_endpoint=rand_endpoint(r), remote_endpoint=rand_endpoint(r),
                       annotations=tuple((1472470996199000 + i, "ann") for i in range(r.randrange(3))),
                       tags=tags, shared=r.choice([None, True]), debug=r.choice([None, True]))


def rand_batch(r, n):
    out = []
    for _ in range(n):
        tid = r.choice(["%016x" % r.randrange(1, 1 << 64), "%032x" % r.randrange(1, 1 << 128),
                        "%016x" % r.randrange(1, 50)])
        out.append(rand_span(r, tid))
    return out


def add_unknown_fields(r, data: bytes) -> bytes:
    """Re-frames every span with extra unknown fields of each wire type (skipValue paths)."""
    b, pos, out = P._Buf(data), 0, bytearray()
    while b.pos < len(data):
        b.read_varint32()
        n = b.length_prefix()
        body = bytes(data[b.pos:b.pos + n])
        b.pos += n
        extra = P._varint(20 << 3 | 0) + P._varint(r.randrange(1 << 40))
        extra += P._varint(21 << 3 | 1) + struct.pack("<q", 7)
        extra += P._varint(22 << 3 | 2) + b"\x03xyz" + P._varint(23 << 3 | 5) + b"abcd"
        body = body + extra if r.random() < 0.5 else extra + body
        out += bytes([0x0a]) + P._varint(len(body)) + body
    return bytes(out)


def oracle_columns(data, svc, ip4, ip6):
    sp, overrun = P.read_list(data)
    return pack_traces([[s] for s in sp], svc, ip4, ip6), overrun


def mutate(r, data: bytes) -> bytes:
    b = bytearray(data)
    for _ in range(r.randrange(1, 4)):
        k = r.randrange(4)
        if k == 0 and b:
            b[r.randrange(len(b))] = r.randrange(256)
        elif k == 1 and b:
            del b[r.randrange(len(b)):]
        elif k == 2:
            b.insert(r.randrange(len(b) + 1), r.randrange(256))
        elif b:
            i = r.randrange(len(b))
            b[i] ^= 1 << r.randrange(8)
    return bytes(b)


def test_oracle_fuzz_never_crashes():
    r = random.Random(7)
    for _ in range(300):
        d = mutate(r, P.write_list(rand_batch(r, 3)))
        try:
            P.read_list(d)
        except P.IllegalArgument:
            pass


# ---------------- device decoder vs oracle (GPU) ----------------

COLS = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
        "timestamp")


def assert_same(got, exp):
    for f in COLS:
        np.testing.assert_array_equal(getattr(got, f), getattr(exp, f), err_msg=f)


def fresh():
    return Dictionary(), Dictionary(), Dictionary()


@pytest.mark.gpu
def test_gpu_decode_golden_spans():
    from zipkin_amd.proto3 import Proto3Decoder
    d = fresh()
    dec = Proto3Decoder(*d)
    o = fresh()
    data = P.write_list(GOLDEN_SPANS)
    exp, _ = oracle_columns(data, *o)
    assert_same(dec.decode_columns(data), exp)
    assert [x.strings for x in d] == [x.strings for x in o]
    dec.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_decode_random_batches(seed):
    """Several batches through one decoder: ids stay first-seen across batches."""
    from zipkin_amd.proto3 import Proto3Decoder
    r = random.Random(seed)
    d, o = fresh(), fresh()
    dec = Proto3Decoder(*d)
    for _ in range(3):
        data = P.write_list(rand_batch(r, r.randrange(1, 400)))
        if seed % 2:
            data = add_unknown_fields(r, data)
        exp, overrun = oracle_columns(data, *o)
        assert not overrun
        assert_same(dec.decode_columns(data), exp)
        assert [x.strings for x in d] == [x.strings for x in o]
    dec.close()


@pytest.mark.gpu
def test_gpu_decode_errors_match_oracle():
    """Mutated batches: the device raises where the reference throws, rejects where the
    reference would read across a message end, and otherwise decodes identically."""
    from zipkin_amd import _native as N
    from zipkin_amd.proto3 import Proto3Decoder
    r = random.Random(99)
    seen = {"ok": 0, "iae": 0, "overrun": 0}
    for _ in range(400):
        d, o = fresh(), fresh()
        dec = Proto3Decoder(*d)
        data = mutate(r, P.write_list(rand_batch(r, r.randrange(1, 6))))
        try:
            exp, overrun = oracle_columns(data, *o)
            kind = "overrun" if overrun else "ok"
        except P.IllegalArgument:
            kind = "iae"
        seen[kind] += 1
        if kind == "iae":
            with pytest.raises(N.ReferenceIllegalArgumentException):
                dec.decode_columns(data)
        elif kind == "overrun":
            with pytest.raises(N.ZdlError) as ei:
                dec.decode_columns(data)
            assert ei.value.code == N.ZDL_EINVAL
        else:
            assert_same(dec.decode_columns(data), exp)
            assert [x.strings for x in d] == [x.strings for x in o]
        dec.close()
    assert min(seen.values()) > 0, seen


@pytest.mark.gpu
def test_gpu_decode_edge_inputs():
    from zipkin_amd import _native as N
    from zipkin_amd.proto3 import Proto3Decoder
    dec = Proto3Decoder(*fresh())
    assert dec.decode(b"").n_spans == 0
    with pytest.raises(N.ReferenceIllegalArgumentException):
        dec.decode(b"hello")
    one = P.write_list([base()])
    assert dec.decode(one + b"\x0a\x00" + one).n_spans == 0  # zero-length span: empty list
    assert dec.decode(one * 3).n_spans == 3
    dec.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ST["cases"], ids=lambda c: c["name"])
def test_gpu_storage_accept_proto3(case):
    """ITDependencies through accept_proto3(encode(batch)) == the transcribed expectations."""
    from golden_io import check_links
    from zipkin_amd.storage import InMemoryStorage
    store = InMemoryStorage(strict_trace_id=True)
    for b in case["batches"]:
        store.accept_proto3(P.write_list(spans(b))).execute()
    for q in case["queries"]:
        check_links(store.get_dependencies(q["endTs"], q["lookback"]).execute(), q["expect"], "only")


@pytest.mark.gpu
def test_gpu_decode_then_link_large():
    """100k synthetic spans: decode on the device, link the device columns (grouped on the device),
    same links as packing the oracle-decoded spans."""
    from zipkin_amd import _native as N
    from zipkin_amd.proto3 import Proto3Decoder
    r = random.Random(5)
    sp = []
    for t in range(10000):
        tid = "%016x" % r.randrange(1, 1 << 64)
        root = r.randrange(1, 1 << 64)
        sp.append(Span.create(tid, root, None, Kind.SERVER, local_endpoint=Endpoint.create(r.choice(SVC))))
        for _ in range(9):
            sp.append(Span.create(tid, r.randrange(1, 1 << 64), root, r.choice([Kind.CLIENT, None]),
                                  local_endpoint=Endpoint.create(r.choice(SVC)),
                                  remote_endpoint=Endpoint.create(r.choice(SVC)),
                                  tags={"error": ""} if r.random() < 0.05 else None))
    r.shuffle(sp)
    data = P.write_list(sp)
    d, o = fresh(), fresh()
    dec = Proto3Decoder(*d)
    b = dec.decode(data)
    ctx = N.Context(len(d[0]))
    ctx.put_spans_device({k: getattr(b.dev, k) for k in COLS}, b.n_spans, None, 0)
    got = sorted(zip(*(a.tolist() for a in ctx.link())))
    exp_cols, _ = oracle_columns(data, *o)
    ctx2 = N.Context(len(o[0]))
    ctx2.put_spans_ungrouped(exp_cols)
    exp = sorted(zip(*(a.tolist() for a in ctx2.link())))
    assert got == exp and len(got) > 0
    dec.close()


@pytest.mark.gpu
def test_gpu_decode_spans_beyond_lds_window():
    """Blocks whose span messages exceed the kernel's LDS window read the rest from HBM."""
    from zipkin_amd.proto3 import Proto3Decoder
    r = random.Random(3)
    sp = rand_batch(r, 600)
    big = [s.to_builder(local_endpoint=Endpoint.create("svc-" + "x" * r.randrange(50, 3000), "10.0.0.1", 80))
           if i % 3 == 0 else s for i, s in enumerate(sp)]
    d, o = fresh(), fresh()
    dec = Proto3Decoder(*d)
    data = P.write_list(big)
    exp, _ = oracle_columns(data, *o)
    assert_same(dec.decode_columns(data), exp)
    assert [x.strings for x in d] == [x.strings for x in o]
    dec.close()
