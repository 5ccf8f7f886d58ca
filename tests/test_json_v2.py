"""JSON v2 ingest: the oracle restatement (gson 2.8.5 strict JsonReader +
V2SpanReader + V2SpanWriter) pinned by the reference's own vectors (CPU), and the device decoder
zdl_decode_json_v2 checked exactly against it (GPU): same columns, same dictionary ids, same
errors, and storage queries fed by accept_json_v2 answering like accept(decodeList(bytes)).

Reference vectors transcribed (zipkin/src/test/java/zipkin2/codec/): SpanBytesEncoderTest
span_JSON_V2 / localSpan_JSON_V2 / span_64bitTraceId_JSON_V2 / span_shared_JSON_V2 /
specialCharsInJson_JSON_V2 / span_minimum_JSON_V2 / span_noLocalServiceName_JSON_V2 /
span_noRemoteServiceName_JSON_V2 (exact bytes, decoded back to the same span), and every
SpanBytesDecoderTest JSON_V2 case (niceErrorOnUppercase_traceId, readsTraceIdHighFromTraceIdField,
ignoresNull_topLevelFields, ignoresNull_endpoint_topLevelFields, skipsIncompleteEndpoint,
niceErrorOnIncomplete_annotation, niceErrorOnNull_traceId / _id / _tagValue / _annotationValue /
_annotationTimestamp, readSpan_local/remoteEndpoint_noServiceName, falseOnEmpty_inputSpans,
niceErrorOnMalformed_inputSpans, traceRoundTrip / spansRoundTrip over the golden traces).
Parity unpinned (no reference-executed result): non-ASCII case mapping of service names, malformed
UTF-8 replacement counts, surrogate escapes in names; non-ASCII digits in quoted numbers beyond
Java 8's table (Character.digit); the gson restatement itself beyond those vectors (gson is a
dependency absent from the reference tree). NUMBER_VECTORS' expected values are derived from IEEE-754
rounding and Java's cast rules, not from a run of the reference.
"""
import random

import numpy as np
import pytest

from golden_io import load, spans
from oracle import json_oracle as J
from test_proto3 import COLS, SVC, assert_same, fresh, rand_batch
from zipkin_amd.columnar import pack_traces
from zipkin_amd.model import Endpoint, Kind, Span

DL = load("dependency_linker.json")
ST = load("storage_dependencies.json")
GOLDEN_SPANS = [s for c in DL["cases"] for t in c["traces"] for s in spans(t)]

TODAY = 1472470996199  # TestObjects.TODAY as the encoder tests print it (ms)
CLIENT_SPAN = Span.create(
    "7180c278b62e8f6a216a2aea45d08fc9", "5b4185666d50f68b", "6b221d5bc9e6496c", Kind.CLIENT, name="get",
    timestamp=1472470996199000, duration=207000,
    local_endpoint=Endpoint.create("frontend", "127.0.0.1"),
    remote_endpoint=Endpoint.create("backend", "192.168.99.101", 9000),
    annotations=((1472470996238000, "foo"), (1472470996403000, "bar")),
    tags={"clnt/finagle.version": "6.45.0", "http.path": "/api"})
LOCAL_SPAN = Span.create("dc955a1d4768875d", "dc955a1d4768875d", None, None, name="encode",
                         timestamp=1510256710021866, duration=1117,
                         local_endpoint=Endpoint.create("isao01", "10.23.14.72"))
UTF8_SPAN = Span.create("1", "1", None, None, name="\"\\\t\b\n\r\f",
                        annotations=((1, "\u2028 and \u2029"),),
                        tags={"\"foo": "Database error: ORA-00942:\u2028 and \u2029 table or view does not exist\n"})
_BODY = (',"kind":"CLIENT","name":"get","timestamp":1472470996199000,"duration":207000,'
         '"localEndpoint":{"serviceName":"frontend","ipv4":"127.0.0.1"},'
         '"remoteEndpoint":{"serviceName":"backend","ipv4":"192.168.99.101","port":9000},'
         '"annotations":[{"timestamp":1472470996238000,"value":"foo"},{"timestamp":1472470996403000,"value":"bar"}],'
         '"tags":{"clnt/finagle.version":"6.45.0","http.path":"/api"}')
ENCODER_VECTORS = [  # SpanBytesEncoderTest: (span, exact JSON_V2 bytes)
    (CLIENT_SPAN, '{"traceId":"7180c278b62e8f6a216a2aea45d08fc9","parentId":"6b221d5bc9e6496c","id":"5b4185666d50f68b"'
     + _BODY + "}"),
    (LOCAL_SPAN, '{"traceId":"dc955a1d4768875d","id":"dc955a1d4768875d","name":"encode","timestamp":1510256710021866,'
     '"duration":1117,"localEndpoint":{"serviceName":"isao01","ipv4":"10.23.14.72"}}'),
    (CLIENT_SPAN.to_builder(trace_id="216a2aea45d08fc9"),
     '{"traceId":"216a2aea45d08fc9","parentId":"6b221d5bc9e6496c","id":"5b4185666d50f68b"' + _BODY + "}"),
    (CLIENT_SPAN.to_builder(kind=Kind.SERVER, shared=True),
     '{"traceId":"7180c278b62e8f6a216a2aea45d08fc9","parentId":"6b221d5bc9e6496c","id":"5b4185666d50f68b"'
     + _BODY.replace('"CLIENT"', '"SERVER"') + ',"shared":true}'),
    (UTF8_SPAN, '{"traceId":"0000000000000001","id":"0000000000000001","name":"\\"\\\\\\t\\b\\n\\r\\f",'
     '"annotations":[{"timestamp":1,"value":"\\u2028 and \\u2029"}],"tags":{"\\"foo":"Database error: '
     'ORA-00942:\\u2028 and \\u2029 table or view does not exist\\n"}}'),
    (Span.create("7180c278b62e8f6a216a2aea45d08fc9", "5b4185666d50f68b"),
     '{"traceId":"7180c278b62e8f6a216a2aea45d08fc9","id":"5b4185666d50f68b"}'),
    (CLIENT_SPAN.to_builder(local_endpoint=Endpoint.create(None, "127.0.0.1")),
     '{"traceId":"7180c278b62e8f6a216a2aea45d08fc9","parentId":"6b221d5bc9e6496c","id":"5b4185666d50f68b"'
     + _BODY.replace('{"serviceName":"frontend","ipv4":"127.0.0.1"}', '{"ipv4":"127.0.0.1"}') + "}"),
    (CLIENT_SPAN.to_builder(remote_endpoint=Endpoint.create(None, "192.168.99.101", 9000)),
     '{"traceId":"7180c278b62e8f6a216a2aea45d08fc9","parentId":"6b221d5bc9e6496c","id":"5b4185666d50f68b"'
     + _BODY.replace('{"serviceName":"backend","ipv4":"192.168.99.101","port":9000}',
                     '{"ipv4":"192.168.99.101","port":9000}') + "}"),
]

_ID = '  "traceId": "6b221d5bc9e6496c",\n'
DECODER_VECTORS = [  # SpanBytesDecoderTest JSON_V2: (span object, None = IllegalArgumentException, else check)
    ('{\n  "traceId": "48485A3953BB6124",\n  "name": "get-traces",\n  "id": "6b221d5bc9e6496c"\n}', None),
    ('{\n' + _ID + '  "parentId": null,\n  "id": "6b221d5bc9e6496c",\n  "name": null,\n  "timestamp": null,\n'
     '  "duration": null,\n  "localEndpoint": null,\n  "remoteEndpoint": null,\n  "annotations": null,\n'
     '  "tags": null,\n  "debug": null,\n  "shared": null\n}', lambda s: s.id == "6b221d5bc9e6496c"),
    ('{\n' + _ID + '  "name": "get-traces",\n  "id": "6b221d5bc9e6496c",\n  "localEndpoint": {\n'
     '    "serviceName": null,\n    "ipv4": "127.0.0.1",\n    "ipv6": null,\n    "port": null\n  }\n}',
     lambda s: s.local_endpoint == Endpoint.create(None, "127.0.0.1")),
    ('{\n' + _ID + '  "id": "6b221d5bc9e6496c",\n  "localEndpoint": {\n    "serviceName": null,\n'
     '    "ipv4": null,\n    "ipv6": null,\n    "port": null\n  }\n}', lambda s: s.local_endpoint is None),
    ('{\n' + _ID + '  "id": "6b221d5bc9e6496c",\n  "localEndpoint": {\n  }\n}', lambda s: s.local_endpoint is None),
    ('{\n' + _ID + '  "id": "6b221d5bc9e6496c",\n  "remoteEndpoint": {\n    "serviceName": null,\n'
     '    "ipv4": null,\n    "ipv6": null,\n    "port": null\n  }\n}', lambda s: s.remote_endpoint is None),
    ('{\n' + _ID + '  "id": "6b221d5bc9e6496c",\n  "remoteEndpoint": {\n  }\n}', lambda s: s.remote_endpoint is None),
    ('{\n' + _ID + '  "name": "get-traces",\n  "id": "6b221d5bc9e6496c",\n  "annotations": [\n'
     '    { "timestamp": 1472470996199000}\n  ]\n}', None),
    ('{\n  "traceId": null,\n  "name": "get-traces",\n  "id": "6b221d5bc9e6496c"\n}', None),
    ('{\n' + _ID + '  "name": "get-traces",\n  "id": null\n}', None),
    ('{\n' + _ID + '  "name": "get-traces",\n  "id": "6b221d5bc9e6496c",\n  "tags": {\n    "foo": NULL\n  }\n}', None),
    ('{\n' + _ID + '  "name": "get-traces",\n  "id": "6b221d5bc9e6496c",\n  "annotations": [\n'
     '    { "timestamp": 1472470996199000, "value": NULL}\n  ]\n}', None),
    ('{\n' + _ID + '  "name": "get-traces",\n  "id": "6b221d5bc9e6496c",\n  "annotations": [\n'
     '    { "timestamp": NULL, "value": "foo"}\n  ]\n}', None),
    ('{\n' + _ID + '  "name": "get-traces",\n  "id": "6b221d5bc9e6496c",\n  "localEndpoint": {\n'
     '    "ipv4": "127.0.0.1"\n  }\n}', lambda s: s.local_service_name is None),
    ('{\n' + _ID + '  "name": "get-traces",\n  "id": "6b221d5bc9e6496c",\n  "remoteEndpoint": {\n'
     '    "ipv4": "127.0.0.1"\n  }\n}', lambda s: s.remote_service_name is None),
]


# ---------------- oracle vs the reference's vectors (CPU) ----------------

@pytest.mark.parametrize("k", range(len(ENCODER_VECTORS)))
def test_writer_and_reader_vectors(k):  # SpanBytesEncoderTest *_JSON_V2 + the decoder round trips
    span, text = ENCODER_VECTORS[k]
    assert J.write_span(span) == text
    assert J.read_list(("[" + text + "]").encode()) == [span]


@pytest.mark.parametrize("k", range(len(DECODER_VECTORS)))
def test_decoder_vectors(k):  # SpanBytesDecoderTest *_JSON_V2 (decodeOne of the object, as a list)
    obj, check = DECODER_VECTORS[k]
    data = ("[" + obj + "]").encode()
    if check is None:
        with pytest.raises(J.IllegalArgument):
            J.read_list(data)
    else:
        (s,) = J.read_list(data)
        assert check(s)


def test_trace_id_high_read_from_trace_id_field():  # readsTraceIdHighFromTraceIdField
    a = J.read_list(b'[{"traceId": "48485a3953bb61246b221d5bc9e6496c", "name": "get-traces", "id": "6b221d5bc9e6496c"}]')
    b = J.read_list(b'[{"traceId": "6b221d5bc9e6496c", "name": "get-traces", "id": "6b221d5bc9e6496c"}]')
    assert a == [b[0].to_builder(trace_id="48485a3953bb61246b221d5bc9e6496c")]


def test_short_zero_id_is_kept():
    """Span.Builder.id("0") pads to 16 zeros and keeps it (Span.java:474-483: only a 16-zero text
    is "all zeros"); the decoder reads it once, as V2SpanReader does."""
    sp = J.read_list(b'[{"traceId":"a","id":"0"}]')
    assert sp[0].id == "0" * 16
    with pytest.raises(J.IllegalArgument):
        J.read_list(b'[{"traceId":"a","id":"0000000000000000"}]')


def test_empty_and_malformed():  # falseOnEmpty_inputSpans / niceErrorOnMalformed_inputSpans
    assert J.read_list(b"") == []
    assert J.read_list(b"[]") == []
    with pytest.raises(J.IllegalArgument):
        J.read_list(b"hello")


def test_golden_traces_round_trip():  # traceRoundTrip_JSON_V2 / spansRoundTrip_JSON_V2
    assert J.read_list(J.write_list(GOLDEN_SPANS)) == GOLDEN_SPANS


@pytest.mark.parametrize("text,v4,v6", [
    ("127.0.0.1", "127.0.0.1", None), ("01.2.3.4", "01.2.3.4", None), ("1.2.3", None, None),
    ("::1", None, "::1"), ("::1.2.3.4", "1.2.3.4", None), ("::ffff:1.2.3.4", "1.2.3.4", None),
    ("::fFfF:1.2.3.4", "1.2.3.4", None), ("::ffff:102:304", None, "::ffff:102:304"),
    ("2001:db8::c001", None, "2001:db8::c001"), ("2001:DB8:0:0:0:0:0:C001", None, "2001:db8::c001"),
    ("1::2::3", None, None), ("1:2:3:4:5:6:7:8", None, "1:2:3:4:5:6:7:8"), ("1:2:3:4:5:6:7:8:9", None, None),
    ("::", None, "::"), (":1::", None, None), ("00000001::", None, "1::"), ("10000::", None, None),
    ("1.2.3.256", None, None), ("abc", None, None), ("::1.2.3.4:5", None, None),
])
def test_parse_ip(text, v4, v6):  # Endpoint.Builder.parseIp(String) restated (Endpoint.java:219-518)
    assert J.parse_ip(text, None, None) == (v4, v6)


def test_gson_strictness():
    ok = b'[{"traceId":"1","id":"2"}]'
    assert len(J.read_list(ok)) == 1
    for bad in [b'[{"traceId":"1","id":"2"},]', b'[{"traceId":"1","id":"2",}]', b"[{'traceId':'1','id':'2'}]",
                b'[{traceId:"1","id":"2"}]', b'[{"traceId":"1";"id":"2"}]', b'[{"traceId"="1","id":"2"}]',
                b'[{"traceId":"1","id":"2"} {"traceId":"1","id":"2"}]', b'[/*c*/{"traceId":"1","id":"2"}]',
                b'[{"traceId":"1","id":"2","x":01}]', b'[{"traceId":"1","id":"2","x":tru}]',
                b'[{"traceId":"1","id":"2","x":"\\x"}]', b'[{"traceId":"1","id":"2","x":"\\u12g4"}]',
                b'[{"traceId":"1","id":"2"}', b'[{"traceId":"1","id":"2","x":[1,]}]']:
        with pytest.raises(J.IllegalArgument):
            J.read_list(bad)
    # accepted by the strict reader: keywords in either case per character, trailing input
    # after the array, escapes in names, numbers as strings, quoted longs
    assert J.read_list(b'[{"traceId":"1","id":"2","shared":tRuE}] trailing') == \
        [Span.create("1", "2", shared=True)]
    assert J.read_list(b'[{"trace\\u0049d":123,"id":"2","timestamp":"77"}]') == [Span.create("123", "2", timestamp=77)]
    with pytest.raises(J.IllegalArgument):  # nextLong: (long) 1.5 != 1.5
        J.read_list(b'[{"traceId":"1","id":"2","timestamp":1.5}]')


# gson 2.8.5 nextLong / nextInt on PEEKED_NUMBER or a quoted text Long.parseLong refuses:
# Double.parseDouble, (long) of it, NumberFormatException unless (double) result == the double.
# Expected values follow from the IEEE-754 double nearest each text (Java's parseDouble rounds
# correctly) and Java's saturating (long) / (int) casts. None = IllegalArgumentException.
_P5 = str(5 ** 1075)  # 2^-1075 = 5^1075 / 10^1075, 752 significant digits
_TWO_M1075 = _P5[0] + "." + _P5[1:] + "e-324"
NUMBER_VECTORS = [
    ("1.472470996199E15", 1472470996199000), ("1.472470996199e+15", 1472470996199000),
    ("147247099619900E1", 1472470996199000), ("1.5", None), ("-1.5", None), ("1.0", 1), ("1e0", 1),
    ("0.5", None), ("0.0", 0), ("-0", 0), ("-0.0", 0), ("0e7", 0), ("1e19", None), ("1E-400", 0),
    ("9223372036854775807", 9223372036854775807),  # PEEKED_LONG
    ("9223372036854775808", 9223372036854775807),  # 2^63: (long) saturates, (double) Long.MAX == 2^63
    ("9223372036854776832", 9223372036854775807),  # the tie above 2^63 rounds to 2^63 (even)
    ("9223372036854776833", None), ("9223372036854777000", None),
    ("-9223372036854775809", -9223372036854775808), ("-9223372036854777856", None),
    ("0.99999999999999999", 1), ("0.999999999999999944488848768742172978818416595458984375", 1),
    ("0.999999999999999944488848768742172978818416595458984374", None),
    ("4503599627370497.4", 4503599627370497), ("4503599627370496.5", 4503599627370496),
    ("4503599627370497.5", 4503599627370498), ("9007199254740993", 9007199254740993),  # PEEKED_LONG
    ("9007199254740993.0", 9007199254740992), ("9007199254740995.0", 9007199254740996), ("2.5000000000000000000001", None),
    ("3.0000000000000004", None), ("3.0000000000000002", 3), ("3.00000000000000022204460492503130808472633361816406", 3),
    ("3.00000000000000022204460492503130808472633361816407", None),
    (_TWO_M1075, 0),  # 2^-1075 exactly: the tie rounds to 0 (even)
    (_TWO_M1075[:-5] + "1e-324", None),  # just above 2^-1075: the smallest subnormal
    ("2.4703282292062327e-324", 0), ("-1e-330", 0),
    ('"77"', 77), ('"+77"', 77), ('"-0"', 0), ('"1.472470996199E15"', 1472470996199000), ('" 12\t"', 12),
    ('"12d"', 12), ('"12.0F"', 12), ('"0x1p4"', 16), ('"0X1.8P1"', 3), ('"-0x.8p1"', -1), ('"0x8.p-3"', 1),
    ('"0x1p63"', 9223372036854775807), ('"-0x1p63"', -9223372036854775808), ('"0x1p64"', None),
    ('"0x1.00000000000008p52"', 4503599627370496), ('"0x1.00000000000018p52"', 4503599627370498),
    ('"0x1p-1075"', 0), ('"0x1.0000001p-1075"', None), ('"0x1p-1076"', 0), ('"0x0p99999999999"', 0),
    ('"\u0031\u0032"', 12), ('"\u0661\u0662"', 12), ('"\uff11"', 1), ('"\u0de7"', None),  # Java 8 digits only
    ('"NaN"', None), ('"Infinity"', None), ('"-Infinity"', None), ('"1e"', None), ('"1e+"', None),
    ('"1.2.3"', None), ('""', None), ('"+"', None), ('"."', None), ('".5"', None), ('"5."', 5), ('"1_0"', None),
    ('"0x1"', None), ('"0x"', None), ('"1d "', 1), ('"1dd"', None), ('"1 d"', None), ('"٣.0"', None),
    ("01", None), ("1.", None), ("-", None), (".5", None), ("1e", None),
]


def _read_ts(text):
    try:
        return J.read_list(('[{"traceId":"1","id":"2","timestamp":%s}]' % text).encode())[0].timestamp
    except J.IllegalArgument:
        return None


@pytest.mark.parametrize("text,exp", NUMBER_VECTORS)
def test_next_long_through_parse_double(text, exp):
    got = _read_ts(text)
    assert got == (None if exp is None else max(exp, 0))  # Span.Builder.timestamp drops negatives
    # nextInt (port): the same double, (int) cast
    try:
        (s,) = J.read_list(('[{"traceId":"1","id":"2","localEndpoint":{"port":%s}}]' % text).encode())
        port = s.local_endpoint.port if s.local_endpoint else 0
        assert exp is not None and -(1 << 31) <= exp <= 0xFFFF and port == max(exp, 0)
    except J.IllegalArgument:
        assert exp is None or not (-(1 << 31) <= exp <= 0xFFFF)


# ---------------- generators: gson-legal formatting variety ----------------

WS = [" ", "\n", "\t", "\r", "  "]


def _ws(r):
    return "".join(r.choice(WS) for _ in range(r.randrange(3))) if r.random() < 0.3 else ""


def _esc_some(r, s: str) -> str:
    """A JSON string literal for s, with some characters written as \\u escapes."""
    out = []
    for c in J.json_escape(s):
        out.append("\\u%04x" % ord(c) if c.isalnum() and r.random() < 0.1 else c)
    return '"' + "".join(out) + '"'


def _kw(r, v: str) -> str:
    return "".join(c.upper() if r.random() < 0.3 else c for c in v)


def _junk_value(r, depth=0):
    k = r.randrange(7)
    if k == 0 and depth < 3:
        return "[" + ",".join(_junk_value(r, depth + 1) for _ in range(r.randrange(3))) + "]"
    if k == 1 and depth < 3:
        return "{" + ",".join(_esc_some(r, "k%d" % i) + ":" + _junk_value(r, depth + 1) for i in range(r.randrange(3))) + "}"
    return r.choice(['"x\\"y"', "12", "-3.5e2", _kw(r, "true"), _kw(r, "null"), "0", '"\\u00e9"', "-0"])


def _endpoint(r, e: Endpoint) -> str:
    m = []
    if e.service_name is not None:
        svc = "".join(c.upper() if r.random() < 0.3 else c for c in e.service_name)
        m.append(('"serviceName"', _esc_some(r, svc)))
    if e.ipv4 is not None:
        v4 = e.ipv4 if r.random() < 0.9 else "::ffff:" + e.ipv4
        m.append(('"ipv4"' if r.random() < 0.8 else '"ipv6"', _esc_some(r, v4) if r.random() < 0.2 else '"%s"' % v4))
    if e.ipv6 is not None:
        v6 = e.ipv6.upper() if r.random() < 0.3 else e.ipv6
        m.append(('"ipv6"', _esc_some(r, v6) if r.random() < 0.2 else '"%s"' % v6))
    if e.port:
        m.append(('"port"', _num_text(r, e.port)))
    if r.random() < 0.2:
        m.append(('"serviceName"' if not e.service_name else '"extra"', _kw(r, "null")))
    if r.random() < 0.2:
        m.append(('"whatever"', _junk_value(r)))
    r.shuffle(m)
    return "{" + ",".join(_ws(r) + k + _ws(r) + ":" + _ws(r) + v + _ws(r) for k, v in m) + "}"


def _num_text(r, v: int) -> str:
    """An integer as some text gson's nextLong / nextInt reads as v."""
    k = r.randrange(10)
    if k < 6:
        return str(v)
    if k == 6:
        return '"%d"' % v
    d = str(v)
    if k == 7:  # exact scientific notation
        return ("%s.%sE%d" % (d[0], d[1:], len(d) - 1)) if len(d) > 1 else d + ".0e0"
    if k == 8:
        return d + "." + "0" * r.randrange(1, 4)
    return '"%s"' % (d + r.choice(["d", "D", ".0f", " "]))


def noisy_span(r, s: Span) -> str:
    m = [('"traceId"', '"%s"' % (s.trace_id if r.random() < 0.8 else s.trace_id.lstrip("0") or "0")),
         ('"id"', '"%s"' % s.id)]
    if s.parent_id:
        m.append(('"parentId"', '"%s"' % s.parent_id))
    elif r.random() < 0.2:
        m.append(('"parentId"', _kw(r, "null")))
    if s.kind is not None:
        m.append(('"kind"', _esc_some(r, Kind(s.kind).name)))
    if s.name:
        m.append(('"name"', _esc_some(r, s.name)))
    if s.timestamp:
        m.append(('"timestamp"', _num_text(r, s.timestamp)))
    if s.duration:
        m.append(('"duration"', _num_text(r, s.duration)))
    if s.local_endpoint:
        m.append(('"localEndpoint"', _endpoint(r, s.local_endpoint)))
    if s.remote_endpoint:
        m.append(('"remoteEndpoint"', _endpoint(r, s.remote_endpoint)))
    if s.annotations:
        m.append(('"annotations"', "[" + ",".join('{"value":%s,"timestamp":%s}' % (_esc_some(r, v), _num_text(r, t))
                                                  for t, v in s.annotations) + "]"))
    if s.tags:
        m.append(('"tags"', "{" + ",".join(_esc_some(r, k) + ":" + _esc_some(r, v) for k, v in s.tags) + "}"))
    if s.shared:
        m.append(('"shared"', _kw(r, "true")))
    elif r.random() < 0.1:
        m.append(('"shared"', _kw(r, "false")))
    if s.debug:
        m.append(('"debug"', _kw(r, "true")))
    if r.random() < 0.3:
        m.append(('"unknown%d"' % r.randrange(9), _junk_value(r)))
    if r.random() < 0.2:
        m.append(('"tr\\u0061ceId"', '"%s"' % s.trace_id))  # an escaped name, the same value again
    r.shuffle(m)
    return "{" + ",".join(_ws(r) + k + _ws(r) + ":" + _ws(r) + v + _ws(r) for k, v in m) + "}"


def noisy_list(r, sp) -> bytes:
    return (_ws(r) + "[" + ",".join(_ws(r) + noisy_span(r, s) + _ws(r) for s in sp) + "]" + _ws(r)).encode()


def oracle_columns(data, svc, ip4, ip6):
    return pack_traces([[s] for s in J.read_list(data)], svc, ip4, ip6)


def mutate(r, data: bytes) -> bytes:
    b = bytearray(data)
    for _ in range(r.randrange(1, 3)):
        k = r.randrange(5)
        i = r.randrange(len(b)) if b else 0
        if k == 0 and b:
            b[i] = ord(r.choice('{}[]:,"\\ 0a-.eE'))
        elif k == 1 and b:
            del b[i:]
        elif k == 2:
            b.insert(i, ord(r.choice('{}[]:,"\\ ')))
        elif k == 3 and b:
            del b[i]
        elif b:
            b[i] = r.randrange(256)
    return bytes(b)


def test_noisy_lists_decode_like_the_spans():
    r = random.Random(11)
    for _ in range(30):
        sp = rand_batch(r, r.randrange(1, 20))
        # (against the plain encoding: Endpoint.create's ipv6 text is Python's, writeIpV6 differs
        # for a zero run after an earlier one, e.g. 2001:db8::1:0:0:0)
        assert J.read_list(noisy_list(r, sp)) == J.read_list(J.write_list(sp))


def test_oracle_fuzz_never_crashes():
    r = random.Random(7)
    for _ in range(300):
        d = mutate(r, noisy_list(r, rand_batch(r, 3)))
        try:
            J.read_list(d)
        except (J.IllegalArgument, J.Unsupported):
            pass


# ---------------- device decoder vs oracle (GPU) ----------------

def _dec(d):
    from zipkin_amd.jsonv2 import JsonV2Decoder
    return JsonV2Decoder(*d)


@pytest.mark.gpu
def test_gpu_decode_reference_vectors():
    from zipkin_amd import _native as N
    d, o = fresh(), fresh()
    dec = _dec(d)
    for span, text in ENCODER_VECTORS:
        data = ("[" + text + "]").encode()
        assert_same(dec.decode_columns(data), oracle_columns(data, *o))
    for obj, check in DECODER_VECTORS:
        data = ("[" + obj + "]").encode()
        if check is None:
            with pytest.raises(N.ReferenceIllegalArgumentException):
                dec.decode(data)
        else:
            assert_same(dec.decode_columns(data), oracle_columns(data, *o))
    assert [x.strings for x in d] == [x.strings for x in o]
    dec.close()


@pytest.mark.gpu
def test_gpu_decode_golden_spans():
    d, o = fresh(), fresh()
    dec = _dec(d)
    data = J.write_list(GOLDEN_SPANS)
    assert_same(dec.decode_columns(data), oracle_columns(data, *o))
    assert [x.strings for x in d] == [x.strings for x in o]
    dec.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_decode_random_batches(seed):
    """Several noisy batches through one decoder: ids stay first-seen across batches."""
    r = random.Random(seed)
    d, o = fresh(), fresh()
    dec = _dec(d)
    for _ in range(3):
        sp = rand_batch(r, r.randrange(1, 400))
        data = noisy_list(r, sp) if seed % 2 else J.write_list(sp)
        assert_same(dec.decode_columns(data), oracle_columns(data, *o))
        assert [x.strings for x in d] == [x.strings for x in o]
    dec.close()


@pytest.mark.gpu
def test_gpu_decode_errors_match_oracle():
    """Mutated batches: the device raises where the reference throws, rejects what it does not
    restate (ZDL_EINVAL), and otherwise decodes identically."""
    from zipkin_amd import _native as N
    r = random.Random(99)
    seen = {"ok": 0, "iae": 0, "unsupported": 0}
    for _ in range(500):
        d, o = fresh(), fresh()
        dec = _dec(d)
        data = mutate(r, noisy_list(r, rand_batch(r, r.randrange(1, 6))))
        try:
            exp = oracle_columns(data, *o)
            kind = "ok"
        except J.IllegalArgument:
            kind = "iae"
        except J.Unsupported:
            kind = "unsupported"
        seen[kind] += 1
        if kind == "iae":
            with pytest.raises(N.ReferenceIllegalArgumentException):
                dec.decode_columns(data)
        elif kind == "unsupported":
            with pytest.raises(N.ZdlError) as ei:
                dec.decode_columns(data)
            assert ei.value.code == N.ZDL_EINVAL
        else:
            assert_same(dec.decode_columns(data), exp)
            assert [x.strings for x in d] == [x.strings for x in o]
        dec.close()
    assert seen["ok"] > 0 and seen["iae"] > 0, seen  # "unsupported": nesting > 64 only, rare here


@pytest.mark.gpu
def test_gpu_numbers_through_parse_double():
    """NUMBER_VECTORS and random texts near the rounding boundaries as timestamp, duration,
    annotation timestamp and port: the device accepts, rejects and reads them like the oracle."""
    from zipkin_amd import _native as N
    r = random.Random(3)
    texts = [t for t, _ in NUMBER_VECTORS]
    for _ in range(400):
        texts.append(_edge_number(r))
    dec = _dec(fresh())
    o = fresh()
    fields = ['"timestamp":%s', '"duration":%s', '"annotations":[{"value":"a","timestamp":%s}]',
              '"localEndpoint":{"serviceName":"s","port":%s}']
    n_ok = 0
    for text in texts:
        for f in fields:
            data = ('[{"traceId":"1","id":"2",' + f % text + '}]').encode()
            try:
                exp = oracle_columns(data, *o)
            except J.IllegalArgument:
                with pytest.raises(N.ReferenceIllegalArgumentException):
                    dec.decode_columns(data)
                    pytest.fail(f"device accepts {data!r}")
                continue
            try:
                got = dec.decode_columns(data)
            except N.ZdlError as ex:
                pytest.fail(f"device rejects {data!r}: {ex}")
            assert_same(got, exp)
            n_ok += 1
    assert n_ok > 300
    dec.close()


def _edge_number(r) -> str:
    """A number text near a rounding boundary of the doubles nextLong / nextInt meet."""
    base = r.choice([r.randrange(1 << 40), (1 << 52) + r.randrange(-3, 4), (1 << 53) + r.randrange(-3, 4),
                     (1 << 63) + r.randrange(-3000, 3000), (1 << 31) + r.randrange(-3, 3), r.randrange(100)])
    sign = "-" if r.random() < 0.2 else ""
    k = r.randrange(7)
    if k == 0:
        t = "%d.%s" % (base, r.choice(["5", "49999999999999999999", "50000000000000000001", "0", "25", "75"]))
    elif k == 1:
        d = str(base)
        t = "%s.%se%d" % (d[0], d[1:] or "0", len(d) - 1 + r.randrange(-2, 3))
    elif k == 2:
        t = "%de%d" % (base, r.randrange(-5, 5))
    elif k == 3:
        t = "0.%s" % ("9" * r.randrange(10, 25) + r.choice(["", "4", "5", "44488848768742172978818416595458984375"]))
    elif k == 4:
        t = "%s1e-%d" % (sign, r.randrange(300, 400))
        sign = ""
    elif k == 5:
        t = "0x%xp%d" % (base, r.randrange(-8, 12))
        return '"' + sign + t + r.choice(["", "d", "F"]) + '"'
    else:
        t = str(base)
    t = sign + t
    return t if r.random() < 0.7 else '"%s%s%s"' % (r.choice(["", " ", "\\t"]), t, r.choice(["", "d", " "]))


@pytest.mark.gpu
def test_gpu_decode_edge_inputs():
    from zipkin_amd import _native as N
    dec = _dec(fresh())
    one = b'{"traceId":"1","id":"2"}'
    for data in (b"", b"[]", b" \n[ \t]", b"[]junk", b"  [  ]  ]"):
        assert dec.decode(data).n_spans == 0, data
    for data in (b"hello", b"[", b"[ ", b"{}", b"[1]", b"[[]]", b"[" + one, b"[" + one + b",]", b"[" + one + one + b"]",
                 b"[" + one + b"," + one, b"[null]", b"[" + one + b"}", b"[" + one + b", 1]", b"[1, " + one + b"]",
                 b"/*x*/[" + one + b"]", b"[" + one.replace(b"}", b',"a":{"b":[}]}') + b"]"):
        with pytest.raises(N.ReferenceIllegalArgumentException):
            dec.decode(data)
    assert dec.decode(b"[" + b",".join([one] * 3) + b"] trailing {[").n_spans == 3
    # more than 4 objects in one 64-byte lane (only "{}"-dense input): the exact starts path
    with pytest.raises(N.ReferenceIllegalArgumentException):
        dec.decode(b"[" + b",".join([b"{}"] * 200) + b"]")
    tight = b'{"traceId":1,"id":2}'  # the shortest span objects: 4 starts in some lanes
    assert dec.decode(b"[" + b",".join([tight] * 500) + b"]").n_spans == 500
    deep = b"[" + one[:-1] + b',"x":' + b"[" * 70 + b"]" * 70 + b"}]"
    with pytest.raises(N.ZdlError) as ei:
        dec.decode(deep)
    assert ei.value.code == N.ZDL_EINVAL
    ok = b"[" + one[:-1] + b',"x":' + b"[" * 60 + b"]" * 60 + b"}]"
    assert dec.decode(ok).n_spans == 1
    dec.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ST["cases"], ids=lambda c: c["name"])
def test_gpu_storage_accept_json_v2(case):
    """ITDependencies through accept_json_v2(encode(batch)) == the transcribed expectations."""
    from golden_io import check_links
    from zipkin_amd.storage import InMemoryStorage
    store = InMemoryStorage(strict_trace_id=True)
    for b in case["batches"]:
        store.accept_json_v2(J.write_list(spans(b))).execute()
    for q in case["queries"]:
        check_links(store.get_dependencies(q["endTs"], q["lookback"]).execute(), q["expect"], "only")
    store.close()


@pytest.mark.gpu
def test_gpu_decode_then_link_large():
    """20k traces of noisy JSON: decode on the device, link the device columns (grouped on the
    device), same links as packing the oracle-decoded spans; objects beyond the LDS window too."""
    from zipkin_amd import _native as N
    r = random.Random(5)
    sp = []
    for t in range(20000):
        tid = "%016x" % r.randrange(1, 1 << 64)
        root = r.randrange(1, 1 << 64)
        sp.append(Span.create(tid, root, None, Kind.SERVER, local_endpoint=Endpoint.create(r.choice(SVC))))
        for _ in range(4):
            sp.append(Span.create(tid, r.randrange(1, 1 << 64), root, r.choice([Kind.CLIENT, None]),
                                  local_endpoint=Endpoint.create(r.choice(SVC) + ("x" * 3000 if r.random() < 0.01 else "")),
                                  remote_endpoint=Endpoint.create(r.choice(SVC)),
                                  tags={"error": ""} if r.random() < 0.05 else None))
    r.shuffle(sp)
    data = noisy_list(r, sp)
    d, o = fresh(), fresh()
    dec = _dec(d)
    b = dec.decode(data)
    ctx = N.Context(len(d[0]))
    ctx.put_spans_device({k: getattr(b.dev, k) for k in COLS}, b.n_spans, None, 0)
    got = sorted(zip(*(a.tolist() for a in ctx.link())))
    exp_cols = oracle_columns(data, *o)
    ctx2 = N.Context(len(o[0]))
    ctx2.put_spans_ungrouped(exp_cols)
    exp = sorted(zip(*(a.tolist() for a in ctx2.link())))
    assert got == exp and len(got) > 0
    assert dec.kernel_ms() > 0 and dec.struct_ms() > 0
    dec.close()


# ---------------- the fast path against the exact reader (GPU) ----------------

def _dec_exact(d):
    """A decoder that reads every span with the exact reader (ZDL_JS_EXACT=1 at creation)."""
    import os
    os.environ["ZDL_JS_EXACT"] = "1"
    try:
        return _dec(d)
    finally:
        del os.environ["ZDL_JS_EXACT"]


def _compact_edge_span(r) -> str:
    """A compact span object (the fast path's shape) with edge values: valid ones the fast path
    reads itself or must hand over (17+ digit numbers, escapes, null, annotations, upper-case
    keywords), and, rarely, invalid ones (all-zero ids, bad kinds, ports above 65535...)."""
    bad = r.random() < 0.03

    def pick(good, worse):
        return r.choice(worse) if bad and r.random() < 0.3 else r.choice(good)
    tid = pick(["%016x" % r.randrange(1, 1 << 64), "%032x" % r.randrange(1, 1 << 128), "%x" % r.randrange(1, 1 << 70),
                "00000000000000000000000000000001", "%020x" % r.randrange(1, 1 << 64), "%x" % r.randrange(1, 99)],
               ["0" * 16, "0" * 32, "", "ABCDEF0123456789", "%033x" % 5])
    m = [('"traceId"', '"%s"' % tid),
         ('"id"', '"%s"' % pick(["%016x" % r.randrange(1, 1 << 64), "1", "%x" % r.randrange(1, 1 << 40), "0"],
                                ["0" * 16, "%017x" % 3, ""]))]
    if r.random() < 0.7:
        m.append(('"parentId"', pick(['"%016x"' % r.randrange(1 << 64), '"0000000000000000"', '"a"', "null"], ['""'])))
    if r.random() < 0.7:
        m.append(('"kind"', pick(['"CLIENT"', '"SERVER"', '"PRODUCER"', '"CONSUMER"', '"\u0043LIENT"'],
                                 ['"client"', '"CLIENTX"', '""', '"CONSUME"'])))
    if r.random() < 0.5:
        m.append(('"name"', pick(['"get"', '""', '"a\\"b"', '"x y"', "12"], ["true"])))
    for k in ('"timestamp"', '"duration"'):
        if r.random() < 0.8:
            m.append((k, pick([str(r.randrange(1, 1 << 53)), "0", "1704067200000010", "12345678901234567", "-5", "1e3",
                               str(r.randrange(10 ** 15, 10 ** 16)), '"77"', "9223372036854775807"],
                              ["0123", "1.5", "99999999999999999999", '"x"'])))

    def ep():
        f = []
        if r.random() < 0.8:
            f.append('"serviceName":%s' % pick(['"svc-%d"' % r.randrange(9), '""', '"Svc"', '"s\\u0041"', "null"], ["[]"]))
        if r.random() < 0.6:
            f.append('"ipv4":%s' % r.choice(['"10.0.0.%d"' % r.randrange(256), '"1.2.3"', '""', '"::ffff:1.2.3.4"',
                                             '"01.2.3.4"', '"256.1.1.1"', '"::1.2.3.4"']))
        if r.random() < 0.3:
            f.append('"ipv6":%s' % r.choice(['"2001:db8::1"', '"::1"', '"fe80::1:2:3:4:5:6:7"', '"1.2.3.4"', '"zz"',
                                             '"1:2:3:4:5:6:7:8"', '"::"']))
        if r.random() < 0.5:
            f.append('"port":%s' % pick(["0", "80", "65535", "-1", "8080", "00"[:1]], ["65536", "1.5"]))
        r.shuffle(f)
        return "{" + ",".join(f) + "}"
    if r.random() < 0.9:
        m.append(('"localEndpoint"', ep()))
    if r.random() < 0.6:
        m.append(('"remoteEndpoint"', ep()))
    if r.random() < 0.3:
        m.append(('"tags"', pick(['{"error":""}', '{}', '{"http.path":"/x","error":"boom"}', '{"a":1}', '{"err":"x"}',
                                  '{"\\u0065rror":"x"}'], ['{"error":null}'])))
    if r.random() < 0.1:
        m.append(('"annotations"', '[{"timestamp":1,"value":"ws"}]'))
    for k in ('"shared"', '"debug"'):
        if r.random() < 0.2:
            m.append((k, pick(["true", "false", "TRUE", "null"], ["1"])))
    if r.random() < 0.05:
        m.append(('"unknown"', '"x"'))
    r.shuffle(m)
    return "{" + ",".join(k + ":" + v for k, v in m) + "}"


def _mixed_list(r, n) -> bytes:
    sp = rand_batch(r, n)
    objs = []
    for s in sp:
        x = r.random()
        if x < 0.5:
            objs.append(J.write_list([s])[1:-1].decode())
        elif x < 0.8:
            objs.append(_compact_edge_span(r))
        else:
            objs.append(noisy_span(r, s))
    return ("[" + ",".join(objs) + "]").encode()


def _d2h(ptr, n, dtype):
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    out = np.empty(n, dtype)
    if n:
        assert hip.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(ptr), C.c_size_t(out.nbytes), 2) == 0
    return out


def _decode_outcome(dec, data):
    """("ok", every column incl. the trace ids' high halves and widths) or (error kind, message)."""
    from zipkin_amd import _native as N
    try:
        b = dec.decode(data)
    except N.ReferenceIllegalArgumentException as e:
        return "iae", str(e)
    except N.ZdlError as e:
        return "err%d" % e.code, str(e)
    n = int(b.n_spans)
    cols = dec._dec.download(n) if n else {}
    if n:
        cols["trace_hi"] = _d2h(b.dev_trace_hi, n, np.uint64)
        cols["trace_wide"] = _d2h(b.dev_trace_wide, n, np.uint8)
    return "ok", cols


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_fast_path_matches_exact_reader(seed):
    """Compact spans (the fast path), edge values and noisy spans mixed in one list: the default
    decoder (fast path + exact hand-over) and an all-exact decoder give the same columns, the same
    dictionaries and the same first error."""
    r = random.Random(1000 + seed)
    fast_seen = 0
    for k in range(40):
        data = _mixed_list(r, r.randrange(1, 300))
        if k % 4 == 3:
            data = mutate(r, data)
        da, db = fresh(), fresh()
        fa, ex = _dec(da), _dec_exact(db)
        a, b = _decode_outcome(fa, data), _decode_outcome(ex, data)
        assert a[0] == b[0], (a[0], b[0], a[1] if a[0] != "ok" else "", b[1] if b[0] != "ok" else "")
        if a[0] == "ok":
            assert sorted(a[1]) == sorted(b[1])
            for c in a[1]:
                np.testing.assert_array_equal(a[1][c], b[1][c], err_msg=c)
            assert [x.strings for x in da] == [x.strings for x in db]
            fast_seen += len(a[1].get("id", ())) - fa.exact_spans()
        else:
            assert a[1] == b[1]
        fa.close()
        ex.close()
    assert fast_seen > 0


@pytest.mark.gpu
def test_gpu_fast_path_takes_compact_lists():
    """The writer's compact encoding without annotations stays on the fast path entirely; with
    annotations those spans (only) go to the exact reader."""
    from zipkin_amd import synth
    w = synth.C2.scaled(300)
    cols = synth.generate(w)
    data = synth.encode_json_v2(cols, synth.service_names(w)).tobytes()
    d, o = fresh(), fresh()
    dec = _dec(d)
    b = dec.decode(data)
    assert b.n_spans == cols.n_spans and dec.exact_spans() == 0
    dec.close()
    dec = _dec(d := fresh())
    r = random.Random(3)
    sp = [s for s in rand_batch(r, 400)]
    data = J.write_list(sp)
    assert_same(dec.decode_columns(data), oracle_columns(data, *o))
    n_ann = sum(1 for s in sp if s.annotations)
    n_esc = sum(1 for s in sp if b"\\" in J.write_list([s]))
    assert dec.exact_spans() <= n_ann + n_esc + 1, (dec.exact_spans(), n_ann, n_esc)
    dec.close()
