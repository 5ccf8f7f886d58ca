"""DependencyLinkBytesEncoder / Decoder JSON_V1 (the bytes `/api/v2/dependencies` returns).

Expected bytes follow the writer in zipkin2/codec/DependencyLinkBytesEncoder.java:57-65 and
JsonCodec.writeList (JsonCodec.java:225-232); sizes follow its sizeInBytes (:45-55).
"""
from zipkin_amd.codec import decode_links, encode_link, encode_links, json_escape
from zipkin_amd.model import DependencyLink


def _size_in_bytes(l):
    # DependencyLinkBytesEncoder.WRITER.sizeInBytes (:45-55)
    n = 37 + len(json_escape(l.parent).encode()) + len(json_escape(l.child).encode())
    n += len(str(l.call_count))
    if l.error_count > 0:
        n += 14 + len(str(l.error_count))
    return n


def test_encode_without_errors():
    l = DependencyLink.create("web", "app", 2, 0)
    assert encode_link(l) == b'{"parent":"web","child":"app","callCount":2}'


def test_encode_with_errors():
    l = DependencyLink.create("web", "app", 10, 3)
    assert encode_link(l) == b'{"parent":"web","child":"app","callCount":10,"errorCount":3}'


def test_encode_list_and_empty():
    a = DependencyLink.create("a", "b", 1, 0)
    b = DependencyLink.create("b", "c", 4, 1)
    assert encode_links([]) == b"[]"
    assert encode_links([a]) == b'[{"parent":"a","child":"b","callCount":1}]'
    assert encode_links([a, b]) == (b'[{"parent":"a","child":"b","callCount":1},'
                                    b'{"parent":"b","child":"c","callCount":4,"errorCount":1}]')


def test_escapes_match_json_escaper():
    # JsonEscaper.REPLACEMENT_CHARS: quote, backslash, short control forms, \u00xx, U+2028/9.
    assert json_escape('a"b\\c') == 'a\\"b\\\\c'
    assert json_escape("\t\b\n\r\f") == "\\t\\b\\n\\r\\f"
    assert json_escape("\x01\x1f") == "\\u0001\\u001f"
    assert json_escape("x\u2028y\u2029") == "x\\u2028y\\u2029"
    assert json_escape("café") == "café"
    l = DependencyLink.create('fr"ont', "café", 1, 0)
    assert encode_link(l) == '{"parent":"fr\\"ont","child":"café","callCount":1}'.encode()


def test_size_and_round_trip():
    links = [DependencyLink.create("web", "app", 2, 0),
             DependencyLink.create("app", "db\n", 123456789012, 7),
             DependencyLink.create("svc ", "kafka", 1, 1)]
    for l in links:
        assert len(encode_link(l)) == _size_in_bytes(l)
    assert decode_links(encode_links(links)) == links


def test_decode_skips_unknown_fields():
    got = decode_links(b'[{"parent":"a","foo":{"x":[1]},"child":"b","callCount":3}]')
    assert got == [DependencyLink.create("a", "b", 3, 0)]
