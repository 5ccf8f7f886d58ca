"""ORACLE — TEST INFRASTRUCTURE ONLY, NEVER A PRODUCT PATH.

Literal CPU restatement of ``SpanBytesDecoder.PROTO3.decodeList(bytes)`` (the proto3
``ListOfSpans`` reader) and of the matching writer, used by ``tests/`` as the checker for the
device decoder ``zdl_decode_proto3``. Nothing under ``zipkin_amd/`` imports it.

Paths are relative to /root/reference/zipkin/src/main/java/zipkin2/:

* ``read_list``        <- internal/Proto3Codec.java readList + codec/SpanBytesDecoder.java:144-152
* ``_read_span``       <- internal/Proto3ZipkinFields.java:309-369 (SpanField.readValue)
* ``_read_endpoint``   <- internal/Proto3ZipkinFields.java:76-101 + Endpoint.java:179-198,269-285
* ``_read_annotation`` <- internal/Proto3ZipkinFields.java:138-162
* ``_read_tag``        <- internal/Proto3ZipkinFields.java:186-210
* ``_Buf``             <- internal/Buffer.java:279-379 (readVarint32's 5th byte does not advance
                          ``pos``, restated as is) and internal/Proto3Fields.java (skipValue,
                          ensureLength, BooleanField.read)
* ``write_ipv6``       <- Endpoint.java:350-407
* ``write_list``       <- internal/Proto3ZipkinFields.java:246-302 + Proto3Fields.java writers

Errors: every exception the reference raises while reading becomes ``IllegalArgument`` (the
reference wraps them all, Proto3Codec.exceptionReading). ``overrun`` is returned True when a
field read ends beyond the end of the message that encloses it (or a length is negative) —
the reference reads on leniently from there; the restatement stops at that point, where the
device decoder rejects the batch (ZDL_EINVAL), and the tests check that through this flag.

Pinned by the reference's own vectors: Proto3ZipkinFieldsTest (write bytes, kind tolerance,
round trips), SpanBytesDecoderTest PROTO3 cases (round trips of TestObjects, empty input,
"Truncated: length 101 > bytes remaining 3" on b"hello"); see tests/test_proto3.py.
"""
from __future__ import annotations

import struct
from typing import List, Optional, Tuple

from zipkin_amd.model import Endpoint, Kind, Span

WIRETYPE_VARINT, WIRETYPE_FIXED64, WIRETYPE_LENGTH_DELIMITED, WIRETYPE_FIXED32 = 0, 1, 2, 5


class IllegalArgument(Exception):
    pass


class _Unsupported(Exception):
    """A read ended beyond its enclosing message: the device decoder rejects the batch here."""


class _Buf:
    def __init__(self, b: bytes):
        self.buf, self.pos, self.overrun = b, 0, False

    def remaining(self) -> int:
        return len(self.buf) - self.pos

    def _check(self, pos):
        if pos > len(self.buf) - 1:
            raise IllegalArgument(f"Truncated reading position {pos}")

    def read_byte(self) -> int:  # signed, like Java's byte
        self._check(self.pos)
        b = self.buf[self.pos]
        self.pos += 1
        return b - 256 if b > 127 else b

    def read_varint32(self) -> int:
        """Buffer.readVarint32 (Buffer.java:300-334): 5th byte read without advancing pos."""
        result = 0
        for i in range(4):
            self._check(self.pos)
            b = self.buf[self.pos]
            self.pos += 1
            if b < 0x80:
                v = result | b << (7 * i)
                return v - (1 << 32) if v >= 1 << 31 else v
            result |= (b & 0x7F) << (7 * i)
        self._check(self.pos)
        b = self.buf[self.pos]
        if b & 0xF0:
            raise IllegalArgument(f"Greater than 32-bit varint at position {self.pos}")
        v = (result | b << 28) & 0xFFFFFFFF
        return v - (1 << 32) if v >= 1 << 31 else v

    def read_varint64(self) -> int:
        """Buffer.readVarint64 (Buffer.java:346-365)."""
        self._check(self.pos)
        b = self.buf[self.pos]
        self.pos += 1
        if b < 0x80:
            return b
        result = b & 0x7F
        i = 1
        while b >= 0x80 and i < 10:
            self._check(self.pos)
            b = self.buf[self.pos]
            self.pos += 1
            if i == 9 and (b & 0xF0) != 0:
                raise IllegalArgument(f"Greater than 64-bit varint at position {self.pos - 1}")
            result |= (b & 0x7F) << (i * 7)
            i += 1
        return result & 0xFFFFFFFFFFFFFFFF

    def read_long_le(self) -> int:
        if 8 > self.remaining():  # Fixed64Field.readValue's ensureLength
            raise IllegalArgument(f"Truncated: length 8 > bytes remaining {self.remaining()}")
        v = struct.unpack_from("<q", self.buf, self.pos)[0]
        self.pos += 8
        return v

    def skip(self, n: int) -> bool:
        nxt = self.pos + n
        if nxt > len(self.buf):
            self.pos = len(self.buf)
            return False
        self.pos = nxt
        return True

    def length_prefix(self) -> int:
        """LengthDelimitedField.readLengthPrefix (Proto3Fields.java) with ensureLength."""
        n = self.read_varint32()
        if n > self.remaining():
            raise IllegalArgument(f"Truncated: length {n} > bytes remaining {self.remaining()}")
        return n

    def read_bytes(self, n: int) -> bytes:
        if n < 0:
            raise IllegalArgument("negative length")  # new byte[negative] in the reference
        v = bytes(self.buf[self.pos:self.pos + n])
        self.pos += n
        return v

    def end(self, end_pos: int):
        if self.pos > end_pos:
            raise _Unsupported()


def _skip_value(b: _Buf, key: int):
    """Proto3ZipkinFields.logAndSkip + Proto3Fields.skipValue."""
    wt = key & 7
    if wt not in (0, 1, 2, 5):
        raise IllegalArgument(f"Malformed: invalid wireType {wt} at byte {b.pos}")
    if wt == WIRETYPE_VARINT:
        for _ in range(b.remaining()):
            if b.read_byte() >= 0:
                return
    elif wt == WIRETYPE_FIXED64:
        b.skip(8)
    elif wt == WIRETYPE_LENGTH_DELIMITED:
        n = b.read_varint32()
        if n < 0:
            raise _Unsupported()  # the reference would move pos backwards
        b.skip(n)
    else:
        b.skip(4)


def _hex(bs: bytes) -> str:
    return bs.hex()


def write_ipv6(ip: bytes) -> str:
    """Endpoint.writeIpV6 (Endpoint.java:350-407), literally (incl. its trailing-run rule)."""
    zci, zcl, zi, all_zeros = -1, -1, -1, True
    for i in range(0, 16, 2):
        if ip[i] == 0 and ip[i + 1] == 0:
            if zi < 0:
                zi = i
            continue
        all_zeros = False
        if zi >= 0:
            zl = i - zi
            if zl > zcl:
                zci, zcl = zi, zl
            zi = -1
    if all_zeros:
        return "::"
    if zci == -1 and zi != -1:
        zci, zcl = zi, 16 - zi
    out, i, H = [], 0, "0123456789abcdef"
    while i < 16:
        if i == zci:
            out.append(":")
            i += zcl
            if i == 16:
                out.append(":")
            continue
        if i != 0:
            out.append(":")
        hi, lo = ip[i], ip[i + 1]
        i += 2
        v = H[hi >> 4]
        lz = v == "0"
        if not lz:
            out.append(v)
        v = H[hi & 0xF]
        lz = lz and v == "0"
        if not lz:
            out.append(v)
        v = H[lo >> 4]
        if not (lz and v == "0"):
            out.append(v)
        out.append(H[lo & 0xF])
    return "".join(out)


def parse_ip_bytes(ip: Optional[bytes]) -> Tuple[Optional[str], Optional[str], bool]:
    """Endpoint.Builder.parseIp(byte[]) (Endpoint.java:179-198, 269-285) -> (ipv4, ipv6, set).

    ``flag != -1`` never holds for a value in [0, 0xffff], so only IPv4-compatible (::a.b.c.d,
    not ::1) addresses become ipv4; IPv4-mapped ones stay ipv6 (restated as is)."""
    if ip is None:
        return None, None, False
    if len(ip) == 4:
        return ".".join(str(x) for x in ip), None, True
    if len(ip) == 16:
        if all(x == 0 for x in ip[:10]) and (ip[10] << 8 | ip[11]) == 0 and ip[12:] != b"\0\0\0\1":
            return ".".join(str(x) for x in ip[12:]), "", True  # "" = ipv4 only (ipv6 untouched)
        return None, write_ipv6(ip), True
    return None, None, False


def _read_endpoint(b: _Buf, length: int) -> Endpoint:
    end = b.pos + length
    svc, ipv4, ipv6, port = None, None, None, 0
    while b.pos < end:
        key = b.read_varint32()
        if key == (1 << 3 | 2):
            n = b.length_prefix()
            s = None if n == 0 else b.read_bytes(n).decode("utf-8", "replace")
            svc = None if not s else s.lower()
        elif key in ((2 << 3 | 2), (3 << 3 | 2)):
            n = b.length_prefix()
            v4, v6, ok = parse_ip_bytes(None if n == 0 else b.read_bytes(n))
            if ok:
                if v6 == "":
                    ipv4 = v4
                elif v4 is not None:
                    ipv4 = v4
                else:
                    ipv6 = v6
        elif key == (4 << 3 | 0):
            p = b.read_varint32()
            if p > 0xFFFF:
                raise IllegalArgument(f"invalid port {p}")
            port = max(p, 0)
        else:
            _skip_value(b, key)
    b.end(end)
    return Endpoint(svc, ipv4, ipv6, port)


def _read_annotation(b: _Buf):
    n = b.length_prefix()
    if n == 0:
        return None
    end = b.pos + n
    ts, value = 0, None
    while b.pos < end:
        key = b.read_varint32()
        if key == (1 << 3 | 1):
            ts = b.read_long_le()
        elif key == (2 << 3 | 2):
            m = b.length_prefix()
            value = None if m == 0 else b.read_bytes(m).decode("utf-8", "replace")
        else:
            _skip_value(b, key)
    b.end(end)
    return None if ts == 0 or value is None else (ts, value)


def _read_tag(b: _Buf):
    n = b.length_prefix()
    if n == 0:
        return None
    end = b.pos + n
    k, v = None, ""
    while b.pos < end:
        key = b.read_varint32()
        if key == (1 << 3 | 2):
            m = b.length_prefix()
            k = None if m == 0 else b.read_bytes(m).decode("utf-8", "replace")
        elif key == (2 << 3 | 2):
            m = b.length_prefix()
            r = None if m == 0 else b.read_bytes(m).decode("utf-8", "replace")
            if r is not None:
                v = r
        else:
            _skip_value(b, key)
    b.end(end)
    return None if k is None else (k, v)


def _read_bool(b: _Buf) -> bool:
    v = b.read_byte()
    if v < 0 or v > 1:
        raise IllegalArgument(f"Malformed: invalid boolean value at byte {b.pos}")
    return v == 1


def _read_span(b: _Buf, length: int) -> Span:
    end = b.pos + length
    f = dict(trace_id=None, id=None, parent_id=None, kind=None, name=None, timestamp=0, duration=0,
             local_endpoint=None, remote_endpoint=None, shared=None, debug=None)
    anns, tags = [], {}
    try:
        while b.pos < end:
            key = b.read_varint32()
            if key in ((1 << 3 | 2), (2 << 3 | 2), (3 << 3 | 2)):
                n = b.length_prefix()
                h = None if n == 0 else _hex(b.read_bytes(n))
                if key == (1 << 3 | 2):
                    if h is None:
                        raise IllegalArgument("traceId == null")
                    Span.create(h, 1)  # Builder.traceId validates now (Span.java:402-405)
                    f["trace_id"] = h
                elif key == (3 << 3 | 2):
                    if h is None:
                        raise IllegalArgument("id == null")
                    Span.create("1", h)  # Builder.id validates now (Span.java:474-484)
                    f["id"] = h
                else:
                    if h is not None:
                        Span.create("1", 1, h)  # Builder.parentId validates now (Span.java:442-456)
                    f["parent_id"] = h
            elif key == (4 << 3 | 0):
                k = b.read_varint32()
                if k == 0 or k > 4:
                    continue
                if k < 0:
                    raise IllegalArgument("ArrayIndexOutOfBounds")  # Kind.values()[kind - 1]
                f["kind"] = Kind(k - 1)
            elif key == (5 << 3 | 2):
                n = b.length_prefix()
                f["name"] = None if n == 0 else b.read_bytes(n).decode("utf-8", "replace")
            elif key == (6 << 3 | 1):
                f["timestamp"] = max(b.read_long_le(), 0)
            elif key == (7 << 3 | 0):
                d = b.read_varint64()
                f["duration"] = d if d < 1 << 63 else 0
            elif key in ((8 << 3 | 2), (9 << 3 | 2)):
                n = b.length_prefix()
                e = None if n == 0 else _read_endpoint(b, n)
                f["local_endpoint" if key == (8 << 3 | 2) else "remote_endpoint"] = e
            elif key == (10 << 3 | 2):
                a = _read_annotation(b)
                if a is not None:
                    anns.append(a)
            elif key == (11 << 3 | 2):
                t = _read_tag(b)
                if t is not None:
                    tags[t[0]] = t[1]
            elif key == (12 << 3 | 0):
                if _read_bool(b):
                    f["debug"] = True
            elif key == (13 << 3 | 0):
                if _read_bool(b):
                    f["shared"] = True
            else:
                _skip_value(b, key)
        b.end(end)
        if f["trace_id"] is None or f["id"] is None:
            raise IllegalArgument("Missing :" + (" traceId" if f["trace_id"] is None else "")
                                  + (" id" if f["id"] is None else ""))
        return Span.create(f["trace_id"], f["id"], f["parent_id"], f["kind"], name=f["name"],
                           timestamp=f["timestamp"], duration=f["duration"],
                           local_endpoint=f["local_endpoint"], remote_endpoint=f["remote_endpoint"],
                           annotations=anns, tags=tags, shared=f["shared"], debug=f["debug"])
    except (ValueError, TypeError) as e:  # Span/Endpoint builder exceptions
        raise IllegalArgument(str(e)) from e


def read_list(data: bytes) -> Tuple[List[Span], bool]:
    """SpanBytesDecoder.PROTO3.decodeList(bytes) -> (spans, overrun).

    Raises IllegalArgument like the reference; an empty input or a zero-length span message
    yields the empty list (readList returns false -> Collections.emptyList())."""
    b = _Buf(bytes(data))
    out: List[Span] = []
    if len(data) == 0:
        return [], False
    try:
        while b.pos < len(data):
            b.read_varint32()  # the key is tossed (SpanField.read)
            n = b.length_prefix()
            if n == 0:
                return [], False
            out.append(_read_span(b, n))
    except _Unsupported:
        return [], True
    return out, False


# ---- writer (Proto3ZipkinFields.java:246-302), for fixtures ----

def _varint(v: int) -> bytes:
    v &= 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(key: int, payload: bytes) -> bytes:
    return b"" if not payload else bytes([key]) + _varint(len(payload)) + payload


def _ip_bytes(s: str) -> bytes:
    import ipaddress
    return ipaddress.ip_address(s).packed


def write_endpoint(e: Optional[Endpoint]) -> bytes:
    if e is None:
        return b""
    out = _ld(1 << 3 | 2, (e.service_name or "").encode())
    out += _ld(2 << 3 | 2, _ip_bytes(e.ipv4) if e.ipv4 else b"")
    out += _ld(3 << 3 | 2, _ip_bytes(e.ipv6) if e.ipv6 else b"")
    if e.port:
        out += bytes([4 << 3]) + _varint(e.port)
    return out


def write_span(s: Span) -> bytes:
    out = _ld(1 << 3 | 2, bytes.fromhex(s.trace_id))
    out += _ld(2 << 3 | 2, bytes.fromhex(s.parent_id) if s.parent_id else b"")
    out += _ld(3 << 3 | 2, bytes.fromhex(s.id))
    if s.kind is not None:
        out += bytes([4 << 3]) + _varint(int(s.kind) + 1)
    out += _ld(5 << 3 | 2, (s.name or "").encode())
    if s.timestamp:
        out += bytes([6 << 3 | 1]) + struct.pack("<q", s.timestamp)
    if s.duration:
        out += bytes([7 << 3]) + _varint(s.duration)
    out += _ld(8 << 3 | 2, write_endpoint(s.local_endpoint))
    out += _ld(9 << 3 | 2, write_endpoint(s.remote_endpoint))
    for ts, v in s.annotations:
        a = (bytes([1 << 3 | 1]) + struct.pack("<q", ts) if ts else b"") + _ld(2 << 3 | 2, v.encode())
        out += _ld(10 << 3 | 2, a)
    for k, v in s.tags:
        out += _ld(11 << 3 | 2, _ld(1 << 3 | 2, k.encode()) + _ld(2 << 3 | 2, v.encode()))
    if s.debug:
        out += bytes([12 << 3, 1])
    if s.shared:
        out += bytes([13 << 3, 1])
    return out


def write_list(spans) -> bytes:
    return b"".join(_ld(1 << 3 | 2, write_span(s)) for s in spans)
