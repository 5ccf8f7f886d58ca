"""JSON v2 ingest on the device: SpanBytesDecoder.JSON_V2.decodeList(bytes) straight to span columns.

Reference: codec/SpanBytesDecoder.java:94-120 -> internal/JsonCodec.java:142-155 ->
internal/V2SpanReader.java:25-135 over gson 2.8.5's strict JsonReader (paths under
/root/reference/zipkin/src/main/java/zipkin2/). The decoding runs in ``k_js_*``
(zipkin_amd/csrc/zdl_json.inc); this module only owns the dictionaries. When the device meets a
key its table lacks it lists it, and the key is normalised here the way the reference's builders
do — a service name's JSON text unescaped (gson readEscapeCharacter) and lower-cased
(Endpoint.Builder.serviceName, Endpoint.java:132-136); an ipv4 text kept as given, unescaped
(Endpoint.java:222-227); an ipv6 text unescaped, parsed to its 16 bytes (textToNumericFormatV6,
Endpoint.java:417-487) and written back by writeIpV6 (:350-407) — given the id of its string in
first-seen order (the ids ``columnar.pack_traces`` assigns to the decoded spans) and bound, and the
kernel re-runs on the resident batch. Malformed input raises like the reference
(IllegalArgumentException); the one input the decoder does not restate (objects or arrays nested deeper than 64
inside a span) raises ZdlError (ZDL_EINVAL).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import _native as N
from .columnar import Columns, Dictionary
from .model import format_ipv6
from .proto3 import DecodedBatch

_ESC = {ord("t"): "\t", ord("b"): "\b", ord("n"): "\n", ord("r"): "\r", ord("f"): "\f"}


def unescape(raw: bytes) -> str:
    """A JSON string token's content as gson's nextQuotedValue returns it: UTF-8 text between
    escapes (malformed bytes -> U+FFFD, like InputStreamReader), each escape one UTF-16 code unit
    (\\uXXXX) or character; surrogate pairs from escapes combine as they do in a Java String."""
    units = []
    i, n = 0, len(raw)
    while i < n:
        j = raw.find(b"\\", i)
        if j < 0:
            j = n
        if j > i:
            units.extend(_utf16_units(raw[i:j].decode("utf-8", "replace")))
        if j == n:
            break
        e = raw[j + 1]
        if e == ord("u"):
            units.append(int(raw[j + 2:j + 6], 16))
            i = j + 6
        else:
            units.append(ord(_ESC.get(e, chr(e))))
            i = j + 2
    return b"".join(u.to_bytes(2, "big") for u in units).decode("utf-16-be", "surrogatepass")


def _utf16_units(s: str):
    b = s.encode("utf-16-be", "surrogatepass")
    return [b[k] << 8 | b[k + 1] for k in range(0, len(b), 2)]


def ipv6_bytes(text: str) -> Optional[bytes]:
    """textToNumericFormatV6 (Guava InetAddresses 23, Endpoint.java:417-487) for a text of hex
    digits and ':' (detectFamily already chose IPv6)."""
    parts = text.split(":")
    if len(parts) > 10:  # String.split(":", 10)
        parts = parts[:9] + [":".join(parts[9:])]
    if not 3 <= len(parts) <= 9:
        return None
    skip = -1
    for i in range(1, len(parts) - 1):
        if parts[i] == "":
            if skip >= 0:
                return None
            skip = i
    if skip >= 0:
        hi, lo = skip, len(parts) - skip - 1
        if parts[0] == "":
            hi -= 1
            if hi != 0:
                return None
        if parts[-1] == "":
            lo -= 1
            if lo != 0:
                return None
    else:
        hi, lo = len(parts), 0
    skipped = 8 - (hi + lo)
    if not (skipped >= 1 if skip >= 0 else skipped == 0):
        return None
    words = []
    for p in parts[:hi] + [None] * skipped + (parts[len(parts) - lo:] if lo else []):
        if p is None:
            words.append(0)
            continue
        if p == "" or int(p, 16) > 0xFFFF:
            return None
        words.append(int(p, 16))
    return b"".join(w.to_bytes(2, "big") for w in words)


class JsonV2Decoder:
    """Decodes JSON v2 span lists on the device with ids from the given dictionaries."""

    def __init__(self, svc: Dictionary, ip4: Dictionary, ip6: Dictionary, device: int = 0):
        self.svc, self.ip4, self.ip6 = svc, ip4, ip6
        self._dec = N.Decoder(device)

    def _bind(self, dict_id: int, raw: bytes):
        if dict_id == N.ZDL_DICT_JSON_SERVICE:
            self._dec.bind(dict_id, raw, self.svc.id(unescape(raw).lower()))  # non-ASCII case mapping unpinned
        elif dict_id == N.ZDL_DICT_JSON_IPV4:
            t = unescape(raw)  # the device lists an escaped text whole: keep the IPv4 after any ':'
            self._dec.bind(dict_id, raw, self.ip4.id(t[t.rfind(":") + 1:]))
        elif dict_id == N.ZDL_DICT_JSON_IPV6TEXT:
            b = ipv6_bytes(unescape(raw))
            if b is None:  # the device only lists texts it parsed
                raise N.ZdlError(N.ZDL_EINVAL, f"ipv6 text {raw!r} does not parse")
            self._dec.bind(N.ZDL_DICT_IPV6, b, self.ip6.id(format_ipv6(b)))
        else:
            raise N.ZdlError(N.ZDL_EINVAL, f"unexpected key kind {dict_id}")

    def decode(self, data: bytes) -> DecodedBatch:
        out = self._dec.decode_json(data)
        while out.n_missing:
            for dict_id, raw in self._dec.missing(int(out.n_missing)):
                self._bind(dict_id, raw)
            out = self._dec.retry()
        n = int(out.n_spans)
        if n == 0:
            return DecodedBatch(0, None)
        return DecodedBatch(n, out.dev, out.dev_trace_hi, self._dec, out.dev_trace_wide)

    def decode_columns(self, data: bytes) -> Columns:
        """Host columns of one decoded batch, one span per trace (as ``accept`` packs them)."""
        b = self.decode(data)
        c = self._dec.download(b.n_spans)
        return Columns(c["trace_lo"], c["id"], c["parent_id"], c["local_svc"], c["remote_svc"], c["local_ip4"],
                       c["local_ip6"], c["port_flags"], c["timestamp"], np.arange(b.n_spans + 1, dtype=np.uint64))

    def kernel_ms(self) -> float:
        return self._dec.kernel_ms()

    def struct_ms(self) -> float:
        return self._dec.struct_ms()

    def exact_spans(self) -> int:
        return self._dec.exact_spans()

    def close(self):
        self._dec.close()
