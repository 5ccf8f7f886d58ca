"""Zipkin v2 JSON <-> model, the field set of SpanBytesEncoder/Decoder.JSON_V2.

Reference: zipkin2/internal/V2SpanWriter.java / V2SpanReader.java (field names
traceId, parentId, id, kind, name, timestamp, duration, localEndpoint,
remoteEndpoint, annotations, tags, debug, shared; endpoint fields serviceName,
ipv4, ipv6, port). Used by the golden fixtures and the storage facade.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

from .model import DependencyLink, Endpoint, Kind, Span


def endpoint_to_json(e: Optional[Endpoint]) -> Optional[Dict[str, Any]]:
    if e is None:
        return None
    d: Dict[str, Any] = {}
    if e.service_name is not None:
        d["serviceName"] = e.service_name
    if e.ipv4 is not None:
        d["ipv4"] = e.ipv4
    if e.ipv6 is not None:
        d["ipv6"] = e.ipv6
    if e.port:
        d["port"] = e.port
    return d


def endpoint_from_json(d: Optional[Dict[str, Any]]) -> Optional[Endpoint]:
    if not d:
        return None
    svc = d.get("serviceName")
    e = Endpoint(svc.lower() if svc else None, d.get("ipv4") or None, d.get("ipv6") or None,
                 int(d.get("port") or 0))
    return None if e.is_empty() else e


def span_to_json(s: Span) -> Dict[str, Any]:
    d: Dict[str, Any] = {"traceId": s.trace_id}
    if s.parent_id is not None:
        d["parentId"] = s.parent_id
    d["id"] = s.id
    if s.kind is not None:
        d["kind"] = s.kind.name
    if s.name is not None:
        d["name"] = s.name
    if s.timestamp:
        d["timestamp"] = s.timestamp
    if s.duration:
        d["duration"] = s.duration
    if s.local_endpoint is not None:
        d["localEndpoint"] = endpoint_to_json(s.local_endpoint)
    if s.remote_endpoint is not None:
        d["remoteEndpoint"] = endpoint_to_json(s.remote_endpoint)
    if s.annotations:
        d["annotations"] = [{"timestamp": t, "value": v} for t, v in s.annotations]
    if s.tags:
        d["tags"] = dict(s.tags)
    if s.debug is not None:
        d["debug"] = s.debug
    if s.shared is not None:
        d["shared"] = s.shared
    return d


def span_from_json(d: Dict[str, Any]) -> Span:
    kind = d.get("kind")
    return Span.create(
        d["traceId"], d["id"], d.get("parentId"), Kind[kind] if kind else None,
        name=d.get("name"), timestamp=d.get("timestamp", 0), duration=d.get("duration", 0),
        local_endpoint=endpoint_from_json(d.get("localEndpoint")),
        remote_endpoint=endpoint_from_json(d.get("remoteEndpoint")),
        annotations=tuple((a["timestamp"], a["value"]) for a in d.get("annotations", [])),
        tags=d.get("tags"), shared=d.get("shared"), debug=d.get("debug"))


def spans_from_json(data) -> List[Span]:
    if isinstance(data, (bytes, str)):
        data = json.loads(data)
    return [span_from_json(x) for x in data]


def link_to_json(l: DependencyLink) -> Dict[str, Any]:
    return {"parent": l.parent, "child": l.child, "callCount": l.call_count, "errorCount": l.error_count}


def link_from_json(d: Dict[str, Any]) -> DependencyLink:
    return DependencyLink.create(d["parent"], d["child"], d.get("callCount", 0), d.get("errorCount", 0))


# JsonEscaper.REPLACEMENT_CHARS (zipkin2/internal/JsonEscaper.java): every control
# character as \u00xx, then the short forms for quote, backslash, \t \b \n \r \f.
_JSON_REPLACEMENTS = {i: "\\u%04x" % i for i in range(0x20)}
_JSON_REPLACEMENTS.update({ord('"'): '\\"', ord("\\"): "\\\\", ord("\t"): "\\t", ord("\b"): "\\b",
                           ord("\n"): "\\n", ord("\r"): "\\r", ord("\f"): "\\f",
                           0x2028: "\\u2028", 0x2029: "\\u2029"})


def json_escape(v: str) -> str:
    """JsonEscaper.jsonEscape: RFC 7159 escapes plus U+2028 / U+2029."""
    return v.translate(_JSON_REPLACEMENTS)


def _utf8(v: str) -> bytes:
    # Buffer.writeUtf8 writes '?' for an unpaired surrogate.
    return v.encode("utf-8", "replace")


def encode_link(l: DependencyLink) -> bytes:
    """DependencyLinkBytesEncoder.JSON_V1.encode (DependencyLinkBytesEncoder.java:35-65).

    ``{"parent":"…","child":"…","callCount":N[,"errorCount":E]}``, errorCount only when > 0,
    no whitespace; the same bytes the reference's ``/api/v2/dependencies`` returns per link.
    """
    out = b'{"parent":"' + _utf8(json_escape(l.parent)) + b'","child":"' + _utf8(json_escape(l.child))
    out += b'","callCount":' + str(int(l.call_count)).encode()
    if l.error_count > 0:
        out += b',"errorCount":' + str(int(l.error_count)).encode()
    return out + b"}"


def encode_links(links) -> bytes:
    """DependencyLinkBytesEncoder.JSON_V1.encodeList via JsonCodec.writeList (JsonCodec.java:206-232)."""
    return b"[" + b",".join(encode_link(l) for l in links) + b"]"


def decode_links(data) -> List[DependencyLink]:
    """DependencyLinkBytesDecoder.JSON_V1.decodeList: the inverse of :func:`encode_links`."""
    if isinstance(data, (bytes, bytearray)):
        data = data.decode("utf-8")
    return [link_from_json(d) for d in json.loads(data)]
