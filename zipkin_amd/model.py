"""Value types of the dependency-link path: Span, Endpoint, DependencyLink, Kind.

Host-side mirror of the reference's immutable model classes, restricted to the
fields and normalisation rules the DependencyLinker path observes:

* ``zipkin2.Span`` (zipkin/src/main/java/zipkin2/Span.java): id/parentId
  normalisation (:442-484), ``parentId == id`` dropped on build (:606-619,
  :730-744), ``shared`` tri-state (:262-266), ``Builder.merge`` (:358-388),
  empty endpoints coerced to null (:527-536), ``equals`` over every field.
* ``zipkin2.Endpoint`` (Endpoint.java): service name lower-cased and
  empty->null (:132-135), ip parsing into ipv4/ipv6 (:219-237), port 0 = null
  (:245-260), ``equals`` on (serviceName, ipv4, ipv6, port) (:554-563).
* ``zipkin2.DependencyLink`` (DependencyLink.java): parent/child lower-cased
  (:72-82), equality on all four fields (:119-127).

Ids are kept as the reference keeps them: lower-hex strings, 16 chars for span
ids and 16 or 32 for trace ids, so lexicographic order equals u64 order.
"""
from __future__ import annotations

import enum
import ipaddress
from dataclasses import dataclass, field, replace
from typing import Dict, Iterable, List, NamedTuple, Optional, Tuple

__all__ = ["Kind", "Endpoint", "Span", "DependencyLink", "span2",
           "normalize_trace_id", "lower_hex", "java_string_key"]


class Kind(enum.IntEnum):
    """Span.Kind (Span.java:107-134). Values are the columnar kind codes."""
    CLIENT = 0
    SERVER = 1
    PRODUCER = 2
    CONSUMER = 3


def java_string_key(s: str) -> bytes:
    """Sort key reproducing ``java.lang.String.compareTo`` (UTF-16 code-unit order)."""
    return s.encode("utf-16-be", "surrogatepass")


_HEX = set("0123456789abcdef")


def _validate_hex(s: str) -> int:
    """Returns the count of leading zeros; raises like Span.validateHexAndReturnZeroPrefix."""
    zeros, in_prefix = 0, s[0] == "0"
    for c in s:
        if c not in _HEX:
            raise ValueError(f"{s} should be lower-hex encoded with no prefix")
        if c != "0":
            in_prefix = False
        elif in_prefix:
            zeros += 1
    return zeros


def normalize_trace_id(trace_id: str) -> str:
    """Span.normalizeTraceId (Span.java:634-649)."""
    if trace_id is None:
        raise TypeError("traceId == null")
    n = len(trace_id)
    if n == 0:
        raise ValueError("traceId is empty")
    if n > 32:
        raise ValueError("traceId.length > 32")
    zeros = _validate_hex(trace_id)
    if zeros == n:
        raise ValueError("traceId is all zeros")
    if n in (16, 32):
        if n == 32 and zeros >= 16:
            return trace_id[16:]
        return trace_id
    return trace_id.rjust(16 if n < 16 else 32, "0")


def lower_hex(v: int) -> str:
    return format(v & 0xFFFFFFFFFFFFFFFF, "016x")


def _norm_id(v, *, parent: bool) -> Optional[str]:
    if v is None:
        if parent:
            return None
        raise TypeError("id == null")
    if isinstance(v, int):
        if v == 0:
            if parent:
                return None
            raise ValueError("empty id")
        return lower_hex(v)
    n = len(v)
    if n == 0:
        raise ValueError(("parentId" if parent else "id") + " is empty")
    if n > 16:
        raise ValueError(("parentId" if parent else "id") + ".length > 16")
    zeros = _validate_hex(v)
    if parent and zeros == n:
        return None
    if not parent and zeros == 16:
        raise ValueError("id is all zeros")
    return v.rjust(16, "0")


@dataclass(frozen=True)
class Endpoint:
    service_name: Optional[str] = None
    ipv4: Optional[str] = None
    ipv6: Optional[str] = None
    port: int = 0

    @staticmethod
    def create(service_name: Optional[str] = None, ip: Optional[str] = None,
               port: Optional[int] = None) -> "Endpoint":
        svc = None if not service_name else service_name.lower()
        ipv4 = ipv6 = None
        if ip:
            ipv4, ipv6 = _parse_ip(ip)
        p = 0 if port is None or port <= 0 else int(port)
        if p > 0xFFFF:
            raise ValueError(f"invalid port {port}")
        return Endpoint(svc, ipv4, ipv6, p)

    def to_builder(self, **changes) -> "Endpoint":
        return replace(self, **changes)

    def is_empty(self) -> bool:
        return self.service_name is None and self.ipv4 is None and self.ipv6 is None and self.port == 0

    def is_full(self) -> bool:
        """All of serviceName, ipv4, ipv6 and port are set: merge(null) cannot NPE (Endpoint.java:121-129)."""
        return (self.service_name is not None and self.ipv4 is not None
                and self.ipv6 is not None and self.port != 0)


def _parse_ip(ip: str) -> Tuple[Optional[str], Optional[str]]:
    """Endpoint.Builder.parseIp(String) (Endpoint.java:219-237)."""
    try:
        addr = ipaddress.ip_address(ip)
    except ValueError:
        return None, None
    if addr.version == 4:
        return ip, None
    packed = addr.packed
    if all(b == 0 for b in packed[:10]):
        flag = packed[10] << 8 | packed[11]
        if flag in (0, 0xFFFF) and not (flag == 0 and packed[12:] == b"\x00\x00\x00\x01"):
            return ".".join(str(b) for b in packed[12:]), None
    return None, addr.compressed


def format_ipv6(ip: bytes) -> str:
    """Endpoint.writeIpV6 (Endpoint.java:350-407): the text of 16 address bytes. The longest run
    of zero groups ending before a non-zero group is compressed (first such run on ties); a
    trailing run only when no earlier run ended."""
    best_at, best_len, run_at, all_zero = -1, -1, -1, True
    for i in range(0, 16, 2):
        if ip[i] == 0 and ip[i + 1] == 0:
            run_at = i if run_at < 0 else run_at
            continue
        all_zero = False
        if run_at >= 0:
            if i - run_at > best_len:
                best_at, best_len = run_at, i - run_at
            run_at = -1
    if all_zero:
        return "::"
    if best_at == -1 and run_at != -1:
        best_at, best_len = run_at, 16 - run_at
    parts, i = [], 0
    while i < 16:
        if i == best_at:
            parts.append(":")
            i += best_len
            if i == 16:
                parts.append(":")
            continue
        if i != 0:
            parts.append(":")
        parts.append(format(ip[i] << 8 | ip[i + 1], "x"))  # hex without leading zeros
        i += 2
    return "".join(parts)


def _norm_endpoint(e: Optional[Endpoint]) -> Optional[Endpoint]:
    if e is None or e.is_empty():
        return None
    return e


_ESC = {'"': '\\"', "\\": "\\\\", "\b": "\\b", "\t": "\\t", "\n": "\\n", "\f": "\\f", "\r": "\\r",
        "\u2028": "\\u2028", "\u2029": "\\u2029"}


def _jstr(v: str) -> str:
    """A quoted JSON string as JsonEscaper.jsonEscape writes it (internal/JsonEscaper.java)."""
    return '"' + "".join(_ESC.get(c, "\\u%04x" % ord(c) if ord(c) < 0x20 else c) for c in v) + '"'


def _endpoint_json(e: "Endpoint") -> str:
    parts = []
    if e.service_name is not None:
        parts.append('"serviceName":' + _jstr(e.service_name))
    if e.ipv4 is not None:
        parts.append('"ipv4":"%s"' % e.ipv4)
    if e.ipv6 is not None:
        parts.append('"ipv6":"%s"' % e.ipv6)
    if e.port:
        parts.append('"port":%d' % e.port)
    return "{" + ",".join(parts) + "}"


@dataclass(frozen=True)
class Span:
    trace_id: str
    id: str
    parent_id: Optional[str] = None
    kind: Optional[Kind] = None
    name: Optional[str] = None
    timestamp: int = 0
    duration: int = 0
    local_endpoint: Optional[Endpoint] = None
    remote_endpoint: Optional[Endpoint] = None
    annotations: Tuple[Tuple[int, str], ...] = ()
    tags: Tuple[Tuple[str, str], ...] = ()
    shared: Optional[bool] = None
    debug: Optional[bool] = None

    @staticmethod
    def create(trace_id, id, parent_id=None, kind=None, *, name=None, timestamp=0, duration=0,
               local_endpoint=None, remote_endpoint=None, annotations=(), tags=None,
               shared=None, debug=None) -> "Span":
        tid = normalize_trace_id(trace_id if isinstance(trace_id, str) else lower_hex(trace_id))
        sid = _norm_id(id, parent=False)
        pid = _norm_id(parent_id, parent=True)
        if pid == sid:  # Span.Builder.build: undoing circular dependency (Span.java:611-617)
            pid = None
        tagt = tuple(sorted((tags or {}).items()))
        return Span(tid, sid, pid, kind, name.lower() if name else None,
                    max(int(timestamp or 0), 0), max(int(duration or 0), 0),
                    _norm_endpoint(local_endpoint), _norm_endpoint(remote_endpoint),
                    tuple(sorted(set(annotations))), tagt, shared, debug)

    def to_builder(self, **changes) -> "Span":
        """Copy with changes, re-applying the normalisation done by Span.Builder.build."""
        d = {f: getattr(self, f) for f in self.__dataclass_fields__}
        d.update(changes)
        if "tags" in changes and isinstance(changes["tags"], dict):
            d["tags"] = tuple(sorted(changes["tags"].items()))
        d["local_endpoint"] = _norm_endpoint(d["local_endpoint"])
        d["remote_endpoint"] = _norm_endpoint(d["remote_endpoint"])
        if "parent_id" in changes:
            d["parent_id"] = _norm_id(changes["parent_id"], parent=True)
        if "trace_id" in changes:
            tid = changes["trace_id"]
            d["trace_id"] = normalize_trace_id(tid if isinstance(tid, str) else lower_hex(tid))
        if d["parent_id"] == d["id"]:
            d["parent_id"] = None
        return Span(**d)

    @property
    def local_service_name(self) -> Optional[str]:
        return self.local_endpoint.service_name if self.local_endpoint else None

    @property
    def remote_service_name(self) -> Optional[str]:
        return self.remote_endpoint.service_name if self.remote_endpoint else None

    @property
    def tag_map(self) -> Dict[str, str]:
        return dict(self.tags)

    @property
    def is_error(self) -> bool:
        """``tags().containsKey("error")`` (DependencyLinker.java:112)."""
        return any(k == "error" for k, _ in self.tags)

    def to_json_v2(self) -> str:
        """Span.toString(): SpanBytesEncoder.JSON_V2 (internal/V2SpanWriter.java member order,
        JsonEscaper.jsonEscape). The FINE messages quote spans this way."""
        out = ['{"traceId":"', self.trace_id, '"']
        if self.parent_id is not None:
            out += [',"parentId":"', self.parent_id, '"']
        out += [',"id":"', self.id, '"']
        if self.kind is not None:
            out += [',"kind":"', Kind(self.kind).name, '"']
        if self.name is not None:
            out += [',"name":', _jstr(self.name)]
        if self.timestamp:
            out.append(',"timestamp":%d' % self.timestamp)
        if self.duration:
            out.append(',"duration":%d' % self.duration)
        for key, ep in (("localEndpoint", self.local_endpoint), ("remoteEndpoint", self.remote_endpoint)):
            if ep is not None:
                out += [',"', key, '":', _endpoint_json(ep)]
        if self.annotations:
            out.append(',"annotations":[' + ",".join(
                '{"timestamp":%d,"value":%s}' % (ts, _jstr(v)) for ts, v in self.annotations) + "]")
        if self.tags:
            out.append(',"tags":{' + ",".join(_jstr(k) + ":" + _jstr(v) for k, v in self.tags) + "}")
        if self.debug:
            out.append(',"debug":true')
        if self.shared:
            out.append(',"shared":true')
        out.append("}")
        return "".join(out)

    @property
    def trace_lo(self) -> str:
        """IMS.lowTraceId (InMemoryStorage.java:465-467)."""
        return self.trace_id[16:] if len(self.trace_id) == 32 else self.trace_id


class DependencyLink(NamedTuple):
    """zipkin2.DependencyLink (DependencyLink.java): immutable, equal by its four fields. A
    NamedTuple: link() builds one per pair, and a frozen dataclass cost ~1 us each (2.3 ms for
    C2's 2 500 links, more than the device's whole step)."""
    parent: str
    child: str
    call_count: int = 0
    error_count: int = 0

    @staticmethod
    def create(parent: str, child: str, call_count: int = 0, error_count: int = 0) -> "DependencyLink":
        # DependencyLink.Builder lower-cases parent and child (DependencyLink.java:72-82)
        return DependencyLink(parent.lower(), child.lower(), int(call_count), int(error_count))

    def to_json_v1(self) -> dict:
        """DependencyLinkBytesEncoder.JSON_V1 field set; errorCount omitted when 0."""
        d = {"parent": self.parent, "child": self.child, "callCount": self.call_count}
        if self.error_count:
            d["errorCount"] = self.error_count
        return d


def span2(trace_id: str, parent_id: Optional[str], id: str, kind: Optional[Kind],
          local: Optional[str], remote: Optional[str], is_error: bool, **kw) -> Span:
    """DependencyLinkerTest.span2 helper (DependencyLinkerTest.java:585-592)."""
    return Span.create(trace_id, id, parent_id, kind,
                       local_endpoint=Endpoint.create(local) if local is not None else None,
                       remote_endpoint=Endpoint.create(remote) if remote is not None else None,
                       tags={"error": ""} if is_error else None, **kw)
