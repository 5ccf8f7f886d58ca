"""Proto3 ingest on the device: SpanBytesDecoder.PROTO3.decodeList(bytes) straight to span columns.

Reference: codec/SpanBytesDecoder.java:144-152 -> internal/Proto3Codec.java readList ->
internal/Proto3ZipkinFields.java:309-369 (paths under /root/reference/zipkin/src/main/java/zipkin2/).
The decoding runs in ``k_proto3_spans`` (zipkin_amd/csrc/zdl_proto3.hip); this module only owns
the dictionaries: when the device meets a raw key its table lacks (a service name before
``toLowerCase``, an ipv4 / ipv6 address), the key is normalised here like Endpoint.Builder does
(``serviceName(..)`` lower-cases, Endpoint.java:132-136; ``parseIp(byte[])`` texts,
Endpoint.java:179-198, 350-407), given the id of its string in first-seen order — the same ids
``columnar.pack_traces`` assigns to the decoded spans — and bound, and the kernel re-runs on the
resident batch. Malformed input raises like the reference (IllegalArgumentException).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _native as N
from .columnar import Columns, Dictionary
from .model import format_ipv6


@dataclass
class DecodedBatch:
    """A decode's result: device columns owned by the decoder until its next decode. The host
    copies of trace_lo / timestamp are downloaded only when read (the storage facade never
    does: accept goes device columns -> store)."""
    n_spans: int
    dev: Optional[N.SpanCols]
    dev_trace_hi: Optional[int] = None  # device pointer: the trace ids' high 64 bits (0 = 64-bit id)
    _dec: Optional[N.Decoder] = None
    dev_trace_wide: Optional[int] = None  # device pointer: the ids' widths (None: 128-bit iff hi != 0)
    _gen: int = 0  # the decoder's generation that produced these columns

    def __post_init__(self):
        if self._dec is not None:
            self._gen = self._dec.gen

    def _host(self, name, dtype):
        if self.n_spans == 0:
            return np.zeros(0, dtype)
        if self._dec.gen != self._gen:
            raise RuntimeError("DecodedBatch: its decoder has decoded another batch since; the device columns "
                               "are valid only until the next decode")
        return self._dec.download(self.n_spans, (name,))[name]

    @property
    def trace_lo(self) -> np.ndarray:
        return self._host("trace_lo", np.uint64)

    @property
    def timestamp(self) -> np.ndarray:
        return self._host("timestamp", np.int64)


def _key_string(dict_id: int, raw: bytes) -> str:
    if dict_id == N.ZDL_DICT_SERVICE:
        # Java: new String(bytes, UTF_8).toLowerCase(Locale.ROOT); Python's lower() agrees on ASCII
        # (non-ASCII case mapping is parity-unpinned)
        return raw.decode("utf-8", "replace").lower()
    if dict_id == N.ZDL_DICT_IPV4:
        return ".".join(str(b) for b in raw)
    return format_ipv6(raw)


class Proto3Decoder:
    """Decodes proto3 ListOfSpans batches on the device with ids from the given dictionaries."""

    def __init__(self, svc: Dictionary, ip4: Dictionary, ip6: Dictionary, device: int = 0):
        self.dicts = {N.ZDL_DICT_SERVICE: svc, N.ZDL_DICT_IPV4: ip4, N.ZDL_DICT_IPV6: ip6}
        self._dec = N.Decoder(device)

    def decode(self, data: bytes) -> DecodedBatch:
        out = self._dec.decode(data)
        while out.n_missing:
            for dict_id, raw in self._dec.missing(int(out.n_missing)):
                self._dec.bind(dict_id, raw, self.dicts[dict_id].id(_key_string(dict_id, raw)))
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

    def close(self):
        self._dec.close()
