"""mysql-v1 getDependencies on the device: AggregateDependencies.apply after its query.

Reference: zipkin-storage/mysql-v1/src/main/java/zipkin2/storage/mysql/v1/
AggregateDependencies.java:55-84 and DependencyLinkV2SpanIterator.java. The SQL cursor (spans
left-joined with their lc/cs/ca/sr/sa/error annotations, grouped by trace then span id) is the
input; the projection of each span's rows to a minimal span and the linking run on the device
(zdl_put_mysql_rows). The returned list has DependencyLinker.link()'s order.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

from .linker import DependencyLinker
from .model import DependencyLink


def aggregate_dependencies(rows: Iterable[Sequence], device: int = 0) -> List[DependencyLink]:
    """rows: (trace_id_high, trace_id, parent_id, id, a_key, a_type, endpoint_service_name)."""
    rows = list(rows)
    if not rows:  # !traces.hasNext() -> emptyList
        return []
    linker = DependencyLinker(device)
    try:
        return linker.put_mysql_rows(rows).link()
    finally:
        linker.close()
