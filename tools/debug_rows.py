"""Diagnostic: zdl_put_mysql_rows on tiny inputs, both context modes."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np
from zipkin_amd import _native as N
from zipkin_amd.linker import DependencyLinker
from zipkin_amd.model import Endpoint, Kind, Span
from test_mysql_rows import with_root, rec, B
rows = with_root([rec("ca", B, "s1"), rec("sa", B, "s2")])
for io in (False, True):
    l = DependencyLinker(insertion_order=io)
    l.put_mysql_rows(rows)
    print("rows io=%s" % io, l.link(), l.svc.strings)
    l2 = DependencyLinker(insertion_order=io)
    l2.put_trace([Span.create(1, 9, None, Kind.SERVER, local_endpoint=Endpoint.create("root")),
                  Span.create(1, 1, 9, None, local_endpoint=Endpoint.create("s1"), remote_endpoint=Endpoint.create("s2"))])
    print("spans io=%s" % io, l2.link())
