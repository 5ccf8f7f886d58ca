"""Random small traces that hit the reference's corner cases: colliding ids,
shared/non-shared mixes, fragments with partial endpoints, missing parents,
duplicate roots, cycles, remote-only services, errors, and (optionally) the
Q1 NPE. Used to cross-check the oracles against each other and the engine."""
import random

from zipkin_amd.model import Endpoint, Kind, Span

SVCS = ["a", "b", "c", "web", "app", "db", "B", "été", "\U0001F600x"]
IP4 = ["10.0.0.1", "10.0.0.2", "9.0.0.1"]
IP6 = ["2001:db8::1", "2001:db8::2"]


def _ep(r, p_null=0.25, full_ok=True):
    if r.random() < p_null:
        return None
    e = Endpoint.create(r.choice(SVCS + [None]), r.choice(IP4 + IP6 + [None, None]),
                        r.choice([0, 0, 80, 8080]))
    return None if e.is_empty() else e


def random_trace(r: random.Random, n=None, allow_npe=True, id_pool=6):
    n = n or r.randint(1, 12)
    ids = [format(r.randint(1, 2 ** 64 - 1), "016x") for _ in range(id_pool)]
    out = []
    for _ in range(n):
        sid = r.choice(ids)
        pid = r.choice(ids + [None, None])
        kind = r.choice([Kind.CLIENT, Kind.SERVER, Kind.PRODUCER, Kind.CONSUMER, None, Kind.SERVER, Kind.CLIENT])
        shared = r.choice([None, None, False, True])
        local = _ep(r)
        remote = None
        if r.random() < 0.6:
            remote = Endpoint.create(r.choice(SVCS), r.choice(IP4 + [None]), r.choice([0, 9000]))
        tags = {"error": ""} if r.random() < 0.2 else None
        out.append(Span.create("a" * 16, sid, pid, kind, local_endpoint=local, remote_endpoint=remote,
                               shared=shared, tags=tags, timestamp=r.choice([0, 1000, 2000, 3000])))
    if not allow_npe:
        # make every remote endpoint full so Builder.merge can never dereference a null one,
        # and local endpoints either null or full
        fix = []
        for s in out:
            re = s.remote_endpoint
            if re is not None:
                re = Endpoint(re.service_name or "x", "1.1.1.1", "::2", 9)
            le = s.local_endpoint
            if le is not None:
                le = Endpoint(le.service_name or "y", le.ipv4 or "2.2.2.2", le.ipv6 or "::3", le.port or 7)
            fix.append(s.to_builder(remote_endpoint=re, local_endpoint=le))
        out = fix
    return out
