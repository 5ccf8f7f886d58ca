"""Debug helper: repeat the C5 insertion-order put in one process and report any run whose
output differs from the C++ restatement (wrong-result flake hunt; no GPU fault involved)."""
import sys

sys.path.insert(0, ".")
from oracle import ref  # noqa: E402
from zipkin_amd import _native as N  # noqa: E402
from zipkin_amd import synth  # noqa: E402

w = synth.C5.scaled(20_000)
w = synth.Workload(**{**w.__dict__, "max_size": 5_000})
cols = synth.generate(w)
st, op, oc, on, oe = ref.link(cols, threads=8)
exp = list(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))
print("oracle links", len(exp), flush=True)
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    ctx = N.Context(w.total_services, insertion_order=True)
    ctx.put_spans(cols)
    p, c, n, e = ctx.link(N.ZDL_ORDER_INSERTION)
    got = list(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))
    sp, sc, sn, se = ctx.link(N.ZDL_ORDER_SORTED)
    srt = sorted(zip(sp.tolist(), sc.tolist(), sn.tolist(), se.tolist()))
    ctx.close()
    print(it, "insertion", len(got), "equal" if got == exp else "DIFF",
          "sorted", len(srt), "equal" if srt == sorted(exp) else "DIFF",
          "calls", sum(x[2] for x in srt), flush=True)
