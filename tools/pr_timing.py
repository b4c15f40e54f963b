import sys, time, os
sys.path.insert(0, 'bn-pp_amd/python')
import bnpp
ctx = bnpp.Context(0)
for name, ev in [("Munin2.uai", None), ("Pigs.uai", "Pigs.uai.evid")]:
    m = bnpp.Model.load("tests/golden/models/" + name)
    e = bnpp.load_evidence("tests/golden/models/" + ev) if ev else {}
    for i in range(3):
        t = time.perf_counter()
        lz, z, up = bnpp.partition(ctx, m, e, "mf", bnpp.F64)
        print(name, i, "uptime %.2f ms wall %.2f ms" % (up, (time.perf_counter() - t) * 1e3), file=sys.stderr, flush=True)
