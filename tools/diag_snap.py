"""Diagnostic: determinism of the general engine's state across identical runs and across a
snapshot/restore (compares device images batch by batch)."""
import importlib, sys
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from test_gpu_general import GENERAL
sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

q = GENERAL[sys.argv[1] if len(sys.argv) > 1 else "c3_min1"]
app = sa.parse_app(q)
cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
mk = lambda: sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=1024, max_batch=20000,
                             partial_capacity=64, match_capacity=1 << 21)
data, seq = [], 0
for b in range(4):
    data.append((seq, synth.stock_ticks(seq, 20000, 1024, seed=41 + b, rate_per_ms=16)))
    seq += 20000
push = lambda e, s, d: e.push(0, s, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
r1, r2 = mk(), mk()
imgs = []
for i, (s, d) in enumerate(data):
    for e in (r1, r2):
        push(e, s, d); e.poll()
    a, b = r1.snapshot(), r2.snapshot()
    print("batch", i, "images equal:", a == b, "live", r1.stats()["partials_live"], r2.stats()["partials_live"], flush=True)
    imgs.append(a)
c = mk()
c.restore(imgs[1])
print("restored live", c.stats()["partials_live"], "image equal after restore:", c.snapshot() == imgs[1])
for i, (s, d) in enumerate(data[2:], start=2):
    push(c, s, d); c.poll()
    x = c.snapshot()
    print("restored batch", i, "image equal:", x == imgs[i], "live", c.stats()["partials_live"], flush=True)
    if x != imgs[i]:
        u, v = np.frombuffer(x, dtype=np.uint8), np.frombuffer(imgs[i], dtype=np.uint8)
        diff = np.nonzero(u != v)[0]
        wi = (diff[diff >= 88] - 88) // 4
        print("  differing bytes:", len(diff), "block words:", sorted(set((wi // 1024).tolist()))[:20],
              "keys:", len(set((wi % 1024).tolist())))
