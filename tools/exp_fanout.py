"""bench.py's fanout_one_gpu leg on its own (two shards of the C-ABI fan-out on one GPU vs the single engine)."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
app = sa.parse_app(synth.C2_QUERY)
cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
print(json.dumps(bench.fanout_one_gpu(sa, synth, torch, torch.device("cuda", 0), cq, 1 << 20, 1 << 22, 6)), flush=True)

# where the fan-out's step goes: push (split + host wait + seq maps + shard pushes) vs poll (shard polls to host,
# seq mapping, merge)
import time  # noqa: E402
B, K = 1 << 22, 1 << 20
eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=64,
                      match_capacity=2 * B, device=0, devices=[0, 0])
dev = torch.device("cuda", 0)
bats = [synth.stock_ticks_torch(torch, s * B, B, K, dev) for s in range(6)]
torch.cuda.synchronize()
tp = tq = 0.0
for s in range(6):
    t = bats[s]
    t0 = time.perf_counter()
    eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(), t["volume"].data_ptr()],
                        t["key"].data_ptr()), [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
    t1 = time.perf_counter()
    n = len(eng.poll(copy=False))
    t2 = time.perf_counter()
    if s >= 2:
        tp += t1 - t0
        tq += t2 - t1
print(json.dumps({"push_ms": tp / 4 * 1e3, "poll_ms": tq / 4 * 1e3, "matches": n}), flush=True)
