"""C4's playback step (advance_time, poll, push, poll) with the host time of each call, averaged over the steps:
where the step's wall time goes beside the kernels.  python tools/exp_c4_host.py [C4|C4_deep_state] [steps]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
dev = torch.device("cuda", 0)
name = sys.argv[1] if len(sys.argv) > 1 else "C4"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 16
K, cb = 1 << 20, 1 << 22
if name == "C4":
    mk, keys, B, cap = (lambda s: synth.burst_ticks(s * cb, cb, K, 1)), K, cb, 16
else:
    mk, keys, B, cap = (lambda s: synth.absent_deep_ticks(s * 4096, 4096, 2048, 16)), 2048, 1 << 16, 512
app = sa.parse_app(synth.C4_QUERY)
cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
warm = 8 if name != "C4" else 2
bats = [bench.to_dev(torch, mk(s), dev) for s in range(warm + steps)]
lastts = [int(b["ts"][-1].item()) for b in bats]
torch.cuda.synchronize()
eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=keys, max_batch=B, partial_capacity=cap,
                      match_capacity=2 * B, device=0)
acc = {"advance": 0.0, "poll_a": 0.0, "push": 0.0, "poll_b": 0.0}


def step(s, rec):
    t = bats[s]
    t0 = time.perf_counter()
    eng.advance_time(lastts[s])
    t1 = time.perf_counter()
    m = eng.poll_device()
    eng.release(m)
    t2 = time.perf_counter()
    eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(), t["volume"].data_ptr()],
                        t["key"].data_ptr()), [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
    t3 = time.perf_counter()
    m = eng.poll_device()
    eng.release(m)
    t4 = time.perf_counter()
    if rec:
        acc["advance"] += t1 - t0
        acc["poll_a"] += t2 - t1
        acc["push"] += t3 - t2
        acc["poll_b"] += t4 - t3


for s in range(warm):
    step(s, False)
eng.synchronize()
t0 = time.perf_counter()
for s in range(warm, warm + steps):
    step(s, True)
eng.synchronize()
el = time.perf_counter() - t0
print(json.dumps({"config": name, "ms_per_step": el / steps * 1e3, "events_per_s": B * steps / el,
                  **{k + "_ms": v / steps * 1e3 for k, v in acc.items()}}), flush=True)
eng.close()
