"""Small C2 driver for profiling: pushes a few 2^24-event batches through the HIP engine."""
import importlib, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
B, K = 1 << 24, 1 << 20
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 3
app = sa.parse_app(synth.C2_QUERY)
cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=64,
                      match_capacity=2 * B, device=0, flags=sa.native.SG_CFG_TIMING)
dev = torch.device("cuda", 0)
bat = []
for s in range(nb):
    d = synth.stock_ticks(s * B, B, K)
    bat.append({k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev) for k, v in d.items()})
torch.cuda.synchronize()
for s in range(nb):
    t = bat[s]
    eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(), t["volume"].data_ptr()],
                        t["key"].data_ptr()), [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
    m = eng.poll_device(); eng.release(m)
eng.synchronize()
st = eng.stats()
print({k: v for k, v in st.items()})
print("advance ms/launch", st["advance_ns"] / 1e6 / st["advance_launches"])
