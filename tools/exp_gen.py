"""General-engine configs of bench.py (C3_min1, C4, C4_deep) at their bench sizes, fewer steps: one JSON
line per config.  SG_HIP_LIBRARY selects an alternative build of the engine (layout experiments)."""
import faulthandler
import importlib
import json
import os
import sys

faulthandler.dump_traceback_later(int(os.environ.get("SG_EXP_WATCHDOG", "150")), exit=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import bench  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
dev = torch.device("cuda", 0)
K, cb = 1 << 20, 1 << 22
steps = int(os.environ.get("SG_EXP_STEPS", "4"))
which = sys.argv[1:] or ["C3", "C3_min1", "C4", "C4_deep"]
cfg = {
    "C3": (synth.C3_QUERY, lambda s: synth.stock_ticks(s * cb, cb, K), K, cb, 8, False),
    "C3_min1": (synth.C3_MIN1_QUERY, lambda s: synth.stock_ticks(s * cb, cb, K), K, cb, 8, False),
    "C3_and": (synth.C3_AND_QUERY, lambda s: synth.stock_ticks(s * cb, cb, K), K, cb, 8, False),
    "P3": (synth.P3_QUERY, lambda s: synth.stock_ticks(s * cb, cb, K), K, cb, 32, False),
    "C4": (synth.C4_QUERY, lambda s: synth.burst_ticks(s * cb, cb, K, 1), K, cb, 16, True),
    "C4_deep": (synth.C4_QUERY, lambda s: synth.burst_ticks(s * (cb // 16), cb // 16, K // 4, 16), K // 4, cb, 64,
                True),
    "C4_deep_state": (synth.C4_QUERY, lambda s: synth.absent_deep_ticks(s * 4096, 4096, 2048, 16), 2048, 1 << 16, 512,
                      True),
}
for name in which:
    print("config", name, flush=True)
    q, mk, keys, b, cap, pb = cfg[name]
    r = bench.run_general(sa, synth, torch, dev, q, mk, keys, b, steps, 8 if name == "C4_deep_state" else 1, cap,
                          playback=pb)
    print(json.dumps(dict(r, config=name, lib=os.environ.get("SG_HIP_LIBRARY", "default"))), flush=True)
