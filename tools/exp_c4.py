"""C4 workload variants on the general engine (keys x burst), for choosing the bench's C4 line."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import bench  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
dev = torch.device("cuda", 0)
for spec in sys.argv[1:]:
    keys, burst, nb, cap = (int(x) for x in spec.split(","))
    per = nb // burst
    r = bench.run_general(sa, synth, torch, dev, synth.C4_QUERY,
                          lambda s: synth.burst_ticks(s * per, per, keys, burst), keys, nb, 3, 1, cap, playback=True)
    print(json.dumps(dict(r, keys=keys, burst=burst, cap=cap)), flush=True)
