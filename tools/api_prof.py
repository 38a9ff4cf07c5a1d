"""Host API legs of bench.py (api_inclusive, api_async, api_columnar) timed, then each again under
cProfile: where a send's host time goes on the GPU box."""
import cProfile
import importlib
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
legs = {
    "api_inclusive": lambda: bench.api_inclusive(sa, synth, 1 << 16, 1 << 16, 16),
    "api_async": lambda: bench.api_async(sa, synth, 1 << 16, 1 << 20),
    "api_columnar": lambda: bench.api_columnar(sa, synth, 1 << 20, 1 << 20, 8),
    "api_columnar_cat": lambda: bench.api_columnar(sa, synth, 1 << 20, 1 << 20, 8, strings="categorical"),
}
want = sys.argv[1:] or list(legs)
for name in want:
    r = legs[name]()
    print(name, {k: v for k, v in r.items() if k != "what"}, flush=True)
for name in want:
    pr = cProfile.Profile()
    pr.enable()
    r = legs[name]()
    pr.disable()
    print(f"== {name} under cProfile: {r['value']:.4g} events/s", flush=True)
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    pstats.Stats(pr).sort_stats("cumtime").print_stats("runtime.py|native.py|bench.py", 25)
