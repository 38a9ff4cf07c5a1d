"""Profile of the columnar host API leg (bench.api_columnar) under cProfile: where a send's host time goes."""
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
pr = cProfile.Profile()
pr.enable()
r = bench.api_columnar(sa, synth, 1 << 20, 1 << 20, 4)
pr.disable()
print({k: v for k, v in r.items() if k != "what"})
pstats.Stats(pr).sort_stats("cumulative").print_stats(28)
