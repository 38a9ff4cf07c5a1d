"""The CPU baseline leg of bench.py alone (C2 sizes): where the partition-parallel threads run and how they
scale.  python tools/cpu_leg.py [seconds]"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
q = bench.cpu_quota()
print("quota", q, "pins", bench.distinct_cores(int(q or 1)), flush=True)
r = bench.cpu_baseline(sa, synth, 1 << 20, 1 << 24, float(sys.argv[1]) if len(sys.argv) > 1 else 12.0)
print(json.dumps(r), flush=True)
