"""Partition-parallel CPU leg of bench.py at several thread counts (SG_CPU_THREADS), C2 sizes: per-thread rate
against one thread on the same shard, the threads' busy times.  python tools/cpu_scaling.py [seconds] T1 T2 ..."""
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
secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
print("quota", bench.cpu_quota(), "nproc", os.cpu_count(), flush=True)
for t in sys.argv[2:] or ["16"]:
    os.environ["SG_CPU_THREADS"] = t
    r = bench.cpu_baseline(sa, synth, 1 << 20, 1 << 24, secs)
    p = r["partition_parallel"]
    print(json.dumps({"threads": int(t), "par": p["value"], "alone": p["one_thread_same_sample"],
                      "per_thread": p["per_thread_scaling"], "busy": p["thread_busy_s"], "pins": p["pinned_cpus"],
                      "single_prefix": r["value"]}), flush=True)
