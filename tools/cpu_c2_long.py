"""The single-thread C2 CPU leg over SURVEY §8(d)'s full sample: the CPU oracle (the faithful single-thread
restatement of the reference engine) on the first N events of the C2 stream (default 1e8; bench.py's cpu_baseline
bounds itself to ~12 s), in 2^19-event chunks, with the rate every 1e7 events (the 10-second windows fill over the
first ~2e7 events, so the rate falls and then holds).

    python tools/cpu_c2_long.py [events] > profiles/<round>_cpu_c2_1e8.json
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from oracle_backend import build_oracle  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")


def main():
    total = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    K = 1 << 20
    bench.keep_heap()
    lib = build_oracle()
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    eng = sa.NativeEngine(lib, "sgo_", cq.ir, n_keys=K)
    chunk = 1 << 19
    done, busy, marks, last = 0, 0.0, [], (0, 0.0)
    while done < total:
        n = min(chunk, total - done)
        d = synth.stock_ticks(done, n, K)
        t = time.perf_counter()
        eng.push(0, done, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        eng.discard()
        busy += time.perf_counter() - t
        done += n
        if done - last[0] >= 10_000_000 or done == total:
            marks.append({"events": done, "rate_since_last": (done - last[0]) / (busy - last[1])})
            last = (done, busy)
            print(json.dumps(marks[-1]), file=sys.stderr, flush=True)
    st = eng.stats()
    eng.close()
    print(json.dumps({"value": done / busy, "unit": "events/s", "cores": 1, "kind": "port", "events": done,
                      "busy_s": busy, "matches": st["matches"], "cpu_model": bench.cpu_model(),
                      "sample": f"first {done} events of the C2 stream (2^20 keys, 2000 events/ms), CPU oracle single "
                                f"thread, pushed in {chunk}-event chunks (generation not timed)",
                      "rate_per_1e7": marks}), flush=True)


if __name__ == "__main__":
    main()
