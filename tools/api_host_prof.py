"""Host-side cost of the row API (InputHandler.send(Event[]) -> QueryCallback) without a device: a stub
engine that accepts pushes and returns, per poll, one match per 2.5 events with the C2 select list
projected "on the device" (synthetic values), so that the profile shows only the runtime's Python work.
    python tools/api_host_prof.py [--async] [--profile]"""
import cProfile
import importlib
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
native = importlib.import_module("siddhi-1_amd.native")


class StubEngine:
    def __init__(self, ir, n_keys):
        self.pending = []
        self.proj_items = 0

    def set_projection(self, code, pc, ln, ty, pa):
        self.proj_items = int(np.sum((np.asarray(ty) & 0x10000) == 0))

    def push(self, stream, seq_base, ts, cols, nulls=None, key=None, mem=0):
        n = len(ts)
        idx = np.arange(0, n, 5, dtype=np.int64)
        idx = np.sort(np.concatenate([idx, idx[::2]]))   # some triggers with two matches
        self.pending.append((seq_base + idx, np.asarray(ts)[idx], np.asarray(cols[1])[idx]))

    def poll(self, copy=True, ready=False):
        if not self.pending:
            z = np.zeros(0, np.uint64)
            return native.Matches(z, np.zeros(0, np.uint32), np.zeros(0, np.int64), np.zeros((0, 2, 1), np.uint64),
                                  np.zeros((0, 2), np.uint32))
        trig = np.concatenate([p[0] for p in self.pending]).astype(np.uint64)
        ts = np.concatenate([p[1] for p in self.pending])
        pr = np.concatenate([p[2] for p in self.pending]).astype(np.float32)
        self.pending = []
        n = len(trig)
        m = native.Matches(trig, np.zeros(n, np.uint32), ts, np.zeros((n, 2, 1), np.uint64), np.ones((n, 2), np.uint32))
        pv = np.zeros((self.proj_items, n), np.uint64)
        pv[0] = 3
        for i in range(1, self.proj_items):
            pv[i] = pr.view(np.uint32)
        m.proj_value, m.proj_null = pv, np.zeros((self.proj_items, n), np.uint8)
        return m

    def advance_time(self, now):
        pass

    def close(self):
        pass


def main():
    asyn = "--async" in sys.argv
    n_keys, chunk, chunks = 1 << 16, 1 << 16, 6
    mgr = sa.SiddhiManager(engine_factory=StubEngine, n_keys=n_keys, max_batch=chunk)
    app = synth.C2_QUERY
    if asyn:
        app = "@async(buffer.size='65536', batch.size.max='65536')\n" + app
    rt = mgr.createSiddhiAppRuntime(app)
    got = [0, 0]

    class Count(sa.QueryCallback):
        def receive(self, timestamp, in_events, remove_events):
            got[0] += 1
            got[1] += len(in_events)

    rt.addCallback("query1", Count())
    rt.start()
    ih = rt.getInputHandler("StockStream")
    names = [f"S{k}" for k in range(n_keys)]
    batches = []
    for c in range(chunks + 1):
        d = synth.stock_ticks(c * chunk, chunk, n_keys)
        batches.append([sa.Event(t, [names[k], p, v]) for t, k, p, v in
                        zip(d["ts"].tolist(), d["key"].tolist(), d["price"].tolist(), d["volume"].tolist())])
    ih.send(batches[0])
    pr = cProfile.Profile() if "--profile" in sys.argv else None
    if pr:
        pr.enable()
    t0 = time.perf_counter()
    for c in range(1, chunks + 1):
        ih.send(batches[c])
    rt.flush()
    el = time.perf_counter() - t0
    if pr:
        pr.disable()
    print(f"{chunk * chunks / el:.4g} events/s host-only, callbacks {got[0]}, matches {got[1]}")
    if pr:
        pstats.Stats(pr).sort_stats("tottime").print_stats(22)


if __name__ == "__main__":
    main()
