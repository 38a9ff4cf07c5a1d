"""P3 (3-state chain) at bench size through the engine: events/s, the chain kernel's hand-overs (window_spills) and
keys, for rocprofv3 kernel traces of the chain kernel against the general kernel (SG_NO_CHN=1).

    python tools/exp_chain.py [steps]
"""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    sa = importlib.import_module("siddhi-1_amd")
    synth = importlib.import_module("siddhi-1_amd.synth")
    K, B = 1 << 20, 1 << 22
    app = sa.parse_app(synth.P3_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    dev = torch.device("cuda", 0)
    bats = []
    for s in range(steps):
        d = synth.stock_ticks(s * B, B, K)
        bats.append({k: torch.from_numpy(v.view("int32") if v.dtype.kind == "u" else v).to(dev) for k, v in d.items()})
    torch.cuda.synchronize()
    eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=32,
                          match_capacity=2 * B, device=0)
    print(eng.describe(), flush=True)
    t0 = None
    for s in range(steps):
        if s == 1:
            eng.synchronize()
            t0 = time.perf_counter()
        t = bats[s]
        eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(), t["volume"].data_ptr()],
                            t["key"].data_ptr()), [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
        m = eng.poll_device()
        eng.release(m)
        if os.environ.get("CHN_PER_STEP"):   # (per push: wall time and the counters, the engine synchronised)
            eng.synchronize()
            st = eng.stats()
            print(f"step {s}: {time.perf_counter() - (t0 or time.perf_counter()):.4f} s, live {st['partials_live']}, "
                  f"spills {st['window_spills']}, matches {st['matches']}", flush=True)
    eng.synchronize()
    el = time.perf_counter() - t0
    st = eng.stats()
    print(f"P3: {B * (steps - 1) / el:.3e} events/s, {el / (steps - 1) * 1e3:.2f} ms per step; stats {st}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
