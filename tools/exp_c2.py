"""Advance-kernel variant sweep on the C2 workload (one process, the same HBM-resident batches).

Each variant sets environment knobs read at engine creation (SG_JIT_EXTRA = JIT #defines,
SGD_STAGE_CHUNKS, SGD_REG_SLOTS) and prints the per-stage device time.  Used to pick the shipped
defaults; not the bench.

    python tools/exp_c2.py [n_batches] "NAME:ENV=VAL;ENV=VAL" ...
"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
B, K = 1 << 24, 1 << 20
KNOBS = ("SG_JIT_EXTRA", "SGD_STAGE_CHUNKS", "SGD_REG_SLOTS", "SG_NO_FUSED", "SG_CUMASK", "SG_STREAM_PRIO")


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    variants = [("base", {})]
    for a in sys.argv[2:]:
        name, _, envs = a.partition(":")
        variants.append((name, dict(x.split("=", 1) for x in envs.split(";") if x)))
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    dev = torch.device("cuda", 0)
    bat = []
    pb = int(os.environ.get("SG_EXP_PIPE", "6"))   # more batches, pushed pipelined after the serial ones
    for s in range(nb + pb):
        d = synth.stock_ticks(s * B, B, K)
        bat.append({k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev) for k, v in d.items()})
    torch.cuda.synchronize()
    for name, env in variants:
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(env)
        eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=64,
                              match_capacity=2 * B, device=0, flags=sa.native.SG_CFG_TIMING)
        st0 = None
        for s in range(nb):
            t = bat[s]
            eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                        t["volume"].data_ptr()], t["key"].data_ptr()),
                     [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
            while True:   # a window that wraps the output ring comes in two polls
                m = eng.poll_device()
                n_m = int(m.n)
                eng.release(m)
                if n_m == 0:
                    break
            if s == 0:
                eng.synchronize()
                st0 = eng.stats()
        eng.synchronize()
        st = eng.stats()
        n = nb - 1
        # the pipelined step (bench.py's loop: ready polls, batch s+1's grouping beside batch s's advance)
        import time
        eng.synchronize()
        t0 = time.perf_counter()
        for s in range(nb, nb + pb):
            t = bat[s]
            eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                        t["volume"].data_ptr()], t["key"].data_ptr()),
                     [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
            while True:
                m = eng.poll_device(ready=True)
                n_m = int(m.n)
                eng.release(m)
                if n_m == 0:
                    break
        eng.synchronize()
        while True:
            m = eng.poll_device()
            n_m = int(m.n)
            eng.release(m)
            if n_m == 0:
                break
        step_ms = (time.perf_counter() - t0) / max(1, pb) * 1e3
        print(json.dumps({"variant": name, "env": env, "pipelined_step_ms": round(step_ms, 4),
                          "group_ms": round((st["group_ns"] - st0["group_ns"]) / 1e6 / n, 4),
                          "advance_ms": round((st["advance_ns"] - st0["advance_ns"]) / 1e6 / n, 4),
                          "order_ms": round((st["order_ns"] - st0["order_ns"]) / 1e6 / n, 4),
                          "hbm_pass_ms": round((st.get("advance_hbm_ns", 0) - st0.get("advance_hbm_ns", 0)) / 1e6 / n, 4),
                          "matches": (st["matches"] - st0["matches"]) / n,
                          "spills": (st["window_spills"] - st0["window_spills"]) / n}), flush=True)
        eng.close()
    for k in KNOBS:
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
