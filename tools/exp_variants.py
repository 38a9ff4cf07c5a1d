"""C2 on the SURVEY §8(d) workload variants (Zipf s=1.1 keys, per-key random-walk prices) against the uniform
stream: per-stage device time and the step, one process, HBM-resident batches.  Experiments only (bench.py has
the reported legs).

    python tools/exp_variants.py [batch_log2] [n_batches] [variant ...]   (variants: uniform zipf walk)
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
K = 1 << 20


def batches(kind, B, nb, dev):
    out = []
    walk = synth.RandomWalk(K, torch=torch, device=dev) if kind == "walk" else None
    for s in range(nb):
        if kind == "zipf":
            d = synth.zipf_ticks_torch(torch, s * B, B, K, dev)
        else:
            d = synth.stock_ticks_torch(torch, s * B, B, K, dev)
        if walk is not None:
            d["price"] = walk.step(d["key"], s * B)
        out.append(d)
    torch.cuda.synchronize()
    return out


def main():
    B = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    kinds = sys.argv[3:] or ["uniform", "zipf", "walk"]
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    dev = torch.device("cuda", 0)
    for kind in kinds:
        bat = batches(kind, B, nb, dev)
        eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=256,
                              match_capacity=4 * B, device=0, flags=sa.native.SG_CFG_TIMING)
        st0 = None
        t0 = 0.0
        warm = min(3, nb - 1)  # (the engine settles its grouping / hot-key choices on the first batches)
        for s, t in enumerate(bat):
            if s == warm:
                eng.synchronize()
                st0 = eng.stats()
                t0 = time.perf_counter()
            eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                        t["volume"].data_ptr()], t["key"].data_ptr()),
                     [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
            while True:
                m = eng.poll_device()
                n_m = int(m.n)
                eng.release(m)
                if n_m == 0:
                    break
        eng.synchronize()
        el = time.perf_counter() - t0
        st = eng.stats()
        n = nb - warm
        print(json.dumps({"variant": kind, "batch": B, "step_ms": round(el / n * 1e3, 3),
                          "events_per_s": B * n / el,
                          "group_ms": round((st["group_ns"] - st0["group_ns"]) / 1e6 / n, 4),
                          "advance_ms": round((st["advance_ns"] - st0["advance_ns"]) / 1e6 / n, 4),
                          "hbm_pass_ms": round((st["advance_hbm_ns"] - st0["advance_hbm_ns"]) / 1e6 / n, 4),
                          "order_ms": round((st["order_ns"] - st0["order_ns"]) / 1e6 / n, 4),
                          "matches": (st["matches"] - st0["matches"]) / n,
                          "spills": (st["window_spills"] - st0["window_spills"]) / n,
                          "hot_pipeline": "k_hot_prep" in eng.describe()}), flush=True)
        eng.close()
        del bat
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
