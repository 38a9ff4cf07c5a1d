"""Benchmark: partitioned 2-step pattern query on MI355X (BASELINE.json configs[1], "C2").

    every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] within 10 sec
    partition with (symbol of StockStream), 1,048,576 synthetic keys

A step = one micro-batch of 2^24 synthetic stock ticks (already resident in HBM) pushed through the
C-ABI (key grouping + NFA advance) and polled (matches ordered by trigger seq, left in HBM).
`value` = input events/sec of the whole job (all ranks).  N > 1: one process per GPU, each rank owns
a disjoint shard of 1,048,576 keys and its own arrival stream (weak scaling, no data-path
collective).  The roofline object prices the NFA advance kernel with the algorithmic byte model of
DESIGN.md over its HIP-event-timed duration; cpu_baseline times the CPU oracle (the
single-threaded restatement of the reference engine) on a bounded prefix of the same stream.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(st):
    """16 B/event in + 16 B per touched key header (r+w) + 2*16 B per live partial of a
    touched key at batch start + 16 B per new partial + 24 B per emitted match."""
    return (16 * st["events"] + 16 * st["keys_touched"] + 32 * st["live_at_batch_start"]
            + 16 * st["partials_created"] + 24 * st["matches"])


def delta(a, b):
    return {k: b[k] - a[k] for k in a}


def cpu_baseline(sa, synth, n_keys, batch, seconds):
    """Single-thread CPU oracle on the first events of the same C2 stream (bounded by `seconds`)."""
    from oracle_backend import build_oracle
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    eng = sa.NativeEngine(build_oracle(), "sgo_", cq.ir, n_keys=n_keys)
    chunk = 1 << 19
    done, busy = 0, 0.0
    while busy < seconds and done < batch * 4:
        d = synth.stock_ticks(done, chunk, n_keys)
        t = time.perf_counter()
        eng.push(0, done, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        eng.poll()
        busy += time.perf_counter() - t
        done += chunk
    eng.close()
    return {"value": done / busy, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": f"first {done} events of the C2 stream ({n_keys} keys), CPU oracle "
                      f"(faithful single-thread restatement of the reference engine; reference JVM "
                      f"unavailable on the box)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    sa = importlib.import_module("siddhi-1_amd")
    synth = importlib.import_module("siddhi-1_amd.synth")
    app = sa.parse_app(synth.C2_QUERY)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    B, K = args.batch, args.keys
    eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=B, partial_capacity=64,
                          match_capacity=2 * B, device=local, flags=sa.native.SG_CFG_TIMING)

    # inputs resident in HBM before timing: one independent stream per rank (its own key shard)
    total = args.warmup + args.steps
    seed = synth.SEED + 7919 * rank
    batches = []
    for s in range(total):
        d = synth.stock_ticks(s * B, B, K, seed=seed)
        batches.append({k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev)
                        for k, v in d.items()})
    torch.cuda.synchronize()

    def step(s):
        t = batches[s]
        eng.push(0, s * B, (B, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                    t["volume"].data_ptr()], t["key"].data_ptr()),
                 [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
        m = eng.poll_device()
        eng.release(m)
        return int(m.n) if hasattr(m, "n") else 0

    for s in range(args.warmup):
        step(s)
    eng.synchronize()
    st0 = eng.stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, total):
        step(s)
    eng.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    st1 = eng.stats()
    el = t1 - t0
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    dst = delta(st0, st1)
    events_all = B * args.steps * world
    value = events_all / el

    launches = max(1, dst["advance_launches"])
    adv_s = dst["advance_ns"] / 1e9 / launches
    alg = algorithmic_bytes(dst) / launches
    achieved = alg / adv_s / 1e9 if adv_s > 0 else 0.0
    out = {
        "metric": "input events/sec, partitioned pattern query, 1/2/4/8 GPU; % of HBM roofline",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (splitmix64 stock ticks, seeded, HBM-resident)",
        "config": {"workload": "C2: every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] "
                               "within 10 sec, partition with (symbol of StockStream)",
                   "keys_per_gpu": K, "batch_events": B, "events_per_ms": 2000,
                   "parallelism": f"key-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "k_p2_advance", "alg_bytes_per_launch": alg,
                     "kernel_ms_per_launch": adv_s * 1e3},
        "stages_ms_per_step": {"group": dst["group_ns"] / 1e6 / args.steps,
                               "advance": dst["advance_ns"] / 1e6 / args.steps,
                               "order": dst["order_ns"] / 1e6 / args.steps},
        "work_per_step": {k: dst[k] / args.steps for k in ("matches", "partials_created", "partials_scanned",
                                                           "keys_touched", "live_at_batch_start")},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(sa, synth, K, B, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
