"""One rank of the multi-GPU ingest rehearsal (tests/test_gpu_multirank.py): this rank's slice of every
step of the global arrival-ordered C2-shaped stream -> BlockResharder (HIP pack into fixed destination
blocks, all_to_all, unpack into a padded batch) -> this rank's engine (SG_CFG_NULL_KEYS) -> matches.
Writes, per step, (global trigger index, global e1 index, global key) of every match to <out>/rank<r>.npy.
Every rank may run on the same GPU (SG_BENCH_DEVICE) with the gloo backend (exchange through host memory)."""
import importlib
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
reshard = importlib.import_module("siddhi-1_amd.reshard")


def main():
    out_dir, K, B, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("SG_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group(os.environ.get("SG_BENCH_BACKEND", "gloo"))
    app = sa.parse_app(synth.C2_QUERY.replace("within 10 sec", "within 1 sec"))
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    lib = sa.load_hip_library()
    rs = reshard.BlockResharder(lib, B, world, ["price", "volume", "gidx"], [torch.float32, torch.int32, torch.int32],
                                dev)
    eng = sa.NativeEngine(lib, "sg_", cq.ir, n_keys=K, max_batch=world * rs.cap, partial_capacity=64,
                          match_capacity=4 * world * rs.cap, device=local, flags=sa.native.SG_CFG_NULL_KEYS)
    import ctypes as C
    lib.sg_wait_stream.argtypes = [C.c_void_p, C.c_void_p]
    rows, hist = [], []
    seq = 0
    for s in range(steps):
        base = s * world * B + rank * B
        d = synth.stock_ticks(base, B, K * world, rate_per_ms=8 * world)
        gidx = np.arange(base, base + B, dtype=np.int64).astype(np.int32)
        t = {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev) for k, v in d.items()}
        t["gidx"] = torch.from_numpy(gidx).to(dev)
        g = rs({"key": t["key"], "ts": t["ts"], "price": t["price"], "volume": t["volume"], "gidx": t["gidx"]})
        assert lib.sg_wait_stream(eng.h, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) == 0
        n = g["key"].numel()
        eng.push(0, seq, (n, g["ts"].data_ptr(), [g["key"].data_ptr(), g["price"].data_ptr(), g["volume"].data_ptr()],
                          g["key"].data_ptr()), [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
        m = eng.poll()
        gi = g["gidx"].cpu().numpy().astype(np.int64)
        trig = gi[(m.trigger_seq.astype(np.int64) - seq)]
        e1_local = m.slot_seq[:, 0, 0].astype(np.int64)
        e1 = np.empty_like(e1_local)
        # e1 may come from an earlier step: map through this rank's per-step gidx history
        hist.append((seq, gi))
        for s0, g0 in hist:
            sel = (e1_local >= s0) & (e1_local < s0 + len(g0))
            e1[sel] = g0[e1_local[sel] - s0]
        key = m.key.astype(np.int64) * world + rank
        rows.append(np.stack([trig, e1, key], axis=1))
        seq += n
    rs.check()
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), np.concatenate(rows) if rows else np.zeros((0, 3), np.int64))
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
