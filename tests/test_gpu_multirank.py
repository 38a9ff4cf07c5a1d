"""Multi-GPU ingest rehearsed on one GPU: two ranks (processes) share device 0, each holds
a contiguous slice of every step of the global arrival-ordered stream, reshards it by key through the
fixed-block pack + all_to_all (gloo: through host memory) and runs its own engine on the keys it owns
(SG_CFG_NULL_KEYS drops the block padding).  The union of the ranks' matches, mapped back to global
keys and arrival indices, equals one engine's matches on the whole stream."""
import importlib
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle_backend import ROOT

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu


def test_two_rank_rehearsal_equals_single_engine(tmp_path):
    world, K, B, steps = 2, 4096, 1 << 16, 3
    env = dict(os.environ, SG_BENCH_DEVICE="0", SG_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", "29517",
           os.path.join(ROOT, "tests", "helpers", "shard_rank.py"), str(tmp_path), str(K), str(B), str(steps)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = np.concatenate([np.load(tmp_path / f"rank{i}.npy") for i in range(world)])
    # one engine on the whole stream (global keys)
    app = sa.parse_app(synth.C2_QUERY.replace("within 10 sec", "within 1 sec"))
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    eng = sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K * world, max_batch=world * B,
                          partial_capacity=64, match_capacity=1 << 22)
    want = []
    for s in range(steps):
        n = world * B
        d = synth.stock_ticks(s * n, n, K * world, rate_per_ms=8 * world)
        eng.push(0, s * n, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])
        m = eng.poll()
        want.append(np.stack([m.trigger_seq.astype(np.int64), m.slot_seq[:, 0, 0].astype(np.int64),
                              m.key.astype(np.int64)], axis=1))
    want = np.concatenate(want)
    assert len(want) > 1000
    order = lambda a: a[np.lexsort((a[:, 1], a[:, 0]))]
    np.testing.assert_array_equal(order(got), order(want))


def test_bench_two_rank_rehearsal_with_host_merge():
    """bench.py's N > 1 path rehearsed on one GPU (two ranks on device 0, gloo exchange): the JSON line of
    rank 0 carries the whole-job value and the host timestamp-order merge leg (sg_merge_ts over the ranks'
    /dev/shm segments), and the segments are removed afterwards"""
    import glob
    import json
    env = dict(os.environ, SG_BENCH_DEVICE="0", SG_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29519", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--keys", "4096", "--batch", str(1 << 16), "--no-cpu", "--no-extra"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert "error" not in out["extra"]["merge_inclusive"], out["extra"]
    mg = json.load(open(os.path.join(ROOT, out["detail"])))["merge_inclusive"]   # (the full record beside the line)
    assert "error" not in mg, mg
    assert mg["value"] > 0 and mg["matches_per_step"] > 0 and mg["merge_records_per_s"] > 0
    assert not glob.glob("/dev/shm/sgmerge_29519_*")
