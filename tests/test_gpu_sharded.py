"""ShardedEngine over HIP engines (two shards on device 0, or one per device when the box has more)
against one HIP engine, bit-exact, incl. purge, snapshot/restore and playback timers; the runtime API
with SiddhiManager(devices=...)."""
import importlib

import pytest
import torch

from test_sharded import SHAPES, run_property

sa = importlib.import_module("siddhi-1_amd")

pytestmark = pytest.mark.gpu


def _devices():
    n = torch.cuda.device_count()
    return tuple(range(min(n, 4))) if n > 1 else (0, 0)


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_sharded_hip_equals_single(shape):
    run_property(shape, sa.load_hip_library(), "sg_", devices=_devices())


def test_null_keys_are_dropped():
    """SG_CFG_NULL_KEYS: SG_KEY_NULL events are dropped (the reshard's padding), the rest is processed as
    if they were never there; a power-of-two key count still sorts them after every valid key"""
    import numpy as np
    synth = importlib.import_module("siddhi-1_amd.synth")
    from test_gpu_parity import _same
    for shape in ("two_state", "count"):
        app = sa.parse_app(SHAPES[shape])
        cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
        K, n = 1024, 20000
        mk = lambda fl: sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=K, max_batch=n,
                                        partial_capacity=64, match_capacity=1 << 20, flags=fl)
        a, b = mk(sa.native.SG_CFG_NULL_KEYS), mk(0)
        d = synth.stock_ticks(0, n, K, rate_per_ms=8)
        keep = np.random.default_rng(1).random(n) < 0.8
        kn = d["key"].copy()
        kn[~keep] = 0xFFFFFFFF
        a.push(0, 0, d["ts"], [d["symbol"], d["price"], d["volume"]], None, kn)
        ma = a.poll()
        # the same events without the dropped ones, at their own seqs
        idx = np.nonzero(keep)[0]
        starts = np.concatenate([[0], np.nonzero(np.diff(idx) != 1)[0] + 1])
        ends = np.concatenate([starts[1:], [len(idx)]])
        for s, t in zip(starts, ends):
            sl = idx[s:t]
            b.push(0, int(sl[0]), d["ts"][sl], [d["symbol"][sl], d["price"][sl], d["volume"][sl]], None, d["key"][sl])
        mb = b.poll()
        assert len(ma) > 100
        _same(ma, mb)
