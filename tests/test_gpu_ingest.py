"""Host-memory ingest through the C-ABI (sg_batch.mem = SG_MEM_HOST) on both device kernels.

A host batch whose key ids leave [0, n_keys) fails at push with SG_ERR_INVALID (the range check runs
after the H2D copies are queued, and waits for them before returning), the engine keeps working, and a
host batch gives the same matches as the same batch pushed from device memory.
"""
import importlib

import numpy as np
import pytest
import torch

from test_gpu_parity import _same
from test_purge import SHAPES

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")

pytestmark = pytest.mark.gpu

NK, N = 256, 4096


def _engine(shape):
    app = sa.parse_app(SHAPES[shape])
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    return sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=NK, max_batch=N, partial_capacity=64,
                           match_capacity=1 << 18)


def _push_host(e, seq, d):
    e.push(0, seq, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])


@pytest.mark.parametrize("shape", ["two_state", "count"])
def test_host_batch_key_range_fails_at_push_and_engine_recovers(shape):
    e = _engine(shape)
    d0 = synth.stock_ticks(0, N, NK)
    bad = {k: v.copy() for k, v in synth.stock_ticks(N, N, NK).items()}
    bad["key"][N // 2] = NK          # one key just past the range
    d2 = synth.stock_ticks(2 * N, N, NK)
    _push_host(e, 0, d0)
    with pytest.raises(sa.EngineError) as ex:
        _push_host(e, N, bad)
    assert ex.value.code == -1 and "n_keys" in str(ex.value)
    _push_host(e, 2 * N, d2)
    m = e.poll()

    ref = _engine(shape)
    _push_host(ref, 0, d0)
    _push_host(ref, 2 * N, d2)
    _same(m, ref.poll())
    e.close()
    ref.close()


@pytest.mark.parametrize("shape", ["two_state", "count"])
def test_host_and_device_batches_agree(shape):
    dev = torch.device("cuda", 0)
    eh, ed = _engine(shape), _engine(shape)
    for s in range(3):
        d = synth.stock_ticks(s * N, N, NK)
        _push_host(eh, s * N, d)
        t = {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev) for k, v in d.items()}
        torch.cuda.synchronize()
        ed.push(0, s * N, (N, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(),
                                                   t["volume"].data_ptr()], t["key"].data_ptr()),
                [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
        ed.synchronize()
        _same(eh.poll(), ed.poll())
    eh.close()
    ed.close()
