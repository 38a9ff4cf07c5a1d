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


@pytest.mark.parametrize("shape", ["two_state", "count"])
def test_rejected_batch_retried_at_the_same_seq_base(shape):
    """a rejected host batch changes no engine state: the caller fixes its keys and pushes it again at
    the SAME seq_base, and the result equals an engine that only ever saw the good batches"""
    e, ref = _engine(shape), _engine(shape)
    d0 = synth.stock_ticks(0, N, NK)
    d1 = synth.stock_ticks(N, N, NK)
    bad = {k: v.copy() for k, v in d1.items()}
    bad["key"][7] = NK + 5
    _push_host(e, 0, d0)
    with pytest.raises(sa.EngineError):
        _push_host(e, N, bad)
    _push_host(e, N, d1)                         # same seq_base: accepted
    for s, d in ((0, d0), (N, d1)):
        _push_host(ref, s, d)
    _same(e.poll(), ref.poll())
    assert e.stats()["events"] == ref.stats()["events"] == 2 * N
    e.close()
    ref.close()


@pytest.mark.parametrize("shape", ["two_state", "count"])
def test_device_batch_key_range_reported_once(shape):
    """a DEVICE batch with an out-of-range key is found on the device: the next poll reports it (the
    valid keys' events were processed), later polls work again"""
    dev = torch.device("cuda", 0)
    e = _engine(shape)
    d = synth.stock_ticks(0, N, NK)
    d["key"][11] = NK
    t = {k: torch.from_numpy(v.view(np.int32) if v.dtype == np.uint32 else v).to(dev) for k, v in d.items()}
    torch.cuda.synchronize()
    e.push(0, 0, (N, t["ts"].data_ptr(), [t["symbol"].data_ptr(), t["price"].data_ptr(), t["volume"].data_ptr()],
                  t["key"].data_ptr()), [0, 1, 2], mem=sa.native.SG_MEM_DEVICE)
    with pytest.raises(sa.EngineError, match="n_keys"):
        e.poll()
    d2 = synth.stock_ticks(N, N, NK)
    _push_host(e, N, d2)
    e.poll()                                     # no error left behind
    e.close()


@pytest.mark.parametrize("shape", ["two_state", "count"])
def test_reset_keys_device_ids_validated_first(shape):
    """sg_reset_keys with device-memory ids: one id == n_keys fails with SG_ERR_INVALID before any key is
    reset (the general engine's k_gen_reset would otherwise write outside the key's block)"""
    dev = torch.device("cuda", 0)
    e, ref = _engine(shape), _engine(shape)
    d0 = synth.stock_ticks(0, N, NK)
    for x in (e, ref):
        _push_host(x, 0, d0)
        x.poll()
    ids = torch.tensor([3, 9, NK], dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    f = e.lib.sg_reset_keys
    import ctypes as C
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32]
    assert f(e.h, C.c_void_p(ids.data_ptr()), 3, sa.native.SG_MEM_DEVICE) == -1
    d1 = synth.stock_ticks(N, N, NK)
    for x in (e, ref):
        _push_host(x, N, d1)
    _same(e.poll(), ref.poll())                  # nothing was reset
    ok = torch.tensor([3, 9], dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    assert f(e.h, C.c_void_p(ok.data_ptr()), 2, sa.native.SG_MEM_DEVICE) == 0
    ref.reset_keys(np.array([3, 9], dtype=np.uint32))
    d2 = synth.stock_ticks(2 * N, N, NK)
    for x in (e, ref):
        _push_host(x, 2 * N, d2)
    _same(e.poll(), ref.poll())
    e.close()
    ref.close()
