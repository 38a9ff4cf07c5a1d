"""Pipelined pushes (two-state kernel): batch i + 1's copies and grouping run on the engine's grouping
stream while batch i advances; SG_POLL_READY polls hand out the complete batches' matches without
waiting; the ordered records form a ring of match_capacity entries that windows wrap around.

Every variant must give exactly the matches (same order) of one blocking push + poll per batch.
"""
import importlib

import numpy as np
import pytest

from test_gpu_parity import _same
from test_purge import SHAPES

sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")
native = importlib.import_module("siddhi-1_amd.native")

pytestmark = pytest.mark.gpu

NK, N, NB = 256, 4096, 12
SG_ERR_CAPACITY = -4


def _engine(mcap, flags=0):
    app = sa.parse_app(SHAPES["two_state"])
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    return sa.NativeEngine(sa.load_hip_library(), "sg_", cq.ir, n_keys=NK, max_batch=N, partial_capacity=64,
                           match_capacity=mcap, flags=flags)


def _batches():
    return [synth.stock_ticks(b * N, N, NK) for b in range(NB)]


def _push(e, b, d):
    e.push(0, b * N, d["ts"], [d["symbol"], d["price"], d["volume"]], None, d["key"])


def _cat(ms):
    ms = [m for m in ms if len(m)]
    return sa.native.Matches(*[np.concatenate([getattr(m, f) for m in ms]) for f in
                               ("trigger_seq", "key", "ts", "slot_seq", "chain_len")])


def _reference(bats):
    e = _engine(1 << 18)
    per = []
    for b, d in enumerate(bats):
        _push(e, b, d)
        per.append(e.poll())
    e.close()
    return per


def test_ready_polls_with_async_host_pushes_wrap_the_ring():
    bats = _batches()
    per = _reference(bats)
    big = max(len(m) for m in per)
    assert big > 0
    # odd size: windows wrap the ring at arbitrary positions; with two batches in flight and ready polls
    # between pushes, at most three batches' matches are pending
    mcap = 3 * big + 17
    e = _engine(mcap, flags=native.SG_CFG_ASYNC_HOST)
    got = []
    for b, d in enumerate(bats):
        _push(e, b, d)
        got.append(e.poll(ready=True))     # the batches complete so far (possibly none)
    e.synchronize()
    got.append(e.poll())
    assert len(e.poll()) == 0
    _same(_cat(got), _cat(per))
    e.close()


def test_device_polls_hand_a_wrapped_window_out_in_two_parts():
    bats = _batches()
    per = _reference(bats)
    mcap = max(len(m) for m in per) + 5
    e = _engine(mcap)
    pos = 0
    for b, d in enumerate(bats):
        _push(e, b, d)
        got = 0
        while True:
            m = e.poll_device()
            n = int(m.n)
            start = pos % mcap
            assert n <= mcap - start      # one contiguous run of the ring per poll
            e.release(m)
            pos += n
            got += n
            if n == 0:
                break
        assert got == len(per[b])
    e.close()


def test_host_poll_of_a_wrapped_window_is_whole():
    bats = _batches()
    per = _reference(bats)
    mcap = max(len(m) for m in per) + 5
    e = _engine(mcap)
    got = []
    for b, d in enumerate(bats):
        _push(e, b, d)
        m = e.poll()
        assert len(m) == len(per[b])
        got.append(m)
    _same(_cat(got), _cat(per))
    e.close()


def test_match_capacity_counts_unpolled_batches():
    bats = _batches()
    per = _reference(bats)
    mcap = max(len(m) for m in per) + 5
    e = _engine(mcap)
    with pytest.raises(sa.EngineError) as ex:
        for b, d in enumerate(bats[:4]):   # nothing polled: the pending windows exceed the ring
            _push(e, b, d)
        e.poll()
    assert ex.value.code == SG_ERR_CAPACITY
    e.close()
