"""A stream the partition does not key, inside a partition: each of its events goes to
every partition key known at that moment, the whole chunk per key, and creates no key
(PartitionStreamReceiver.receive -> send(ComplexEvent), C/partition/PartitionStreamReceiver.java:83-92,
275-283).  Pinned by the reference's PatternPartitionTestCase.testPatternPartitionQuery30 (one key, in
the KAT suite) and here, hand-worked, with several keys and a key that appears only later."""
import importlib

from oracle_backend import oracle_manager

sa = importlib.import_module("siddhi-1_amd")

APP = ("define stream Trades (symbol string, price float);\n"
       "define stream Alerts (level int);\n"
       "partition with (symbol of Trades) begin\n"
       "@info(name='q') from every e1=Trades[price > 20] -> e2=Alerts[level > 2] "
       "select e1.symbol as s, e1.price as p, e2.level as l insert into O; end;")


def run(manager, sends):
    rt = manager.createSiddhiAppRuntime(APP)
    got = []
    rt.addCallback("O", lambda evs: got.append([tuple(e.data) for e in evs]))
    rt.start()
    for stream, row in sends:
        h = rt.getInputHandler(stream)
        if isinstance(row, list) and row and isinstance(row[0], sa.Event):
            h.send(row)
        else:
            h.send(list(row))
    rt.shutdown()
    return got


SENDS = [("Alerts", (5,)),              # no key known yet: goes nowhere, creates nothing
         ("Trades", ("A", 25.0)),
         ("Trades", ("B", 30.0)),
         ("Alerts", (1,)),              # to A and B: filter fails
         ("Alerts", (3,)),              # to A and B: both match
         ("Trades", ("C", 21.0)),
         ("Trades", ("A", 26.0)),
         ("Alerts", [sa.Event(0, [4]), sa.Event(0, [9])])]   # a chunk: per key, the whole chunk


def test_broadcast_to_known_keys_on_the_oracle():
    got = run(oracle_manager(), SENDS)
    flat = [r for call in got for r in call]
    assert sorted(flat[:2]) == [("A", 25.0, 3), ("B", 30.0, 3)]
    # the chunk [4, 9]: A (26.0) and C (21.0) have one partial each, both consumed by level 4
    assert sorted(flat[2:]) == [("A", 26.0, 4), ("C", 21.0, 4)]
    assert len(flat) == 4


import pytest  # noqa: E402


@pytest.mark.gpu
def test_broadcast_to_known_keys_on_the_device_equals_oracle():
    from test_gpu_parity import hip_manager
    assert run(hip_manager(), SENDS) == run(oracle_manager(), SENDS)
