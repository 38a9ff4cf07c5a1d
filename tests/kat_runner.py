"""Replay a transcribed reference KAT (tests/golden/kat/*.json) through the host API and check it.

The fixtures hold the reference tests' inputs and hard-coded expected outputs (see make_kat.py).
"""
import glob
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
KAT_DIR = os.path.join(HERE, "golden", "kat")

_TYPE_OF = {"FLOAT": "float", "DOUBLE": "double", "INT": "int", "LONG": "long", "STRING": "string",
            "BOOL": "bool"}


def load_cases(files=None):
    out = []
    for f in sorted(glob.glob(os.path.join(KAT_DIR, "*.json"))):
        base = os.path.splitext(os.path.basename(f))[0]
        if files and base not in files:
            continue
        d = json.load(open(f))
        for c in d["cases"]:
            out.append((base, c))
    return out


def py_value(v):
    if v is None:
        return None
    t = v["t"]
    if t == "float":
        return np.float32(v["v"])
    return v["v"]


def same(exp, act):
    if exp is None or act is None:
        return exp is None and act is None
    t = exp["t"]
    if t == "list":   # a count state's attribute over its chain (List / Object[] compared element-wise)
        return isinstance(act, (list, tuple)) and len(act) == len(exp["v"]) and \
            all(same(e, a) for e, a in zip(exp["v"], act))
    if t in ("float", "double"):
        a = np.float32(act) if t == "float" else float(act)
        e = np.float32(exp["v"]) if t == "float" else float(exp["v"])
        return bool(a == e) or (np.isnan(a) and np.isnan(e))
    if t in ("int", "long"):
        return isinstance(act, (int, np.integer)) and not isinstance(act, bool) and int(act) == exp["v"]
    if t == "bool":
        return bool(act) == exp["v"]
    return act == exp["v"]


class Recorder:
    def __init__(self):
        self.calls = []     # list of list[Event]

    def events(self):
        return [e for c in self.calls for e in c]


def run_case(case, manager):
    """Returns (ok, message)."""
    from importlib import import_module
    sa = import_module("siddhi-1_amd")
    rt = manager.createSiddhiAppRuntime(case["app"])
    recs = []
    for cb in case["callbacks"]:
        rec = Recorder()
        if cb["kind"] == "QueryCallback":
            class QC(sa.QueryCallback):
                def receive(self, ts, ins, rem, rec=rec):
                    if ins:
                        rec.calls.append(list(ins))
            rt.addCallback(cb["target"], QC())
        else:
            class SC(sa.StreamCallback):
                def receive(self, evs, rec=rec):
                    rec.calls.append(list(evs))
            rt.addCallback(cb["target"], SC())
        recs.append(rec)
    # virtual wall clock: Thread.sleep / waitFor* steps of the reference test advance it, so absent
    # states' timers fire at the same virtual times as in the Java test
    clock = case.get("start_clock", 1_000_000)
    rt.set_wall_clock(clock)
    rt.start()

    def in_count():
        cb = case["callbacks"][0]
        return len(recs[0].events()) if cb.get("count_per") == "event" or cb.get("testutil") else len(recs[0].calls)

    for s in case["sends"]:
        if "sleep" in s:
            clock += s["sleep"]
            rt.advance_wall_clock(clock)
            continue
        if "wait_in" in s:   # TestUtil.waitForInEvents: until exactly one in-event arrived or retries run out
            w = s["wait_in"]
            for _ in range(w["retry"]):
                clock += w["sleep"]
                rt.advance_wall_clock(clock)
                if in_count() == 1:
                    break
            continue
        if "wait_count" in s:  # SiddhiTestHelper.waitForEvents(sleep, expected, counter, timeout)
            w = s["wait_count"]
            waited = 0
            while in_count() < w["expected"] and waited < w["timeout"]:
                clock += w["sleep"]
                waited += w["sleep"]
                rt.advance_wall_clock(clock)
            continue
        ih = rt.getInputHandler(s["stream"])
        if "batch" in s:
            ih.send([sa.Event(e["ts"], [py_value(x) for x in e["data"]]) for e in s["batch"]])
        elif s.get("wall"):
            ih.send([py_value(x) for x in s["data"]])
        else:
            ih.send(s["ts"], [py_value(x) for x in s["data"]])
    rt.shutdown()
    msgs = []
    for cb, rec in zip(case["callbacks"], recs):
        evs = rec.events()
        if "ordered" in cb:
            for k, spec in cb["ordered"].items():
                i = int(k) - 1
                if i >= len(evs):
                    if not cb.get("testutil"):  # TestUtil callbacks check only the events that arrive
                        msgs.append(f"{cb['target']}: expected event #{k}, only {len(evs)} arrived")
                    continue
                d = evs[i].data
                if "row" in spec:
                    row = spec["row"]
                    if len(row) != len(d) or not all(same(e, a) for e, a in zip(row, d)):
                        msgs.append(f"{cb['target']}: event #{k} = {d}, expected {[py_value(x) for x in row]}")
                else:
                    for ci, e in spec["cols"].items():
                        if not same(e, d[int(ci)]):
                            msgs.append(f"{cb['target']}: event #{k} col {ci} = {d[int(ci)]}, expected {e}")
        if "first_of_each_call" in cb:
            row = cb["first_of_each_call"]
            for c in rec.calls:
                d = c[0].data
                if len(row) != len(d) or not all(same(e, a) for e, a in zip(row, d)):
                    msgs.append(f"{cb['target']}: call first event {d}, expected {[py_value(x) for x in row]}")
                    break
        if "first_at_count" in cb:
            cum = 0
            seen = set()
            for c in rec.calls:
                cum += len(c) if cb.get("count_per") == "event" else 1
                if str(cum) in cb["first_at_count"]:
                    seen.add(str(cum))
                    row = cb["first_at_count"][str(cum)]
                    d = c[0].data
                    if len(row) != len(d) or not all(same(e, a) for e, a in zip(row, d)):
                        msgs.append(f"{cb['target']}: at count {cum} first event {d}, "
                                    f"expected {[py_value(x) for x in row]}")
            for k in cb["first_at_count"]:
                if k not in seen:
                    msgs.append(f"{cb['target']}: cumulative count never reached {k}")
        if "every_event" in cb:
            row = cb["every_event"]
            for e_ in evs:
                if len(row) != len(e_.data) or not all(same(e, a) for e, a in zip(row, e_.data)):
                    msgs.append(f"{cb['target']}: event {e_.data}, expected {[py_value(x) for x in row]}")
                    break
    # counts refer to the (single) counting callback of the test
    exp = case.get("expect", {})
    if "in" in exp and recs:
        cb = case["callbacks"][0]
        n = len(recs[0].events()) if cb.get("count_per") == "event" else len(recs[0].calls)
        if len(case["callbacks"]) > 1:
            n = sum(len(r.events()) for r in recs) if cb.get("count_per") == "event" else \
                sum(len(r.calls) for r in recs)
        if n != exp["in"]:
            msgs.append(f"in-event count {n}, expected {exp['in']}")
    if exp.get("arrived") is False and any(r.calls for r in recs):
        msgs.append("events arrived, expected none")
    if exp.get("arrived") is True and not any(r.calls for r in recs):
        msgs.append("no event arrived")
    return (not msgs), "; ".join(msgs)
