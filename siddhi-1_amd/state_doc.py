"""The NFA state in the reference's per-state-processor form (sg_state_export / sg_state_import).

The engines write a flat document (layout: `csrc/state_doc.h`): per initialised partition key, each
pre-state processor's lists of StateEvents and its flags, the StateEvents and StreamEvents numbered once
so that shared references survive.  This module reads and writes that document and turns it into the
nested map the reference persists (PartitionStateHolder.java:37-80):

    {partition key: {processor id: {"FirstEvent": None,
                                    "PendingStateEventList": [StateEvent, ...],
                                    "NewAndEveryStateEventList": [StateEvent, ...],
                                    "Initialized": bool, "Started": bool,
                                    + count: "SuccessCondition", "StartStateReset"
                                    + absent stream: "IsActive", "LastScheduledTime"
                                    + absent logical: "IsActive", "LastArrivalTime"},
                     "Scheduler:<processor id>": {"ToNotifyQueue": [...]}}}

(StreamPreStateProcessor.java:450-469, CountPreStateProcessor.java:206-219,
AbsentStreamPreStateProcessor.java:328-341, AbsentLogicalPreStateProcessor.java:407-420,
Scheduler.java:331-368).  StateEvent / StreamEvent objects are shared exactly as the document shares them.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional

MAGIC = 0x44534753
VERSION = 1
INITIALIZED, STARTED, SUCCESS, SSRESET, ACTIVE = 1, 2, 4, 8, 16


@dataclass
class DocStream:
    seq: int
    ts: int
    null_bits: int = 0
    present: int = 0
    attr: List[int] = field(default_factory=list)


@dataclass
class DocState:
    ts: int
    type: int
    chains: List[List[int]]


@dataclass
class DocProc:
    flags: int = 0
    last_scheduled: int = 0
    last_arrival: int = 0
    pending: List[int] = field(default_factory=list)
    newev: List[int] = field(default_factory=list)
    queue: List[int] = field(default_factory=list)
    running: int = 0
    fire_at: int = 0
    order: int = 0


@dataclass
class DocKey:
    key: int
    streams: List[DocStream] = field(default_factory=list)
    states: List[DocState] = field(default_factory=list)
    procs: List[DocProc] = field(default_factory=list)


@dataclass
class ProcDesc:
    kind: int     # 0 stream, 1 count, 2 logical
    absent: int
    slot: int


KIND_NAMES = {0: "Stream", 1: "Count", 2: "Logical"}


@dataclass
class StateDoc:
    n_procs: int
    n_slots: int
    desc: List[ProcDesc] = field(default_factory=list)
    now: int = 0
    last_event_ts: int = 0
    clock_flags: int = 0
    keys: List[DocKey] = field(default_factory=list)


class _R:
    def __init__(self, b: bytes):
        self.b, self.o = b, 0

    def get(self, fmt):
        v = struct.unpack_from("<" + fmt, self.b, self.o)
        self.o += struct.calcsize("<" + fmt)
        return v[0] if len(v) == 1 else v

    def arr(self, fmt, n):
        if n == 0:
            return []
        v = list(struct.unpack_from(f"<{n}{fmt}", self.b, self.o))
        self.o += struct.calcsize(f"<{n}{fmt}")
        return v


def parse(b: bytes) -> StateDoc:
    r = _R(bytes(b))
    magic, ver, n_procs, n_slots = r.get("IIII")
    if magic != MAGIC or ver != VERSION:
        raise ValueError("not a state document of this version")
    d = StateDoc(n_procs, n_slots)
    d.desc = [ProcDesc(*r.get("III")) for _ in range(n_procs)]
    d.now, d.last_event_ts, d.clock_flags = r.get("qqQ")
    for _ in range(r.get("I")):
        key, ns, nt = r.get("III")
        k = DocKey(key)
        for _ in range(ns):
            seq, ts, nb, present, na = r.get("QqIII")
            k.streams.append(DocStream(seq, ts, nb, present, r.arr("Q", na)))
        for _ in range(nt):
            ts, typ = r.get("qI")
            chains = [r.arr("I", r.get("I")) for _ in range(n_slots)]
            k.states.append(DocState(ts, typ, chains))
        for _ in range(n_procs):
            p = DocProc()
            p.flags, p.last_scheduled, p.last_arrival = r.get("Iqq")
            p.pending = r.arr("I", r.get("I"))
            p.newev = r.arr("I", r.get("I"))
            p.queue = r.arr("q", r.get("I"))
            p.running, p.fire_at, p.order = r.get("IqQ")
            k.procs.append(p)
        d.keys.append(k)
    if r.o != len(r.b):
        raise ValueError("state document has trailing bytes")
    return d


def write(d: StateDoc) -> bytes:
    out = [struct.pack("<IIII", MAGIC, VERSION, d.n_procs, d.n_slots)]
    for x in d.desc:
        out.append(struct.pack("<III", x.kind, x.absent, x.slot))
    out.append(struct.pack("<qqQI", d.now, d.last_event_ts, d.clock_flags, len(d.keys)))
    for k in d.keys:
        out.append(struct.pack("<III", k.key, len(k.streams), len(k.states)))
        for s in k.streams:
            out.append(struct.pack(f"<QqIII{len(s.attr)}Q", s.seq & (2**64 - 1), s.ts, s.null_bits, s.present,
                                   len(s.attr), *s.attr))
        for s in k.states:
            out.append(struct.pack("<qI", s.ts, s.type))
            for c in s.chains:
                out.append(struct.pack(f"<I{len(c)}I", len(c), *c))
        for p in k.procs:
            out.append(struct.pack("<Iqq", p.flags, p.last_scheduled, p.last_arrival))
            out.append(struct.pack(f"<I{len(p.pending)}I", len(p.pending), *p.pending))
            out.append(struct.pack(f"<I{len(p.newev)}I", len(p.newev), *p.newev))
            out.append(struct.pack(f"<I{len(p.queue)}q", len(p.queue), *p.queue))
            out.append(struct.pack("<IqQ", p.running, p.fire_at, p.order))
    return b"".join(out)


def logical(d: StateDoc, seed_ts=False):
    """Engine-independent view for comparisons: per key, per processor, the lists as tuples
    (ts, type, ((seq, ts) chain per slot)); StateEvent sharing between lists as index pairs.  The
    two-state kernel does not keep a start-state seed's timestamp: seed_ts=False drops it."""
    out = {}
    for k in d.keys:
        def st(i):
            s = k.states[i]
            chains = tuple(tuple((k.streams[x].seq, k.streams[x].ts) for x in c) for c in s.chains)
            empty = all(len(c) == 0 for c in s.chains)
            return (None if (empty and not seed_ts) else s.ts, s.type, chains)
        procs = []
        where = {}
        for pi, p in enumerate(k.procs):
            for li, lst in enumerate((p.pending, p.newev)):
                for x in lst:
                    where.setdefault(x, []).append((pi, li))
            procs.append((p.flags, p.last_scheduled, p.last_arrival, tuple(st(x) for x in p.pending),
                          tuple(st(x) for x in p.newev), tuple(p.queue), p.running, p.fire_at, p.order))
        shared = tuple(sorted(tuple(v) for v in where.values() if len(v) > 1))
        out[k.key] = (tuple(procs), shared)
    return out


# ---- the reference's nested map ------------------------------------------------------------------------
class StreamEventState:
    """io.siddhi.core.event.stream.StreamEvent as persisted: timestamp, data; `seq` is the engine's arrival
    number of the event (the host event store resolves it)."""
    __slots__ = ("seq", "timestamp", "data", "next", "stream")

    def __init__(self, seq, timestamp, data, nxt=None, stream=None):
        self.seq, self.timestamp, self.data, self.next, self.stream = seq, timestamp, data, nxt, stream

    def __repr__(self):
        return f"StreamEvent(seq={self.seq}, ts={self.timestamp}, data={self.data})"


class StateEventState:
    """io.siddhi.core.event.state.StateEvent as persisted: timestamp, type, one StreamEvent chain head
    per slot (StateEvent.java:42-258)"""
    __slots__ = ("timestamp", "type", "stream_events")

    def __init__(self, timestamp, typ, stream_events):
        self.timestamp, self.type, self.stream_events = timestamp, typ, stream_events

    def chain(self, slot) -> List[StreamEventState]:
        out, e = [], self.stream_events[slot]
        while e is not None:
            out.append(e)
            e = e.next
        return out

    def __repr__(self):
        return (f"StateEvent(ts={self.timestamp}, type={'EXPIRED' if self.type else 'CURRENT'}, "
                f"slots={[self.chain(s) for s in range(len(self.stream_events))]})")


def proc_names(desc: List[ProcDesc], slot_name=lambda s: f"slot{s}"):
    """element id of each pre-state processor: its class and the state (event reference) it owns"""
    return [f"{'Absent' if x.absent else ''}{KIND_NAMES.get(x.kind, 'Stream')}PreStateProcessor:{slot_name(x.slot)}"
            for x in desc]


def to_reference_map(d: StateDoc, key_name=str, event_data=None, slot_name=lambda s: f"slot{s}", slot_stream=None):
    """key_name(key id) -> partition key String; event_data(DocStream, slot) -> the event's attribute values
    (None: the document's value bits); slot_stream(slot) -> stream name recorded on each StreamEvent."""
    names = proc_names(d.desc, slot_name)
    out = {}
    for k in d.keys:
        evs = [StreamEventState(s.seq, s.ts, None) for s in k.streams]
        filled = [False] * len(evs)
        sts = []
        for s in k.states:
            for sl, c in enumerate(s.chains):
                for x in c:
                    if not filled[x]:
                        filled[x] = True
                        ds = k.streams[x]
                        evs[x].data = event_data(ds, sl) if event_data else list(ds.attr)
                        evs[x].stream = slot_stream(sl) if slot_stream else sl
                for a, b in zip(c, c[1:]):
                    evs[a].next = evs[b]
            sts.append(StateEventState(s.ts, s.type, [evs[c[0]] if c else None for c in s.chains]))
        m = {}
        for name, x, p in zip(names, d.desc, k.procs):
            st = {"FirstEvent": None,
                  "PendingStateEventList": [sts[i] for i in p.pending],
                  "NewAndEveryStateEventList": [sts[i] for i in p.newev],
                  "Initialized": bool(p.flags & INITIALIZED), "Started": bool(p.flags & STARTED)}
            if x.kind == 1:
                st["SuccessCondition"] = bool(p.flags & SUCCESS)
                st["StartStateReset"] = bool(p.flags & SSRESET)
            if x.absent:
                st["IsActive"] = bool(p.flags & ACTIVE)
                if x.kind == 2:
                    st["LastArrivalTime"] = p.last_arrival
                else:
                    st["LastScheduledTime"] = p.last_scheduled
                sch = {"ToNotifyQueue": list(p.queue)}
                if p.running:   # the wall-clock EventCaller scheduled for this key (Scheduler.java:238-298)
                    sch["EventCaller"] = {"FireAt": p.fire_at, "Order": p.order}
                m[f"Scheduler:{name}"] = sch
            m[name] = st
        out[key_name(k.key)] = m
    return out


def from_reference_map(states, desc: List[ProcDesc], n_slots, key_id, event_bits, slot_name=lambda s: f"slot{s}",
                       now=0, last_event_ts=0, clock_flags=1) -> StateDoc:
    """The inverse of to_reference_map: key_id(partition key String) -> dense key id;
    event_bits(StreamEventState) -> (attribute value bits, null bits, present mask)."""
    names = proc_names(desc, slot_name)
    d = StateDoc(len(desc), n_slots, list(desc), now, last_event_ts, clock_flags)
    for pk, m in states.items():
        k = DocKey(key_id(pk))
        st_ix, ev_ix = {}, {}

        def ev(e):
            if id(e) in ev_ix:
                return ev_ix[id(e)]
            bits, nb, present = event_bits(e)
            k.streams.append(DocStream(e.seq, e.timestamp, nb, present, list(bits)))
            ev_ix[id(e)] = len(k.streams) - 1
            return ev_ix[id(e)]

        def state(s):
            if id(s) in st_ix:
                return st_ix[id(s)]
            k.states.append(DocState(s.timestamp, s.type, []))
            i = len(k.states) - 1
            st_ix[id(s)] = i
            k.states[i].chains = [[ev(x) for x in s.chain(sl)] for sl in range(n_slots)]
            return i

        for name in names:
            st = m.get(name, {})
            p = DocProc()
            p.flags = ((INITIALIZED if st.get("Initialized") else 0) | (STARTED if st.get("Started") else 0) |
                       (SUCCESS if st.get("SuccessCondition") else 0) | (SSRESET if st.get("StartStateReset") else 0) |
                       (ACTIVE if st.get("IsActive", True) else 0))
            p.last_scheduled = int(st.get("LastScheduledTime", 0))
            p.last_arrival = int(st.get("LastArrivalTime", 0))
            p.pending = [state(s) for s in st.get("PendingStateEventList", [])]
            p.newev = [state(s) for s in st.get("NewAndEveryStateEventList", [])]
            sch = m.get(f"Scheduler:{name}", {})
            p.queue = list(sch.get("ToNotifyQueue", []))
            if "EventCaller" in sch:
                p.running, p.fire_at, p.order = 1, int(sch["EventCaller"]["FireAt"]), int(sch["EventCaller"]["Order"])
            k.procs.append(p)
        d.keys.append(k)
    d.keys.sort(key=lambda x: x.key)
    return d
