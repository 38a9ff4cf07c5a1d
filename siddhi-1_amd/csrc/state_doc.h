// state_doc.h — the per-key NFA state in the reference's per-state-processor form, as a flat
// document (sg_state_export / sg_state_import, include/siddhi_gpu.h).  Host-only C++.
//
// The reference persists a partitioned pattern query as PartitionStateHolder's map
//   partition key -> (group-by key "") -> State of each pre-state processor
// (C/util/snapshot/state/PartitionStateHolder.java:37-80), where each State snapshots to
//   {FirstEvent, PendingStateEventList, NewAndEveryStateEventList, Initialized, Started}
// (C/query/input/stream/state/StreamPreStateProcessor.java:450-469) plus SuccessCondition /
// StartStateReset for count states (CountPreStateProcessor.java:206-219), IsActive /
// LastScheduledTime for absent stream states (AbsentStreamPreStateProcessor.java:328-341) and IsActive /
// LastArrivalTime for absent logical states (AbsentLogicalPreStateProcessor.java:407-420); the
// Scheduler of an absent state keeps its per-key toNotifyQueue (C/util/Scheduler.java:331-368).  The
// lists hold StateEvent objects that share StreamEvents (and StateEvents between lists), so the
// document numbers every distinct StateEvent and StreamEvent of a key once and the lists refer to them
// by index.  Numbering is canonical — processors in order, pending before newAndEvery, a StateEvent's
// slots in order and each slot's chain in order — so two engines in the same logical state write the
// same bytes (FirstEvent, a transient of one processing call, is always empty between batches).
//
// Layout (little endian): "SGSD" u32 version n_procs n_slots | per processor: u32 kind (0 stream, 1 count,
// 2 logical), absent, slot | i64 now, last_event_ts | u64 clock_flags |
// u32 n_keys | per key: u32 key n_stream n_state | stream events: u64 seq, i64 ts, u32 null_bits,
// u32 present (attribute bitmask), u32 n_attr, u64 attr[n_attr] | state events: i64 ts, u32 type,
// per slot: u32 len, u32 stream_index[len] | per processor: u32 flags, i64 last_scheduled_time,
// i64 last_arrival_time, u32 n_pending, u32 state_index[], u32 n_new, u32 state_index[], u32 n_queue,
// i64 queue[], u32 running, i64 fire_at, u64 order.
#pragma once

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#define SD_MAGIC 0x44534753u  // "SGSD"
#define SD_VERSION 1u

// processor flags
enum {
    SD_INITIALIZED = 1u,   // StreamPreState.initialized
    SD_STARTED = 2u,       // StreamPreState.started
    SD_SUCCESS = 4u,       // CountStreamPreState.successCondition
    SD_SSRESET = 8u,       // CountStreamPreState.startStateReset
    SD_ACTIVE = 16u,       // LogicalStreamPreState.active (absent states)
};

struct SdStream {
    uint64_t seq = 0;
    int64_t ts = -1;
    uint32_t null_bits = 0;
    uint32_t present = 0;            // attributes whose value the document carries
    std::vector<uint64_t> attr;      // value bits per attribute of the event's stream
};

struct SdState {
    int64_t ts = -1;
    uint32_t type = 0;               // 0 CURRENT, 1 EXPIRED
    std::vector<std::vector<uint32_t>> chains;  // per slot: stream-event indices, chain order
};

struct SdProc {
    uint32_t flags = 0;
    int64_t last_scheduled = 0, last_arrival = 0;
    std::vector<uint32_t> pending, newev;   // state-event indices
    std::vector<int64_t> queue;             // Scheduler toNotifyQueue, FIFO order
    uint32_t running = 0;                   // wall clock: an EventCaller is scheduled
    int64_t fire_at = 0;
    uint64_t order = 0;                     // rank of that caller among the key's callers (1-based)
};

struct SdKey {
    uint32_t key = 0;
    std::vector<SdStream> streams;
    std::vector<SdState> states;
    std::vector<SdProc> procs;
};

struct SdProcDesc {
    uint32_t kind = 0, absent = 0, slot = 0;   // the pre-state processor: stream / count / logical, its slot
    bool operator==(const SdProcDesc& o) const { return kind == o.kind && absent == o.absent && slot == o.slot; }
};

struct SdDoc {
    uint32_t n_procs = 0, n_slots = 0;
    std::vector<SdProcDesc> desc;   // [n_procs]
    int64_t now = 0, last_event_ts = 0;
    uint64_t clock_flags = 0;   // bit 0: the engine clock has been set (an event or a time advance)
    std::vector<SdKey> keys;
};

// ---- serialisation -------------------------------------------------------------------------------
struct SdWriter {
    std::vector<uint8_t> b;
    template <class T> void put(T v) {
        const size_t n = b.size();
        b.resize(n + sizeof(T));
        memcpy(b.data() + n, &v, sizeof(T));
    }
};
struct SdReader {
    const uint8_t* p;
    size_t n, off = 0;
    template <class T> T get() {
        if (off + sizeof(T) > n) throw std::runtime_error("state document truncated");
        T v;
        memcpy(&v, p + off, sizeof(T));
        off += sizeof(T);
        return v;
    }
    uint32_t count(size_t elem) {  // a length, checked against the bytes left
        const uint32_t c = get<uint32_t>();
        if ((uint64_t)c * elem > n - off) throw std::runtime_error("state document length out of range");
        return c;
    }
};

inline std::vector<uint8_t> sd_write(const SdDoc& d) {
    SdWriter w;
    w.put<uint32_t>(SD_MAGIC);
    w.put<uint32_t>(SD_VERSION);
    w.put<uint32_t>(d.n_procs);
    w.put<uint32_t>(d.n_slots);
    if (d.desc.size() != d.n_procs) throw std::runtime_error("processor descriptors missing");
    for (const SdProcDesc& x : d.desc) {
        w.put<uint32_t>(x.kind);
        w.put<uint32_t>(x.absent);
        w.put<uint32_t>(x.slot);
    }
    w.put<int64_t>(d.now);
    w.put<int64_t>(d.last_event_ts);
    w.put<uint64_t>(d.clock_flags);
    w.put<uint32_t>((uint32_t)d.keys.size());
    for (const SdKey& k : d.keys) {
        w.put<uint32_t>(k.key);
        w.put<uint32_t>((uint32_t)k.streams.size());
        w.put<uint32_t>((uint32_t)k.states.size());
        for (const SdStream& s : k.streams) {
            w.put<uint64_t>(s.seq);
            w.put<int64_t>(s.ts);
            w.put<uint32_t>(s.null_bits);
            w.put<uint32_t>(s.present);
            w.put<uint32_t>((uint32_t)s.attr.size());
            for (uint64_t a : s.attr) w.put<uint64_t>(a);
        }
        for (const SdState& s : k.states) {
            w.put<int64_t>(s.ts);
            w.put<uint32_t>(s.type);
            if (s.chains.size() != d.n_slots) throw std::runtime_error("state event slot count differs");
            for (const auto& c : s.chains) {
                w.put<uint32_t>((uint32_t)c.size());
                for (uint32_t x : c) w.put<uint32_t>(x);
            }
        }
        if (k.procs.size() != d.n_procs) throw std::runtime_error("processor count differs");
        for (const SdProc& p : k.procs) {
            w.put<uint32_t>(p.flags);
            w.put<int64_t>(p.last_scheduled);
            w.put<int64_t>(p.last_arrival);
            w.put<uint32_t>((uint32_t)p.pending.size());
            for (uint32_t x : p.pending) w.put<uint32_t>(x);
            w.put<uint32_t>((uint32_t)p.newev.size());
            for (uint32_t x : p.newev) w.put<uint32_t>(x);
            w.put<uint32_t>((uint32_t)p.queue.size());
            for (int64_t x : p.queue) w.put<int64_t>(x);
            w.put<uint32_t>(p.running);
            w.put<int64_t>(p.fire_at);
            w.put<uint64_t>(p.order);
        }
    }
    return w.b;
}

inline SdDoc sd_read(const void* buf, size_t len) {
    SdReader r{(const uint8_t*)buf, len};
    if (r.get<uint32_t>() != SD_MAGIC) throw std::runtime_error("not a state document");
    if (r.get<uint32_t>() != SD_VERSION) throw std::runtime_error("state document version differs");
    SdDoc d;
    d.n_procs = r.get<uint32_t>();
    d.n_slots = r.get<uint32_t>();
    if ((uint64_t)d.n_procs * 12 > len) throw std::runtime_error("state document length out of range");
    d.desc.resize(d.n_procs);
    for (SdProcDesc& x : d.desc) {
        x.kind = r.get<uint32_t>();
        x.absent = r.get<uint32_t>();
        x.slot = r.get<uint32_t>();
    }
    d.now = r.get<int64_t>();
    d.last_event_ts = r.get<int64_t>();
    d.clock_flags = r.get<uint64_t>();
    const uint32_t nk = r.count(12);
    d.keys.resize(nk);
    for (SdKey& k : d.keys) {
        k.key = r.get<uint32_t>();
        const uint32_t ns = r.count(28), nt = r.count(12);
        k.streams.resize(ns);
        for (SdStream& s : k.streams) {
            s.seq = r.get<uint64_t>();
            s.ts = r.get<int64_t>();
            s.null_bits = r.get<uint32_t>();
            s.present = r.get<uint32_t>();
            s.attr.resize(r.count(8));
            for (uint64_t& a : s.attr) a = r.get<uint64_t>();
        }
        k.states.resize(nt);
        for (SdState& s : k.states) {
            s.ts = r.get<int64_t>();
            s.type = r.get<uint32_t>();
            s.chains.resize(d.n_slots);
            for (auto& c : s.chains) {
                c.resize(r.count(4));
                for (uint32_t& x : c) {
                    x = r.get<uint32_t>();
                    if (x >= ns) throw std::runtime_error("stream event index out of range");
                }
            }
        }
        k.procs.resize(d.n_procs);
        for (SdProc& p : k.procs) {
            p.flags = r.get<uint32_t>();
            p.last_scheduled = r.get<int64_t>();
            p.last_arrival = r.get<int64_t>();
            p.pending.resize(r.count(4));
            for (uint32_t& x : p.pending) {
                x = r.get<uint32_t>();
                if (x >= nt) throw std::runtime_error("state event index out of range");
            }
            p.newev.resize(r.count(4));
            for (uint32_t& x : p.newev) {
                x = r.get<uint32_t>();
                if (x >= nt) throw std::runtime_error("state event index out of range");
            }
            p.queue.resize(r.count(8));
            for (int64_t& x : p.queue) x = r.get<int64_t>();
            p.running = r.get<uint32_t>();
            p.fire_at = r.get<int64_t>();
            p.order = r.get<uint64_t>();
        }
    }
    if (r.off != len) throw std::runtime_error("state document has trailing bytes");
    return d;
}

// ---- canonical numbering while an engine walks one key ------------------------------------------------
// Object ids are the engine's own (a pool index, a pointer); the builder numbers them in first-visit order.
// Visit order: for each processor, pending then newAndEvery; a StateEvent is numbered when its list entry
// is visited, its slots' chains right after.
template <class StId, class EvId> struct SdKeyBuilder {
    SdKey k;
    std::map<StId, uint32_t> st_ix;
    std::map<EvId, uint32_t> ev_ix;
    // the caller fills the stream event's fields when `fresh`
    uint32_t stream(const EvId& id, bool& fresh) {
        auto it = ev_ix.find(id);
        fresh = it == ev_ix.end();
        if (!fresh) return it->second;
        const uint32_t i = (uint32_t)k.streams.size();
        ev_ix.emplace(id, i);
        k.streams.emplace_back();
        return i;
    }
    uint32_t state(const StId& id, bool& fresh) {
        auto it = st_ix.find(id);
        fresh = it == st_ix.end();
        if (!fresh) return it->second;
        const uint32_t i = (uint32_t)k.states.size();
        st_ix.emplace(id, i);
        k.states.emplace_back();
        return i;
    }
};

// wall-clock callers: the order values of one key's running processors become ranks 1..n (engines keep
// a per-key or a global counter; only the order within a key is observable)
inline void sd_rank_orders(SdKey& k) {
    std::vector<std::pair<uint64_t, size_t>> o;
    for (size_t i = 0; i < k.procs.size(); i++)
        if (k.procs[i].running) o.emplace_back(k.procs[i].order, i);
        else k.procs[i].order = 0;
    std::sort(o.begin(), o.end());
    for (size_t r = 0; r < o.size(); r++) k.procs[o[r].second].order = r + 1;
}
