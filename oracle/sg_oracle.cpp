/*
 * sg_oracle.cpp — CPU ORACLE (test infrastructure only).
 *
 * A faithful single-threaded restatement of the reference engine's pattern/sequence state machine,
 * used by tests/ as the parity checker for the HIP engine and by bench.py as the CPU baseline
 * ("port").  It is never linked into or called by the product (siddhi-1_amd/).
 *
 * Parity of this restatement is pinned by the reference's own known-answer tests, transcribed into
 * tests/golden/kat_*.json by tests/golden/make_kat.py (see tests/test_oracle_kat.py).  The reference
 * (Java 8, Maven) cannot be built or run in this image (no JDK), so no oracle/_ref exists.
 *
 * Structure follows the reference object graph (paths relative to
 * /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/):
 *   StateEvent / StreamEvent            event/state/StateEvent.java:42-258, event/stream/StreamEvent
 *   StateEventCloner (shallow clone)    event/state/StateEventCloner.java:48-60
 *   PreProc  = StreamPreStateProcessor  query/input/stream/state/StreamPreStateProcessor.java:46-498
 *   CountPre = CountPreStateProcessor   query/input/stream/state/CountPreStateProcessor.java:36-220
 *   LogicalPre = LogicalPreStateProcessor query/input/stream/state/LogicalPreStateProcessor.java:43-202
 *   PostProc = StreamPostStateProcessor query/input/stream/state/StreamPostStateProcessor.java:31-160
 *   CountPost, LogicalPost              .../CountPostStateProcessor.java:39-89, LogicalPostStateProcessor.java:59-129
 *   Inner runtimes (init/reset/update)  .../runtime/*.java
 *   wiring (build)                      util/parser/StateInputStreamParser.java:76-408
 *   receivers (stabilize + order)       query/input/MultiProcessStreamReceiver.java:93-247,
 *                                       query/input/SingleProcessStreamReceiver.java:55-78,
 *                                       query/input/StateMultiProcessStreamReceiver.java:47-68,
 *                                       query/input/stream/state/receiver/*.java
 *   per-key state (partition flow)      util/snapshot/state/PartitionStateHolder.java:43-80,
 *                                       partition/PartitionStreamReceiver.java:148-272,
 *                                       partition/PartitionRuntimeImpl.java:346-367
 *   filter expression semantics         executor/condition/**, executor/math/** (see eval())
 *   absent states (`not S[..] for T`)   AbsentStreamPreStateProcessor.java:67-308,
 *                                       AbsentStreamPostStateProcessor.java:36-56,
 *                                       AbsentLogicalPreStateProcessor.java:65-388,
 *                                       AbsentLogicalPostStateProcessor.java:37-49
 *   timers / clock                      util/Scheduler.java:65-368 (per-key FIFO queue; EventCaller in
 *                                       wall-clock mode, time-change listener in playback mode),
 *                                       util/timestamp/TimestampGeneratorImpl.java:77-122
 *
 * Memory: StateEvent / StreamEvent are intrusively reference counted (the Java originals are GC'd
 * objects that are shared between lists and chains; identity matters for the shared-alias
 * semantics).
 */
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <list>
#include <set>
#include <tuple>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../include/siddhi_gpu.h"
#include "../include/siddhi_gpu_ir.h"
#include "../siddhi-1_amd/csrc/state_doc.h"   // the state document's format (sgo_state_export/import)

namespace {

// ------------------------------------------------------------------------------------------------
// intrusive refcount
// ------------------------------------------------------------------------------------------------
template <class T> class Ref {
  public:
    Ref() : p_(nullptr) {}
    Ref(T* p) : p_(p) { if (p_) p_->rc++; }
    Ref(const Ref& o) : p_(o.p_) { if (p_) p_->rc++; }
    Ref(Ref&& o) noexcept : p_(o.p_) { o.p_ = nullptr; }
    ~Ref() { release(); }
    Ref& operator=(const Ref& o) { if (o.p_) o.p_->rc++; release(); p_ = o.p_; return *this; }
    Ref& operator=(Ref&& o) noexcept { if (this != &o) { release(); p_ = o.p_; o.p_ = nullptr; } return *this; }
    T* operator->() const { return p_; }
    T* get() const { return p_; }
    explicit operator bool() const { return p_ != nullptr; }
    bool operator==(const Ref& o) const { return p_ == o.p_; }
    bool operator!=(const Ref& o) const { return p_ != o.p_; }
  private:
    void release() { if (p_ && --p_->rc == 0) delete p_; p_ = nullptr; }
    T* p_;
};

struct StreamEvent {
    int rc = 0;
    uint64_t seq;
    int64_t ts;
    Ref<StreamEvent> next;  // count-state chains (StreamEvent.next)
    StreamEvent(uint64_t s, int64_t t) : seq(s), ts(t) {}
};

enum EvType { CURRENT = 0, EXPIRED = 1 };

struct StateEvent {
    int rc = 0;
    std::vector<Ref<StreamEvent>> slots;
    int64_t ts = -1;
    EvType type = CURRENT;
    explicit StateEvent(int n) : slots(n) {}
};

using SE = Ref<StateEvent>;
using SEList = std::list<SE>;

// StateEvent.getStreamEvent(int[] position) for (slot, index-in-chain)  (StateEvent.java:138-182)
StreamEvent* chain_at(const StateEvent* se, int slot, int idx) {
    StreamEvent* s = se->slots[slot].get();
    if (!s) return nullptr;
    if (idx >= 0) {
        for (int i = 1; i <= idx; i++) {
            s = s->next.get();
            if (!s) return nullptr;
        }
        return s;
    }
    if (idx == -1) {  // CURRENT
        while (s->next) s = s->next.get();
        return s;
    }
    if (idx == -2) {  // LAST
        if (!s->next) return nullptr;
        while (s->next->next) s = s->next.get();
        return s;
    }
    std::vector<StreamEvent*> all;
    while (s) { all.push_back(s); s = s->next.get(); }
    long index = (long)all.size() + idx;
    if (index < 0) return nullptr;
    return all[index];
}

// StateEvent.addEvent / removeLastEvent (StateEvent.java:212-236)
void add_event(StateEvent* se, int slot, Ref<StreamEvent> ev) {
    StreamEvent* s = se->slots[slot].get();
    if (!s) { se->slots[slot] = ev; return; }
    while (s->next) s = s->next.get();
    s->next = ev;
}
void remove_last_event(StateEvent* se, int slot) {
    StreamEvent* s = se->slots[slot].get();
    if (!s) return;
    while (s->next) {
        if (!s->next->next) { s->next = Ref<StreamEvent>(); return; }
        s = s->next.get();
    }
    se->slots[slot] = Ref<StreamEvent>();
}

// StateEventCloner.copyStateEvent: shallow copy of the slot references (StateEventCloner.java:48-60)
SE clone_state(const StateEvent* se) {
    SE c(new StateEvent((int)se->slots.size()));
    c->slots = se->slots;
    c->type = se->type;
    c->ts = se->ts;
    return c;
}

// ------------------------------------------------------------------------------------------------
// event store (host ring stand-in: attribute values by seq)
// ------------------------------------------------------------------------------------------------
struct Column {
    int type;
    std::vector<uint64_t> v;   // value bits
    std::vector<uint8_t> null;
};
struct StreamStore {
    std::vector<int> types;
    std::vector<Column> cols;
};
struct EvLoc { uint32_t stream; uint32_t row; };

struct Val { uint64_t b; bool null; };

inline float f32(uint64_t b) { uint32_t u = (uint32_t)b; float f; memcpy(&f, &u, 4); return f; }
inline double f64(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
inline uint64_t bf32(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
inline uint64_t bf64(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
inline int32_t i32(uint64_t b) { return (int32_t)(uint32_t)b; }
inline int64_t i64(uint64_t b) { return (int64_t)b; }

struct Engine;

// ------------------------------------------------------------------------------------------------
// processors
// ------------------------------------------------------------------------------------------------
enum ProcKind { P_STREAM = 0, P_COUNT = 1, P_LOGICAL = 2 };

struct PreProc;

struct KeyState {  // StreamPreState (+ Count extras) of ONE processor for ONE partition key
    SEList pending;        // pendingStateEventList
    SEList newAndEvery;    // newAndEveryStateEventList
    bool stateChanged = false;
    bool initialized = false;
    bool successCondition = false;   // CountStreamPreState
    bool startStateReset = false;    // CountStreamPreState
    // LogicalStreamPreState of the absent processors
    int64_t lastScheduledTime = 0;   // AbsentStreamPreStateProcessor.java:312-318
    int64_t lastArrivalTime = 0;     // AbsentLogicalPreStateProcessor.java:360-365
    bool active = true;
    bool started = false;            // StreamPreState.started (partitionCreated once per key)
    // SchedulerState of this processor's Scheduler for this key (Scheduler.java:331-368)
    std::deque<int64_t> toNotify;    // toNotifyQueue: FIFO, NOT sorted
    bool running = false;            // an EventCaller is scheduled (wall-clock mode)
    int64_t fireAt = 0;              // when that EventCaller runs
    uint64_t order = 0;              // schedule order (ties of fireAt)
};

struct PostProc {
    int kind = P_STREAM;
    bool absent = false;              // Absent{Stream,Logical}PostStateProcessor
    int stateId = 0;
    PreProc* nextStatePre = nullptr;
    PreProc* nextEveryStatePre = nullptr;
    PreProc* thisPre = nullptr;
    PreProc* callbackPre = nullptr;   // CountPreStateProcessor callback (StreamPostStateProcessor.java:37)
    bool hasNext = false;             // nextProcessor (QuerySelector) attached
    bool isEventReturned = false;
    // count
    int minCount = 0, maxCount = 0;
    // logical
    int logicalType = 0;
    PreProc* partnerPre = nullptr;
    PostProc* partnerPost = nullptr;
    Engine* eng = nullptr;

    void process(StateEvent* se);
    void streamProcess(StateEvent* se);
    void processMinCountReached(StateEvent* se);
    void setNextStatePre(PreProc* p);
    void setNextEveryStatePre(PreProc* p);
};

struct PreProc {
    int id = 0;          // index in Engine::procs (state storage)
    int kind = P_STREAM;
    bool absent = false;           // Absent{Stream,Logical}PreStateProcessor
    int64_t waitingTime = -1;      // `for` time of the absent state
    int stateId = 0;
    bool isStart = false;
    int stateType = SG_Q_PATTERN;
    int64_t withinTime = -1;
    std::vector<int> startStateIds;
    PreProc* withinEveryPre = nullptr;
    PostProc* thisPost = nullptr;
    PostProc* thisLast = nullptr;
    uint32_t filterPc = 0, filterLen = 0;
    // count
    int minCount = 0, maxCount = 0;
    PostProc* countPost = nullptr;
    // logical
    int logicalType = 0;
    PreProc* partner = nullptr;
    Engine* eng = nullptr;
    int resetDepth = 0;

    KeyState& st();

    bool isExpired(const StateEvent* se, int64_t now) const {
        if (withinTime == -1) return false;
        for (int s : startStateIds) {
            StreamEvent* ev = se->slots[s].get();
            if (ev && std::llabs(ev->ts - now) > withinTime) return true;
        }
        return false;
    }

    void init();
    void addState(SE se);
    void addEveryState(const SE& se);
    void resetState();
    void updateState();
    void expireEvents(int64_t ts);
    void stateChanged() { st().stateChanged = true; }
    void successCondition() { st().successCondition = true; }
    void startStateReset();
    void runChain(StateEvent* se);  // StreamPreStateProcessor.process(StateEvent)
    void processAndReturn(Ref<StreamEvent> ev, std::vector<SE>& ret);
    // absent states
    void notifyAt(int64_t t);                       // Scheduler.notifyAt (Scheduler.java:114-128)
    void updateLastArrivalTime(int64_t ts);
    void partitionCreated();
    void processTimer(int64_t currentTime);         // Absent*PreStateProcessor.process(chunk)
    void sendAbsentEvent(const SE& se);             // Absent*PreStateProcessor.sendEvent
    bool partnerCanProceed(StateEvent* se);         // AbsentLogicalPreStateProcessor.java:391-422
    void processAndReturnAbsentLogical(Ref<StreamEvent> ev);
};

// ------------------------------------------------------------------------------------------------
// inner state runtimes (query/input/stream/state/runtime/*.java)
// ------------------------------------------------------------------------------------------------
struct InnerRT {
    int tag;               // SG_N_*
    PreProc* first = nullptr;
    PostProc* last = nullptr;
    InnerRT* a = nullptr;  // current / inner / rt1
    InnerRT* b = nullptr;  // next / rt2
    int stream = -1;       // stream runtimes: stream of the state

    void init() {
        switch (tag) {
        case SG_N_NEXT: a->init(); b->init(); break;
        case SG_N_EVERY: a->init(); break;
        case SG_N_LOGICAL: b->init(); a->init(); break;
        default: first->init();
        }
    }
    void reset() {
        switch (tag) {
        case SG_N_NEXT: b->reset(); a->reset(); break;
        case SG_N_LOGICAL: b->reset(); break;
        default: first->resetState();  // Stream, Count, and Every (inherits StreamInnerStateRuntime)
        }
    }
    void update() {
        switch (tag) {
        case SG_N_NEXT: a->update(); b->update(); break;
        case SG_N_LOGICAL: b->update(); break;
        default: first->updateState();
        }
    }
    void setQuerySelector() {
        switch (tag) {
        case SG_N_NEXT: b->setQuerySelector(); break;
        case SG_N_EVERY: a->setQuerySelector(); break;
        case SG_N_LOGICAL: b->setQuerySelector(); a->setQuerySelector(); break;
        default: last->hasNext = true;
        }
    }
};

struct Receiver {  // ProcessStreamReceiver family for one stream
    bool multi = false;
    bool sequence = false;
    std::vector<PreProc*> nextProcessors;     // setup order
    std::vector<PreProc*> stateProcessorsForStream;
    std::vector<int> eventSequence;           // Multi receivers: reversed for pattern/sequence
};

struct Match {
    uint64_t trigger;
    uint32_t key;
    int64_t ts;
    std::vector<std::vector<uint64_t>> chains;
};

struct Engine {
    // IR
    std::vector<uint32_t> ir;
    int qtype = SG_Q_PATTERN;
    int nslots = 0;
    int64_t within = -1;
    bool partitioned = false;
    const uint32_t* code = nullptr;
    uint32_t codeLen = 0;

    std::vector<std::unique_ptr<PreProc>> procs;
    std::vector<std::unique_ptr<PostProc>> posts;
    std::vector<std::unique_ptr<InnerRT>> rts;
    std::vector<PreProc*> allStateProcessors;   // preStateProcessors list (expire order)
    InnerRT* root = nullptr;
    std::vector<Receiver> receivers;            // per IR stream

    // per-key state: keyStates[key][proc]
    std::vector<std::vector<KeyState>> keyStates;
    std::vector<uint8_t> keyInit;
    uint32_t curKey = 0;

    // event store
    std::vector<StreamStore> streams;
    std::vector<EvLoc> seqLoc;
    // events that entered through sgo_state_import (before this engine's first push): seq -> attribute
    // value bits + null bits
    std::unordered_map<uint64_t, std::pair<std::vector<uint64_t>, uint32_t>> importedAttrs;
    uint64_t seq0 = 0;
    bool haveSeq0 = false;

    // output
    std::vector<Match> matches;
    std::vector<SE> toProject;          // Single receivers project after the chunk
    uint64_t curTrigger = 0;

    // polled buffers
    std::vector<uint64_t> outTrig, outSlot;
    std::vector<uint32_t> outKey, outLen;
    std::vector<int64_t> outTs;

    sg_stats stats{};

    // clock (TimestampGeneratorImpl): wall clock, or the last event time in playback mode
    bool playback = false;
    int64_t now = 0;
    int64_t lastEventTs = 0;
    bool clockSet = false;                      // an event or a time advance has reached the engine
    uint64_t schedOrder = 0;
    std::vector<PreProc*> startup;              // startupPreStateProcessors (absent pres, parse order)
    // per scheduler (absent pre): keys whose queue is not empty, by head (playback listener)
    std::vector<std::set<std::pair<int64_t, uint32_t>>> heads;   // [proc id]
    // scheduled EventCallers (wall-clock mode): (fireAt, key, order, proc).  Callers of different keys
    // due at the same time run in key order (in the reference they race on the executor's threads).
    std::set<std::tuple<int64_t, uint32_t, uint64_t, int>> callers;

    KeyState& state(int proc) { return keyStates[curKey][proc]; }
    void advanceTime(int64_t t);
    void sendTimerEvents(PreProc* p);

    // ---- attribute access ----
    bool stored(uint64_t seq) const {
        return haveSeq0 && seq >= seq0 && seq - seq0 < seqLoc.size() && seqLoc[seq - seq0].stream != UINT32_MAX;
    }
    Val attr(uint64_t seq, uint32_t a) const {
        if (!stored(seq)) {
            auto it = importedAttrs.find(seq);
            if (it == importedAttrs.end() || a >= it->second.first.size())
                throw std::runtime_error("attributes of an event not in the store");
            return Val{it->second.first[a], ((it->second.second >> a) & 1u) != 0};
        }
        const EvLoc& l = seqLoc[seq - seq0];
        const Column& c = streams[l.stream].cols[a];
        return Val{c.v[l.row], c.null.empty() ? false : (bool)c.null[l.row]};
    }
    bool eval(const StateEvent* se, uint32_t pc, uint32_t len) const;
    void project(const StateEvent* se);
    void processEventMulti(int stream, uint64_t seq, int64_t ts);
    void processChunkSingle(int stream, const std::vector<std::pair<uint64_t, int64_t>>& evs);
    void stabilize(const Receiver& r, int64_t ts);
};

KeyState& PreProc::st() { return eng->state(id); }

// ---------------------------------------------------------------------- StreamPreStateProcessor
void PreProc::init() {  // StreamPreStateProcessor.java:178-194
    KeyState& s = st();
    if (isStart && (!s.initialized || thisPost->nextEveryStatePre != nullptr ||
                    (stateType == SG_Q_SEQUENCE && thisPost->nextStatePre != nullptr &&
                     thisPost->nextStatePre->absent))) {
        SE se(new StateEvent(eng->nslots));
        addState(se);
        st().initialized = true;
    }
}

void PreProc::addState(SE se) {
    KeyState& s = st();
    if (absent && !s.active) return;  // Absent*PreStateProcessor.addState: 'every' not used, already fired
    if (absent && kind == P_STREAM) {  // AbsentStreamPreStateProcessor.java:83-103
        if (stateType == SG_Q_SEQUENCE) s.newAndEvery.clear();
        s.newAndEvery.push_back(se);
        if (!isStart) {
            st().lastScheduledTime = se->ts + waitingTime;
            notifyAt(st().lastScheduledTime);
        }
        return;
    }
    if (kind == P_LOGICAL) {  // LogicalPreStateProcessor.java:43-62
        if (isStart || stateType == SG_Q_SEQUENCE) {
            if (s.newAndEvery.empty()) s.newAndEvery.push_back(se);
            if (partner && partner->st().newAndEvery.empty()) partner->st().newAndEvery.push_back(se);
        } else {
            s.newAndEvery.push_back(se);
            if (partner) partner->st().newAndEvery.push_back(se);
        }
        if (absent && !isStart && waitingTime != -1) {  // AbsentLogicalPreStateProcessor.java:77-97
            notifyAt(se->ts + waitingTime);
            if (partner && partner->absent) partner->notifyAt(se->ts + partner->waitingTime);
        }
        return;
    }
    // StreamPreStateProcessor.java:214-227 (and CountPreStateProcessor.java:114-128)
    if (stateType == SG_Q_SEQUENCE) {
        if (s.newAndEvery.empty()) s.newAndEvery.push_back(se);
    } else {
        s.newAndEvery.push_back(se);
    }
    if (kind == P_COUNT && minCount == 0 && !se->slots[stateId]) {  // CountPreStateProcessor.java:129-136
        countPost->processMinCountReached(se.get());
    }
}

void PreProc::addEveryState(const SE& se) {
    SE c = clone_state(se.get());
    c->type = CURRENT;
    if (absent && kind == P_LOGICAL) {  // AbsentLogicalPreStateProcessor.java:99-118
        if (c->slots[stateId]) c->ts = c->slots[stateId]->ts;
        c->slots[stateId] = Ref<StreamEvent>();
        c->slots[partner->stateId] = Ref<StreamEvent>();
        st().newAndEvery.push_back(c);
        partner->st().newAndEvery.push_back(c);
        eng->stats.partials_created++;
        return;
    }
    if (absent) {  // AbsentStreamPreStateProcessor.java:105-123
        for (size_t i = stateId; i < c->slots.size(); i++) c->slots[i] = Ref<StreamEvent>();
        st().newAndEvery.push_back(c);
        st().lastScheduledTime = se->ts + waitingTime;
        notifyAt(st().lastScheduledTime);
        eng->stats.partials_created++;
        return;
    }
    if (kind == P_LOGICAL) {  // LogicalPreStateProcessor.java:64-84
        c->slots[stateId] = Ref<StreamEvent>();
        for (size_t i = stateId; i < c->slots.size(); i++) c->slots[i] = Ref<StreamEvent>();
        st().newAndEvery.push_back(c);
        if (partner) {
            c->slots[partner->stateId] = Ref<StreamEvent>();
            partner->st().newAndEvery.push_back(c);
        }
        eng->stats.partials_created++;
        return;
    }
    // StreamPreStateProcessor.java:229-247 / CountPreStateProcessor.java:140-157
    for (size_t i = stateId; i < c->slots.size(); i++) c->slots[i] = Ref<StreamEvent>();
    st().newAndEvery.push_back(c);
    eng->stats.partials_created++;
}

void PreProc::resetState() {
    KeyState& s = st();
    if (kind == P_LOGICAL) {  // LogicalPreStateProcessor.java:96-124
        if (logicalType == SG_L_OR || s.pending.size() == partner->st().pending.size()) {
            s.pending.clear();
            partner->st().pending.clear();
            if (isStart && s.newAndEvery.empty()) {
                if (stateType == SG_Q_SEQUENCE && thisPost->nextEveryStatePre == nullptr &&
                    !thisPost->nextStatePre->st().pending.empty())
                    return;
                init();
            }
        }
        return;
    }
    // StreamPreStateProcessor.java:287-305
    s.pending.clear();
    if (isStart && s.newAndEvery.empty()) {
        if (stateType == SG_Q_SEQUENCE && thisPost->nextEveryStatePre == nullptr &&
            !thisPost->nextStatePre->st().pending.empty())
            return;
        init();
    }
}

static void sort_by_ts(SEList& l) {
    // eventTimeComparator (StreamPreStateProcessor.java:66-80): ts -1 sorts last; List.sort is stable
    l.sort([](const SE& a, const SE& b) {
        if (a->ts == -1) return false;
        if (b->ts == -1) return true;
        return a->ts < b->ts;
    });
}

void PreProc::updateState() {
    KeyState& s = st();
    if (kind == P_COUNT && s.startStateReset) {  // CountPreStateProcessor.java:168-180
        s.startStateReset = false;
        init();
    }
    KeyState& s2 = st();
    sort_by_ts(s2.newAndEvery);
    s2.pending.splice(s2.pending.end(), s2.newAndEvery);
    if (kind == P_LOGICAL) {  // LogicalPreStateProcessor.java:126-140 + moveAll...():181-190
        KeyState& p = partner->st();
        sort_by_ts(p.newAndEvery);
        p.pending.splice(p.pending.end(), p.newAndEvery);
    }
}

void PreProc::expireEvents(int64_t ts) {  // StreamPreStateProcessor.java:325-361
    KeyState& s = st();
    StateEvent* expired = nullptr;
    SE keep;
    for (auto it = s.pending.begin(); it != s.pending.end();) {
        if (isExpired(it->get(), ts)) {
            SE se = *it;
            it = s.pending.erase(it);
            if (se->type != EXPIRED) { se->type = EXPIRED; expired = se.get(); keep = se; }
        } else {
            break;
        }
    }
    for (auto it = s.newAndEvery.begin(); it != s.newAndEvery.end();) {
        if (isExpired(it->get(), ts)) {
            SE se = *it;
            it = s.newAndEvery.erase(it);
            if (se->type != EXPIRED) { se->type = EXPIRED; expired = se.get(); keep = se; }
        } else {
            ++it;
        }
    }
    if (expired && withinEveryPre) {
        withinEveryPre->addEveryState(keep);
        withinEveryPre->updateState();
    }
}

void PreProc::startStateReset() {  // CountPreStateProcessor.java:155-166
    if (++resetDepth > 64) {
        resetDepth = 0;
        throw std::runtime_error("startStateReset recursion (the reference overflows its stack here)");
    }
    st().startStateReset = true;
    if (thisPost->callbackPre != nullptr) {
        countPost->thisPre->startStateReset();
    }
    resetDepth = 0;
}

void PreProc::runChain(StateEvent* se) {  // StreamPreStateProcessor.process(StateEvent) :131-142
    st().stateChanged = false;
    if (filterLen == 0 || eng->eval(se, filterPc, filterLen)) {  // FilterProcessor.java:48-60
        thisPost->process(se);
    }
}

void PreProc::processAndReturn(Ref<StreamEvent> ev, std::vector<SE>& ret) {
    KeyState& s = st();
    if (absent) {
        if (!s.active) return;
        if (kind == P_LOGICAL) { processAndReturnAbsentLogical(ev); return; }
    }
    const size_t ret0 = ret.size();
    for (auto it = s.pending.begin(); it != s.pending.end();) {
        SE se = *it;
        eng->stats.partials_scanned++;
        if (kind == P_COUNT) {  // CountPreStateProcessor.java:53-95
            int n = (int)se->slots.size();
            if ((n > stateId + 1 && se->slots[stateId + 1]) || (n > stateId + 2 && se->slots[stateId + 2])) {
                it = s.pending.erase(it);
                continue;
            }
            add_event(se.get(), stateId, Ref<StreamEvent>(new StreamEvent(ev->seq, ev->ts)));
            st().successCondition = false;
            runChain(se.get());
            if (thisLast->isEventReturned) {
                thisLast->isEventReturned = false;
                ret.push_back(se);
            }
            bool removed = false;
            if (st().stateChanged) { it = s.pending.erase(it); removed = true; }
            if (!st().successCondition) {
                remove_last_event(se.get(), stateId);
                if (stateType == SG_Q_SEQUENCE && !removed) { it = s.pending.erase(it); removed = true; }
            }
            if (!removed) ++it;
            continue;
        }
        if (kind == P_LOGICAL && logicalType == SG_L_OR && se->slots[partner->stateId]) {
            it = s.pending.erase(it);  // LogicalPreStateProcessor.java:153-157
            continue;
        }
        // StreamPreStateProcessor.java:371-397 (LogicalPreStateProcessor.java:158-176)
        se->slots[stateId] = Ref<StreamEvent>(new StreamEvent(ev->seq, ev->ts));
        runChain(se.get());
        if (thisLast->isEventReturned) {
            thisLast->isEventReturned = false;
            ret.push_back(se);
        }
        if (st().stateChanged) {
            it = s.pending.erase(it);
        } else {
            se->slots[stateId] = Ref<StreamEvent>();
            if (stateType == SG_Q_SEQUENCE) {
                // removeOnNoStateChange: SEQUENCE, except absent (AbsentStreamPreStateProcessor.java:289-291)
                if (kind == P_STREAM && absent) ++it;
                else it = s.pending.erase(it);
                if (kind == P_STREAM && thisPost->callbackPre) thisPost->callbackPre->startStateReset();
            } else {
                ++it;
            }
        }
    }
    if (absent) ret.resize(ret0);  // AbsentStreamPreStateProcessor.processAndReturn: always empty (:265-283)
}

// AbsentLogicalPreStateProcessor.processAndReturn (AbsentLogicalPreStateProcessor.java:255-318)
void PreProc::processAndReturnAbsentLogical(Ref<StreamEvent> ev) {
    KeyState& s = st();
    for (auto it = s.pending.begin(); it != s.pending.end();) {
        SE se = *it;
        eng->stats.partials_scanned++;
        if (logicalType == SG_L_OR && se->slots[partner->stateId]) {
            it = s.pending.erase(it);
            continue;
        }
        Ref<StreamEvent> cur = se->slots[stateId];
        se->slots[stateId] = Ref<StreamEvent>(new StreamEvent(ev->seq, ev->ts));
        runChain(se.get());
        if (waitingTime != -1 ||
            (stateType == SG_Q_SEQUENCE && logicalType == SG_L_AND && thisPost->nextEveryStatePre != nullptr))
            se->slots[stateId] = cur;  // reset to the original state after processing
        bool removed = false;
        if (thisLast->isEventReturned) {
            thisLast->isEventReturned = false;
            it = s.pending.erase(it);  // passed the filter: no longer an absent candidate
            removed = true;
            if (stateType == SG_Q_SEQUENCE) {
                auto& pp = partner->st().pending;
                for (auto jt = pp.begin(); jt != pp.end(); ++jt)
                    if (*jt == se) { pp.erase(jt); break; }
            }
        }
        if (!st().stateChanged) {
            se->slots[stateId] = cur;
            if (stateType == SG_Q_SEQUENCE) {
                if (removed) throw std::runtime_error("iterator removed twice (IllegalStateException in the reference)");
                it = s.pending.erase(it);
                removed = true;
            }
        }
        if (!removed) ++it;
    }
}

// ---------------------------------------------------------------------- post processors
void PostProc::streamProcess(StateEvent* se) {  // StreamPostStateProcessor.java:64-83
    thisPre->stateChanged();
    se->ts = se->slots[stateId]->ts;
    if (hasNext) isEventReturned = true;
    SE keep(se);
    if (nextStatePre) nextStatePre->addState(keep);
    if (nextEveryStatePre) nextEveryStatePre->addEveryState(keep);
    if (callbackPre) callbackPre->startStateReset();
}

void PostProc::processMinCountReached(StateEvent* se) {  // CountPostStateProcessor.java:68-80
    if (hasNext) {
        thisPre->stateChanged();
        isEventReturned = true;
    }
    SE keep(se);
    if (nextStatePre) nextStatePre->addState(keep);
    if (nextEveryStatePre) nextEveryStatePre->addEveryState(keep);
}

void PostProc::process(StateEvent* se) {
    if (absent) {
        StreamEvent* ev = se->slots[stateId].get();
        thisPre->stateChanged();
        isEventReturned = true;  // the notification to the absent pre that the event was processed
        if (kind == P_STREAM) {  // AbsentStreamPostStateProcessor.java:36-56
            se->ts = ev->ts;
            if (thisPre->isStart && nextEveryStatePre != nullptr && nextEveryStatePre == thisPre)
                thisPre->addEveryState(SE(se));
        }                        // AbsentLogicalPostStateProcessor.java:37-49
        thisPre->updateLastArrivalTime(ev->ts);
        return;
    }
    if (kind == P_COUNT) {  // CountPostStateProcessor.java:39-66
        StreamEvent* s = se->slots[stateId].get();
        int n = 1;
        while (s->next) { n++; s = s->next.get(); }
        thisPre->successCondition();
        se->ts = s->ts;
        if (n >= minCount) {
            if (thisPre->stateType == SG_Q_SEQUENCE) {
                SE keep(se);
                if (nextStatePre) nextStatePre->addState(keep);
                if (n != maxCount) thisPre->addState(keep);
            } else if (n == minCount) {
                processMinCountReached(se);
            }
            if (n == maxCount) thisPre->stateChanged();
        }
        return;
    }
    if (kind == P_LOGICAL) {  // LogicalPostStateProcessor.java:59-83
        if (logicalType == SG_L_AND) {
            const bool go = partnerPre->absent ? partnerPre->partnerCanProceed(se)
                                               : (bool)se->slots[partnerPre->stateId];
            if (go) streamProcess(se);
            else thisPre->stateChanged();
        } else {
            streamProcess(se);
            if (partnerPost->hasNext && thisPre->thisLast == partnerPost) partnerPost->isEventReturned = true;
        }
        return;
    }
    streamProcess(se);
}

void PostProc::setNextStatePre(PreProc* p) {
    nextStatePre = p;
    if (kind == P_LOGICAL) partnerPost->nextStatePre = p;  // LogicalPostStateProcessor.java:117-120
    if (kind == P_COUNT && thisPre->isStart && thisPre->stateType == SG_Q_SEQUENCE && minCount == 0) {
        p->thisPost->callbackPre = thisPre;  // CountPostStateProcessor.java:82-88
    }
}
void PostProc::setNextEveryStatePre(PreProc* p) {
    nextEveryStatePre = p;
    if (kind == P_LOGICAL) partnerPost->nextEveryStatePre = p;
}

// ------------------------------------------------------------------------------------------------
// absent states and their timers
// ------------------------------------------------------------------------------------------------
void PreProc::notifyAt(int64_t t) {  // Scheduler.notifyAt + schedule (Scheduler.java:114-156)
    KeyState& s = st();
    const bool wasEmpty = s.toNotify.empty();
    s.toNotify.push_back(t);
    if (wasEmpty) eng->heads[id].insert({t, eng->curKey});
    if (!eng->playback && !s.running && s.toNotify.size() == 1) {
        // EventCaller scheduled after (time - now), or at once when that is <= 0
        s.running = true;
        s.fireAt = std::max(t, eng->now);
        s.order = ++eng->schedOrder;
        eng->callers.insert({s.fireAt, eng->curKey, s.order, id});
    }
}

void PreProc::updateLastArrivalTime(int64_t ts) {
    KeyState& s = st();
    if (kind == P_LOGICAL) {  // AbsentLogicalPreStateProcessor.java:65-74
        s.lastArrivalTime = ts;
        return;
    }
    s.lastScheduledTime = ts + waitingTime;  // AbsentStreamPreStateProcessor.java:70-81
    notifyAt(s.lastScheduledTime);
}

// PartitionCreationListener.partitionCreated (AbsentStreamPreStateProcessor.java:290-308,
// AbsentLogicalPreStateProcessor.java:370-389), called by StateStreamRuntime.initPartition :90-97
void PreProc::partitionCreated() {
    KeyState& s = st();
    if (s.started) return;
    s.started = true;
    if (isStart && waitingTime != -1 && s.active) {
        if (kind == P_STREAM) s.lastScheduledTime = eng->now + waitingTime;
        notifyAt(eng->now + waitingTime);
    }
}

// AbsentLogicalPreStateProcessor.partnerCanProceed (:391-422)
bool PreProc::partnerCanProceed(StateEvent* se) {
    KeyState& s = st();
    if (stateType == SG_Q_SEQUENCE && thisPost->nextEveryStatePre == nullptr && s.lastArrivalTime > 0) return false;
    if (waitingTime == -1) {
        if (thisPost->nextEveryStatePre == nullptr) return !se->slots[stateId];
        if (s.lastArrivalTime > 0) {
            s.lastArrivalTime = 0;
            init();
            return false;
        }
        return true;
    }
    return (bool)se->slots[stateId];
}

// Absent*PreStateProcessor.sendEvent (AbsentStreamPreStateProcessor.java:229-246,
// AbsentLogicalPreStateProcessor.java:228-247): the timer thread delivers the match at once
void PreProc::sendAbsentEvent(const SE& se) {
    if (thisPost->hasNext) eng->project(se.get());
    if (thisPost->nextStatePre) thisPost->nextStatePre->addState(se);
    if (thisPost->nextEveryStatePre) {
        thisPost->nextEveryStatePre->addEveryState(se);
    } else if (isStart) {
        st().active = false;
        if (kind == P_LOGICAL && logicalType == SG_L_OR && partner->absent) partner->st().active = false;
    }
    if (thisPost->callbackPre) thisPost->callbackPre->startStateReset();
}

// the TIMER event of this processor's scheduler for the current key, at `currentTime`
void PreProc::processTimer(int64_t currentTime) {
    KeyState& s = st();
    if (!s.active) return;
    std::vector<SE> ret;
    if (kind == P_STREAM) {  // AbsentStreamPreStateProcessor.process (:151-227)
        bool initialize = isStart && s.newAndEvery.empty() && s.pending.empty();
        if (initialize && stateType == SG_Q_SEQUENCE && thisPost->nextEveryStatePre == nullptr &&
            s.lastScheduledTime > 0)
            initialize = false;
        if (initialize) {
            addState(SE(new StateEvent(eng->nslots)));
        } else if (stateType == SG_Q_SEQUENCE && !s.newAndEvery.empty()) {
            resetState();
        }
        updateState();
        for (auto it = s.pending.begin(); it != s.pending.end();) {
            SE se = *it;
            eng->stats.partials_scanned++;
            if (isExpired(se.get(), currentTime)) {
                it = s.pending.erase(it);
                if (withinEveryPre != nullptr && thisPost->nextEveryStatePre != this) {
                    if (!thisPost->nextEveryStatePre) throw std::runtime_error("NullPointerException in the reference timer path");
                    thisPost->nextEveryStatePre->addEveryState(se);
                }
                continue;
            }
            if ((se->ts == -1 && currentTime >= s.lastScheduledTime) ||
                (se->ts != -1 && currentTime >= se->ts + waitingTime)) {
                it = s.pending.erase(it);
                se->ts = currentTime;
                ret.push_back(se);
                continue;
            }
            ++it;
        }
        if (withinEveryPre) withinEveryPre->updateState();
        const bool notProcessed = ret.empty();
        for (auto& se : ret) sendAbsentEvent(se);
        KeyState& s2 = st();
        const int64_t actual = eng->now;  // TimestampGenerator.currentTime()
        if (actual > waitingTime + currentTime) s2.lastScheduledTime = actual + waitingTime;
        if (notProcessed && s2.lastScheduledTime < currentTime) {
            s2.lastScheduledTime = currentTime + waitingTime;
            notifyAt(s2.lastScheduledTime);
        }
        return;
    }
    // AbsentLogicalPreStateProcessor.process (:121-209)
    bool notProcessed = true;
    if (currentTime >= s.lastArrivalTime + waitingTime) {
        if (isStart && stateType == SG_Q_SEQUENCE && s.newAndEvery.empty() && s.pending.empty()) {
            addState(SE(new StateEvent(eng->nslots)));
        } else if (stateType == SG_Q_SEQUENCE && !s.newAndEvery.empty()) {
            resetState();
        }
        updateState();
        SE expired;
        for (auto it = s.pending.begin(); it != s.pending.end();) {
            SE se = *it;
            eng->stats.partials_scanned++;
            if (isExpired(se.get(), currentTime)) {
                expired = se;
                it = s.pending.erase(it);
                continue;
            }
            StreamEvent* own = se->slots[stateId].get();
            const bool passed = own ? currentTime >= own->ts + waitingTime : currentTime >= se->ts + waitingTime;
            if (passed) {
                it = s.pending.erase(it);
                const bool partnerIn = (bool)se->slots[partner->stateId];
                if (logicalType == SG_L_OR && !partnerIn) {
                    add_event(se.get(), stateId, Ref<StreamEvent>(new StreamEvent(SG_BLANK_SEQ, -1)));
                    ret.push_back(se);
                } else if (logicalType == SG_L_AND && partnerIn) {
                    ret.push_back(se);
                } else if (logicalType == SG_L_AND && !partnerIn) {
                    add_event(se.get(), stateId, Ref<StreamEvent>(new StreamEvent(SG_BLANK_SEQ, -1)));
                }
                continue;
            }
            ++it;
        }
        if (expired && withinEveryPre) {
            withinEveryPre->addEveryState(expired);
            withinEveryPre->updateState();
        }
        notProcessed = ret.empty();
        for (auto& se : ret) {
            se->ts = currentTime;
            sendAbsentEvent(se);
        }
        st().lastArrivalTime = 0;
    }
    if (thisPost->nextEveryStatePre != nullptr || (notProcessed && isStart)) {
        const int64_t nextBreak = st().lastArrivalTime == 0 ? eng->now + waitingTime : st().lastArrivalTime + waitingTime;
        notifyAt(nextBreak);
    }
}

// Scheduler.sendTimerEvents (Scheduler.java:172-210) for the current key
void Engine::sendTimerEvents(PreProc* p) {
    curTrigger = SG_TIMER_SEQ;
    for (;;) {
        KeyState& s = state(p->id);
        if (s.toNotify.empty() || s.toNotify.front() > now) break;
        const int64_t t = s.toNotify.front();
        s.toNotify.pop_front();
        heads[p->id].erase({t, curKey});
        if (!s.toNotify.empty()) heads[p->id].insert({s.toNotify.front(), curKey});
        p->processTimer(t);
    }
}

void Engine::advanceTime(int64_t t) {
    if (playback) {
        // TimestampGeneratorImpl.setCurrentTimestamp -> each Scheduler's time-change listener, in
        // registration order (Scheduler.java:73-104)
        if (t < lastEventTs) return;
        lastEventTs = t;
        now = t;
        for (PreProc* p : startup) {
            std::vector<std::pair<int64_t, uint32_t>> due;
            for (auto& h : heads[p->id]) {
                if (h.first > t) break;
                due.push_back(h);
            }
            // TreeMultimap<Long, SchedulerState> with SchedulerState.compareTo == 0 keeps ONE state per
            // distinct due time; which one depends on Java HashMap order
            for (size_t i = 1; i < due.size(); i++)
                if (due[i].first == due[i - 1].first)
                    throw std::runtime_error("two partition keys share a timer due time at one clock advance "
                                             "(reference Scheduler collapse quirk, SURVEY A.10): input not supported");
            const uint32_t save = curKey;
            for (auto& d : due) {
                curKey = d.second;
                sendTimerEvents(p);
            }
            curKey = save;
        }
        return;
    }
    // wall clock: the EventCallers run in time order (Scheduler.EventCaller.run, Scheduler.java:264-298)
    const uint32_t save = curKey;
    while (!callers.empty() && std::get<0>(*callers.begin()) <= t) {
        auto c = *callers.begin();
        callers.erase(callers.begin());
        now = std::max(now, std::get<0>(c));
        PreProc* p = procs[std::get<3>(c)].get();
        curKey = std::get<1>(c);
        sendTimerEvents(p);
        KeyState& s = state(p->id);
        if (!s.toNotify.empty()) {
            s.fireAt = std::max(s.toNotify.front(), now);
            s.order = ++schedOrder;
            callers.insert({s.fireAt, curKey, s.order, p->id});
        } else {
            s.running = false;
        }
    }
    curKey = save;
    if (t > now) now = t;
}

// ------------------------------------------------------------------------------------------------
// filter bytecode with Java semantics
// ------------------------------------------------------------------------------------------------
static Val cvt(Val v, int from, int to) {
    if (v.null) return v;
    switch (from) {
    case SG_T_INT: {
        int32_t x = i32(v.b);
        if (to == SG_T_LONG) return {(uint64_t)(int64_t)x, false};
        if (to == SG_T_FLOAT) return {bf32((float)x), false};
        if (to == SG_T_DOUBLE) return {bf64((double)x), false};
        break;
    }
    case SG_T_LONG: {
        int64_t x = i64(v.b);
        if (to == SG_T_FLOAT) return {bf32((float)x), false};
        if (to == SG_T_DOUBLE) return {bf64((double)x), false};
        break;
    }
    case SG_T_FLOAT:
        if (to == SG_T_DOUBLE) return {bf64((double)f32(v.b)), false};
        break;
    }
    return v;
}

static Val arith(int op, int t, Val l, Val r) {
    if (l.null || r.null) return {0, true};
    switch (t) {
    case SG_T_INT: {
        int32_t a = i32(l.b), b = i32(r.b);
        uint32_t ua = (uint32_t)a, ub = (uint32_t)b;
        switch (op) {
        case SG_OP_ADD: return {(uint64_t)(uint32_t)(ua + ub), false};
        case SG_OP_SUB: return {(uint64_t)(uint32_t)(ua - ub), false};
        case SG_OP_MUL: return {(uint64_t)(uint32_t)(ua * ub), false};
        case SG_OP_DIV:
            if (b == 0) return {0, true};
            if (a == INT32_MIN && b == -1) return {(uint64_t)(uint32_t)a, false};
            return {(uint64_t)(uint32_t)(a / b), false};
        case SG_OP_MOD:
            if (b == 0) return {0, true};
            if (b == -1) return {0, false};
            return {(uint64_t)(uint32_t)(a % b), false};
        }
        break;
    }
    case SG_T_LONG: {
        int64_t a = i64(l.b), b = i64(r.b);
        uint64_t ua = (uint64_t)a, ub = (uint64_t)b;
        switch (op) {
        case SG_OP_ADD: return {ua + ub, false};
        case SG_OP_SUB: return {ua - ub, false};
        case SG_OP_MUL: return {ua * ub, false};
        case SG_OP_DIV:
            if (b == 0) return {0, true};
            if (a == INT64_MIN && b == -1) return {(uint64_t)a, false};
            return {(uint64_t)(a / b), false};
        case SG_OP_MOD:
            if (b == 0) return {0, true};
            if (b == -1) return {0, false};
            return {(uint64_t)(a % b), false};
        }
        break;
    }
    case SG_T_FLOAT: {
        float a = f32(l.b), b = f32(r.b);
        switch (op) {
        case SG_OP_ADD: return {bf32(a + b), false};
        case SG_OP_SUB: return {bf32(a - b), false};
        case SG_OP_MUL: return {bf32(a * b), false};
        case SG_OP_DIV: if (b == 0.0f) return {0, true}; return {bf32(a / b), false};
        case SG_OP_MOD: if (b == 0.0f) return {0, true}; return {bf32(std::fmod(a, b)), false};
        }
        break;
    }
    case SG_T_DOUBLE: {
        double a = f64(l.b), b = f64(r.b);
        switch (op) {
        case SG_OP_ADD: return {bf64(a + b), false};
        case SG_OP_SUB: return {bf64(a - b), false};
        case SG_OP_MUL: return {bf64(a * b), false};
        case SG_OP_DIV: if (b == 0.0) return {0, true}; return {bf64(a / b), false};
        case SG_OP_MOD: if (b == 0.0) return {0, true}; return {bf64(std::fmod(a, b)), false};
        }
        break;
    }
    }
    throw std::runtime_error("bad arithmetic instruction");
}

template <class T> static bool cmp_op(int op, T a, T b) {
    switch (op) {
    case SG_OP_EQ: return a == b;
    case SG_OP_NE: return a != b;
    case SG_OP_GT: return a > b;
    case SG_OP_GE: return a >= b;
    case SG_OP_LT: return a < b;
    case SG_OP_LE: return a <= b;
    }
    return false;
}

static bool compare(int op, int dom, Val l, Val r) {
    // CompareConditionExpressionExecutor.java:38-42: null operand -> false;
    // NotEqualCompareConditionExpressionExecutor: null operand -> true
    if (l.null || r.null) return op == SG_OP_NE;
    switch (dom) {
    case SG_T_INT: return cmp_op(op, i32(l.b), i32(r.b));
    case SG_T_LONG: return cmp_op(op, i64(l.b), i64(r.b));
    case SG_T_FLOAT: return cmp_op(op, f32(l.b), f32(r.b));
    case SG_T_DOUBLE: return cmp_op(op, f64(l.b), f64(r.b));
    case SG_T_STRING: return cmp_op(op, (uint32_t)l.b, (uint32_t)r.b);
    case SG_T_BOOL: return cmp_op(op, (uint32_t)(l.b & 1), (uint32_t)(r.b & 1));
    }
    return false;
}

bool Engine::eval(const StateEvent* se, uint32_t pc, uint32_t len) const {
    Val stk[64];
    int sp = 0;
    uint32_t end = pc + len;
    while (pc < end) {
        uint32_t w = code[pc];
        uint32_t op = w & 0xff, a = (w >> 8) & 0xff, b = (w >> 16) & 0xff;
        if (sp > 60) throw std::runtime_error("filter stack overflow");
        switch (op) {
        case SG_OP_VAR: {
            StreamEvent* ev = chain_at(se, (int)b, (int32_t)code[pc + 2]);
            stk[sp++] = ev ? attr(ev->seq, code[pc + 1]) : Val{0, true};
            break;
        }
        case SG_OP_CONST:
            stk[sp++] = Val{(uint64_t)code[pc + 1] | ((uint64_t)code[pc + 2] << 32), b != 0};
            break;
        case SG_OP_CVT: stk[sp - 1] = cvt(stk[sp - 1], (int)a, (int)b); break;
        case SG_OP_ADD: case SG_OP_SUB: case SG_OP_MUL: case SG_OP_DIV: case SG_OP_MOD:
            stk[sp - 2] = arith((int)op, (int)a, stk[sp - 2], stk[sp - 1]);
            sp--;
            break;
        case SG_OP_EQ: case SG_OP_NE: case SG_OP_GT: case SG_OP_GE: case SG_OP_LT: case SG_OP_LE:
            stk[sp - 2] = Val{(uint64_t)compare((int)op, (int)a, stk[sp - 2], stk[sp - 1]), false};
            sp--;
            break;
        case SG_OP_AND: {  // AndConditionExpressionExecutor.java:65-74
            bool l = !stk[sp - 2].null && (stk[sp - 2].b & 1);
            bool r = !stk[sp - 1].null && (stk[sp - 1].b & 1);
            stk[sp - 2] = Val{(uint64_t)(l && r), false};
            sp--;
            break;
        }
        case SG_OP_OR: {  // OrConditionExpressionExecutor.java:65-75
            bool l = !stk[sp - 2].null && (stk[sp - 2].b & 1);
            bool r = !stk[sp - 1].null && (stk[sp - 1].b & 1);
            stk[sp - 2] = Val{(uint64_t)(l || r), false};
            sp--;
            break;
        }
        case SG_OP_NOT: {  // NotConditionExpressionExecutor.java:43-49
            bool t = !stk[sp - 1].null && (stk[sp - 1].b & 1);
            stk[sp - 1] = Val{(uint64_t)(!t), false};
            break;
        }
        case SG_OP_ISNULL: stk[sp - 1] = Val{(uint64_t)stk[sp - 1].null, false}; break;
        case SG_OP_ISNULL_EV: {
            StreamEvent* ev = chain_at(se, (int)b, (int32_t)code[pc + 1]);
            stk[sp++] = Val{(uint64_t)(ev == nullptr), false};
            break;
        }
        case SG_OP_IFELSE: {  // IfThenElseFunctionExecutor.java:127-133, 148-159: Boolean.TRUE.equals(cond)
            const bool c = !stk[sp - 3].null && (stk[sp - 3].b & 1);
            stk[sp - 3] = c ? stk[sp - 2] : stk[sp - 1];
            sp -= 2;
            break;
        }
        default: throw std::runtime_error("bad opcode");
        }
        pc += sg_op_len(op);
    }
    return sp > 0 && !stk[sp - 1].null && (stk[sp - 1].b & 1);
}

// ------------------------------------------------------------------------------------------------
// receivers (stabilize + per-event processing)
// ------------------------------------------------------------------------------------------------
void Engine::stabilize(const Receiver& r, int64_t ts) {
    for (PreProc* p : allStateProcessors) p->expireEvents(ts);
    if (qtype == SG_Q_SEQUENCE) {  // Sequence*ProcessStreamReceiver.stabilizeStates -> resetAndUpdate
        root->reset();
        root->update();
    } else if (r.multi) {  // PatternMultiProcessStreamReceiver.java:42-51
        for (PreProc* p : r.stateProcessorsForStream) p->updateState();
    } else if (!r.stateProcessorsForStream.empty()) {  // PatternSingleProcessStreamReceiver.java:34-41
        r.stateProcessorsForStream[0]->updateState();
    }
}

void Engine::project(const StateEvent* se) {
    Match m;
    m.trigger = curTrigger;
    m.key = curKey;
    m.ts = se->ts;
    m.chains.resize(nslots);
    for (int s = 0; s < nslots; s++) {
        for (StreamEvent* e = se->slots[s].get(); e; e = e->next.get()) m.chains[s].push_back(e->seq);
    }
    matches.push_back(std::move(m));
    stats.matches++;
}

// MultiProcessStreamReceiver.receive (one event) + StateMultiProcessStreamReceiver.processAndClear
void Engine::processEventMulti(int stream, uint64_t seq, int64_t ts) {
    Receiver& r = receivers[stream];
    curTrigger = seq;
    stabilize(r, ts);
    for (int idx : r.eventSequence) {
        std::vector<SE> ret;
        r.nextProcessors[idx]->processAndReturn(Ref<StreamEvent>(new StreamEvent(seq, ts)), ret);
        for (auto& se : ret) project(se.get());  // projected immediately (QuerySelector.process)
    }
}

// SingleProcessStreamReceiver.processAndClear: matches projected after the whole chunk
void Engine::processChunkSingle(int stream, const std::vector<std::pair<uint64_t, int64_t>>& evs) {
    Receiver& r = receivers[stream];
    std::vector<std::pair<uint64_t, SE>> collected;
    for (auto& e : evs) {
        stabilize(r, e.second);
        std::vector<SE> ret;
        r.nextProcessors[0]->processAndReturn(Ref<StreamEvent>(new StreamEvent(e.first, e.second)), ret);
        for (auto& se : ret) collected.emplace_back(e.first, se);
    }
    for (auto& c : collected) {
        curTrigger = c.first;
        project(c.second.get());
    }
}

// ------------------------------------------------------------------------------------------------
// build = StateInputStreamParser.parse
// ------------------------------------------------------------------------------------------------
struct Builder {
    Engine* e;
    const uint32_t* w;
    size_t n;
    size_t pos;

    uint32_t next() {
        if (pos >= n) throw std::runtime_error("truncated IR node tree");
        return w[pos++];
    }

    PreProc* newPre(int kind) {
        auto p = std::make_unique<PreProc>();
        p->id = (int)e->procs.size();
        p->kind = kind;
        p->stateType = e->qtype;
        p->eng = e;
        e->procs.push_back(std::move(p));
        return e->procs.back().get();
    }
    PostProc* newPost(int kind) {
        auto p = std::make_unique<PostProc>();
        p->kind = kind;
        p->eng = e;
        e->posts.push_back(std::move(p));
        return e->posts.back().get();
    }
    InnerRT* newRT(int tag) {
        e->rts.push_back(std::make_unique<InnerRT>());
        e->rts.back()->tag = tag;
        return e->rts.back().get();
    }

    // returns the inner runtime; `pre/post` are supplied by logical/count parents
    InnerRT* parse(PreProc* pre, PostProc* post, std::vector<PreProc*>& preList, bool isStart) {
        uint32_t tag = next();
        switch (tag) {
        case SG_N_STREAM: {  // StateInputStreamParser.java:167-225
            uint32_t slot = next(), stream = next(), fpc = next(), flen = next(), absent = next();
            uint32_t flo = next(), fhi = next();
            const int64_t forMs = (int64_t)((uint64_t)flo | ((uint64_t)fhi << 32));
            if (!pre) {
                pre = newPre(P_STREAM);
                if (absent) {
                    if (forMs < 0) throw std::runtime_error("absent stream state needs a 'for' time");
                    e->startup.push_back(pre);  // startupPreStateProcessors (StateInputStreamParser.java:181-197)
                }
            }
            pre->absent = absent != 0;
            pre->waitingTime = absent ? forMs : -1;
            pre->stateId = (int)slot;
            pre->isStart = isStart;
            pre->filterPc = fpc;
            pre->filterLen = flen;
            if (!post) post = newPost(P_STREAM);
            post->absent = absent != 0;
            post->stateId = (int)slot;
            post->thisPre = pre;
            pre->thisPost = post;
            pre->thisLast = post;
            InnerRT* rt = newRT(SG_N_STREAM);
            rt->first = pre;
            rt->last = post;
            rt->stream = (int)stream;
            preList.push_back(pre);
            return rt;
        }
        case SG_N_NEXT: {  // :227-259
            InnerRT* cur = parse(pre, post, preList, isStart);
            InnerRT* nx = parse(pre, post, preList, false);
            cur->last->setNextStatePre(nx->first);
            InnerRT* rt = newRT(SG_N_NEXT);
            rt->a = cur;
            rt->b = nx;
            rt->first = cur->first;
            rt->last = nx->last;
            return rt;
        }
        case SG_N_EVERY: {  // :261-287
            std::vector<PreProc*> withinEvery;
            InnerRT* inner = parse(pre, post, withinEvery, isStart);
            InnerRT* rt = newRT(SG_N_EVERY);
            rt->a = inner;
            rt->first = inner->first;
            rt->last = inner->last;
            rt->last->setNextEveryStatePre(rt->first);
            for (PreProc* p : withinEvery) p->withinEveryPre = rt->first;
            preList.insert(preList.end(), withinEvery.begin(), withinEvery.end());
            return rt;
        }
        case SG_N_LOGICAL: {  // :289-378
            uint32_t ltype = next();
            PreProc* lp1 = newPre(P_LOGICAL);
            PostProc* lpost1 = newPost(P_LOGICAL);
            PreProc* lp2 = newPre(P_LOGICAL);
            PostProc* lpost2 = newPost(P_LOGICAL);
            lp1->logicalType = lp2->logicalType = (int)ltype;
            lpost1->logicalType = lpost2->logicalType = (int)ltype;
            lpost1->partnerPre = lp2;
            lpost2->partnerPre = lp1;
            lpost1->partnerPost = lpost2;
            lpost2->partnerPost = lpost1;
            lp1->partner = lp2;
            lp2->partner = lp1;
            // AbsentLogicalPreStateProcessor pres join startupPreStateProcessors at creation, element 1
            // first (StateInputStreamParser.java:289-320)
            {
                size_t q = pos;
                const bool a1 = peekAbsent(q);
                skip_at(q);
                const bool a2 = peekAbsent(q);
                if (a1) e->startup.push_back(lp1);
                if (a2) e->startup.push_back(lp2);
            }
            // element 1 is encoded first, but element 2 must be parsed (and slotted) first
            size_t save = pos;
            skip();               // element 1
            InnerRT* rt2 = parse(lp2, lpost2, preList, isStart);
            size_t after = pos;
            pos = save;
            InnerRT* rt1 = parse(lp1, lpost1, preList, isStart);
            pos = after;
            InnerRT* rt = newRT(SG_N_LOGICAL);
            rt->a = rt1;
            rt->b = rt2;
            rt->first = rt1->first;
            rt->last = rt2->last;
            return rt;
        }
        case SG_N_COUNT: {  // :380-403
            uint32_t mn = next(), mx = next();
            PreProc* cp = newPre(P_COUNT);
            PostProc* cpost = newPost(P_COUNT);
            cp->minCount = (int)mn;
            cp->maxCount = mx == SG_COUNT_ANY ? INT32_MAX : (int)mx;
            cpost->minCount = cp->minCount;
            cpost->maxCount = cp->maxCount;
            cp->countPost = cpost;
            InnerRT* inner = parse(cp, cpost, preList, isStart);
            InnerRT* rt = newRT(SG_N_COUNT);
            rt->first = inner->first;
            rt->last = inner->last;
            rt->stream = inner->stream;
            return rt;
        }
        }
        throw std::runtime_error("bad node tag in IR");
    }

    bool peekAbsent(size_t q) const {  // the node at q is an absent stream state
        return q < n && w[q] == SG_N_STREAM && q + 5 < n && w[q + 5] != 0;
    }
    void skip_at(size_t& q) {
        size_t save = pos;
        pos = q;
        skip();
        q = pos;
        pos = save;
    }

    void skip() {
        uint32_t tag = next();
        switch (tag) {
        case SG_N_STREAM: pos += 7; return;
        case SG_N_NEXT: skip(); skip(); return;
        case SG_N_EVERY: skip(); return;
        case SG_N_LOGICAL: next(); skip(); skip(); return;
        case SG_N_COUNT: next(); next(); skip(); return;
        }
        throw std::runtime_error("bad node tag in IR");
    }

    // InnerStateRuntime.setup: register first processors with the stream receivers
    void setup(InnerRT* rt) {
        switch (rt->tag) {
        case SG_N_NEXT: setup(rt->a); setup(rt->b); return;
        case SG_N_EVERY: setup(rt->a); return;
        case SG_N_LOGICAL: setup(rt->b); setup(rt->a); return;
        default: {
            Receiver& r = e->receivers.at(rt->stream);
            r.nextProcessors.push_back(rt->first);
            r.stateProcessorsForStream.push_back(rt->first);
        }
        }
    }
};

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

void build(Engine* e, const void* ir, size_t len) {
    if (len < SG_IR_HDR_WORDS * 4 || len % 4) throw std::runtime_error("IR too short");
    e->ir.assign((const uint32_t*)ir, (const uint32_t*)ir + len / 4);
    const uint32_t* w = e->ir.data();
    if (w[0] != SG_IR_MAGIC || w[1] != SG_IR_VERSION) throw std::runtime_error("bad IR magic/version");
    e->qtype = (int)w[2];
    uint32_t nstreams = w[3];
    e->nslots = (int)w[4];
    e->within = (int64_t)((uint64_t)w[5] | ((uint64_t)w[6] << 32));
    uint32_t offStreams = w[7], offNodes = w[8], nNodes = w[9], offCode = w[10], nCode = w[11];
    e->partitioned = (w[12] & SG_IR_F_PARTITIONED) != 0;
    e->playback = (w[12] & SG_IR_F_PLAYBACK) != 0;
    size_t nw = e->ir.size();
    if (offCode + nCode > nw || offNodes + nNodes > nw) throw std::runtime_error("IR offsets out of range");
    e->code = w + offCode;
    e->codeLen = nCode;
    e->streams.resize(nstreams);
    e->receivers.resize(nstreams);
    size_t p = offStreams;
    for (uint32_t s = 0; s < nstreams; s++) {
        uint32_t na = w[p++];
        e->streams[s].types.assign(w + p, w + p + na);
        p += na;
        e->streams[s].cols.resize(na);
        for (uint32_t a = 0; a < na; a++) e->streams[s].cols[a].type = (int)e->streams[s].types[a];
    }
    Builder b{e, w + offNodes, nNodes, 0};
    std::vector<PreProc*> preList;
    e->root = b.parse(nullptr, nullptr, preList, true);
    e->allStateProcessors = preList;
    // QueryParser -> StateStreamRuntime.setCommonProcessor: query selector + setup
    e->root->setQuerySelector();
    b.setup(e->root);
    // StateInputStreamParser.java:129-143: within + start state ids, first.thisLast = last
    if (e->within != -1) {
        std::vector<int> startIds;
        for (PreProc* pp : preList) if (pp->isStart) startIds.push_back(pp->stateId);
        for (PreProc* pp : preList) {
            pp->startStateIds = startIds;
            pp->withinTime = e->within;
        }
    }
    e->root->first->thisLast = e->root->last;
    e->heads.resize(e->procs.size());
    // receiver kinds: Pattern/Sequence Multi when the stream appears more than once (:91-110)
    for (auto& r : e->receivers) {
        r.sequence = e->qtype == SG_Q_SEQUENCE;
        r.multi = r.nextProcessors.size() > 1;
        r.eventSequence.clear();
        for (int i = (int)r.nextProcessors.size() - 1; i >= 0; i--) r.eventSequence.push_back(i);
    }
}

void ensure_key(Engine* e, uint32_t key) {
    if (key >= e->keyStates.size()) {
        size_t n = std::max<size_t>(key + 1, e->keyStates.size() * 2);
        e->keyStates.resize(n);
        e->keyInit.resize(n, 0);
    }
    if (e->keyStates[key].empty()) e->keyStates[key].resize(e->procs.size());
}

// PartitionRuntimeImpl.initPartition -> StateStreamRuntime.initPartition (first event of a key)
void init_key(Engine* e, uint32_t key) {
    ensure_key(e, key);
    if (!e->keyInit[key]) {
        e->keyInit[key] = 1;
        uint32_t save = e->curKey;
        e->curKey = key;
        e->root->init();
        for (PreProc* p : e->startup) p->partitionCreated();  // StateStreamRuntime.initPartition :90-97
        e->curKey = save;
    }
}

}  // namespace

// ================================================================================================
// C-ABI (same signatures as include/siddhi_gpu.h, prefixed sgo_ so both can be loaded together)
// ================================================================================================
struct sgo_engine {
    Engine e;
};

extern "C" {

const char* sgo_last_error(void) { return g_err.c_str(); }

int sgo_engine_create(const void* ir, size_t ir_len, const sg_config* cfg, sgo_engine** out) {
    if (!ir || !out) return fail(SG_ERR_INVALID, "null argument");
    try {
        auto* h = new sgo_engine();
        build(&h->e, ir, ir_len);
        (void)cfg;
        // unpartitioned: QueryRuntimeImpl.start seeds once, at the first sgo_advance_time / push
        *out = h;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_UNSUPPORTED, ex.what());
    }
}

void sgo_engine_destroy(sgo_engine* h) { delete h; }

// partition purge (PartitionRuntimeImpl.java:368-401): the key is removed from partitionKeys and every
// state holder of the partition's queries drops its states (cleanGroupByStates), the schedulers' per-key
// queues included; its next event runs initPartition again
int sgo_reset_keys(sgo_engine* h, const uint32_t* keys, uint64_t n, uint32_t mem) {
    if (!h || (!keys && n)) return fail(SG_ERR_INVALID, "null argument");
    if (mem != SG_MEM_HOST) return fail(SG_ERR_INVALID, "oracle takes host key lists only");
    Engine& e = h->e;
    if (!e.partitioned) return SG_OK;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t k = keys[i];
        if (k >= e.keyStates.size()) continue;  // never seen: nothing to drop
        e.keyStates[k].clear();
        e.keyInit[k] = 0;
        for (auto& hs : e.heads)
            for (auto it = hs.begin(); it != hs.end();) it = (it->second == k) ? hs.erase(it) : std::next(it);
        for (auto it = e.callers.begin(); it != e.callers.end();)
            it = (std::get<1>(*it) == k) ? e.callers.erase(it) : std::next(it);
    }
    return SG_OK;
}

int sgo_push_batch(sgo_engine* h, const sg_batch* b) {
    if (!h || !b) return fail(SG_ERR_INVALID, "null argument");
    Engine& e = h->e;
    try {
        if (b->mem != SG_MEM_HOST) return fail(SG_ERR_INVALID, "oracle takes host batches only");
        if (b->stream >= e.streams.size()) return fail(SG_ERR_INVALID, "stream index out of range");
        StreamStore& ss = e.streams[b->stream];
        if (b->n_cols != ss.cols.size()) return fail(SG_ERR_INVALID, "column count mismatch");
        if (e.partitioned && !b->key) return fail(SG_ERR_INVALID, "partitioned query needs key ids");
        if (!e.haveSeq0) {
            e.seq0 = b->seq_base;
            e.haveSeq0 = true;
        }
        e.clockSet = true;
        if (b->seq_base < e.seq0 + e.seqLoc.size()) return fail(SG_ERR_INVALID, "sequence numbers must increase");
        if (!e.partitioned) init_key(&e, 0);
        // store rows
        uint32_t row0 = ss.cols.empty() ? 0 : (uint32_t)ss.cols[0].v.size();
        if (ss.cols.empty()) row0 = (uint32_t)(e.seqLoc.size());  // stream without attributes
        for (uint32_t a = 0; a < b->n_cols; a++) {
            Column& c = ss.cols[a];
            const uint8_t* nl = b->nulls ? b->nulls[a] : nullptr;
            for (uint64_t i = 0; i < b->n; i++) {
                uint64_t v = 0;
                switch (c.type) {
                case SG_T_INT: case SG_T_FLOAT: case SG_T_STRING: v = ((const uint32_t*)b->cols[a])[i]; break;
                case SG_T_LONG: case SG_T_DOUBLE: v = ((const uint64_t*)b->cols[a])[i]; break;
                case SG_T_BOOL: v = ((const uint8_t*)b->cols[a])[i] ? 1 : 0; break;
                }
                c.v.push_back(v);
                if (nl || !c.null.empty()) {
                    if (c.null.size() < c.v.size() - 1) c.null.resize(c.v.size() - 1, 0);
                    c.null.push_back(nl ? nl[i] : 0);
                }
            }
        }
        e.seqLoc.resize(b->seq_base - e.seq0, EvLoc{UINT32_MAX, 0});
        for (uint64_t i = 0; i < b->n; i++) e.seqLoc.push_back(EvLoc{b->stream, row0 + (uint32_t)i});
        e.stats.events += b->n;
        e.stats.batches++;

        Receiver& r = e.receivers[b->stream];
        // chunking: PartitionStreamReceiver.receive(Event[]) sends runs of consecutive same-key events
        uint64_t i = 0;
        while (i < b->n) {
            uint32_t key = e.partitioned ? b->key[i] : 0;
            uint64_t j = i + 1;
            if (e.partitioned)
                while (j < b->n && b->key[j] == key) j++;
            else
                j = b->n;
            init_key(&e, key);
            e.curKey = key;
            if (r.nextProcessors.empty()) { i = j; continue; }
            if (r.multi) {
                for (uint64_t k = i; k < j; k++) e.processEventMulti((int)b->stream, b->seq_base + k, b->ts[k]);
            } else {
                std::vector<std::pair<uint64_t, int64_t>> evs;
                for (uint64_t k = i; k < j; k++) evs.emplace_back(b->seq_base + k, b->ts[k]);
                e.processChunkSingle((int)b->stream, evs);
            }
            i = j;
        }
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_STATE, ex.what());
    }
}

int sgo_advance_time(sgo_engine* h, int64_t now) {
    if (!h) return fail(SG_ERR_INVALID, "null argument");
    Engine& e = h->e;
    try {
        e.clockSet = true;
        if (!e.partitioned && (e.keyInit.empty() || !e.keyInit[0])) {
            if (!e.playback) e.now = std::max(e.now, now);  // start(): wall clock now
            init_key(&e, 0);
        }
        e.advanceTime(now);
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_STATE, ex.what());
    }
}

int sgo_poll_matches(sgo_engine* h, uint32_t mem, sg_match_batch* out) {
    if (!h || !out) return fail(SG_ERR_INVALID, "null argument");
    // (SG_POLL_READY: every batch of the oracle is complete when its push returns)
    if ((mem & ~SG_POLL_READY) != SG_MEM_HOST) return fail(SG_ERR_INVALID, "oracle returns host memory only");
    Engine& e = h->e;
    uint32_t maxc = 1;
    for (auto& m : e.matches)
        for (auto& c : m.chains) maxc = std::max<uint32_t>(maxc, (uint32_t)c.size());
    size_t n = e.matches.size();
    e.outTrig.resize(n);
    e.outKey.resize(n);
    e.outTs.resize(n);
    e.outSlot.assign(n * e.nslots * maxc, SG_NULL_SEQ);
    e.outLen.assign(n * e.nslots, 0);
    for (size_t i = 0; i < n; i++) {
        const Match& m = e.matches[i];
        e.outTrig[i] = m.trigger;
        e.outKey[i] = m.key;
        e.outTs[i] = m.ts;
        for (int s = 0; s < e.nslots; s++) {
            e.outLen[i * e.nslots + s] = (uint32_t)m.chains[s].size();
            for (size_t c = 0; c < m.chains[s].size(); c++) e.outSlot[(i * e.nslots + s) * maxc + c] = m.chains[s][c];
        }
    }
    e.matches.clear();
    out->n = n;
    out->n_slots = (uint32_t)e.nslots;
    out->max_chain = maxc;
    out->trigger_seq = e.outTrig.data();
    out->key = e.outKey.data();
    out->ts = e.outTs.data();
    out->slot_seq = e.outSlot.data();
    out->chain_len = e.outLen.data();
    out->mem = SG_MEM_HOST;
    out->reserved = 0;
    return SG_OK;
}

int sgo_release_matches(sgo_engine* h, sg_match_batch* m) {
    (void)h;
    if (m) memset(m, 0, sizeof(*m));
    return SG_OK;
}

// ---- the per-key state in the reference's per-state-processor form (state_doc.h) ----------------------
// StreamPreState.snapshot (StreamPreStateProcessor.java:450-469) + Count / Absent extras + the
// Scheduler's toNotifyQueue, per initialised key
int sgo_state_export(sgo_engine* h, void** buf, size_t* len) {
    if (!h || !buf || !len) return fail(SG_ERR_INVALID, "null argument");
    Engine& e = h->e;
    try {
        SdDoc d;
        d.n_procs = (uint32_t)e.procs.size();
        d.n_slots = (uint32_t)e.nslots;
        for (const auto& p : e.procs) d.desc.push_back(SdProcDesc{(uint32_t)p->kind, p->absent ? 1u : 0u, (uint32_t)p->stateId});
        d.now = e.now;
        d.last_event_ts = e.lastEventTs;
        d.clock_flags = e.clockSet ? 1u : 0u;
        for (uint32_t k = 0; k < e.keyInit.size(); k++) {
            if (!e.keyInit[k]) continue;
            SdKeyBuilder<const StateEvent*, const StreamEvent*> B;
            B.k.key = k;
            auto visit_ev = [&](const StreamEvent* ev) -> uint32_t {
                bool fresh;
                const uint32_t i = B.stream(ev, fresh);
                if (!fresh) return i;
                SdStream s;
                s.seq = ev->seq;
                s.ts = ev->ts;
                if (ev->seq == SG_BLANK_SEQ) {
                    s.null_bits = 0xffffffffu;
                } else if (e.stored(ev->seq)) {
                    const EvLoc& l = e.seqLoc[ev->seq - e.seq0];
                    const StreamStore& ss = e.streams[l.stream];
                    for (uint32_t a = 0; a < ss.cols.size(); a++) {
                        const Val v = e.attr(ev->seq, a);
                        s.attr.push_back(v.b);
                        if (v.null) s.null_bits |= 1u << a;
                    }
                    s.present = ss.cols.size() >= 32 ? 0xffffffffu : ((1u << ss.cols.size()) - 1u);
                } else {
                    auto it = e.importedAttrs.find(ev->seq);
                    if (it != e.importedAttrs.end()) {
                        s.attr = it->second.first;
                        s.null_bits = it->second.second;
                        s.present = s.attr.size() >= 32 ? 0xffffffffu : ((1u << s.attr.size()) - 1u);
                    }
                }
                B.k.streams[i] = s;
                return i;
            };
            auto visit_st = [&](const StateEvent* se) -> uint32_t {
                bool fresh;
                const uint32_t i = B.state(se, fresh);
                if (!fresh) return i;
                SdState st;
                st.ts = se->ts;
                st.type = se->type == EXPIRED ? 1u : 0u;
                st.chains.resize(e.nslots);
                for (int sl = 0; sl < e.nslots; sl++)
                    for (const StreamEvent* ev = se->slots[sl].get(); ev; ev = ev->next.get())
                        st.chains[sl].push_back(visit_ev(ev));
                B.k.states[i] = st;
                return i;
            };
            for (size_t p = 0; p < e.procs.size(); p++) {
                const KeyState& ks = e.keyStates[k][p];
                SdProc P;
                P.flags = (ks.initialized ? (uint32_t)SD_INITIALIZED : 0u) | (ks.started ? (uint32_t)SD_STARTED : 0u) |
                          (ks.successCondition ? (uint32_t)SD_SUCCESS : 0u) |
                          (ks.startStateReset ? (uint32_t)SD_SSRESET : 0u) | (ks.active ? (uint32_t)SD_ACTIVE : 0u);
                P.last_scheduled = ks.lastScheduledTime;
                P.last_arrival = ks.lastArrivalTime;
                for (const SE& se : ks.pending) P.pending.push_back(visit_st(se.get()));
                for (const SE& se : ks.newAndEvery) P.newev.push_back(visit_st(se.get()));
                P.queue.assign(ks.toNotify.begin(), ks.toNotify.end());
                P.running = ks.running ? 1u : 0u;
                P.fire_at = ks.running ? ks.fireAt : 0;
                P.order = ks.order;
                B.k.procs.push_back(P);
            }
            sd_rank_orders(B.k);
            d.keys.push_back(std::move(B.k));
        }
        std::vector<uint8_t> bytes = sd_write(d);
        void* out = malloc(bytes.size());
        if (!out) return fail(SG_ERR_CAPACITY, "state document allocation failed");
        memcpy(out, bytes.data(), bytes.size());
        *buf = out;
        *len = bytes.size();
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_STATE, ex.what());
    }
}

int sgo_free_buffer(void* buf) {
    free(buf);
    return SG_OK;
}

// replaces the whole NFA state (keys absent from the document become never-seen); the document's events
// keep their attributes for the filters and projections that read them later
int sgo_state_import(sgo_engine* h, const void* buf, size_t len) {
    if (!h || !buf) return fail(SG_ERR_INVALID, "null argument");
    Engine& e = h->e;
    try {
        const SdDoc d = sd_read(buf, len);
        bool same = d.n_procs == e.procs.size() && d.n_slots == (uint32_t)e.nslots;
        for (size_t p = 0; same && p < e.procs.size(); p++)
            same = d.desc[p] == SdProcDesc{(uint32_t)e.procs[p]->kind, e.procs[p]->absent ? 1u : 0u,
                                           (uint32_t)e.procs[p]->stateId};
        if (!same) return fail(SG_ERR_INVALID, "state document of a different query shape");
        for (auto& ks : e.keyStates) ks.clear();
        std::fill(e.keyInit.begin(), e.keyInit.end(), 0);
        for (auto& hs : e.heads) hs.clear();
        e.callers.clear();
        e.now = d.now;
        e.lastEventTs = d.last_event_ts;
        e.clockSet = (d.clock_flags & 1u) != 0;
        uint64_t maxRank = 0;
        for (const SdKey& k : d.keys) {
            if (e.partitioned ? false : k.key != 0) return fail(SG_ERR_INVALID, "unpartitioned query with a key other than 0");
            ensure_key(&e, k.key);
            e.keyInit[k.key] = 1;
            std::vector<Ref<StreamEvent>> evs;
            for (const SdStream& s : k.streams) {
                evs.emplace_back(new StreamEvent(s.seq, s.ts));
                if (s.seq != SG_BLANK_SEQ && !e.stored(s.seq)) e.importedAttrs[s.seq] = {s.attr, s.null_bits};
            }
            std::vector<SE> sts;
            for (const SdState& st : k.states) {
                SE se(new StateEvent(e.nslots));
                se->ts = st.ts;
                se->type = st.type ? EXPIRED : CURRENT;
                for (int sl = 0; sl < e.nslots; sl++) {
                    const auto& c = st.chains[sl];
                    if (c.empty()) continue;
                    se->slots[sl] = evs[c[0]];
                    for (size_t i = 0; i + 1 < c.size(); i++) evs[c[i]]->next = evs[c[i + 1]];
                }
                sts.push_back(se);
            }
            for (size_t p = 0; p < e.procs.size(); p++) {
                const SdProc& P = k.procs[p];
                KeyState& ks = e.keyStates[k.key][p];
                ks.initialized = (P.flags & SD_INITIALIZED) != 0;
                ks.started = (P.flags & SD_STARTED) != 0;
                ks.successCondition = (P.flags & SD_SUCCESS) != 0;
                ks.startStateReset = (P.flags & SD_SSRESET) != 0;
                ks.active = (P.flags & SD_ACTIVE) != 0;
                ks.lastScheduledTime = P.last_scheduled;
                ks.lastArrivalTime = P.last_arrival;
                for (uint32_t x : P.pending) ks.pending.push_back(sts[x]);
                for (uint32_t x : P.newev) ks.newAndEvery.push_back(sts[x]);
                ks.toNotify.assign(P.queue.begin(), P.queue.end());
                if (!ks.toNotify.empty()) e.heads[p].insert({ks.toNotify.front(), k.key});
                ks.running = P.running != 0;
                if (ks.running) {
                    ks.fireAt = P.fire_at;
                    ks.order = e.schedOrder + P.order;
                    maxRank = std::max<uint64_t>(maxRank, P.order);
                    e.callers.insert({ks.fireAt, k.key, ks.order, (int)p});
                }
            }
        }
        e.schedOrder += maxRank;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_INVALID, ex.what());
    }
}

int sgo_get_stats(sgo_engine* h, sg_stats* out) {
    if (!h || !out) return fail(SG_ERR_INVALID, "null argument");
    Engine& e = h->e;
    // live partial matches: StateEvents holding at least one event (start-state seeds excluded)
    uint64_t live = 0;
    auto count = [&](const SEList& l) {
        for (auto& se : l) {
            for (auto& sl : se->slots)
                if (sl) { live++; break; }
        }
    };
    for (auto& ks : e.keyStates)
        for (auto& s : ks) { count(s.pending); count(s.newAndEvery); }
    e.stats.partials_live = live;
    *out = e.stats;
    return SG_OK;
}

}  // extern "C"
