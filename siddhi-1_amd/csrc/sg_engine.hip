// sg_engine.hip — host side of the C-ABI (include/siddhi_gpu.h) for the MI355X engine.
//
// Per engine (= one compiled query on one HIP device) it keeps the partial-match state of every
// partition key resident in HBM (SoA slabs sized n_keys x partial_capacity), and per pushed
// micro-batch runs:
//   1. (host batches only) H2D copy of the SoA columns the filters read
//   2. key grouping (part_kernels.hip, hand-written): the batch stably partitioned by key tile (the 256 keys of
//      one advance workgroup), the split by key happening inside the advance kernel's LDS staging (fused); or,
//      for batches too dense per tile, LSD passes to a key-sorted payload + per-key segment bounds — replaces
//      the key-run grouping of PartitionStreamReceiver.receive(Event[]) (partition/PartitionStreamReceiver.java:
//      175-260) and the per-key state lookup (util/snapshot/state/PartitionStateHolder.java:43-80)
//   3. k_adv_m: one lane per key advances that key's NFA over its events in arrival order
//      (query/input/stream/state/StreamPreStateProcessor.java:308-403 and friends)
// and on poll orders the accumulated matches by trigger seq (stable: per-key emission order kept).
//
// Query shapes outside the specialised two-state kernel (count, logical, SEQUENCE, absent states,
// longer chains) run on the general device engine (gen_host.hip / gen_kernels.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <map>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/siddhi_gpu.h"
#include "../../include/siddhi_gpu_ir.h"
#include "gen_engine.h"
#include "gen_host.h"
#include "pack.h"
#include "part.h"
#include "pinned.h"
#include "sg_sharded.h"
#include "state_doc.h"
#include "sg_engine.h"
#include "sg_jit.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define HIP_OK(x)                                                                                       \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess)                                                                           \
            throw HipError(std::string(#x) + ": " + hipGetErrorString(e_));                             \
    } while (0)

struct IRStream {
    std::vector<uint32_t> types;
};

// P2 plan: the lowered two-state query
struct Plan {
    int mode = 0;
    int s0 = -1, s1 = -1;     // stream of state 0 / 1
    uint32_t slot0 = 0, slot1 = 1;
    int64_t within = -1;
    bool partitioned = false;
    // per stream: event columns the kernel loads (attr indices)
    std::vector<std::vector<uint32_t>> evcols;
    std::vector<uint32_t> caps;          // slot-0 attrs captured into partials
    std::vector<uint8_t> cap_col;        // index of each capture in evcols[s0]
    std::vector<uint8_t> cap_type;
    DProg f0{}, f1{};
};

uint32_t op_words(uint32_t op) { return (op == SG_OP_VAR || op == SG_OP_CONST) ? 3u : (op == SG_OP_ISNULL_EV ? 2u : 1u); }

uint32_t bits_for(uint64_t n) {
    uint32_t b = 1;
    while (b < 64 && (1ull << b) < n) b++;
    return b;
}

template <class T> T* dalloc(size_t n, std::vector<void*>& owned) {
    void* p = nullptr;
    if (n == 0) n = 1;
    HIP_OK(hipMalloc(&p, n * sizeof(T)));
    owned.push_back(p);
    return (T*)p;
}

size_t type_size(uint32_t t) {
    switch (t) {
    case SG_T_LONG: case SG_T_DOUBLE: return 8;
    case SG_T_BOOL: return 1;
    default: return 4;
    }
}



}  // namespace

struct sg_engine {
    ShardEngine* shard = nullptr;   // n_devices > 1: the multi-device fan-out (sg_sharded.cpp) behind this handle
    int device = 0;
    hipStream_t stream = nullptr;
    GenEngine* gen = nullptr;  // the general engine, when the query is not a two-state pattern
    sg_config cfg{};
    std::vector<uint32_t> ir;
    uint64_t ir_hash = 0;  // FNV-1a of the IR words: a snapshot restores only into the same query
    std::vector<IRStream> streams;
    Plan plan;
    uint32_t K = 1, cap = 64, maxb = 0;
    bool null_keys = false;
    uint64_t mcap = 0;
    uint64_t raw_cap = 0;  // mcap + one reservation chunk of slack per advance-kernel wave
    std::vector<void*> owned;

    // state
    uint32_t* hdr = nullptr;
    int64_t* p_ts = nullptr;
    uint64_t* p_seq = nullptr;
    uint32_t* p_capw = nullptr;
    uint32_t n_capw = 0;
    uint32_t* p_capnull = nullptr;
    bool nullable = false;
    // query-specialised kernels (sg_jit.cpp), one code object per null variant
    struct Variant {
        hipModule_t mod = nullptr;
        hipFunction_t adv[2] = {nullptr, nullptr};   // [0]: multi / state-0 stream, [1]: state-1 stream
        hipFunction_t adv_h[2] = {nullptr, nullptr}; // the HBM pass over the waves the staged pass deferred
        hipFunction_t adv_k[2] = {nullptr, nullptr}; // ... and over the keys it stopped (wider window)
        hipFunction_t pack[2] = {nullptr, nullptr};
        hipFunction_t hot[14] = {};                  // the hot-key pipeline (k_hot_prep .. k_hot_final_big)
        uint32_t adv_static_lds = 0;                 // the staged pass's static LDS (beside its dynamic staging)
    };
    JitQuery jq;
    std::vector<uint64_t> consts;
    std::map<int, Variant> variants;  // key: evnull | capnull << 1
    // Batch pipeline: batch i's H2D copies and key grouping run on `gstream` into buffer slot i % 2
    // while batch i-1's advance, ordering and projection run on `stream`; a slot is reused once the
    // batch two back has finished reading it (slot.free), the advance waits for its grouping
    // (slot.grouped).  Per-key state, raw matches and the ordered output live on `stream` only.
    hipStream_t gstream = nullptr;
    hipStream_t pstream = nullptr;            // device->host copies of polls
    struct Slot {
        int64_t* b_ts = nullptr;            // host batches: staging of the copied columns
        uint32_t* b_key = nullptr;
        std::vector<void*> b_cols;          // per filter column
        std::vector<uint8_t*> b_nulls;
        std::vector<void*> b_pcols;         // per projection column
        std::vector<uint8_t*> b_pnulls;
        uint32_t* sidx = nullptr;           // wide payloads: batch positions in key order
        uint32_t* seg_begin = nullptr;
        uint32_t* seg_end = nullptr;
        void* pay = nullptr;                // key-sorted payload [max_batch] x pay_words
        void* tpay = nullptr;               // fused grouping: the payload grouped by key tile [max_batch] x pay_words
        uint32_t* tile_lo = nullptr;        // fused grouping: [n_tiles + 1]
        hipEvent_t grouped = nullptr, copied = nullptr, free_ev = nullptr;
        bool used = false;
    };
    Slot slots[2];
    uint64_t nbatch = 0;
    // grouping scratch (part.h), shared by the slots: both slots' groupings run on gstream, one after the other
    PartScratch pscr{};
    bool fused_ok = false;        // the fused tile grouping is possible for this engine (K <= 2^20, max_batch <= 2^24)
    bool fused_last = false;      // the last batch took it (sg_engine_describe)
    uint32_t pay_words = 0;
    // per pushed batch, after its ordering: the {match count, error word} status block copied to pinned
    // host memory and an event, so a poll finds the completed batches without waiting for the others
    static constexpr uint32_t RING = 64;
    unsigned long long* h_status = nullptr;   // pinned [RING][2]
    hipEvent_t done_ev[RING] = {};
    std::vector<uint32_t> inflight;            // ring indices of batches not yet seen complete, in order
    uint64_t done_count = 0;                   // out_count after the newest completed batch
    uint32_t done_err = 0;
    uint64_t win = 0;                          // matches handed out so far (the poll window's start)
    bool async_host = false;                   // SG_CFG_ASYNC_HOST
    // matches
    uint64_t* raw_e1 = nullptr;
    unsigned long long* raw_count = nullptr;
    uint64_t raw_static = 0;       // raw slots owned by the staged pass's waves (no atomics)
    unsigned long long* wstats = nullptr;  // per-wave counters of the staged pass (one batch)
    uint64_t* t_desc = nullptr;    // per batch event: match count << 32 | first raw slot
    uint32_t* deferred = nullptr;  // per advance wave: left by the staged pass to the HBM pass
    unsigned long long* prof = nullptr;  // SG_PROF: walk-phase clocks of the staged pass (experiments)
    size_t prof_rows = 0;
    uint32_t* resume = nullptr;    // per key: where the HBM pass resumes a key the staged pass stopped
    // hot keys (`every e1 -> e2` on one stream, p2_jit.hip k_hot_*): the staged pass lists a key with >= hot_min
    // events; the pipeline runs after it while recent batches had such keys (hot_on: their count comes back in
    // the status block), otherwise the HBM pass walks them
    bool hot_ok = false;
    bool hot_on = true;
    uint32_t hot_idle = 0;         // drained batches in a row without hot keys (the pipeline's buffers are given
                                   // back after SGD_HOT_IDLE of them)
    std::vector<void*> hot_owned;  // the pipeline's per-event / per-partial buffers (hot_buffers)
    bool skewed = false;           // recent batches had workgroup ranges > SGD_BIG_TILE events: sorted grouping
    uint32_t hot_min = 0, hot_cap = 0, hot_exmax = 0;
    uint32_t hot_n0 = 0;           // carried-in live partials that make a key hot (0: the HBM pass's window + 1:
                                   // keys with more go to the pipeline, C2_walk 2.35 -> 1.94 ms against 13)
    uint64_t hot_factor = 4;       // "hot": also >= hot_factor x the batch's mean events per key (SG_HOT_FACTOR)
    uint32_t *hot_ctl = nullptr, *hot_list = nullptr, *hot_info = nullptr, *hot_death = nullptr, *hot_wl = nullptr;
    uint32_t *hot_tcnt = nullptr, *hot_tbase = nullptr, *hot_alive = nullptr, *hot_fh = nullptr, *hot_fbi = nullptr, *hot_cur = nullptr;
    uint64_t hot_batches = 0;      // batches the pipeline ran on (sg_engine_describe)
    uint32_t hbm_grid = 2048;      // work-groups of the HBM pass (SG_HBM_GRID: experiments)
    uint32_t* dlist = nullptr;     // the waves the HBM pass takes, and their number
    uint32_t* dlist_n = nullptr;
    uint32_t* klist = nullptr;     // the keys the staged pass stopped (the HBM pass's lanes)
    uint32_t* tile_sum = nullptr;  // ordering: matches per tile of triggers
    uint32_t td_epoch = 0;         // the current batch's t_desc tag (1..0xffff; t_desc cleared at the wrap)
    unsigned long long* out_count = nullptr;
    unsigned long long* batch_total = nullptr;
    unsigned long long* stats = nullptr;
    uint32_t* err = nullptr;
    // ordered output
    uint64_t* o_trig = nullptr;
    uint64_t* o_slot = nullptr;
    uint32_t* o_key = nullptr;
    int64_t* o_ts = nullptr;
    uint32_t* o_len = nullptr;
    // host copies
    PinnedVec<uint64_t> h_trig, h_slot;
    PinnedVec<uint32_t> h_key, h_len;
    PinnedVec<int64_t> h_ts;
    uint64_t poll_base = 0;
    bool have_base = false;
    uint64_t next_seq = 0;
    bool held = false;
    sg_stats st{};
    // SG_CFG_TIMING: event pairs per stage, resolved at the next synchronisation point
    struct Span { hipEvent_t a, b; int stage; };
    std::vector<Span> spans;
    std::vector<hipEvent_t> free_events;
    bool timing = false;
    // on-device projection of the select list (sg_set_projection)
    uint32_t proj_n = 0;
    std::vector<uint32_t> proj_attrs;     // trigger-stream attributes the projection reads
    uint32_t* d_proj = nullptr;           // rewritten code | item pc | item len | capture word offsets | types
    ProjParams pp{};
    uint32_t* raw_capw = nullptr;
    uint32_t* raw_capnull = nullptr;
    uint32_t* o_capw = nullptr;
    uint32_t* o_capnull = nullptr;
    uint64_t* pval = nullptr;
    uint8_t* pnull = nullptr;
    uint32_t proj_out = 0;                // output items: select list + having
    // aggregators of the selector (QuerySelector + their per-key states, PartitionStateHolder)
    uint32_t n_agg = 0;
    const uint32_t* d_agg_type = nullptr;
    uint64_t* aggv = nullptr;             // [n_agg][mcap] argument, then value, per output record
    uint8_t* aggnull = nullptr;
    int64_t* agg_n = nullptr;             // [n_agg][K] per-key state
    uint64_t* agg_v = nullptr;
    uint8_t* agg_has = nullptr;
    uint64_t* out_first = nullptr;        // [max_batch] per batch event: its records (ScatterParams)
    uint64_t polled = 0;
    PinnedVec<uint64_t> h_pval;
    PinnedVec<uint8_t> h_pnull;
    uint32_t reg_slots = 14;  // SGD_REG_SLOTS: partials per key held in registers by the advance kernel (14 against
                              // 12: staged pass 4.5 % faster, fewer keys stopped for the HBM pass, same occupancy —
                              // LDS-bound at three workgroups per CU, where 168 VGPRs are free; 16: slower)
    uint32_t reg_slots_hbm = 16;  // SGD_REG_SLOTS_HBM: the HBM pass's window (the keys the staged pass stopped;
                                  // 24 walks C2_walk 10 % faster but compiles 3.5x slower per query)
    uint32_t stage_override = 0;  // SGD_STAGE_CHUNKS: fixed LDS staging per wave (tests force the HBM path)
    uint64_t spills = 0;

    hipEvent_t ev() {
        hipEvent_t x;
        if (!free_events.empty()) { x = free_events.back(); free_events.pop_back(); return x; }
        if (hipEventCreate(&x) != hipSuccess) throw std::runtime_error("hipEventCreate failed");
        return x;
    }
    void mark(hipEvent_t x, hipStream_t s = nullptr) {
        if (hipEventRecord(x, s ? s : stream) != hipSuccess) throw std::runtime_error("hipEventRecord failed");
    }
    void resolve_spans() {  // call after the stream is synchronised
        for (auto& s : spans) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, s.a, s.b) == hipSuccess) {
                uint64_t ns = (uint64_t)((double)ms * 1e6);
                if (s.stage == 0) st.group_ns += ns;
                else if (s.stage == 1) st.advance_ns += ns;
                else if (s.stage == 3) { st.advance_ns += ns; st.advance_hbm_ns += ns; }
                else st.order_ns += ns;
            }
            free_events.push_back(s.a);
            free_events.push_back(s.b);
        }
        spans.clear();
    }

    ~sg_engine() {
        if (device >= 0) (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (prof) {  // SG_PROF experiments: s_memtime ticks per walk phase, summed over waves
            std::vector<unsigned long long> rows(prof_rows * 8);
            unsigned long long h[8] = {0};
            if (hipMemcpy(rows.data(), prof, rows.size() * 8, hipMemcpyDeviceToHost) == hipSuccess)
                for (size_t r = 0; r < prof_rows; ++r)
                    for (int i = 0; i < 8; ++i) h[i] += rows[r * 8 + i];
            if (true)
                fprintf(stderr, "SG_PROF phases: stop/decode %llu stabilize %llu f1 %llu emit %llu seed %llu\n",
                        h[0], h[1], h[2], h[3], h[4]);
        }
        if (gstream) (void)hipStreamSynchronize(gstream);
        if (gen) gen_destroy(gen);
        for (auto& sl : slots)
            for (hipEvent_t x : {sl.grouped, sl.copied, sl.free_ev})
                if (x) (void)hipEventDestroy(x);
        for (hipEvent_t x : done_ev)
            if (x) (void)hipEventDestroy(x);
        if (h_status) (void)hipHostFree(h_status);
        for (auto& sp : spans) { (void)hipEventDestroy(sp.a); (void)hipEventDestroy(sp.b); }
        for (auto x : free_events) (void)hipEventDestroy(x);
        for (void* p : owned) (void)hipFree(p);
        if (!hot_owned.empty()) {   // (stream-ordered allocations: freed on the stream, then drained)
            for (void* p : hot_owned) (void)hipFreeAsync(p, stream);
            (void)hipStreamSynchronize(stream);
        }
        for (auto& kv : variants)
            if (kv.second.mod) (void)hipModuleUnload(kv.second.mod);
        if (stream) (void)hipStreamDestroy(stream);
        if (gstream) (void)hipStreamDestroy(gstream);
        if (pstream) (void)hipStreamDestroy(pstream);
    }
};

namespace {

// ------------------------------------------------------------------------------------------------
// IR -> Plan (two-state pattern shapes)
// ------------------------------------------------------------------------------------------------
struct Node {
    uint32_t tag = 0;
    uint32_t slot = 0, stream = 0, fpc = 0, flen = 0, absent = 0;
    uint32_t a = 0, b = 0;  // logical type / count min,max
    std::vector<Node> kids;
};

Node read_node(const uint32_t* w, size_t n, size_t& pos) {
    if (pos >= n) throw std::runtime_error("truncated IR node tree");
    Node x;
    x.tag = w[pos++];
    switch (x.tag) {
    case SG_N_STREAM:
        if (pos + 7 > n) throw std::runtime_error("truncated IR node");
        x.slot = w[pos]; x.stream = w[pos + 1]; x.fpc = w[pos + 2]; x.flen = w[pos + 3]; x.absent = w[pos + 4];
        pos += 7;
        break;
    case SG_N_NEXT: x.kids.push_back(read_node(w, n, pos)); x.kids.push_back(read_node(w, n, pos)); break;
    case SG_N_EVERY: x.kids.push_back(read_node(w, n, pos)); break;
    case SG_N_LOGICAL: x.a = w[pos++]; x.kids.push_back(read_node(w, n, pos)); x.kids.push_back(read_node(w, n, pos)); break;
    case SG_N_COUNT: x.a = w[pos++]; x.b = w[pos++]; x.kids.push_back(read_node(w, n, pos)); break;
    default: throw std::runtime_error("bad IR node tag");
    }
    return x;
}

uint32_t col_index(std::vector<uint32_t>& cols, uint32_t attr) {
    for (size_t i = 0; i < cols.size(); i++)
        if (cols[i] == attr) return (uint32_t)i;
    if (cols.size() >= SGD_MAX_EVCOLS) throw std::runtime_error("filters read too many attributes");
    cols.push_back(attr);
    return (uint32_t)cols.size() - 1;
}

// lower one filter's bytecode: `own` = slot of the state the filter belongs to
void lower_filter(const uint32_t* code, uint32_t pc, uint32_t len, uint32_t own, Plan& pl,
                  std::vector<uint32_t>& evcols, DProg& out, bool is_state1) {
    out = DProg{};
    uint32_t end = pc + len;
    int sp = 0, maxsp = 0;
    while (pc < end) {
        uint32_t w = code[pc];
        uint32_t op = w & 0xff, a = (w >> 8) & 0xff, b = (w >> 16) & 0xff;
        if (out.len >= SGD_MAX_PROG) throw std::runtime_error("filter program too long for the device");
        DInst I{};
        I.op = (uint8_t)op;
        switch (op) {
        case SG_OP_VAR: {
            uint32_t attr = code[pc + 1];
            int32_t chain = (int32_t)code[pc + 2];
            bool single = (chain == 0 || chain == -1);  // a stream slot holds exactly one event
            I.t = (uint8_t)a;
            if (!single) {
                I.src = SGD_SRC_NULL;
            } else if (b == own) {
                I.src = SGD_SRC_EV;
                I.arg = (int32_t)col_index(evcols, attr);
            } else if (is_state1 && b == pl.slot0) {
                I.src = SGD_SRC_CAP;
                uint32_t ci = 0;
                for (; ci < pl.caps.size(); ci++)
                    if (pl.caps[ci] == attr) break;
                if (ci == pl.caps.size()) {
                    if (pl.caps.size() >= SGD_MAX_CAPS) throw std::runtime_error("too many captured attributes");
                    pl.caps.push_back(attr);
                }
                I.arg = (int32_t)ci;
            } else {
                throw std::runtime_error("filter refers to a state that is not visible");
            }
            sp++;
            break;
        }
        case SG_OP_CONST:
            I.t = (uint8_t)a;
            I.t2 = (uint8_t)(b != 0);
            I.imm = (uint64_t)code[pc + 1] | ((uint64_t)code[pc + 2] << 32);
            sp++;
            break;
        case SG_OP_ISNULL_EV: {
            int32_t chain = (int32_t)code[pc + 1];
            bool exists = (chain == 0 || chain == -1) && (b == own || (is_state1 && b == pl.slot0));
            I.op = SG_OP_CONST;
            I.t = SG_T_BOOL;
            I.imm = exists ? 0 : 1;
            sp++;
            break;
        }
        case SG_OP_CVT: I.t = (uint8_t)a; I.t2 = (uint8_t)b; break;
        case SG_OP_ADD: case SG_OP_SUB: case SG_OP_MUL: case SG_OP_DIV: case SG_OP_MOD:
        case SG_OP_EQ: case SG_OP_NE: case SG_OP_GT: case SG_OP_GE: case SG_OP_LT: case SG_OP_LE:
        case SG_OP_AND: case SG_OP_OR:
            I.t = (uint8_t)a;
            sp--;
            break;
        case SG_OP_NOT: case SG_OP_ISNULL: break;
        default: throw std::runtime_error("unknown bytecode op");
        }
        maxsp = std::max(maxsp, sp);
        out.ins[out.len++] = I;
        pc += sg_op_len(op);
    }
    if (maxsp > SGD_MAX_STACK) throw std::runtime_error("filter expression too deep for the device");
}

void build_plan(sg_engine* e, const void* ir, size_t len) {
    if (len < SG_IR_HDR_WORDS * 4 || len % 4) throw std::runtime_error("IR too short");
    e->ir.assign((const uint32_t*)ir, (const uint32_t*)ir + len / 4);
    const uint32_t* w = e->ir.data();
    size_t nw = e->ir.size();
    if (w[0] != SG_IR_MAGIC || w[1] != SG_IR_VERSION) throw std::runtime_error("bad IR magic/version");
    uint32_t qtype = w[2], nstreams = w[3], nslots = w[4];
    int64_t within = (int64_t)((uint64_t)w[5] | ((uint64_t)w[6] << 32));
    uint32_t offS = w[7], offN = w[8], nN = w[9], offC = w[10], nC = w[11];
    if (offN + nN > nw || offC + nC > nw || offS > nw) throw std::runtime_error("IR offsets out of range");
    Plan& pl = e->plan;
    pl.partitioned = (w[12] & SG_IR_F_PARTITIONED) != 0;
    pl.within = within;
    size_t p = offS;
    e->streams.resize(nstreams);
    for (uint32_t s = 0; s < nstreams; s++) {
        if (p >= nw) throw std::runtime_error("IR stream table truncated");
        uint32_t na = w[p++];
        if (p + na > nw) throw std::runtime_error("IR stream table truncated");
        e->streams[s].types.assign(w + p, w + p + na);
        p += na;
    }
    size_t pos = 0;
    Node root = read_node(w + offN, nN, pos);
    // shapes outside the two-state kernel run on the general device engine (gen_host.hip)
    if (qtype != SG_Q_PATTERN) throw std::runtime_error("SEQUENCE query: general device engine");
    if (nslots != 2) throw std::runtime_error("not a two-state pattern: general device engine");
    const Node *a = nullptr, *b = nullptr;
    if (root.tag == SG_N_NEXT) {
        const Node& x = root.kids[0];
        if (x.tag == SG_N_EVERY && x.kids[0].tag == SG_N_STREAM) {
            a = &x.kids[0];
            pl.mode = SGD_P2_EVERY_FIRST;
        } else if (x.tag == SG_N_STREAM) {
            a = &x;
            pl.mode = 0;
        }
        if (root.kids[1].tag == SG_N_STREAM) b = &root.kids[1];
    } else if (root.tag == SG_N_EVERY && root.kids[0].tag == SG_N_NEXT &&
               root.kids[0].kids[0].tag == SG_N_STREAM && root.kids[0].kids[1].tag == SG_N_STREAM) {
        a = &root.kids[0].kids[0];
        b = &root.kids[0].kids[1];
        pl.mode = SGD_P2_EVERY_BOTH;
    }
    if (!a || !b) throw std::runtime_error("pattern shape outside the two-state kernel: general device engine");
    if (a->absent || b->absent) throw std::runtime_error("absent state: general device engine");
    pl.s0 = (int)a->stream;
    pl.s1 = (int)b->stream;
    pl.slot0 = a->slot;
    pl.slot1 = b->slot;
    if ((int)nstreams <= std::max(pl.s0, pl.s1)) throw std::runtime_error("IR stream index out of range");
    pl.evcols.assign(nstreams, {});
    const uint32_t* code = w + offC;
    if (a->fpc + a->flen > nC || b->fpc + b->flen > nC) throw std::runtime_error("IR filter out of range");
    lower_filter(code, b->fpc, b->flen, b->slot, pl, pl.evcols[pl.s1], pl.f1, true);
    lower_filter(code, a->fpc, a->flen, a->slot, pl, pl.evcols[pl.s0], pl.f0, false);
    for (uint32_t attr : pl.caps) {
        pl.cap_col.push_back((uint8_t)col_index(pl.evcols[pl.s0], attr));
        pl.cap_type.push_back((uint8_t)e->streams[pl.s0].types.at(attr));
    }
    for (size_t s = 0; s < nstreams; s++)
        for (uint32_t attr : pl.evcols[s])
            if (attr >= e->streams[s].types.size()) throw std::runtime_error("attribute index out of range");
}

void allocate(sg_engine* e) {
    const size_t K = e->K, C = e->cap, B = e->maxb, M = e->mcap;
    auto& o = e->owned;
    e->hdr = dalloc<uint32_t>(K, o);
    HIP_OK(hipMemsetAsync(e->hdr, 0, K * 4, e->stream));
    e->p_ts = dalloc<int64_t>(C * K, o);
    e->p_seq = dalloc<uint64_t>(C * K, o);
    e->n_capw = 0;
    for (uint8_t t : e->plan.cap_type) e->n_capw += (t == SG_T_LONG || t == SG_T_DOUBLE) ? 2 : 1;
    e->p_capw = dalloc<uint32_t>(std::max<size_t>(1, e->n_capw) * C * K, o);
    e->p_capnull = dalloc<uint32_t>(C * K, o);
    HIP_OK(hipMemsetAsync(e->p_capnull, 0, C * K * 4, e->stream));
    size_t maxattr = 0;
    for (auto& s : e->streams) maxattr = std::max(maxattr, s.types.size());
    for (auto& sl : e->slots) {
        sl.b_ts = dalloc<int64_t>(B, o);
        sl.b_key = dalloc<uint32_t>(B, o);
        for (size_t a = 0; a < maxattr; a++) {
            sl.b_cols.push_back(dalloc<uint64_t>(B, o));
            sl.b_nulls.push_back(dalloc<uint8_t>(B, o));
        }
        sl.sidx = dalloc<uint32_t>(B, o);
        sl.seg_begin = dalloc<uint32_t>(K, o);
        sl.seg_end = dalloc<uint32_t>(K, o);
        HIP_OK(hipEventCreateWithFlags(&sl.grouped, hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&sl.free_ev, hipEventDisableTiming));
    }
    for (auto& x : e->done_ev) HIP_OK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    HIP_OK(hipHostMalloc((void**)&e->h_status, sizeof(unsigned long long) * 2 * sg_engine::RING, hipHostMallocDefault));
    e->pscr = sgd_part_scratch(dalloc<uint8_t>(sgd_part_scratch_bytes(B), o), B);
    {
        uint32_t maxw = 1;  // payload words of the widest stream (+ null word)
        for (int s : {e->plan.s0, e->plan.s1}) {
            std::vector<uint32_t> ty;
            for (uint32_t a : e->plan.evcols[s]) ty.push_back(e->streams[s].types[a]);
            maxw = std::max(maxw, sgj_stride(sgj_col_words(ty) + 1));
        }
        e->pay_words = maxw;
        e->fused_ok = e->plan.partitioned && sgd_fused_ok(K, B, 1) && maxw <= 6 && !getenv("SG_NO_FUSED");
        for (auto& sl : e->slots) {  // + one 16-B chunk: the LDS copy rounds up
            sl.pay = dalloc<uint32_t>((size_t)maxw * B + 4, o);
            if (e->fused_ok) {
                sl.tpay = dalloc<uint32_t>((size_t)maxw * B + 4, o);
                sl.tile_lo = dalloc<uint32_t>((K + SGD_BLOCK - 1) / SGD_BLOCK + 1, o);
            }
        }
    }
    // raw match slots per batch: waves reserve at most sum(live partials + events) up front, or
    // (every (e1 -> e2)) chunks of SGD_RAW_CHUNK with two chunks of slack per wave (p2_jit.hip)
    // [0, raw_static): the staged pass's per-wave ranges (rlo + w*64R ..., p2_jit.hip); above: the
    // atomically reserved slots of the HBM pass and of `every (e1 -> e2)`
    const uint64_t nw = (K + SGD_BLOCK - 1) / SGD_BLOCK * (SGD_BLOCK / SGD_WAVE);  // waves of one launch
    e->raw_static = (uint64_t)B + (nw + 1) * SGD_WAVE * e->reg_slots;
    e->raw_cap = e->raw_static + std::max<uint64_t>(2 * (B + (uint64_t)K * C), M + nw * 2 * SGD_RAW_CHUNK);
    if (e->raw_cap >= (1ull << 32)) throw std::invalid_argument("n_keys x partial_capacity too large for one engine");
    e->wstats = dalloc<unsigned long long>(nw * SGD_ST_N, o);
    e->raw_e1 = dalloc<uint64_t>(e->raw_cap, o);
    e->raw_count = dalloc<unsigned long long>(1, o);  // zeroed here, then by k_stats_reduce after every advance
    HIP_OK(hipMemsetAsync(e->raw_count, 0, 8, e->stream));
    e->t_desc = dalloc<uint64_t>(B, o);
    e->deferred = dalloc<uint32_t>((K + SGD_BLOCK - 1) / SGD_BLOCK * (SGD_BLOCK / SGD_WAVE), o);
    e->resume = dalloc<uint32_t>(K, o);
    e->dlist = dalloc<uint32_t>((K + SGD_BLOCK - 1) / SGD_BLOCK * (SGD_BLOCK / SGD_WAVE), o);
    e->dlist_n = dalloc<uint32_t>(2, o);  // zeroed here, then by k_stats_reduce after every advance
    e->klist = dalloc<uint32_t>(K, o);
    if (const char* x = getenv("SG_HBM_GRID")) e->hbm_grid = std::max(1u, (uint32_t)strtoul(x, nullptr, 0));
    HIP_OK(hipMemsetAsync(e->dlist_n, 0, 8, e->stream));
    if (getenv("SG_PROF")) {
        e->prof = dalloc<unsigned long long>(nw * 8, o);
        HIP_OK(hipMemsetAsync(e->prof, 0, nw * 64, e->stream));
        e->prof_rows = nw;
    }
    HIP_OK(hipMemsetAsync(e->resume, 0xff, K * 4, e->stream));  // SGD_NO_RESUME
    e->hot_ok = e->plan.s0 == e->plan.s1 && e->plan.mode == SGD_P2_EVERY_FIRST;
    e->hot_ctl = dalloc<uint32_t>(SGD_HOT_CTL, o);  // (every engine: the big-tile count lives here too)
    HIP_OK(hipMemsetAsync(e->hot_ctl, 0, SGD_HOT_CTL * 4, e->stream));
    {
        const char* x = getenv("SG_HOT_MIN");  // 0: off
        e->hot_min = x ? (uint32_t)strtoul(x, nullptr, 0) : 64u;
        if (const char* f = getenv("SG_HOT_FACTOR")) e->hot_factor = std::max(1ul, strtoul(f, nullptr, 0));
        if (const char* f = getenv("SG_HOT_N0")) e->hot_n0 = (uint32_t)strtoul(f, nullptr, 0);
        if (e->hot_min == 0) e->hot_ok = false;
    }
    if (e->hot_ok) {
        // hot keys: up to every key (those with more live partials than the window are hot too); their carried-in
        // partials get up to hot_exmax flat indices (further keys are given back to the HBM pass; SG_HOT_EXMAX bounds
        // it, tests force the give-back that way).  Only the key list is allocated here: the pipeline's per-event and
        // per-partial buffers (hot_buffers, ~2.3 GB at 2^24-event batches) come with the first batch that runs it and
        // are given back once SGD_HOT_IDLE batches in a row had no hot key: an engine whose stream has none (uniform
        // C2) holds them only over its first batches.  The first batch runs the pipeline: the host cannot know in
        // advance whether a device batch has hot keys, and a hot key left to the HBM pass is walked by one lane,
        // quadratic in its run (a Zipf stream's first batch: 1.85 s).
        e->hot_cap = (uint32_t)std::min<size_t>(K, 1u << 20);
        e->hot_exmax = (uint32_t)std::min<size_t>((size_t)K * C, std::max<size_t>(1u << 22, 2 * B));
        if (const char* x = getenv("SG_HOT_EXMAX")) e->hot_exmax = std::max(1u, (uint32_t)strtoul(x, nullptr, 0));
        e->hot_list = dalloc<uint32_t>(e->hot_cap, o);
        e->hot_info = dalloc<uint32_t>((size_t)e->hot_cap * SGD_HOT_INFO, o);
    }
    e->tile_sum = dalloc<uint32_t>(B / SGD_ORDER_TILE + 1, o);
    // the match count and the error word share 16 bytes, so poll reads both with one D2H copy
    e->out_count = dalloc<unsigned long long>(2, o);
    e->err = (uint32_t*)(e->out_count + 1);
    e->batch_total = dalloc<unsigned long long>(1, o);
    e->stats = dalloc<unsigned long long>(SGD_ST_N, o);
    HIP_OK(hipMemsetAsync(e->t_desc, 0, B * 8, e->stream));
    HIP_OK(hipMemsetAsync(e->out_count, 0, 16, e->stream));
    HIP_OK(hipMemsetAsync(e->stats, 0, SGD_ST_N * 8, e->stream));
    HIP_OK(hipMemsetAsync(e->err, 0, 4, e->stream));
    e->o_trig = dalloc<uint64_t>(M, o);
    e->o_slot = dalloc<uint64_t>(2 * M, o);
    e->o_key = dalloc<uint32_t>(M, o);
    e->o_ts = dalloc<int64_t>(M, o);
    e->o_len = dalloc<uint32_t>(2 * M, o);
    HIP_OK(hipMemsetD32((hipDeviceptr_t)e->o_len, 1, 2 * M));  // every two-state match: chain lengths 1, 1
    HIP_OK(hipDeviceSynchronize());
}

JitQuery make_jit_query(sg_engine* e) {
    const Plan& pl = e->plan;
    JitQuery q;
    q.mode = pl.mode;
    q.multi = pl.s0 == pl.s1;
    q.within = pl.within >= 0;
    q.reg_slots = e->reg_slots;
    q.reg_slots_hbm = e->reg_slots_hbm;
    for (int r = 0; r < 2; r++) {
        const int s = r == 0 ? pl.s0 : pl.s1;
        for (uint32_t a : pl.evcols[s]) q.coltypes[r].push_back(e->streams[s].types[a]);
    }
    q.f0 = &pl.f0;
    q.f1 = &pl.f1;
    q.cap_col = pl.cap_col;
    q.cap_type = pl.cap_type;
    return q;
}

// the code object of one null variant (compiled on first use; cached across engines)
sg_engine::Variant& variant(sg_engine* e, bool evnull, bool capnull) {
    const int key = (evnull ? 1 : 0) | (capnull ? 2 : 0);
    auto it = e->variants.find(key);
    if (it != e->variants.end()) return it->second;
    JitQuery q = e->jq;
    q.evnull = evnull;
    q.capnull = capnull;
    std::vector<uint64_t> consts;
    const std::string hdr = sgj_generate(q, consts);
    std::vector<char> code;
    std::string log;
    if (!sgj_compile(hdr, code, log)) throw HipError("advance kernel JIT compilation failed: " + log);
    sg_engine::Variant v;
    HIP_OK(hipModuleLoadData(&v.mod, code.data()));
    e->variants[key] = v;  // owned (unloaded by ~sg_engine) before any further call can throw
    sg_engine::Variant& r = e->variants[key];
    if (q.multi) {
        HIP_OK(hipModuleGetFunction(&r.adv[0], r.mod, "k_adv_m"));
        HIP_OK(hipModuleGetFunction(&r.adv_h[0], r.mod, "k_adv_m_h"));
        HIP_OK(hipModuleGetFunction(&r.adv_k[0], r.mod, "k_adv_m_k"));
        r.adv_k[1] = r.adv_k[0];
        r.adv[1] = r.adv[0];
        r.adv_h[1] = r.adv_h[0];
    } else {
        HIP_OK(hipModuleGetFunction(&r.adv[0], r.mod, "k_adv_s0"));
        HIP_OK(hipModuleGetFunction(&r.adv[1], r.mod, "k_adv_s1"));
        HIP_OK(hipModuleGetFunction(&r.adv_h[0], r.mod, "k_adv_s0_h"));
        HIP_OK(hipModuleGetFunction(&r.adv_h[1], r.mod, "k_adv_s1_h"));
        HIP_OK(hipModuleGetFunction(&r.adv_k[0], r.mod, "k_adv_s0_k"));
        HIP_OK(hipModuleGetFunction(&r.adv_k[1], r.mod, "k_adv_s1_k"));
    }
    if (e->hot_ok) {
        static const char* const names[14] = {"k_hot_prep",  "k_hot_scan",  "k_hot_fill", "k_hot_r0",
                                              "k_hot_r1",    "k_hot_r1c",   "k_hot_rn",   "k_hot_rc",
                                              "k_hot_emit",  "k_hot_trig",  "k_hot_place", "k_hot_sort",
                                              "k_hot_final", "k_hot_final_big"};
        for (int i = 0; i < 14; i++) HIP_OK(hipModuleGetFunction(&r.hot[i], r.mod, names[i]));
    }
    {
        int sh = 0;
        HIP_OK(hipFuncGetAttribute(&sh, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, r.adv[0]));
        r.adv_static_lds = (uint32_t)sh;
    }
    HIP_OK(hipModuleGetFunction(&r.pack[0], r.mod, "k_pack0"));
    HIP_OK(hipModuleGetFunction(&r.pack[1], r.mod, "k_pack1"));
    return r;
}

void launch(hipFunction_t f, uint32_t blocks, uint32_t threads, void* arg, hipStream_t stream, uint32_t lds = 0) {
    void* args[] = {arg};
    HIP_OK(hipModuleLaunchKernel(f, blocks, 1, 1, threads, 1, 1, lds, stream, args, nullptr));
}

// LDS staging per advance-kernel wave, in 16-B chunks (a workgroup stages its keys' runs in one region of
// SGD_BLOCK / 64 times this): the payload bytes of the workgroup's keys at this batch's density (n / K
// events per key) plus 4 standard deviations of a Poisson count, so that practically every workgroup of
// a uniform key stream is staged (the rest read HBM directly, exactly); a smaller region means more
// resident workgroups per CU (160 KB LDS).
uint32_t stage_chunks_for(uint64_t n, uint64_t K, uint32_t stride_words) {
    const uint32_t wpb = SGD_BLOCK / SGD_WAVE;
    const double mean = (double)n * SGD_BLOCK / (double)(K ? K : 1);
    const double want = mean + 4.0 * std::sqrt(mean) + 32.0;
    const double chunks = std::ceil((std::ceil(want * stride_words * 4.0 / 16.0) + 1.0) / wpb);
    const double hi = std::floor((double)SGD_STAGE_MAX_BYTES / wpb / 16.0);
    return (uint32_t)std::max(64.0, std::min(chunks, hi));
}

// fused grouping: the LDS staging of a workgroup's tile (its events at this density plus 3.5 standard deviations
// of a Poisson count, the few larger tiles split in HBM and walked by the HBM pass), sized so that three workgroups
// share a CU at the C2 density (with the split's 2 KB of counters beside it); and whether the batch takes the fused
// grouping at all (the split holds SGD_SPLIT_CHUNKS rounds of 64 events per wave in registers)
static uint32_t stage_chunks_fused(uint64_t n, uint64_t K, uint32_t stride_words, uint32_t static_lds) {
    const uint32_t wpb = SGD_BLOCK / SGD_WAVE;
    const double mean = (double)n * SGD_BLOCK / (double)(K ? K : 1);
    const double want = mean + 3.5 * std::sqrt(mean);
    const double chunks = std::ceil((std::ceil(want * stride_words * 4.0 / 16.0) + 1.0) / wpb);
    // three workgroups per CU: LDS is allocated in granules of 1,280 B on gfx950 (measured: a 54,064-B workgroup
    // held two per CU, 53,360 B three), so a workgroup keeps within 42 granules = 53,760 B
    const double three = std::floor((53760.0 - SGD_SPLIT_CNT_BYTES - (double)static_lds) / wpb / 16.0);
    const double hi = std::floor((double)(SGD_STAGE_MAX_BYTES - SGD_SPLIT_CNT_BYTES) / wpb / 16.0);
    if (chunks <= three + 16.0) return (uint32_t)std::max(64.0, std::min(chunks, three));
    return (uint32_t)std::max(64.0, std::min(chunks, hi));
}
static bool fused_density_ok(uint64_t n, uint64_t K, uint32_t stride_words) {
    const double mean = (double)n * SGD_BLOCK / (double)(K ? K : 1);
    return mean + 3.0 * std::sqrt(mean) <= (double)SGD_SPLIT_CHUNKS(stride_words) * SGD_BLOCK;
}

// largest key id of a host batch (branch-free, so it vectorises; range-checked after the H2D is queued);
// with SG_CFG_NULL_KEYS the dropped SG_KEY_NULL ids do not count
static uint32_t sgd_max_key(const uint32_t* k, uint32_t n, bool skip_null) {
    uint32_t m = 0;
    if (skip_null)
        for (uint32_t i = 0; i < n; i++) m = (k[i] > m && k[i] != SG_KEY_NULL) ? k[i] : m;
    else
        for (uint32_t i = 0; i < n; i++) m = k[i] > m ? k[i] : m;
    return m;
}

// the hot-key pipeline's buffers, allocated the first time a batch runs it: B + hot_exmax flat slots (events of the
// hot runs, then the carried-in partials) x 10 words, 3 x B words.  Stream-ordered (hipMallocAsync on the engine's
// main stream, the one every k_hot_* kernel runs on), so neither taking nor giving them back waits on the host: a
// hipFree in the middle of a pipelined run drained both batches in flight (a one-time stall of a few ms)
template <class T> static T* hot_alloc(sg_engine* e, size_t n) {
    void* p = nullptr;
    HIP_OK(hipMallocAsync(&p, n * sizeof(T), e->stream));
    e->hot_owned.push_back(p);
    return (T*)p;
}
static void hot_buffers(sg_engine* e) {
    if (e->hot_death) return;
    const size_t B = e->maxb, slots = B + (size_t)e->hot_exmax;
    e->hot_death = hot_alloc<uint32_t>(e, slots);
    e->hot_wl = hot_alloc<uint32_t>(e, 2 * 3 * slots);
    e->hot_tcnt = hot_alloc<uint32_t>(e, B);
    e->hot_tbase = hot_alloc<uint32_t>(e, B);
    e->hot_alive = hot_alloc<uint32_t>(e, slots);
    e->hot_fh = hot_alloc<uint32_t>(e, slots);
    e->hot_cur = hot_alloc<uint32_t>(e, slots);
    e->hot_fbi = hot_alloc<uint32_t>(e, B);
}

// ... and given back, on the same stream behind the last kernel that could read them (no batch in flight runs the
// pipeline: it ran only while the batches drained before it had hot keys, and the last SGD_HOT_IDLE had none)
static void hot_release(sg_engine* e) {
    if (!e->hot_death) return;
    for (void* p : e->hot_owned) HIP_OK(hipFreeAsync(p, e->stream));
    e->hot_owned.clear();
    e->hot_death = e->hot_wl = e->hot_tcnt = e->hot_tbase = e->hot_alive = e->hot_fh = e->hot_cur = e->hot_fbi = nullptr;
}

// a batch is complete once its ordering ran: record its status block into the pinned ring
static void drain_one(sg_engine* e) {  // wait for the oldest in-flight batch
    const uint32_t ri = e->inflight.front();
    HIP_OK(hipEventSynchronize(e->done_ev[ri]));
    e->done_count = e->h_status[2 * ri];
    e->done_err |= (uint32_t)e->h_status[2 * ri + 1];
    // the batch's hot keys and giant workgroup ranges (p2_jit.hip hbm_pass): the hot-key pipeline runs while
    // batches have hot keys, the sorted grouping replaces the fused one while they have giant tiles (split by one
    // workgroup each in the fused grouping)
    const uint32_t w1 = (uint32_t)(e->h_status[2 * ri + 1] >> 32);
    if (e->hot_ok) {
        e->hot_on = (w1 & 0xffffu) != 0;
        e->hot_idle = e->hot_on ? 0 : e->hot_idle + 1;
    }
    e->skewed = (w1 >> 16) != 0;
    e->inflight.erase(e->inflight.begin());
}

int push(sg_engine* e, const sg_batch* b) {
    const Plan& pl = e->plan;
    // rocPRIM reads the thread's last HIP error after its launches: an error some unrelated earlier call left
    // on this thread (freeing another engine's buffers, say) must not fail this batch
    (void)hipGetLastError();
    if (b->stream >= e->streams.size()) return fail(SG_ERR_INVALID, "stream index out of range");
    const auto& types = e->streams[b->stream].types;
    if (b->n_cols != types.size()) return fail(SG_ERR_INVALID, "column count does not match the stream");
    if (b->n == 0) return SG_OK;
    if (b->n > e->maxb) return fail(SG_ERR_INVALID, "batch larger than max_batch");
    if (pl.partitioned && !b->key) return fail(SG_ERR_INVALID, "partitioned query needs key ids");
    if (!b->ts) return fail(SG_ERR_INVALID, "timestamps missing");
    if (e->have_base && b->seq_base < e->next_seq) return fail(SG_ERR_INVALID, "sequence numbers must increase");
    if (e->held) return fail(SG_ERR_STATE, "release the polled matches before pushing");
    const bool is0 = (int)b->stream == pl.s0, is1 = (int)b->stream == pl.s1;
    if (!is0 && !is1) return SG_OK;  // stream not read by this query
    const uint32_t n = (uint32_t)b->n;
    const int role = is0 ? 0 : 1;    // multi: both, kernel 0
    const auto& cols = pl.evcols[b->stream];
    const bool dev = b->mem == SG_MEM_DEVICE;
    const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    sg_engine::Slot& sl = e->slots[e->nbatch & 1];
    const hipStream_t gs = e->gstream;
    // at most two batches in flight: batch i's copies + grouping overlap batch i - 1's advance, and the
    // matches pending in the output ring stay within three batches (the caller polls between pushes)
    while (e->inflight.size() >= 2) drain_one(e);
    // the slot's buffers were last read by the batch two back (its advance, ordering, projection)
    if (sl.used) HIP_OK(hipStreamWaitEvent(gs, sl.free_ev, 0));

    // timestamps / key ids / the columns the filters read (host batches: H2D on the grouping stream)
    const int64_t* ts = b->ts;
    if (!dev) {
        HIP_OK(hipMemcpyAsync(sl.b_ts, b->ts, (size_t)n * 8, kind, gs));
        ts = sl.b_ts;
    }
    PackParams pk{};
    pk.n = n;
    pk.ts = ts;
    bool any_null = false;
    std::vector<uint32_t> coltypes;
    for (size_t c = 0; c < cols.size(); c++) {
        const uint32_t attr = cols[c];
        coltypes.push_back(types[attr]);
        if (dev) {
            pk.col[c] = b->cols[attr];
            pk.nul[c] = b->nulls ? b->nulls[attr] : nullptr;
        } else {
            HIP_OK(hipMemcpyAsync(sl.b_cols[c], b->cols[attr], (size_t)n * type_size(types[attr]), kind, gs));
            pk.col[c] = sl.b_cols[c];
            pk.nul[c] = nullptr;
            if (b->nulls && b->nulls[attr]) {
                HIP_OK(hipMemcpyAsync(sl.b_nulls[c], b->nulls[attr], n, kind, gs));
                pk.nul[c] = sl.b_nulls[c];
            }
        }
        if (pk.nul[c]) any_null = true;
    }
    // the projection's trigger columns (read after the ordering, on the main stream)
    ProjParams q = e->pp;
    const bool proj = e->proj_n && is1;
    if (proj) {
        q.seq_base = b->seq_base;
        for (size_t j = 0; j < e->proj_attrs.size(); j++) {
            const uint32_t a = e->proj_attrs[j];
            if (dev) {
                q.col[a] = b->cols[a];
                q.col_null[a] = b->nulls ? b->nulls[a] : nullptr;
            } else {
                HIP_OK(hipMemcpyAsync(sl.b_pcols[j], b->cols[a], (size_t)n * type_size(types[a]), kind, gs));
                q.col[a] = sl.b_pcols[j];
                q.col_null[a] = nullptr;
                if (b->nulls && b->nulls[a]) {
                    HIP_OK(hipMemcpyAsync(sl.b_pnulls[j], b->nulls[a], n, kind, gs));
                    q.col_null[a] = sl.b_pnulls[j];
                }
            }
            q.col_type[a] = types[a];
        }
    }
    // the engine state (sequence window, null variant, counters) changes only once the batch has
    // passed validation: a rejected batch leaves the engine as it was, so the caller may fix it and
    // push again at the same seq_base
    const bool nullable = e->nullable || any_null;
    sg_engine::Variant& v = variant(e, any_null, nullable);
    const uint32_t words = sgj_col_words(coltypes) + (any_null ? 1u : 0u);
    const uint32_t stride = sgj_stride(words);
    if (stride > e->pay_words) throw HipError("payload stride above the allocated payload");
    pk.payload = (uint32_t*)sl.pay;

    // ---- grouping by key: the batch as key-sorted payload elements + per-key segment bounds ----
    hipEvent_t g0 = nullptr, g1 = nullptr;
    const uint32_t pack_blocks = (n + 255) / 256;
    const uint32_t* keys = b->key;
    if (pl.partitioned && !dev) {
        // the copy is queued first, so the host range check overlaps the DMA (pinned batches); the
        // staging buffers it fills are not engine state
        HIP_OK(hipMemcpyAsync(sl.b_key, b->key, (size_t)n * 4, kind, gs));
        keys = sl.b_key;
        if (sgd_max_key(b->key, n, e->null_keys) >= e->K) {
            HIP_OK(hipStreamSynchronize(gs));  // the queued copies read the caller's buffers
            return fail(SG_ERR_INVALID, "key id outside [0, n_keys)");
        }
    }
    if (!dev) HIP_OK(hipEventRecord(sl.copied, gs));
    e->nullable = nullable;
    if (!e->have_base) {
        e->poll_base = b->seq_base;
        e->have_base = true;
    }
    e->next_seq = b->seq_base + b->n;
    e->st.events += b->n;
    e->st.batches++;
    if (e->timing) { g0 = e->ev(); e->mark(g0, gs); }
    bool fused = false;
    if (pl.partitioned) {
        GroupArgs ga{};
        ga.n = n;
        ga.K = e->K;
        ga.drop_null = e->null_keys ? 1u : 0u;
        ga.keys = keys;
        ga.seg_begin = sl.seg_begin;
        ga.seg_end = sl.seg_end;
        ga.err = e->err;
        ga.s = e->pscr;
        if (words <= 4) {
            // the events WITH their payload (gathered from the SoA columns by the first pass): the advance kernel
            // then reads one contiguous range per workgroup
            PackSrc ps{};
            ps.ts = ts;
            uint32_t wi = 0;
            for (size_t c = 0; c < cols.size(); c++) {
                const uint32_t ty = coltypes[c];
                if (ty == SG_T_LONG || ty == SG_T_DOUBLE) {
                    ps.p[wi] = pk.col[c]; ps.kind[wi++] = 1;
                    ps.p[wi] = pk.col[c]; ps.kind[wi++] = 2;
                } else {
                    ps.p[wi] = pk.col[c]; ps.kind[wi++] = ty == SG_T_BOOL ? 3 : 0;
                }
            }
            if (any_null) {
                for (size_t c = 0; c < cols.size(); c++) ps.nul[c] = pk.nul[c];
                ps.kind[wi++] = 4;
            }
            if (wi == 0) ps.kind[wi++] = 5;
            ga.W = wi;
            ga.src = ps;
            fused = e->fused_ok && !e->skewed && sgd_fused_ok(e->K, n, wi) && fused_density_ok(n, e->K, stride);
            if (fused) {
                // grouped by key tile only; the split by key is the advance kernel's (tile_split_lds)
                ga.out = sl.tpay;
                HIP_OK(sgd_group_tiles_fused(ga, sl.tile_lo, gs));
            } else {
                ga.out = sl.pay;
                HIP_OK(sgd_group_sorted(ga, gs));
            }
        } else {
            // wide payloads: batch positions in key order, then the payload packed from them
            ga.W = 0;
            ga.out = sl.sidx;
            HIP_OK(sgd_group_sorted(ga, gs));
            pk.sidx = sl.sidx;
            launch(v.pack[role], pack_blocks, 256, &pk, gs);
        }
    } else {
        pk.sidx = nullptr;  // one key: arrival order
        launch(v.pack[role], pack_blocks, 256, &pk, gs);
        HIP_OK(hipMemsetD32Async((hipDeviceptr_t)sl.seg_begin, 0u, 1, gs));
        HIP_OK(hipMemsetD32Async((hipDeviceptr_t)sl.seg_end, (int)n, 1, gs));
    }
    e->fused_last = fused;
    if (e->timing) { g1 = e->ev(); e->mark(g1, gs); e->spans.push_back({g0, g1, 0}); }
    HIP_OK(hipEventRecord(sl.grouped, gs));
    HIP_OK(hipStreamWaitEvent(e->stream, sl.grouped, 0));

    // ---- the NFA advance ----
    P2Params p{};
    p.n_keys = e->K;
    p.cap = e->cap;
    p.seq_base = b->seq_base;
    p.within = pl.within;
    p.payload = (const uint32_t*)sl.pay;
    p.tile_lo = fused ? sl.tile_lo : nullptr;
    p.tpay = (const uint32_t*)sl.tpay;
    p.write_sorted = (fused && proj && e->n_agg) ? 1u : 0u;
    p.hbm_stage_chunks = SGD_HBM_STAGE_BYTES / 16u;
    p.ts_col = ts;
    p.seg_begin = sl.seg_begin;
    p.seg_end = sl.seg_end;
    p.hdr = e->hdr;
    p.p_ts = e->p_ts;
    p.p_seq = e->p_seq;
    p.p_capw = e->p_capw;
    p.p_capnull = e->p_capnull;
    p.raw_e1 = e->raw_e1;
    p.raw_count = e->raw_count;
    p.raw_capacity = e->raw_cap;
    p.t_desc = e->t_desc;
    p.deferred = e->deferred;
    p.prof = e->prof;
    p.resume = e->resume;
    p.dlist = e->dlist;
    p.dlist_n = e->dlist_n;
    p.klist = getenv("SG_NO_KLIST") ? nullptr : e->klist;
    p.stats = e->stats;
    p.wstats = e->wstats;
    p.raw_static = e->raw_static;
    p.err = e->err;
    p.raw_capw = e->raw_capw;
    p.raw_capnull = e->raw_capnull;
    p.hot_ctl = e->hot_ctl;
    if (e->hot_ok && e->hot_on) hot_buffers(e);
    else if (e->hot_ok && e->hot_idle >= SGD_HOT_IDLE) hot_release(e);
    if (e->hot_ok) {
        // a partitioned batch's keys hold n / K events on average: "hot" is far above that (and above hot_min)
        p.hot_min = pl.partitioned ? std::max<uint32_t>(e->hot_min, (uint32_t)std::min<uint64_t>(e->hot_factor * n / e->K, 1u << 30))
                                   : e->hot_min;
        p.hot_cap = e->hot_cap;
        p.hot_exmax = e->hot_exmax;
        p.hot_n0 = e->hot_n0 ? e->hot_n0 : std::max(e->reg_slots, e->reg_slots_hbm) + 1;
        p.max_batch = (uint32_t)e->maxb;
        p.hot_list = e->hot_list;
        p.hot_info = e->hot_info;
        p.hot_death = e->hot_death;
        p.hot_wl = e->hot_wl;
        p.hot_tcnt = e->hot_tcnt;
        p.hot_tbase = e->hot_tbase;
        p.hot_alive = e->hot_alive;
        p.hot_fh = e->hot_fh;
        p.hot_cur = e->hot_cur;
        p.hot_fbi = e->hot_fbi;
    }
    for (size_t i = 0; i < e->consts.size(); i++) p.cst[i] = e->consts[i];
    // this batch's t_desc tag: entries of earlier batches read as empty, so the ordering clears nothing; at the
    // tag's wrap t_desc is cleared once
    if (++e->td_epoch > 0xffffu) {
        HIP_OK(hipMemsetAsync(e->t_desc, 0, e->maxb * 8, e->stream));
        e->td_epoch = 1;
    }
    p.td_tag = SGD_TD_TAG(e->td_epoch);
    hipEvent_t a0 = nullptr, a1 = nullptr;
    if (e->timing) { a0 = e->ev(); e->mark(a0); }
    {
        p.stage_chunks = e->stage_override ? std::max(64u, e->stage_override)
                         : fused ? stage_chunks_fused(n, e->K, stride, v.adv_static_lds) : stage_chunks_for(n, e->K, stride);
        const uint32_t blocks = (e->K + SGD_BLOCK - 1) / SGD_BLOCK;
        // (fused: the split's per-(wave, key) counters after the staging region)
        launch(v.adv[role], blocks, SGD_BLOCK, &p, e->stream,
               p.stage_chunks * 16u * (SGD_BLOCK / SGD_WAVE) + (fused ? SGD_SPLIT_CNT_BYTES : 0u));
        if (e->timing) { a1 = e->ev(); e->mark(a1); e->spans.push_back({a0, a1, 1}); a0 = e->ev(); e->mark(a0); }
        if (e->hot_ok && e->hot_on) {  // the hot keys the staged pass listed (fixed grids: the counts are on the device)
            launch(v.hot[0], 512, 256, &p, e->stream);   // k_hot_prep
            launch(v.hot[1], 1, 1024, &p, e->stream);    // k_hot_scan
            launch(v.hot[2], 1024, 256, &p, e->stream);  // k_hot_fill
            launch(v.hot[3], 2048, 256, &p, e->stream);  // k_hot_r0
            launch(v.hot[4], 1024, 256, &p, e->stream);  // k_hot_r1
            uint64_t covered = 128 + 512;
            if (covered < e->maxb) launch(v.hot[5], 512, 256, &p, e->stream);  // k_hot_r1c
            // rounds 2.. until the spans scanned cover the longest possible run (round r: 512 << 3 (r - 1) events)
            for (uint32_t r = 2; covered < e->maxb; r++) {
                p.hot_round = r;
                covered += 512ull << (3 * (r - 1));
                launch(v.hot[6], 1024, 256, &p, e->stream);  // k_hot_rn
                if (covered < e->maxb) launch(v.hot[7], 256, 256, &p, e->stream);  // k_hot_rc
            }
            for (int i = 8; i < 12; i++) launch(v.hot[i], 1024, 256, &p, e->stream);  // emit, trig, place, sort
            launch(v.hot[12], 1024, 256, &p, e->stream);  // k_hot_final
            launch(v.hot[13], 64, 256, &p, e->stream);    // k_hot_final_big
            e->hot_batches++;
        }
        // one wave per work-group over the listed waves (a fixed grid: the list's length is on the device)
        launch(v.adv_h[role], std::min<uint32_t>(blocks * (SGD_BLOCK / SGD_WAVE), e->hbm_grid), SGD_WAVE, &p, e->stream,
               p.hbm_stage_chunks * 16u);
        launch(v.adv_k[role], std::min<uint32_t>(blocks * (SGD_BLOCK / SGD_WAVE), e->hbm_grid), SGD_WAVE, &p, e->stream,
               p.hbm_stage_chunks * 16u);
        if (e->timing) { a1 = e->ev(); e->mark(a1); e->spans.push_back({a0, a1, 3}); }
        if (sgd_launch_stats_reduce(e->wstats, blocks * (SGD_BLOCK / SGD_WAVE), e->stats, e->raw_count, e->dlist_n, e->stream) != 0)
            throw HipError("k_stats_reduce launch failed");
    }
    e->st.advance_launches++;
    // order this batch's matches by trigger (exclusive scan of per-event counts + scatter) into the ring
    // of match_capacity output records
    hipEvent_t o0 = nullptr, o1 = nullptr;
    if (e->timing) { o0 = e->ev(); e->mark(o0); }
    {
        ScatterParams sp{};
        sp.n = n;
        sp.seq_base = b->seq_base;
        sp.key = pl.partitioned ? (dev ? b->key : sl.b_key) : nullptr;
        sp.ts = ts;
        sp.t_desc = e->t_desc;
        sp.epoch = e->td_epoch;
        sp.tile_sum = e->tile_sum;
        sp.raw_e1 = e->raw_e1;
        sp.out_count = e->out_count;
        sp.batch_total = e->batch_total;
        sp.capacity = e->mcap;
        sp.win_start = e->win;
        sp.o_trig = e->o_trig;
        sp.o_slot = e->o_slot;
        sp.o_key = e->o_key;
        sp.o_ts = e->o_ts;
        sp.err = e->err;
        sp.raw_capw = e->raw_capw;
        sp.raw_capnull = e->raw_capnull;
        sp.raw_capacity = e->raw_cap;
        sp.o_capw = proj ? e->o_capw : nullptr;
        sp.o_capnull = e->o_capnull;
        sp.n_capw = e->n_capw;
        sp.out_first = (proj && e->n_agg) ? e->out_first : nullptr;
#ifdef SG_EXPERIMENTS
        if (const char* x = getenv("SG_ORDER_EXP")) sp.exp = (uint32_t)strtoul(x, nullptr, 0);
#endif
        if (sgd_launch_scatter(sp, e->stream) != 0)
            throw HipError("ordering launch failed");
        if (proj) {
            if (e->n_agg) {  // aggregator arguments, then their per-key values in output order
                q.phase = 0;
                if (sgd_launch_project(q, e->stream) != 0) throw HipError("projection launch failed");
                AggParams ag{};
                ag.K = pl.partitioned ? e->K : 1u;
                ag.n_agg = e->n_agg;
                ag.seg_begin = sl.seg_begin;
                ag.seg_end = sl.seg_end;
                ag.payload = (const uint32_t*)sl.pay;
                ag.stride = stride;
                ag.out_first = e->out_first;
                ag.capacity = e->mcap;
                ag.agg_type = e->d_agg_type;
                ag.aggv = e->aggv;
                ag.aggnull = e->aggnull;
                ag.st_n = e->agg_n;
                ag.st_v = e->agg_v;
                ag.st_has = e->agg_has;
                if (sgd_launch_agg(ag, e->stream) != 0) throw HipError("aggregator launch failed");
            }
            q.phase = 1;
            if (sgd_launch_project(q, e->stream) != 0) throw HipError("projection launch failed");
        }
    }
    if (e->timing) { o1 = e->ev(); e->mark(o1); e->spans.push_back({o0, o1, 2}); }
    // the slot is free again once this batch's kernels ran; its status goes to the pinned ring
    HIP_OK(hipEventRecord(sl.free_ev, e->stream));
    sl.used = true;
    const uint32_t ri = (uint32_t)(e->nbatch % sg_engine::RING);
    HIP_OK(hipMemcpyAsync(e->h_status + 2 * ri, e->out_count, 16, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipEventRecord(e->done_ev[ri], e->stream));
    e->inflight.push_back(ri);
    e->nbatch++;
    // host buffers may be reused by the caller once their copies ran (SG_CFG_ASYNC_HOST: the caller keeps
    // them until the next poll / synchronize instead)
    if (!dev && !e->async_host) HIP_OK(hipEventSynchronize(sl.copied));
    return SG_OK;
}

// every queued batch done (both streams), their status blocks taken
static void sync_all(sg_engine* e) {
    HIP_OK(hipStreamSynchronize(e->gstream));
    HIP_OK(hipStreamSynchronize(e->stream));
    while (!e->inflight.empty()) drain_one(e);
    e->resolve_spans();
}

// n records of w bytes each from ring position start (of a ring of cap records) to contiguous host memory
static void ring_to_host(void* dst, const void* ring, size_t w, uint64_t start, uint64_t n, uint64_t cap,
                         hipStream_t st) {
    const uint64_t a = std::min<uint64_t>(n, cap - start);
    if (a) HIP_OK(hipMemcpyAsync(dst, (const char*)ring + start * w, a * w, hipMemcpyDeviceToHost, st));
    if (n > a) HIP_OK(hipMemcpyAsync((char*)dst + a * w, ring, (n - a) * w, hipMemcpyDeviceToHost, st));
}

// SG_POLL_READY: the matches of the batches already complete (no wait); else of every pushed batch.
// The ordered records form a ring of match_capacity entries: a host poll copies the whole window; a device
// poll of a window that wraps hands it out in two polls (the part up to the ring's end first).
int poll(sg_engine* e, uint32_t memflags, sg_match_batch* out) {
    if (e->held) return fail(SG_ERR_STATE, "previous matches not released");
    const bool ready = (memflags & SG_POLL_READY) != 0;
    const uint32_t mem = memflags & ~(uint32_t)SG_POLL_READY;
    if (ready) {
        while (!e->inflight.empty() && hipEventQuery(e->done_ev[e->inflight.front()]) == hipSuccess) drain_one(e);
        if (e->inflight.empty()) {
            HIP_OK(hipStreamSynchronize(e->gstream));  // (idle by now: its work precedes the advances)
            e->resolve_spans();
        }
    } else {
        sync_all(e);
    }
    const uint32_t err = e->done_err;
    if (err & SGD_ERR_KEY_RANGE) {
        // reported once: the events with valid keys were processed, the others dropped; the engine
        // goes on (capacity errors below stay: partials were lost)
        sync_all(e);
        uint32_t cur = 0;
        HIP_OK(hipMemcpy(&cur, e->err, 4, hipMemcpyDeviceToHost));
        cur &= ~(uint32_t)SGD_ERR_KEY_RANGE;
        HIP_OK(hipMemcpy(e->err, &cur, 4, hipMemcpyHostToDevice));
        e->done_err &= ~(uint32_t)SGD_ERR_KEY_RANGE;
        return fail(SG_ERR_INVALID, "a batch carried key ids outside [0, n_keys) (those events were dropped)");
    }
    if (err & SGD_ERR_PARTIAL_CAP)
        return fail(SG_ERR_CAPACITY, "a partition key exceeded partial_capacity live partial matches");
    if (err & SGD_ERR_PROJ) return fail(SG_ERR_STATE, "malformed projection program");
    if (err & SGD_ERR_MATCH_CAP) return fail(SG_ERR_CAPACITY, "more matches than match_capacity between two polls");
    const uint64_t avail = e->done_count - e->win;
    const uint64_t start = e->win % e->mcap;
    const unsigned long long n = mem == SG_MEM_DEVICE ? std::min<uint64_t>(avail, e->mcap - start) : avail;
    out->n = n;
    out->n_slots = 2;
    out->max_chain = 1;
    out->reserved = 0;
    if (mem == SG_MEM_DEVICE) {
        out->trigger_seq = e->o_trig + start;
        out->slot_seq = e->o_slot + 2 * start;
        out->key = e->o_key + start;
        out->ts = e->o_ts + start;
        out->chain_len = e->o_len + 2 * start;
        out->mem = SG_MEM_DEVICE;
    } else {
        e->h_trig.resize(n);
        e->h_slot.resize(2 * n);
        e->h_key.resize(n);
        e->h_ts.resize(n);
        e->h_len.resize(2 * n);
        if (n) {  // (a separate stream would not see the records any sooner: they are complete)
            ring_to_host(e->h_trig.data(), e->o_trig, 8, start, n, e->mcap, e->pstream);
            ring_to_host(e->h_slot.data(), e->o_slot, 16, start, n, e->mcap, e->pstream);
            ring_to_host(e->h_key.data(), e->o_key, 4, start, n, e->mcap, e->pstream);
            ring_to_host(e->h_ts.data(), e->o_ts, 8, start, n, e->mcap, e->pstream);
            ring_to_host(e->h_len.data(), e->o_len, 8, start, n, e->mcap, e->pstream);
            HIP_OK(hipStreamSynchronize(e->pstream));
        }
        out->trigger_seq = e->h_trig.data();
        out->slot_seq = e->h_slot.data();
        out->key = e->h_key.data();
        out->ts = e->h_ts.data();
        out->chain_len = e->h_len.data();
        out->mem = SG_MEM_HOST;
    }
    e->poll_base = e->next_seq;
    e->held = true;
    e->polled = n;
    return SG_OK;
}

// ---- on-device projection (two-state kernel) -------------------------------------------------------
// VAR of e1 (slot0) becomes "capture c" (the partial carries the attribute; added to the capture list if
// the filters do not capture it already), VAR of e2 (slot1) "trigger column a"; e1's partition attribute
// in a single-stream query is read from the trigger (same key, so the same value).
int set_projection(sg_engine* e, const uint32_t* code, uint32_t words, const uint32_t* pc, const uint32_t* len,
                   const uint32_t* types, uint32_t n, const int32_t* part_attr, uint32_t n_streams) {
    Plan& pl = e->plan;
    if (e->have_base || e->held) return fail(SG_ERR_STATE, "set the projection before the first push");
    if (e->proj_n) return fail(SG_ERR_STATE, "the projection is already set");
    if (n == 0 || n > SGD_MAX_PROJ) return fail(SG_ERR_UNSUPPORTED, "select list size outside the device projection");
    for (uint32_t i = 0; i < n; i++)
        if (pc[i] + len[i] > words) return fail(SG_ERR_INVALID, "projection item outside its code");
    // roles (siddhi_gpu_ir.h): aggregator arguments, then the select list, then at most one `having`
    uint32_t A = 0, S = 0, H = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (types[i] & SG_PROJ_AGG_ITEM) {
            if (S || H) return fail(SG_ERR_INVALID, "aggregator items must come first");
            const uint32_t fn = (types[i] >> 8) & 0xffu;
            if (fn < SG_AGG_COUNT || fn > SG_AGG_MAX) return fail(SG_ERR_INVALID, "unknown aggregator");
            A++;
        } else if (types[i] & SG_PROJ_HAVING) {
            if (H) return fail(SG_ERR_INVALID, "more than one having item");
            H = 1;
        } else {
            if (H) return fail(SG_ERR_INVALID, "select items after the having item");
            S++;
        }
    }
    if (A > SGD_MAX_AGG) return fail(SG_ERR_UNSUPPORTED, "too many aggregators for the device projection");
    std::vector<uint32_t> c(code, code + words);
    std::vector<uint32_t> caps = pl.caps;
    std::vector<uint32_t> attrs;
    const int32_t part0 = (part_attr && (uint32_t)pl.s0 < n_streams) ? part_attr[pl.s0] : -1;
    for (uint32_t i = 0; i < n; i++) {
        const bool is_agg = i < A, is_having = H && i == n - 1;
        for (uint32_t w = pc[i]; w < pc[i] + len[i];) {
            const uint32_t op = c[w] & 0xffu, b = (c[w] >> 16) & 0xffu;
            const bool known = op == SG_OP_VAR || op == SG_OP_CONST || op == SG_OP_CVT || op == SG_OP_ISNULL_EV ||
                               (op >= SG_OP_ADD && op <= SG_OP_MOD) || (op >= SG_OP_EQ && op <= SG_OP_LE) ||
                               (op >= SG_OP_AND && op <= SG_OP_ISNULL) || op == SG_OP_IFELSE;
            if (!known) return fail(SG_ERR_INVALID, "unknown opcode in the projection");
            if (w + op_words(op) > pc[i] + len[i]) return fail(SG_ERR_INVALID, "projection item truncated");
            if (op == SG_OP_VAR && (b == SG_PROJ_SLOT_AGG || b == SG_PROJ_SLOT_OUT)) {
                const uint32_t x = c[w + 1];
                if (b == SG_PROJ_SLOT_AGG ? (is_agg || x >= A) : (!is_having || x >= S))
                    return fail(SG_ERR_INVALID, "projection reads an aggregator or output item it cannot see");
                c[w] = (c[w] & ~(0xffu << 16)) | ((b == SG_PROJ_SLOT_AGG ? 3u : 2u) << 16);
                w += 3;
                continue;
            }
            if (op == SG_OP_VAR || op == SG_OP_ISNULL_EV) {
                if (b != pl.slot0 && b != pl.slot1) return fail(SG_ERR_INVALID, "projection reads an unknown slot");
            }
            if (op == SG_OP_VAR) {
                const uint32_t attr = c[w + 1];
                uint32_t src, x;
                if (b == pl.slot1 || (pl.s0 == pl.s1 && (int32_t)attr == part0)) {
                    if (attr >= e->streams[pl.s1].types.size() || attr >= SGD_MAX_ATTR)
                        return fail(SG_ERR_UNSUPPORTED, "projection attribute outside the device projection");
                    src = 1;
                    x = attr;
                    if (std::find(attrs.begin(), attrs.end(), attr) == attrs.end()) attrs.push_back(attr);
                } else {
                    if (attr >= e->streams[pl.s0].types.size()) return fail(SG_ERR_INVALID, "attribute out of range");
                    size_t ci = std::find(caps.begin(), caps.end(), attr) - caps.begin();
                    if (ci == caps.size()) {
                        if (caps.size() >= SGD_MAX_CAPS) return fail(SG_ERR_UNSUPPORTED, "too many captured attributes");
                        caps.push_back(attr);
                    }
                    src = 0;
                    x = (uint32_t)ci;
                }
                c[w] = (c[w] & ~(0xffu << 16)) | (src << 16);
                c[w + 1] = x;
            }
            w += op_words(op);
        }
    }
    try {
        // the new capture list: payload columns, capture layout, JIT code, slabs (empty: no push yet)
        for (size_t i = pl.caps.size(); i < caps.size(); i++) {
            pl.caps.push_back(caps[i]);
            pl.cap_col.push_back((uint8_t)col_index(pl.evcols[pl.s0], caps[i]));
            pl.cap_type.push_back((uint8_t)e->streams[pl.s0].types.at(caps[i]));
        }
        {
            uint32_t maxw = 1;
            for (int s : {pl.s0, pl.s1}) {
                std::vector<uint32_t> ty;
                for (uint32_t a : pl.evcols[s]) ty.push_back(e->streams[s].types[a]);
                maxw = std::max(maxw, sgj_stride(sgj_col_words(ty) + 1));
            }
            if (maxw > e->pay_words) {
                e->pay_words = maxw;
                for (auto& sl : e->slots) {
                    sl.pay = dalloc<uint32_t>((size_t)maxw * e->maxb + 4, e->owned);
                    if (e->fused_ok) sl.tpay = dalloc<uint32_t>((size_t)maxw * e->maxb + 4, e->owned);
                }
                if (maxw > 6) e->fused_ok = false;
            }
        }
        const size_t K = e->K, C = e->cap, M = e->mcap;
        e->n_capw = 0;
        std::vector<uint32_t> woff;
        for (uint8_t t : pl.cap_type) {
            woff.push_back(e->n_capw);
            e->n_capw += (t == SG_T_LONG || t == SG_T_DOUBLE) ? 2 : 1;
        }
        e->p_capw = dalloc<uint32_t>(std::max<size_t>(1, e->n_capw) * C * K, e->owned);
        e->p_capnull = dalloc<uint32_t>(C * K, e->owned);
        HIP_OK(hipMemsetAsync(e->p_capnull, 0, C * K * 4, e->stream));
        e->raw_capw = dalloc<uint32_t>(std::max<size_t>(1, e->n_capw) * e->raw_cap, e->owned);
        e->raw_capnull = dalloc<uint32_t>(e->raw_cap, e->owned);
        HIP_OK(hipMemsetAsync(e->raw_capnull, 0, e->raw_cap * 4, e->stream));
        e->o_capw = dalloc<uint32_t>(std::max<size_t>(1, e->n_capw) * M, e->owned);
        e->o_capnull = dalloc<uint32_t>(M, e->owned);
        e->pval = dalloc<uint64_t>((size_t)(S + H) * M, e->owned);
        e->pnull = dalloc<uint8_t>((size_t)(S + H) * M, e->owned);
        if (A) {
            e->aggv = dalloc<uint64_t>((size_t)A * M, e->owned);
            e->aggnull = dalloc<uint8_t>((size_t)A * M, e->owned);
            e->agg_n = dalloc<int64_t>((size_t)A * K, e->owned);
            e->agg_v = dalloc<uint64_t>((size_t)A * K, e->owned);
            e->agg_has = dalloc<uint8_t>((size_t)A * K, e->owned);
            HIP_OK(hipMemsetAsync(e->agg_n, 0, (size_t)A * K * 8, e->stream));
            HIP_OK(hipMemsetAsync(e->agg_v, 0, (size_t)A * K * 8, e->stream));
            HIP_OK(hipMemsetAsync(e->agg_has, 0, (size_t)A * K, e->stream));
            e->out_first = dalloc<uint64_t>(e->maxb, e->owned);
        }
        for (auto& sl : e->slots)
            for (size_t j = 0; j < attrs.size(); j++) {
                sl.b_pcols.push_back(dalloc<uint64_t>(e->maxb, e->owned));
                sl.b_pnulls.push_back(dalloc<uint8_t>(e->maxb, e->owned));
            }
        // device tables: code | item pc | item len | capture word offsets | capture types
        std::vector<uint32_t> tab(c);
        const size_t o_pc = tab.size();
        tab.insert(tab.end(), pc, pc + n);
        const size_t o_len = tab.size();
        tab.insert(tab.end(), len, len + n);
        const size_t o_off = tab.size();
        tab.insert(tab.end(), woff.begin(), woff.end());
        const size_t o_ty = tab.size();
        for (uint8_t t : pl.cap_type) tab.push_back(t);
        tab.push_back(0);
        const size_t o_at = tab.size();
        tab.insert(tab.end(), types, types + A);
        tab.push_back(0);
        e->d_proj = dalloc<uint32_t>(tab.size(), e->owned);
        HIP_OK(hipMemcpy(e->d_proj, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
        ProjParams& q = e->pp;
        q = ProjParams{};
        q.code = e->d_proj;
        q.item_pc = e->d_proj + o_pc;
        q.item_len = e->d_proj + o_len;
        q.capw_off = e->d_proj + o_off;
        q.cap_type = e->d_proj + o_ty;
        q.n_items = n;
        q.o_trig = e->o_trig;
        q.o_capw = e->o_capw;
        q.o_capnull = e->o_capnull;
        q.capacity = M;
        q.out_count = e->out_count;
        q.batch_total = e->batch_total;
        q.pval = e->pval;
        q.pnull = e->pnull;
        q.err = e->err;
        q.n_agg = A;
        q.aggv = e->aggv;
        q.aggnull = e->aggnull;
        e->d_agg_type = e->d_proj + o_at;
        // recompile the advance kernel: matches now carry the partials' captures
        for (auto& kv : e->variants)
            if (kv.second.mod) (void)hipModuleUnload(kv.second.mod);
        e->variants.clear();
        e->jq = make_jit_query(e);
        e->jq.proj = true;
        e->consts.clear();
        (void)sgj_generate(e->jq, e->consts);
        (void)variant(e, false, false);
        e->proj_attrs = attrs;
        e->proj_n = n;
        e->proj_out = S + H;
        e->n_agg = A;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
    return SG_OK;
}

}  // namespace

// the other host-side translation units (sg_dict.cpp) report through the same sg_last_error
int sg_set_error(int code, const char* msg) { return fail(code, msg); }

// the multi-device engine (sg_sharded.cpp): the smallest event seq a live partial references (UINT64_MAX: none),
// after every queued batch; and an event recorded behind everything queued so far (its reads of a pushed device
// batch included: the two-state engine's grouping stream joins the main stream before the advance)
uint64_t sg_internal_min_seq(sg_engine* e) {
    HIP_OK(hipSetDevice(e->device));
    if (e->gen) return gen_min_seq(e->gen);
    sync_all(e);
    unsigned long long h = ~0ull;
    unsigned long long* m = nullptr;
    HIP_OK(hipMalloc(&m, 8));
    HIP_OK(hipMemcpyAsync(m, &h, 8, hipMemcpyHostToDevice, e->stream));
    if (sgd_launch_min_seq(e->hdr, e->p_seq, e->K, m, e->stream) != 0) throw HipError("k_min_seq launch failed");
    HIP_OK(hipMemcpyAsync(&h, m, 8, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    HIP_OK(hipFree(m));
    return h;
}
void sg_internal_record(sg_engine* e, hipEvent_t ev) {
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipEventRecord(ev, e->stream));
}

bool sg_internal_keep_heads(sg_engine* e) { return e && e->gen ? gen_keep_timer_heads(e->gen, true) : false; }
void sg_internal_heads(sg_engine* e, std::vector<uint32_t>& keys, std::vector<int64_t>& heads) {
    keys.clear();
    heads.clear();
    if (e && e->gen) gen_timer_heads(e->gen, keys, heads);
}

extern "C" {

const char* sg_last_error(void) { return g_err.c_str(); }
int sg_abi_version(void) { return SG_ABI_VERSION; }

int sg_engine_create(const void* ir, size_t ir_len, const sg_config* cfg, sg_engine** out) {
    if (!ir || !out || !cfg) return fail(SG_ERR_INVALID, "null argument");
    // (the fields before n_devices are the round-2 sg_config: such a caller gets one device)
    if (cfg->struct_size < offsetof(sg_config, n_devices)) return fail(SG_ERR_INVALID, "sg_config too small");
    sg_config full{};
    memcpy(&full, cfg, std::min<size_t>(cfg->struct_size, sizeof(sg_config)));
    full.struct_size = sizeof(sg_config);
    if (cfg->struct_size < sizeof(sg_config)) {
        full.n_devices = 1;
        full.devices = nullptr;
    }
    cfg = &full;
    if (cfg->n_devices > 1) {
        if (!cfg->devices) return fail(SG_ERR_INVALID, "n_devices > 1 needs the devices list");
        int rc = SG_OK;
        ShardEngine* sh = shd_create(ir, ir_len, cfg, &rc);
        if (!sh) return rc;
        sg_engine* e = new sg_engine();
        e->shard = sh;
        e->cfg = *cfg;
        *out = e;
        return SG_OK;
    }
    sg_engine* e = nullptr;
    try {
        e = new sg_engine();
        e->cfg = *cfg;
        e->device = cfg->device;
        e->timing = (cfg->flags & SG_CFG_TIMING) != 0;
        if (const char* d = getenv("SGD_REG_SLOTS")) {
            e->reg_slots = (uint32_t)strtoul(d, nullptr, 0);
            e->reg_slots_hbm = e->reg_slots;  // (a forced window: the HBM pass spills at the same size)
        }
        if (const char* d = getenv("SGD_REG_SLOTS_HBM")) e->reg_slots_hbm = (uint32_t)strtoul(d, nullptr, 0);
        if (e->reg_slots < 1 || e->reg_slots > SGD_MAX_REG) throw std::invalid_argument("SGD_REG_SLOTS out of [1, 16]");
        if (e->reg_slots_hbm < 1 || e->reg_slots_hbm > SGD_MAX_REG_HBM)
            throw std::invalid_argument("SGD_REG_SLOTS_HBM out of [1, 31]");
        if (const char* d = getenv("SGD_STAGE_CHUNKS")) e->stage_override = (uint32_t)strtoul(d, nullptr, 0);
        if (e->stage_override * 16ull * (SGD_BLOCK / SGD_WAVE) > SGD_STAGE_MAX_BYTES)
            throw std::invalid_argument("SGD_STAGE_CHUNKS above the LDS staging bound");
        e->K = cfg->n_keys ? cfg->n_keys : 1;
        e->null_keys = (cfg->flags & SG_CFG_NULL_KEYS) != 0;
        e->cap = cfg->partial_capacity ? cfg->partial_capacity : 64;
        e->maxb = cfg->max_batch ? cfg->max_batch : (1u << 20);
        e->mcap = cfg->match_capacity ? cfg->match_capacity : (uint64_t)e->maxb * 4;
        if (e->cap > SGD_MAX_CAP) throw std::invalid_argument("partial_capacity above 4095");
        // the register window never holds more partials than the key's slab can take when it spills
        if (e->reg_slots > e->cap) e->reg_slots = e->cap;
        if (e->reg_slots_hbm > e->cap) e->reg_slots_hbm = e->cap;
        if (e->mcap >= (1ull << 31)) throw std::invalid_argument("match_capacity must be < 2^31");
        if (ir_len < SG_IR_HDR_WORDS * 4 || ir_len % 4) throw std::invalid_argument("IR too short");
        if (((const uint32_t*)ir)[0] != SG_IR_MAGIC || ((const uint32_t*)ir)[1] != SG_IR_VERSION)
            throw std::invalid_argument("bad IR magic/version");
        // every shape must lower onto the general engine (validates the IR); the specialised
        // two-state kernel takes the shapes it covers
        delete gen_build_program((const uint32_t*)ir, ir_len / 4, e->cap);
        e->ir_hash = 1469598103934665603ull;
        for (size_t i = 0; i < ir_len / 4; i++) e->ir_hash = (e->ir_hash ^ ((const uint32_t*)ir)[i]) * 1099511628211ull;
        bool general = getenv("SG_FORCE_GENERAL") != nullptr;
        if (!general) {
            try {
                build_plan(e, ir, ir_len);
            } catch (const std::runtime_error&) {
                general = true;
            }
        }
        if (general) {
            int ndev = 0;
            HIP_OK(hipGetDeviceCount(&ndev));
            if (cfg->device < 0 || cfg->device >= ndev) throw HipError("no such HIP device");
            HIP_OK(hipSetDevice(cfg->device));
            HIP_OK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
            e->gen = gen_create((const uint32_t*)ir, ir_len / 4, *cfg, e->stream);
            *out = e;
            return SG_OK;
        }
        e->jq = make_jit_query(e);
        (void)sgj_generate(e->jq, e->consts);  // validates the filters, fixes the constant table
        if (!e->plan.partitioned && e->K != 1) e->K = 1;
        int ndev = 0;
        HIP_OK(hipGetDeviceCount(&ndev));
        if (cfg->device < 0 || cfg->device >= ndev) throw HipError("no such HIP device");
        HIP_OK(hipSetDevice(cfg->device));
        // SG_STREAM_PRIO (experiments): "g" = the grouping stream at the higher priority, "m" = the main one
        const char* pr = getenv("SG_STREAM_PRIO");
        int plo = 0, phi = 0;
        HIP_OK(hipDeviceGetStreamPriorityRange(&plo, &phi));
        // SG_CUMASK (experiments): "g:a/b" = the grouping stream on the CUs i with i % b < a, "m:a/b" = the main
        // stream likewise, upper case ("G:a/b", "M:a/b") = the complement (i % b >= a); comma-separated, so that
        // the two batches in flight can run on disjoint CU sets
        const char* cm = getenv("SG_CUMASK");
        auto masked = [&](char which, hipStream_t* st) -> bool {
            if (!cm) return false;
            for (const char* q = cm; *q; q++) {
                if ((q[0] == which || q[0] == which - 32) && q[1] == ':') {
                    const bool comp = q[0] == which - 32;
                    unsigned a = 0, b = 1;
                    if (sscanf(q + 2, "%u/%u", &a, &b) != 2 || b == 0) return false;
                    int ncu = 0;
                    HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg->device));
                    std::vector<uint32_t> mk(((size_t)ncu + 31) / 32, 0u);
                    for (int i = 0; i < ncu; i++)
                        if (((unsigned)i % b < a) != comp) mk[(size_t)i / 32] |= 1u << (i % 32);
                    HIP_OK(hipExtStreamCreateWithCUMask(st, (uint32_t)mk.size(), mk.data()));
                    return true;
                }
            }
            return false;
        };
        if (!masked('m', &e->stream))
            HIP_OK(hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, (pr && pr[0] == 'm') ? phi : plo));
        if (!masked('g', &e->gstream))
            HIP_OK(hipStreamCreateWithPriority(&e->gstream, hipStreamNonBlocking, (pr && pr[0] == 'g') ? phi : plo));
        HIP_OK(hipStreamCreateWithFlags(&e->pstream, hipStreamNonBlocking));
        e->async_host = (cfg->flags & SG_CFG_ASYNC_HOST) != 0;
        allocate(e);
        (void)variant(e, false, false);  // compile (or fetch) the advance kernel now: fail at creation
        *out = e;
        return SG_OK;
    } catch (const HipError& ex) {
        delete e;
        return fail(SG_ERR_DEVICE, ex.what());
    } catch (const std::invalid_argument& ex) {
        delete e;
        return fail(SG_ERR_INVALID, ex.what());
    } catch (const std::exception& ex) {
        delete e;
        return fail(SG_ERR_UNSUPPORTED, ex.what());
    }
}

void sg_engine_destroy(sg_engine* e) {
    if (e && e->shard) {
        shd_destroy(e->shard);
        e->shard = nullptr;
    }
    delete e;
}

int sg_push_batch(sg_engine* e, const sg_batch* b) {
    if (!e || !b) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_push(e->shard, b);
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->gen) {
            std::string msg;
            const int rc = gen_push(e->gen, b, msg);
            return rc == SG_OK ? rc : fail(rc, msg);
        }
        return push(e, b);
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_advance_time(sg_engine* e, int64_t now_ms) {
    if (!e) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_advance(e->shard, now_ms);
    if (!e->gen) return SG_OK;  // the two-state kernel's shapes have no timers
    try {
        HIP_OK(hipSetDevice(e->device));
        std::string msg;
        const int rc = gen_advance(e->gen, now_ms, msg);
        return rc == SG_OK ? rc : fail(rc, msg);
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_set_projection(sg_engine* e, const uint32_t* code, uint32_t code_words, const uint32_t* item_pc,
                      const uint32_t* item_len, const uint32_t* item_type, uint32_t n_items, const int32_t* part_attr,
                      uint32_t n_streams) {
    if (!e || !code || !item_pc || !item_len || !item_type) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard)
        return shd_set_projection(e->shard, code, code_words, item_pc, item_len, item_type, n_items, part_attr, n_streams);
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->gen) {
            std::string msg;
            const int rc = gen_set_projection(e->gen, code, code_words, item_pc, item_len, item_type, n_items, msg);
            return rc == SG_OK ? rc : fail(rc, msg);
        }
        return set_projection(e, code, code_words, item_pc, item_len, item_type, n_items, part_attr, n_streams);
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_get_projection(sg_engine* e, uint32_t mem, sg_projection* out) {
    if (!e || !out) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_get_projection(e->shard, mem, out);
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->gen) {
            std::string msg;
            const int rc = gen_get_projection(e->gen, mem, out, msg);
            return rc == SG_OK ? rc : fail(rc, msg);
        }
        if (!e->held) return fail(SG_ERR_STATE, "poll the matches first");
        if (!e->proj_n) return fail(SG_ERR_STATE, "no projection set");
        const uint32_t n = e->proj_out;   // select items + having (the aggregators feed them)
        const size_t m = (size_t)e->polled;
        const size_t start = (size_t)((e->win) % e->mcap);
        out->n = m;
        out->n_items = n;
        if (mem == SG_MEM_DEVICE) {
            if (m && n > 1) return fail(SG_ERR_INVALID, "device projection rows are capacity-strided: poll to host");
            out->value = e->pval + start;
            out->null = e->pnull + start;
            out->mem = SG_MEM_DEVICE;
            return SG_OK;
        }
        e->h_pval.resize(m * n);
        e->h_pnull.resize(m * n);
        for (uint32_t i = 0; i < n && m; i++) {
            ring_to_host(e->h_pval.data() + i * m, e->pval + (size_t)i * e->mcap, 8, start, m, e->mcap, e->pstream);
            ring_to_host(e->h_pnull.data() + i * m, e->pnull + (size_t)i * e->mcap, 1, start, m, e->mcap, e->pstream);
        }
        HIP_OK(hipStreamSynchronize(e->pstream));
        out->value = e->h_pval.data();
        out->null = e->h_pnull.data();
        out->mem = SG_MEM_HOST;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_wait_stream(sg_engine* e, void* stream) {
    if (!e) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_wait_stream(e->shard, stream);
    try {
        HIP_OK(hipSetDevice(e->device));
        hipEvent_t x = e->ev();
        HIP_OK(hipEventRecord(x, (hipStream_t)stream));
        HIP_OK(hipStreamWaitEvent(e->stream, x, 0));
        // the two-state engine reads a pushed batch first on its grouping stream (copies + sort): it waits too
        if (e->gstream) HIP_OK(hipStreamWaitEvent(e->gstream, x, 0));
        e->free_events.push_back(x);  // reusable once recorded again (a wait captures the recorded work)
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_poll_matches(sg_engine* e, uint32_t mem, sg_match_batch* out) {
    if (!e || !out) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_poll(e->shard, mem, out);
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->gen) {  // (the general engine's polls always wait for every pushed batch)
            std::string msg;
            const int rc = gen_poll(e->gen, mem & ~(uint32_t)SG_POLL_READY, out, msg);
            return rc == SG_OK ? rc : fail(rc, msg);
        }
        return poll(e, mem, out);
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_release_matches(sg_engine* e, sg_match_batch* m) {
    if (!e) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_release(e->shard, m);
    if (e->gen) gen_release(e->gen);
    else if (e->held) e->win += e->polled;  // those ring records are free again
    e->held = false;
    if (m) memset(m, 0, sizeof(*m));
    return SG_OK;
}

int sg_synchronize(sg_engine* e) {
    if (!e) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_synchronize(e->shard);
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->gen) {
            HIP_OK(hipStreamSynchronize(e->stream));
            e->resolve_spans();
        } else {
            sync_all(e);
        }
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_get_stats_sized(sg_engine* e, sg_stats* out, size_t out_size) {
    if (!out || out_size == 0) return fail(SG_ERR_INVALID, "null stats or zero size");
    sg_stats full{};
    const int rc = sg_get_stats(e, &full);
    if (rc == SG_OK) memcpy(out, &full, std::min(out_size, sizeof(sg_stats)));
    return rc;
}

int sg_get_stats(sg_engine* e, sg_stats* out) {
    if (!e || !out) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_stats(e->shard, out);
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->gen) {
            gen_stats(e->gen, out);
            return SG_OK;
        }
        unsigned long long s[SGD_ST_N];
        sync_all(e);
        HIP_OK(hipMemcpyAsync(s, e->stats, sizeof(s), hipMemcpyDeviceToHost, e->stream));
        HIP_OK(hipStreamSynchronize(e->stream));
        *out = e->st;
        out->partials_scanned = s[SGD_ST_SCANNED];
        out->partials_created = s[SGD_ST_CREATED];
        out->matches = s[SGD_ST_MATCHES];
        out->keys_touched = s[SGD_ST_KEYS];
        out->live_at_batch_start = s[SGD_ST_LIVE0];
        out->window_spills = s[SGD_ST_SPILLS];
        out->hot_keys = s[SGD_ST_HOTK];
        out->hot_events = s[SGD_ST_HOTE];
        // live partials now: sum of the headers' counts (host reduction; diagnostics only)
        std::vector<uint32_t> h(e->K);
        HIP_OK(hipMemcpy(h.data(), e->hdr, (size_t)e->K * 4, hipMemcpyDeviceToHost));
        uint64_t live = 0;
        for (uint32_t x : h) live += SGD_H_NPEND(x) + SGD_H_NSTG(x);
        out->partials_live = live;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_engine_describe(sg_engine* e, char* out, size_t out_len) {
    if (!e || (!out && out_len)) return fail(SG_ERR_INVALID, "null argument");
    std::string d;
    sg_engine* one = e->shard ? shd_first(e->shard) : e;
    if (one->gen) {
        d = gen_describe(one->gen);
    } else {
        d = std::string("push: ") +
            (one->fused_last ? "k_part_hist + k_part_scan + k_part_scatter x2 + k_tile_bounds (grouping by key tile, stream 2); "
                               "k_adv_m (key split in LDS + NFA advance, LDS-staged, lane per key)"
                             : "k_part_hist + k_part_scan + k_part_scatter per 8-bit digit + k_part_bounds (grouping, stream 2); "
                               "k_adv_m (NFA advance, LDS-staged, lane per key)") +
            (one->hot_batches ? " + k_hot_prep..k_hot_final (hot keys, partials in parallel, " +
                                    std::to_string(one->hot_batches) + " batches)" : std::string()) +
            " + k_adv_m_h / k_adv_m_k (NFA advance, HBM pass: the waves left whole / the keys stopped) + k_stats_reduce; k_order_sums + scan + k_order_scatter (ordering)";
        if (one->proj_n) d += " + k_project" + std::string(one->n_agg ? " + k_agg" : "");
    }
    if (e->shard) d = std::to_string(shd_count(e->shard)) + " shards, each " + d;
    if (out_len) {
        const size_t n = std::min(out_len - 1, d.size());
        memcpy(out, d.data(), n);
        out[n] = 0;
    }
    return SG_OK;
}

// ---- partition purge (PartitionRuntimeImpl.java:368-401) ----------------------------------------
int sg_reset_keys(sg_engine* e, const uint32_t* keys, uint64_t n, uint32_t mem) {
    if (!e || (!keys && n)) return fail(SG_ERR_INVALID, "null argument");
    if (n == 0) return SG_OK;
    if (e->shard) return shd_reset_keys(e->shard, keys, n, mem);
    if (n >= (1ull << 32)) return fail(SG_ERR_INVALID, "too many keys in one reset");
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->held) return fail(SG_ERR_STATE, "release the polled matches before resetting keys");
        const uint32_t K = e->gen ? (e->cfg.n_keys ? e->cfg.n_keys : 1) : e->K;
        const uint32_t* dk = keys;
        uint32_t* tmp = nullptr;
        if (mem == SG_MEM_HOST) {
            for (uint64_t i = 0; i < n; i++)
                if (keys[i] >= K) return fail(SG_ERR_INVALID, "key id outside [0, n_keys)");
            HIP_OK(hipMalloc(&tmp, n * 4 + 4));
            HIP_OK(hipMemcpyAsync(tmp, keys, n * 4, hipMemcpyHostToDevice, e->stream));
            dk = tmp;
        } else {
            // device ids: validated before any state changes (all or nothing, as for host ids)
            HIP_OK(hipMalloc(&tmp, 4));
            if (sgd_launch_check_keys(dk, (uint32_t)n, K, tmp, e->stream) != 0)
                throw HipError("k_check_keys launch failed");
            uint32_t bad = 0;
            HIP_OK(hipMemcpyAsync(&bad, tmp, 4, hipMemcpyDeviceToHost, e->stream));
            HIP_OK(hipStreamSynchronize(e->stream));
            if (bad) {
                HIP_OK(hipFree(tmp));
                return fail(SG_ERR_INVALID, "key id outside [0, n_keys)");
            }
        }
        int rc = SG_OK;
        std::string msg;
        if (e->gen) {
            rc = gen_reset_keys(e->gen, dk, (uint32_t)n, msg);
        } else if (e->plan.partitioned) {
            if (sgd_launch_reset_keys(dk, (uint32_t)n, e->K, e->hdr, e->err, e->stream) != 0) rc = SG_ERR_DEVICE;
            if (sgd_launch_reset_agg(dk, (uint32_t)n, e->K, e->n_agg, e->agg_n, e->agg_v, e->agg_has, e->stream) != 0)
                rc = SG_ERR_DEVICE;
            msg = "k_reset_keys launch failed";
        }
        HIP_OK(hipStreamSynchronize(e->stream));
        if (tmp) HIP_OK(hipFree(tmp));
        if (rc != SG_OK) return fail(rc, msg);
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

// ---- persistence -------------------------------------------------------------
// The reference snapshots, per partition key, each pre-state processor's pending and newAndEvery lists
// (StreamPreStateProcessor.StreamPreState.snapshot/restore, StreamPreStateProcessor.java:450-469) through
// PartitionStateHolder (util/snapshot/state/PartitionStateHolder.java:43-80).  The device keeps exactly
// that state in HBM, so the image is a header plus the state buffers:
//   two-state kernel: hdr[K] (list counts, start-state seeds, init bit) and the first `rows` rows of
//     every slab plane (partial j of key k at j*K + k; rows = the deepest key's pending + staged count)
//   general kernel:  the interleaved per-key state blocks and the engine clock (gen_snapshot).
// Matches are output, not state: a snapshot or restore with matches waiting to be polled fails with
// SG_ERR_STATE (the reference has delivered its callbacks by the time a snapshot completes).  A
// restore needs an engine created from the same IR with the same n_keys; the two-state image needs
// partial_capacity >= rows, the general one the same partial_capacity (block layout).
struct SnapHeader {
    uint32_t magic;       // SG_SNAP_MAGIC
    uint32_t version;
    uint32_t kind;        // 1 = two-state kernel, 2 = general kernel
    uint32_t K;
    uint64_t ir_hash;
    uint32_t cap;         // partial_capacity of the source engine
    uint32_t rows;        // two-state: slab rows in the image
    uint32_t n_capw;
    uint32_t nullable;
    uint64_t next_seq;    // sequence numbers must keep increasing across a restore
    uint32_t have_base;
    uint32_t n_agg;       // two-state: per-key aggregator states in the image (selector aggregators)
    GenClock clk;
    uint64_t body_bytes;
};
#define SG_SNAP_MAGIC 0x4e534753u  // "SGSN"
#define SG_SNAP_VERSION 2u

static bool outputs_pending(sg_engine* e) {
    sync_all(e);
    return e->done_count != e->win;
}

int sg_snapshot(sg_engine* e, void** buf, size_t* len) {
    if (!e || !buf || !len) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_snapshot(e->shard, buf, len);
    try {
        HIP_OK(hipSetDevice(e->device));
        SnapHeader h{};
        h.magic = SG_SNAP_MAGIC;
        h.version = SG_SNAP_VERSION;
        h.K = e->gen ? 0 : e->K;
        h.ir_hash = e->ir_hash;
        h.next_seq = e->next_seq;
        h.have_base = e->have_base ? 1u : 0u;
        if (e->gen) {
            h.kind = 2;
            const uint64_t words = gen_state_words(e->gen);
            h.body_bytes = words * 4;
            uint8_t* out = (uint8_t*)malloc(sizeof(h) + h.body_bytes);
            if (!out) return fail(SG_ERR_CAPACITY, "snapshot buffer allocation failed");
            std::string msg;
            const int rc = gen_snapshot(e->gen, (uint32_t*)(out + sizeof(h)), &h.clk, msg);
            if (rc != SG_OK) { free(out); return fail(rc, msg); }
            h.cap = e->cap;
            h.K = e->cfg.n_keys ? e->cfg.n_keys : 1;
            memcpy(out, &h, sizeof(h));
            *buf = out;
            *len = sizeof(h) + h.body_bytes;
            return SG_OK;
        }
        if (e->held) return fail(SG_ERR_STATE, "release the polled matches before a snapshot");
        if (outputs_pending(e)) return fail(SG_ERR_STATE, "poll the emitted matches before a snapshot");
        const size_t K = e->K;
        std::vector<uint32_t> hdr(K);
        HIP_OK(hipMemcpy(hdr.data(), e->hdr, K * 4, hipMemcpyDeviceToHost));
        uint32_t rows = 0;
        for (uint32_t x : hdr) rows = std::max(rows, (uint32_t)(SGD_H_NPEND(x) + SGD_H_NSTG(x)));
        h.kind = 1;
        h.cap = e->cap;
        h.rows = rows;
        h.n_capw = e->n_capw;
        h.nullable = e->nullable ? 1u : 0u;
        h.n_agg = e->n_agg;
        const size_t plane = (size_t)rows * K;  // elements per saved plane
        h.body_bytes = K * 4 + plane * (8 + 8 + 4 * (size_t)e->n_capw + 4) + (size_t)e->n_agg * K * 17;
        uint8_t* out = (uint8_t*)malloc(sizeof(h) + h.body_bytes);
        if (!out) return fail(SG_ERR_CAPACITY, "snapshot buffer allocation failed");
        uint8_t* q = out + sizeof(h);
        memcpy(q, hdr.data(), K * 4);
        q += K * 4;
        HIP_OK(hipMemcpyAsync(q, e->p_ts, plane * 8, hipMemcpyDeviceToHost, e->stream));
        q += plane * 8;
        HIP_OK(hipMemcpyAsync(q, e->p_seq, plane * 8, hipMemcpyDeviceToHost, e->stream));
        q += plane * 8;
        for (uint32_t w = 0; w < e->n_capw; w++) {
            HIP_OK(hipMemcpyAsync(q, e->p_capw + (size_t)w * e->cap * K, plane * 4, hipMemcpyDeviceToHost, e->stream));
            q += plane * 4;
        }
        HIP_OK(hipMemcpyAsync(q, e->p_capnull, plane * 4, hipMemcpyDeviceToHost, e->stream));
        q += plane * 4;
        if (e->n_agg) {
            const size_t na = (size_t)e->n_agg * K;
            HIP_OK(hipMemcpyAsync(q, e->agg_n, na * 8, hipMemcpyDeviceToHost, e->stream));
            HIP_OK(hipMemcpyAsync(q + na * 8, e->agg_v, na * 8, hipMemcpyDeviceToHost, e->stream));
            HIP_OK(hipMemcpyAsync(q + na * 16, e->agg_has, na, hipMemcpyDeviceToHost, e->stream));
        }
        HIP_OK(hipStreamSynchronize(e->stream));
        memcpy(out, &h, sizeof(h));
        *buf = out;
        *len = sizeof(h) + h.body_bytes;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_restore(sg_engine* e, const void* buf, size_t len) {
    if (!e || !buf) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_restore(e->shard, buf, len);
    SnapHeader h;
    if (len < sizeof(h)) return fail(SG_ERR_INVALID, "snapshot too short");
    memcpy(&h, buf, sizeof(h));
    if (h.magic != SG_SNAP_MAGIC || h.version != SG_SNAP_VERSION) return fail(SG_ERR_INVALID, "not a snapshot of this engine version");
    if (len != sizeof(h) + h.body_bytes) return fail(SG_ERR_INVALID, "snapshot length does not match its header");
    if (h.ir_hash != e->ir_hash) return fail(SG_ERR_INVALID, "snapshot of a different query");
    if (h.kind != (e->gen ? 2u : 1u)) return fail(SG_ERR_INVALID, "snapshot of a different engine kind");
    const uint8_t* q = (const uint8_t*)buf + sizeof(h);
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->gen) {
            const uint64_t K = e->cfg.n_keys ? e->cfg.n_keys : 1;
            const uint64_t words = gen_state_words(e->gen);
            if (h.K != K || h.body_bytes != words * 4)
                return fail(SG_ERR_INVALID, "snapshot taken with a different n_keys / partial_capacity");
            std::string msg;
            const int rc = gen_restore(e->gen, (const uint32_t*)q, h.clk, msg);
            if (rc != SG_OK) return fail(rc, msg);
        } else {
            const size_t K = e->K;
            if (h.K != K) return fail(SG_ERR_INVALID, "snapshot taken with a different n_keys");
            if (h.rows > e->cap) return fail(SG_ERR_CAPACITY, "snapshot holds more partials per key than partial_capacity");
            if (h.n_capw != e->n_capw) return fail(SG_ERR_INVALID, "snapshot capture layout differs");
            if (h.n_agg != e->n_agg) return fail(SG_ERR_INVALID, "snapshot aggregator layout differs");
            const size_t plane = (size_t)h.rows * K;
            if (h.body_bytes != K * 4 + plane * (8 + 8 + 4 * (size_t)h.n_capw + 4) + (size_t)h.n_agg * K * 17)
                return fail(SG_ERR_INVALID, "snapshot body size does not match its header");
            if (e->held) return fail(SG_ERR_STATE, "release the polled matches before a restore");
            if (outputs_pending(e)) return fail(SG_ERR_STATE, "poll the emitted matches before a restore");
            HIP_OK(hipMemcpyAsync(e->hdr, q, K * 4, hipMemcpyHostToDevice, e->stream));
            q += K * 4;
            HIP_OK(hipMemcpyAsync(e->p_ts, q, plane * 8, hipMemcpyHostToDevice, e->stream));
            q += plane * 8;
            HIP_OK(hipMemcpyAsync(e->p_seq, q, plane * 8, hipMemcpyHostToDevice, e->stream));
            q += plane * 8;
            for (uint32_t w = 0; w < h.n_capw; w++) {
                HIP_OK(hipMemcpyAsync(e->p_capw + (size_t)w * e->cap * K, q, plane * 4, hipMemcpyHostToDevice, e->stream));
                q += plane * 4;
            }
            HIP_OK(hipMemcpyAsync(e->p_capnull, q, plane * 4, hipMemcpyHostToDevice, e->stream));
            q += plane * 4;
            if (e->n_agg) {
                const size_t na = (size_t)e->n_agg * K;
                HIP_OK(hipMemcpyAsync(e->agg_n, q, na * 8, hipMemcpyHostToDevice, e->stream));
                HIP_OK(hipMemcpyAsync(e->agg_v, q + na * 8, na * 8, hipMemcpyHostToDevice, e->stream));
                HIP_OK(hipMemcpyAsync(e->agg_has, q + na * 16, na, hipMemcpyHostToDevice, e->stream));
            }
            HIP_OK(hipStreamSynchronize(e->stream));
            if (h.nullable) e->nullable = true;
        }
        e->next_seq = h.next_seq;
        e->have_base = h.have_base != 0;
        e->poll_base = e->next_seq;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}
int sg_free_buffer(void* buf) {
    free(buf);
    return SG_OK;
}

// ---- the per-key state in the reference's per-state-processor form (state_doc.h) -----------------------
// Two-state kernel: processor 0 is e1's pre-state (its pending / newAndEvery lists hold the start-state
// seeds: StateEvents with no slot filled, counted in the key header), processor 1 is e2's (its lists are
// the partials: one StateEvent per slab row, slot0 = the e1 StreamEvent with the attributes the partial
// captured; the other attributes are not on the device and are marked absent in `present`).  A seed's
// timestamp is not kept (it does not affect matching) and is written as -1.
static int twostate_export(sg_engine* e, SdDoc& d) {
    const Plan& pl = e->plan;
    const size_t K = e->K;
    if (e->held) return fail(SG_ERR_STATE, "release the polled matches before exporting the state");
    if (outputs_pending(e)) return fail(SG_ERR_STATE, "poll the emitted matches before exporting the state");
    std::vector<uint32_t> hdr(K);
    HIP_OK(hipMemcpy(hdr.data(), e->hdr, K * 4, hipMemcpyDeviceToHost));
    uint32_t rows = 0;
    for (uint32_t x : hdr) rows = std::max(rows, (uint32_t)(SGD_H_NPEND(x) + SGD_H_NSTG(x)));
    const size_t plane = (size_t)rows * K;
    std::vector<int64_t> ts(plane);
    std::vector<uint64_t> seq(plane);
    std::vector<uint32_t> capw((size_t)e->n_capw * plane), capn(plane);
    if (plane) {
        HIP_OK(hipMemcpy(ts.data(), e->p_ts, plane * 8, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(seq.data(), e->p_seq, plane * 8, hipMemcpyDeviceToHost));
        for (uint32_t w = 0; w < e->n_capw; w++)
            HIP_OK(hipMemcpy(capw.data() + w * plane, e->p_capw + (size_t)w * e->cap * K, plane * 4, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(capn.data(), e->p_capnull, plane * 4, hipMemcpyDeviceToHost));
    }
    const uint32_t na = (uint32_t)e->streams[pl.s0].types.size();
    d.n_procs = 2;
    d.n_slots = 2;
    d.desc = {SdProcDesc{0, 0, pl.slot0}, SdProcDesc{0, 0, pl.slot1}};
    for (uint32_t k = 0; k < K; k++) {
        const uint32_t h = hdr[k];
        if (!SGD_H_INIT(h)) continue;
        SdKey x;
        x.key = k;
        x.procs.resize(2);
        for (auto& P : x.procs) P.flags = SD_ACTIVE;
        x.procs[0].flags |= SD_INITIALIZED;  // the start state's init() ran with the key's first event
        auto seed = [&]() {
            SdState st;
            st.chains.resize(2);
            x.states.push_back(st);
            return (uint32_t)x.states.size() - 1;
        };
        for (uint32_t i = 0; i < SGD_H_SPEND(h); i++) x.procs[0].pending.push_back(seed());
        for (uint32_t i = 0; i < SGD_H_SSTG(h); i++) x.procs[0].newev.push_back(seed());
        const uint32_t np = SGD_H_NPEND(h), ns = SGD_H_NSTG(h);
        for (uint32_t j = 0; j < np + ns; j++) {
            const size_t r = (size_t)j * K + k;
            SdStream ev;
            ev.seq = seq[r];
            ev.ts = ts[r];
            ev.attr.assign(na, 0);
            uint32_t w = 0;
            for (size_t c = 0; c < pl.caps.size(); c++) {
                const uint32_t a = pl.caps[c], t = pl.cap_type[c];
                uint64_t v = capw[(size_t)w * plane + r];
                if (t == SG_T_LONG || t == SG_T_DOUBLE) v |= (uint64_t)capw[(size_t)(w + 1) * plane + r] << 32;
                w += (t == SG_T_LONG || t == SG_T_DOUBLE) ? 2 : 1;
                ev.attr[a] = v;
                ev.present |= 1u << a;
                if ((capn[r] >> c) & 1u) ev.null_bits |= 1u << a;
            }
            x.streams.push_back(ev);
            SdState st;
            st.ts = ts[r];
            st.chains.resize(2);
            st.chains[pl.slot0].push_back((uint32_t)x.streams.size() - 1);
            x.states.push_back(st);
            (j < np ? x.procs[1].pending : x.procs[1].newev).push_back((uint32_t)x.states.size() - 1);
        }
        d.keys.push_back(std::move(x));
    }
    return SG_OK;
}

static int twostate_import(sg_engine* e, const SdDoc& d) {
    const Plan& pl = e->plan;
    const size_t K = e->K;
    if (d.n_procs != 2 || d.n_slots != 2 || !(d.desc[0] == SdProcDesc{0, 0, pl.slot0}) ||
        !(d.desc[1] == SdProcDesc{0, 0, pl.slot1}))
        return fail(SG_ERR_INVALID, "state document of a different query shape");
    if (e->held) return fail(SG_ERR_STATE, "release the polled matches before a state import");
    if (outputs_pending(e)) return fail(SG_ERR_STATE, "poll the emitted matches before a state import");
    uint32_t rows = 0;
    for (const SdKey& x : d.keys) rows = std::max<uint32_t>(rows, (uint32_t)(x.procs[1].pending.size() + x.procs[1].newev.size()));
    if (rows > e->cap) return fail(SG_ERR_CAPACITY, "state document holds more partials per key than partial_capacity");
    const size_t plane = (size_t)rows * K;
    std::vector<uint32_t> hdr(K, 0u);
    std::vector<int64_t> ts(plane, 0);
    std::vector<uint64_t> seq(plane, 0);
    std::vector<uint32_t> capw((size_t)e->n_capw * plane, 0u), capn(plane, 0u);
    bool nulls = false;
    for (const SdKey& x : d.keys) {
        if (x.key >= K) return fail(SG_ERR_INVALID, "state document key id outside [0, n_keys)");
        for (int p = 0; p < 1; p++)
            for (const auto* l : {&x.procs[0].pending, &x.procs[0].newev})
                for (uint32_t si : *l)
                    for (const auto& c : x.states[si].chains)
                        if (!c.empty()) return fail(SG_ERR_UNSUPPORTED, "a start-state list entry holds an event");
        const size_t spend = x.procs[0].pending.size(), sstg = x.procs[0].newev.size();
        if (spend > 3 || sstg > 3) return fail(SG_ERR_UNSUPPORTED, "more than 3 start-state seeds in one list");
        const size_t np = x.procs[1].pending.size(), ns = x.procs[1].newev.size();
        const bool init = (x.procs[0].flags & SD_INITIALIZED) != 0 || spend + sstg + np + ns > 0;
        hdr[x.key] = SGD_H_MAKE(np, ns, spend, sstg, init ? 1 : 0);
        for (size_t j = 0; j < np + ns; j++) {
            const SdState& st = x.states[j < np ? x.procs[1].pending[j] : x.procs[1].newev[j - np]];
            for (uint32_t sl = 0; sl < 2; sl++)
                if ((sl == pl.slot0) != (st.chains[sl].size() == 1) || st.chains[sl].size() > 1)
                    return fail(SG_ERR_UNSUPPORTED, "a partial that is not one e1 event");
            const SdStream& ev = x.streams[st.chains[pl.slot0][0]];
            const size_t r = j * K + x.key;
            ts[r] = ev.ts;
            seq[r] = ev.seq;
            uint32_t w = 0;
            for (size_t c = 0; c < pl.caps.size(); c++) {
                const uint32_t a = pl.caps[c], t = pl.cap_type[c];
                if (a >= ev.attr.size() || !((ev.present >> a) & 1u))
                    return fail(SG_ERR_INVALID, "a partial's event lacks an attribute the query reads");
                capw[(size_t)w * plane + r] = (uint32_t)ev.attr[a];
                if (t == SG_T_LONG || t == SG_T_DOUBLE) capw[(size_t)(w + 1) * plane + r] = (uint32_t)(ev.attr[a] >> 32);
                w += (t == SG_T_LONG || t == SG_T_DOUBLE) ? 2 : 1;
                if ((ev.null_bits >> a) & 1u) {
                    capn[r] |= 1u << c;
                    nulls = true;
                }
            }
        }
    }
    HIP_OK(hipMemcpy(e->hdr, hdr.data(), K * 4, hipMemcpyHostToDevice));
    if (plane) {
        HIP_OK(hipMemcpy(e->p_ts, ts.data(), plane * 8, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(e->p_seq, seq.data(), plane * 8, hipMemcpyHostToDevice));
        for (uint32_t w = 0; w < e->n_capw; w++)
            HIP_OK(hipMemcpy(e->p_capw + (size_t)w * e->cap * K, capw.data() + w * plane, plane * 4, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(e->p_capnull, capn.data(), plane * 4, hipMemcpyHostToDevice));
    }
    if (nulls) e->nullable = true;
    return SG_OK;
}

int sg_state_export(sg_engine* e, void** buf, size_t* len) {
    if (!e || !buf || !len) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_state_export(e->shard, buf, len);
    try {
        HIP_OK(hipSetDevice(e->device));
        SdDoc d;
        if (e->gen) {
            std::string msg;
            const int rc = gen_state_export(e->gen, d, msg);
            if (rc != SG_OK) return fail(rc, msg);
        } else {
            const int rc = twostate_export(e, d);
            if (rc != SG_OK) return rc;
        }
        std::vector<uint8_t> bytes = sd_write(d);
        void* out = malloc(bytes.size());
        if (!out) return fail(SG_ERR_CAPACITY, "state document allocation failed");
        memcpy(out, bytes.data(), bytes.size());
        *buf = out;
        *len = bytes.size();
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_state_import(sg_engine* e, const void* buf, size_t len) {
    if (!e || !buf) return fail(SG_ERR_INVALID, "null argument");
    if (e->shard) return shd_state_import(e->shard, buf, len);
    SdDoc d;
    try {
        d = sd_read(buf, len);
    } catch (const std::exception& ex) {
        return fail(SG_ERR_INVALID, ex.what());
    }
    try {
        HIP_OK(hipSetDevice(e->device));
        if (e->gen) {
            std::string msg;
            const int rc = gen_state_import(e->gen, d, msg);
            return rc == SG_OK ? rc : fail(rc, msg);
        }
        return twostate_import(e, d);
    } catch (const std::exception& ex) {
        return fail(SG_ERR_DEVICE, ex.what());
    }
}

int sg_jit_check(const void* ir, size_t ir_len, uint32_t variant_flags, char* out, size_t out_len) {
    if (!ir) return fail(SG_ERR_INVALID, "null argument");
    sg_engine* e = nullptr;
    int rc = SG_OK;
    std::string text;
    try {
        e = new sg_engine();
        e->device = -1;
        if (const char* d = getenv("SGD_REG_SLOTS")) e->reg_slots = e->reg_slots_hbm = (uint32_t)strtoul(d, nullptr, 0);
        if (const char* d = getenv("SGD_REG_SLOTS_HBM")) e->reg_slots_hbm = (uint32_t)strtoul(d, nullptr, 0);
        build_plan(e, ir, ir_len);
        JitQuery q = make_jit_query(e);
        q.evnull = (variant_flags & 1u) != 0;
        q.capnull = (variant_flags & 2u) != 0;
        std::vector<uint64_t> consts;
        text = sgj_generate(q, consts);
        std::vector<char> code;
        std::string log;
        if (!sgj_compile(text, code, log)) {
            text = log;
            rc = fail(SG_ERR_DEVICE, "JIT compilation failed: " + log);
        }
    } catch (const std::exception& ex) {
        text = ex.what();
        rc = fail(SG_ERR_UNSUPPORTED, ex.what());
    }
    delete e;
    if (out && out_len) {
        const size_t m = std::min(out_len - 1, text.size());
        memcpy(out, text.data(), m);
        out[m] = 0;
    }
    return rc;
}

}  // extern "C"
