// gen_host.hip — host side of the general NFA engine (gen_engine.h, gen_kernels.hip).
//
// Lowers the IR's state tree into GenProgram the way StateInputStreamParser.parse wires processors
// (util/parser/StateInputStreamParser.java:148-408: Stream :167-225, Next :227-259, Every :261-287,
// Logical :289-378, Count :380-403; then parseInputStream :76-146 for within / start states /
// thisLast), allocates the per-key state in HBM and runs per push:
//   key grouping (stable radix sort of key ids, per-key segments) -> k_gen_batch -> ordering
// and per sg_advance_time: k_gen_timers -> ordering of the timer matches.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_merge_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/siddhi_gpu.h"
#include "../../include/siddhi_gpu_ir.h"
#include "gen_engine.h"
#include "pack.h"
#include "part.h"
#include "gen_host.h"
#include "pinned.h"
#include "state_doc.h"

extern "C" __global__ void k_gen_batch(const GenArgs ap);
#define ABS_DECL(NW) extern "C" __global__ void k_abs_batch_##NW(const GenArgs ap); \
                     extern "C" __global__ void k_abs_batchf_##NW(const GenArgs ap); \
                     extern "C" __global__ void k_abs_timers_##NW(const GenArgs ap);
ABS_DECL(1) ABS_DECL(2) ABS_DECL(3) ABS_DECL(4) ABS_DECL(5) ABS_DECL(6) ABS_DECL(7) ABS_DECL(8)
typedef void (*AbsKernel)(const GenArgs);
static const AbsKernel kAbsBatch[ABS_MAXNW + 1] = {nullptr, k_abs_batch_1, k_abs_batch_2, k_abs_batch_3, k_abs_batch_4,
                                                   k_abs_batch_5, k_abs_batch_6, k_abs_batch_7, k_abs_batch_8};
static const AbsKernel kAbsBatchF[ABS_MAXNW + 1] = {nullptr, k_abs_batchf_1, k_abs_batchf_2, k_abs_batchf_3,
                                                    k_abs_batchf_4, k_abs_batchf_5, k_abs_batchf_6, k_abs_batchf_7,
                                                    k_abs_batchf_8};
#define ABSD_DECL(NW) extern "C" __global__ void k_absd_batch_##NW(const GenArgs ap); \
                      extern "C" __global__ void k_absd_timers_##NW(const GenArgs ap); \
                      extern "C" __global__ void k_absd_batchf_##NW(const GenArgs ap); \
                      extern "C" __global__ void k_absd_timersf_##NW(const GenArgs ap); \
                      extern "C" __global__ void k_absd_flush_##NW(const GenArgs ap);
ABSD_DECL(1) ABSD_DECL(2) ABSD_DECL(3) ABSD_DECL(4) ABSD_DECL(5) ABSD_DECL(6) ABSD_DECL(7) ABSD_DECL(8)
static const AbsKernel kAbsdBatch[ABS_MAXNW + 1] = {nullptr, k_absd_batch_1, k_absd_batch_2, k_absd_batch_3,
                                                    k_absd_batch_4, k_absd_batch_5, k_absd_batch_6, k_absd_batch_7,
                                                    k_absd_batch_8};
static const AbsKernel kAbsdTimers[ABS_MAXNW + 1] = {nullptr, k_absd_timers_1, k_absd_timers_2, k_absd_timers_3,
                                                     k_absd_timers_4, k_absd_timers_5, k_absd_timers_6, k_absd_timers_7,
                                                     k_absd_timers_8};
static const AbsKernel kAbsdBatchF[ABS_MAXNW + 1] = {nullptr, k_absd_batchf_1, k_absd_batchf_2, k_absd_batchf_3,
                                                     k_absd_batchf_4, k_absd_batchf_5, k_absd_batchf_6, k_absd_batchf_7,
                                                     k_absd_batchf_8};
static const AbsKernel kAbsdTimersF[ABS_MAXNW + 1] = {nullptr, k_absd_timersf_1, k_absd_timersf_2, k_absd_timersf_3,
                                                      k_absd_timersf_4, k_absd_timersf_5, k_absd_timersf_6,
                                                      k_absd_timersf_7, k_absd_timersf_8};
static const AbsKernel kAbsdFlush[ABS_MAXNW + 1] = {nullptr, k_absd_flush_1, k_absd_flush_2, k_absd_flush_3,
                                                    k_absd_flush_4, k_absd_flush_5, k_absd_flush_6, k_absd_flush_7,
                                                    k_absd_flush_8};
#define CNT_DECL(NW) extern "C" __global__ void k_cnt_batch_##NW(const GenArgs ap); \
    extern "C" __global__ void k_cnt_flush_##NW(const GenArgs ap);
CNT_DECL(1) CNT_DECL(2) CNT_DECL(3) CNT_DECL(4) CNT_DECL(5) CNT_DECL(6) CNT_DECL(7) CNT_DECL(8)
static const AbsKernel kCntBatch[ABS_MAXNW + 1] = {nullptr, k_cnt_batch_1, k_cnt_batch_2, k_cnt_batch_3, k_cnt_batch_4,
                                                   k_cnt_batch_5, k_cnt_batch_6, k_cnt_batch_7, k_cnt_batch_8};
#define CHN_DECL(NE) extern "C" __global__ void k_chn_batch_##NE##_0(const GenArgs ap); \
    extern "C" __global__ void k_chn_batch_##NE##_1(const GenArgs ap); extern "C" __global__ void k_chn_batch_##NE##_2(const GenArgs ap);
CHN_DECL(1) CHN_DECL(2) CHN_DECL(3)
#define CHNW_DECL(NE) extern "C" __global__ void k_chn_wide_##NE##_0(const GenArgs ap); \
    extern "C" __global__ void k_chn_wide_##NE##_1(const GenArgs ap); extern "C" __global__ void k_chn_wide_##NE##_2(const GenArgs ap);
CHNW_DECL(1) CHNW_DECL(2) CHNW_DECL(3)
// [n - 2][kept words]: the chain kernels (chn_kernels.hip), and their wide-window kernels over the keys handed over
static const AbsKernel kChnBatch[CHN_MAXN - 1][3] = {{k_chn_batch_1_0, k_chn_batch_1_1, k_chn_batch_1_2},
                                                     {k_chn_batch_2_0, k_chn_batch_2_1, k_chn_batch_2_2},
                                                     {k_chn_batch_3_0, k_chn_batch_3_1, k_chn_batch_3_2}};
static const AbsKernel kChnWide[CHN_MAXN - 1][3] = {{k_chn_wide_1_0, k_chn_wide_1_1, k_chn_wide_1_2},
                                                    {k_chn_wide_2_0, k_chn_wide_2_1, k_chn_wide_2_2},
                                                    {k_chn_wide_3_0, k_chn_wide_3_1, k_chn_wide_3_2}};
#define ABSF_DECL(NW) extern "C" __global__ void k_abs_flush_##NW(const GenArgs ap);
ABSF_DECL(1) ABSF_DECL(2) ABSF_DECL(3) ABSF_DECL(4) ABSF_DECL(5) ABSF_DECL(6) ABSF_DECL(7) ABSF_DECL(8)
static const AbsKernel kAbsFlush[ABS_MAXNW + 1] = {nullptr, k_abs_flush_1, k_abs_flush_2, k_abs_flush_3, k_abs_flush_4,
                                                   k_abs_flush_5, k_abs_flush_6, k_abs_flush_7, k_abs_flush_8};
static const AbsKernel kCntFlush[ABS_MAXNW + 1] = {nullptr, k_cnt_flush_1, k_cnt_flush_2, k_cnt_flush_3, k_cnt_flush_4,
                                                   k_cnt_flush_5, k_cnt_flush_6, k_cnt_flush_7, k_cnt_flush_8};
#define ABS4_DECL(NW) extern "C" __global__ void k_abs_batchf4_##NW(const GenArgs ap); \
    extern "C" __global__ void k_abs_timers4_##NW(const GenArgs ap);
ABS4_DECL(1) ABS4_DECL(2) ABS4_DECL(3)
static const AbsKernel kAbsBatchF4[4] = {nullptr, k_abs_batchf4_1, k_abs_batchf4_2, k_abs_batchf4_3};
static const AbsKernel kAbsTimers4[4] = {nullptr, k_abs_timers4_1, k_abs_timers4_2, k_abs_timers4_3};
static const AbsKernel kAbsTimers[ABS_MAXNW + 1] = {nullptr, k_abs_timers_1, k_abs_timers_2, k_abs_timers_3,
                                                    k_abs_timers_4, k_abs_timers_5, k_abs_timers_6, k_abs_timers_7,
                                                    k_abs_timers_8};
extern "C" __global__ void k_gen_timers(const GenArgs ap);
extern "C" __global__ void k_cnt_split(const GenArgs a);
extern "C" __global__ void k_gen_deadlines(const GenArgs ap);
extern "C" __global__ void k_gen_due(const int64_t* nd, uint32_t K, int64_t now, uint32_t* due,
                                     unsigned long long* ndue);
extern "C" __global__ void k_gen_collapse(const unsigned long long* key, const uint32_t* li, uint64_t n,
                                          uint32_t* err);

namespace {

#define GH_OK(x)                                                                                        \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ---------------------------------------------------------------------------------------------
// IR -> GenProgram (mirrors the reference parser's wiring)
// ---------------------------------------------------------------------------------------------
struct RT {  // InnerStateRuntime
    int tag = 0, first = -1, last = -1, a = -1, b = -1, stream = -1;
};

struct Builder {
    GenProgram& G;
    const uint32_t* w;
    size_t n, pos = 0;
    std::vector<RT> rts;
    int64_t forMsCur = -1;

    uint32_t next() {
        if (pos >= n) throw std::runtime_error("truncated IR node tree");
        return w[pos++];
    }
    int newPre(int kind) {
        if (G.nprocs >= GEN_MAXP) throw std::runtime_error("too many states for the device engine");
        const int id = G.nprocs++;
        GenPre& P = G.pre[id];
        P = GenPre{};
        P.kind = kind;
        P.withinEvery = P.thisPost = P.thisLast = P.countPost = P.partner = GEN_NONE;
        P.waiting = -1;
        GenPost& Q = G.post[id];
        Q = GenPost{};
        Q.kind = kind;
        Q.nextStatePre = Q.nextEveryStatePre = Q.callbackPre = Q.partnerPre = Q.partnerPost = Q.thisPre = GEN_NONE;
        return id;  // pre and post share the index
    }
    int newRT(int tag) {
        rts.push_back(RT{});
        rts.back().tag = tag;
        return (int)rts.size() - 1;
    }
    bool peekAbsent(size_t q) const { return q + 5 < n && w[q] == SG_N_STREAM && w[q + 5] != 0; }
    void skip() {
        const uint32_t tag = next();
        switch (tag) {
        case SG_N_STREAM: pos += 7; return;
        case SG_N_NEXT: skip(); skip(); return;
        case SG_N_EVERY: skip(); return;
        case SG_N_LOGICAL: next(); skip(); skip(); return;
        case SG_N_COUNT: next(); next(); skip(); return;
        }
        throw std::runtime_error("bad IR node tag");
    }
    void setNextStatePre(int post, int pre) {  // StreamPost/LogicalPost/CountPost.setNextStatePreProcessor
        GenPost& Q = G.post[post];
        Q.nextStatePre = pre;
        if (Q.kind == GK_LOGICAL) G.post[Q.partnerPost].nextStatePre = pre;  // LogicalPostStateProcessor.java:117-120
        if (Q.kind == GK_COUNT && G.pre[Q.thisPre].isStart && G.qtype == SG_Q_SEQUENCE && Q.minCount == 0)
            G.post[G.pre[pre].thisPost].callbackPre = Q.thisPre;  // CountPostStateProcessor.java:82-88
    }
    void setNextEveryStatePre(int post, int pre) {
        GenPost& Q = G.post[post];
        Q.nextEveryStatePre = pre;
        if (Q.kind == GK_LOGICAL) G.post[Q.partnerPost].nextEveryStatePre = pre;
    }

    int parse(int pre, std::vector<int>& preList, bool isStart) {
        const uint32_t tag = next();
        switch (tag) {
        case SG_N_STREAM: {
            const uint32_t slot = next(), stream = next(), fpc = next(), flen = next(), absent = next();
            const uint32_t flo = next(), fhi = next();
            const int64_t forMs = (int64_t)((uint64_t)flo | ((uint64_t)fhi << 32));
            if (pre < 0) {
                pre = newPre(GK_STREAM);
                if (absent) {
                    if (forMs < 0) throw std::runtime_error("absent stream state needs a 'for' time");
                    G.startup[G.nStartup++] = pre;
                }
            }
            if (slot >= GEN_MAXSLOT || stream >= GEN_MAXS) throw std::runtime_error("IR slot or stream index out of range");
            G.slotStream[slot] = (int)stream;  // the stream of the events this slot holds (their attribute types)
            GenPre& P = G.pre[pre];
            P.absent = absent != 0;
            P.waiting = absent ? forMs : -1;
            P.stateId = (int)slot;
            P.isStart = isStart;
            P.fpc = fpc;
            P.flen = flen;
            GenPost& Q = G.post[pre];
            Q.absent = absent != 0;
            Q.stateId = (int)slot;
            Q.thisPre = pre;
            P.thisPost = pre;
            P.thisLast = pre;
            const int rt = newRT(SG_N_STREAM);
            rts[rt].first = pre;
            rts[rt].last = pre;
            rts[rt].stream = (int)stream;
            preList.push_back(pre);
            return rt;
        }
        case SG_N_NEXT: {
            const int cur = parse(pre, preList, isStart);
            const int nx = parse(pre, preList, false);
            setNextStatePre(rts[cur].last, rts[nx].first);
            const int rt = newRT(SG_N_NEXT);
            rts[rt].a = cur;
            rts[rt].b = nx;
            rts[rt].first = rts[cur].first;
            rts[rt].last = rts[nx].last;
            return rt;
        }
        case SG_N_EVERY: {
            std::vector<int> withinEvery;
            const int inner = parse(pre, withinEvery, isStart);
            const int rt = newRT(SG_N_EVERY);
            rts[rt].a = inner;
            rts[rt].first = rts[inner].first;
            rts[rt].last = rts[inner].last;
            setNextEveryStatePre(rts[rt].last, rts[rt].first);
            for (int p : withinEvery) G.pre[p].withinEvery = rts[rt].first;
            preList.insert(preList.end(), withinEvery.begin(), withinEvery.end());
            return rt;
        }
        case SG_N_LOGICAL: {
            const uint32_t ltype = next();
            const int lp1 = newPre(GK_LOGICAL), lp2 = newPre(GK_LOGICAL);
            for (int x : {lp1, lp2}) {
                G.pre[x].logicalType = (int)ltype;
                G.post[x].logicalType = (int)ltype;
            }
            G.post[lp1].partnerPre = lp2;
            G.post[lp2].partnerPre = lp1;
            G.post[lp1].partnerPost = lp2;
            G.post[lp2].partnerPost = lp1;
            G.pre[lp1].partner = lp2;
            G.pre[lp2].partner = lp1;
            {  // absent logical pres join the startup list at creation, element 1 first
                const size_t save = pos;
                const bool a1 = peekAbsent(pos);
                skip();
                const bool a2 = peekAbsent(pos);
                pos = save;
                if (a1) G.startup[G.nStartup++] = lp1;
                if (a2) G.startup[G.nStartup++] = lp2;
            }
            const size_t save = pos;
            skip();  // element 1 is encoded first, element 2 is parsed (and slotted) first
            const int rt2 = parse(lp2, preList, isStart);
            const size_t after = pos;
            pos = save;
            const int rt1 = parse(lp1, preList, isStart);
            pos = after;
            const int rt = newRT(SG_N_LOGICAL);
            rts[rt].a = rt1;
            rts[rt].b = rt2;
            rts[rt].first = rts[rt1].first;
            rts[rt].last = rts[rt2].last;
            return rt;
        }
        case SG_N_COUNT: {
            const uint32_t mn = next(), mx = next();
            const int cp = newPre(GK_COUNT);
            GenPre& P = G.pre[cp];
            P.minCount = (int)mn;
            P.maxCount = mx == SG_COUNT_ANY ? 0x7fffffff : (int)mx;
            G.post[cp].minCount = P.minCount;
            G.post[cp].maxCount = P.maxCount;
            P.countPost = cp;
            const int inner = parse(cp, preList, isStart);
            const int rt = newRT(SG_N_COUNT);
            rts[rt].first = rts[inner].first;
            rts[rt].last = rts[inner].last;
            rts[rt].stream = rts[inner].stream;
            return rt;
        }
        }
        throw std::runtime_error("bad IR node tag");
    }

    // InnerStateRuntime init / reset / update / setQuerySelector / setup, flattened
    void initOrder(int rt) {
        const RT& r = rts[rt];
        switch (r.tag) {
        case SG_N_NEXT: initOrder(r.a); initOrder(r.b); return;
        case SG_N_EVERY: initOrder(r.a); return;
        case SG_N_LOGICAL: initOrder(r.b); initOrder(r.a); return;
        default: G.initOrder[G.nInit++] = r.first;
        }
    }
    void resetOrder(int rt) {
        const RT& r = rts[rt];
        switch (r.tag) {
        case SG_N_NEXT: resetOrder(r.b); resetOrder(r.a); return;
        case SG_N_LOGICAL: resetOrder(r.b); return;
        default: G.resetOrder[G.nReset++] = r.first;  // Stream, Count and Every reset their first
        }
    }
    void updateOrder(int rt) {
        const RT& r = rts[rt];
        switch (r.tag) {
        case SG_N_NEXT: updateOrder(r.a); updateOrder(r.b); return;
        case SG_N_LOGICAL: updateOrder(r.b); return;
        default: G.updateOrder[G.nUpdate++] = r.first;
        }
    }
    void setQuerySelector(int rt) {
        const RT& r = rts[rt];
        switch (r.tag) {
        case SG_N_NEXT: setQuerySelector(r.b); return;
        case SG_N_EVERY: setQuerySelector(r.a); return;
        case SG_N_LOGICAL: setQuerySelector(r.b); setQuerySelector(r.a); return;
        default: G.post[r.last].hasNext = 1;
        }
    }
    void setup(int rt) {
        const RT& r = rts[rt];
        switch (r.tag) {
        case SG_N_NEXT: setup(r.a); setup(r.b); return;
        case SG_N_EVERY: setup(r.a); return;
        case SG_N_LOGICAL: setup(r.b); setup(r.a); return;
        default: {
            if (r.stream < 0 || r.stream >= G.nstreams) throw std::runtime_error("IR stream index out of range");
            GenRecv& R = G.recv[r.stream];
            if (R.n >= GEN_MAXP) throw std::runtime_error("too many states on one stream");
            R.procs[R.n++] = r.first;
            R.stateProcs[R.nStateProcs++] = r.first;
        }
        }
    }
};

uint32_t ceil32(uint32_t x) { return (x + 31) / 32; }

// deepest stack a filter program reaches; -1 when it uses ifThenElse (abs_kernels.hip evaluates programs
// at most two deep without a stack array)
int prog_depth(const uint32_t* code, uint32_t pc, uint32_t n) {
    int sp = 0, mx = 0;
    for (uint32_t end = pc + n; pc < end;) {
        const uint32_t op = code[pc] & 0xffu;
        switch (op) {
        case SG_OP_VAR: case SG_OP_CONST: case SG_OP_ISNULL_EV: sp++; break;
        case SG_OP_CVT: case SG_OP_NOT: case SG_OP_ISNULL: break;
        case SG_OP_IFELSE: return -1;
        default: sp--;
        }
        mx = std::max(mx, sp);
        pc += (uint32_t)sg_op_len(op);
    }
    return mx;
}

// a filter the register-window kernels evaluate without a stack (jo_eval<false>)
bool shallow(const GenProgram& G, const GenPre& P) {
    const int d = prog_depth(G.code, P.fpc, P.flen);
    return d >= 0 && d <= 2;
}

// the register-window kernels' word layout of stream 0's event (absOff / absNW: long and double take two words)
bool reg_layout(GenProgram& G) {
    uint32_t o = 0;
    for (int a = 0; a < G.nattr[0]; a++) {
        G.absOff[a] = o;
        const bool wide = G.attrType[0][a] == SG_T_LONG || G.attrType[0][a] == SG_T_DOUBLE;
        if (o < ABS_MAXNW) G.absWordAt[o] = SE_ATTR + 2 * (uint32_t)a;
        if (wide && o + 1 < ABS_MAXNW) G.absWordAt[o + 1] = SE_ATTR + 2 * (uint32_t)a + 1;
        o += wide ? 2u : 1u;
    }
    if (o == 0 || o > ABS_MAXNW) return false;
    G.absNW = o;
    return true;
}

// the counting sequence shape of cnt_kernels.hip:
//     every e1=S[f0]<m:n>, e2=S[fA] or e3=S[fB] [within W]      (SEQUENCE, partitioned, one stream)
// with the processors wired as StateInputStreamParser wires that query (a count state inside `every`, its
// post processor feeding a logical OR pair whose post processors reach the selector); 1 <= m, n <= CNT_R.
// Anything else stays on the general kernels.
void cnt_shape(GenProgram& G) {
    G.cntOk = 0;
    G.cntAnd = 0;
    if (G.qtype != SG_Q_SEQUENCE || !G.partitioned || G.nstreams != 1 || G.nprocs != 3 || G.nslots != 3 ||
        G.nStartup != 0)
        return;
    const GenRecv& R = G.recv[0];
    if (R.n != 3 || R.nStateProcs != 3) return;
    const int p0 = R.procs[0], pA = R.procs[2], pB = R.procs[1];  // an event visits procs[2], [1], [0]
    const GenPre &P0 = G.pre[p0], &PA = G.pre[pA], &PB = G.pre[pB];
    const GenPost &Q0 = G.post[p0], &QA = G.post[pA], &QB = G.post[pB];
    if (P0.kind != GK_COUNT || P0.absent || !P0.isStart || P0.minCount < 1 || P0.maxCount > CNT_R ||
        P0.minCount > P0.maxCount || P0.countPost != p0)
        return;
    if (PA.kind != GK_LOGICAL || PB.kind != GK_LOGICAL || PA.absent || PB.absent || PA.isStart || PB.isStart ||
        PA.logicalType != PB.logicalType || (PA.logicalType != SG_L_OR && PA.logicalType != SG_L_AND) ||
        PA.partner != pB || PB.partner != pA)
        return;
    if (Q0.nextStatePre != pA && Q0.nextStatePre != pB) return;
    if (Q0.nextEveryStatePre != p0 || Q0.callbackPre != GEN_NONE || Q0.hasNext) return;
    for (const GenPost* Q : {&QA, &QB})
        if (Q->nextStatePre != GEN_NONE || Q->nextEveryStatePre != GEN_NONE || Q->callbackPre != GEN_NONE || !Q->hasNext)
            return;
    if (PA.withinEvery != GEN_NONE || PB.withinEvery != GEN_NONE || (P0.withinEvery != GEN_NONE && P0.withinEvery != p0))
        return;
    // expiry visits p0 first (its expired partial is the one withinEvery clones)
    if (G.nAll != 3 || G.allProcs[0] != p0) return;
    if (G.within != -1 && (G.nStartIds != 1 || G.startIds[0] != P0.stateId)) return;
    if (G.slotStream[P0.stateId] != 0 || G.slotStream[PA.stateId] != 0 || G.slotStream[PB.stateId] != 0) return;
    if (P0.stateId == PA.stateId || P0.stateId == PB.stateId || PA.stateId == PB.stateId) return;
    // CountPreStateProcessor drops a partial once slot stateId + 1 or + 2 is filled (:97-103): the logical
    // pair's slots
    const int s1 = P0.stateId + 1, s2 = P0.stateId + 2;
    if (!((PA.stateId == s1 && PB.stateId == s2) || (PA.stateId == s2 && PB.stateId == s1))) return;
    if ((uint32_t)P0.maxCount > G.MC) return;
    if (!shallow(G, P0) || !shallow(G, PA) || !shallow(G, PB) || !reg_layout(G)) return;
    G.cntP0 = p0;
    G.cntPA = pA;
    G.cntPB = pB;
    G.cntWE = P0.withinEvery == p0 ? 1 : 0;
    G.cntAnd = PA.logicalType == SG_L_AND ? 1 : 0;
    G.cntOk = getenv("SG_NO_CNT") ? 0 : 1;  // (SG_NO_CNT: A/B timing against the general kernels; same results)
}

// the chained stream-state shape of chn_kernels.hip:
//     [every] e1=S[f0] -> e2=S[f1] -> ... -> en=S[f(n-1)] [within W]      (PATTERN, partitioned, one stream, 2 <= n <= 4)
// with the processors wired as StateInputStreamParser wires that query (each state's post processor feeding the next
// state's addState, the last one's reaching the selector; `every` only around e1), no timers, single-event slots.
// The attribute words the filters read of earlier events are kept in the kernel's window (at most two words).
// Anything else stays on the general kernels.
void chn_shape(GenProgram& G) {
    G.chnOk = 0;
    G.chnWide = 0;
    const int n = G.nprocs;
    if (G.qtype != SG_Q_PATTERN || !G.partitioned || G.nstreams != 1 || n < 2 || n > CHN_MAXN || G.nslots != n ||
        G.nStartup != 0 || G.MC != 1 || G.nAll != n)
        return;
    const GenRecv& R = G.recv[0];
    if (R.n != n || R.nStateProcs != n || !R.multi) return;
    for (int i = 0; i < n; i++) {
        const int p = R.procs[i];
        if (p < 0 || p >= n) return;
        const GenPre& P = G.pre[p];
        const GenPost& Q = G.post[p];
        // (p0's withinEvery is p0 itself under `every ... within`: it clones an EXPIRED entry of p0's own lists, which
        // hold only blank seeds, never expired — StreamPreStateProcessor.java:118-129 reads the start event)
        if (P.kind != GK_STREAM || P.absent || P.isStart != (i == 0) ||
            !(P.withinEvery == GEN_NONE || (i == 0 && P.withinEvery == p)))
            return;
        if (Q.callbackPre != GEN_NONE || P.thisPost != p) return;
        if (i + 1 < n) {
            if (Q.nextStatePre != R.procs[i + 1] || Q.hasNext) return;
        } else if (Q.nextStatePre != GEN_NONE || !Q.hasNext) {
            return;
        }
        if (Q.nextEveryStatePre != GEN_NONE && !(i == 0 && Q.nextEveryStatePre == p)) return;
        if (P.stateId < 0 || P.stateId >= n || G.slotStream[P.stateId] != 0) return;
        for (int j = 0; j < i; j++)
            if (G.pre[R.procs[j]].stateId == P.stateId) return;
        if (!shallow(G, P)) return;
        G.chnP[i] = p;
    }
    if (G.within != -1 && (G.nStartIds != 1 || G.startIds[0] != G.pre[G.chnP[0]].stateId)) return;
    // (every attribute word of the event in the kernel's registers: its filters read them there, and a captured event
    // is written to its pool entry from them)
    if (!reg_layout(G) || G.absNW > CHN_MAXNW) return;
    const int R_ = CHN_R(n);
    // (the window's lists, StateEvents 0 .. R and its events below min(64, SECAP) fit the block; 16-bit pool entries)
    if (G.L < (uint32_t)R_ || G.STCAP < (uint32_t)R_ + 1u || (uint32_t)(R_ * (n - 1)) > std::min<uint32_t>(64u, G.SECAP) ||
        G.SECAP >= 0xffffu)
        return;
    for (int s = 0; s < GEN_MAXSLOT; s++) G.chnSlotEv[s] = -1;
    for (int i = 0; i < n; i++) G.chnSlotEv[G.pre[G.chnP[i]].stateId] = i;
    // the attributes the filters read of an earlier state's event
    uint32_t want = 0;
    for (int t = 0; t < n; t++) {
        const GenPre& P = G.pre[G.chnP[t]];
        for (uint32_t pc = P.fpc, end = P.fpc + P.flen; pc < end;) {
            const uint32_t w = G.code[pc], op = w & 0xffu, b = (w >> 16) & 0xffu;
            if (op == SG_OP_VAR && (int)b != P.stateId) {
                const uint32_t a = G.code[pc + 1];
                if (a >= (uint32_t)G.nattr[0]) return;
                want |= 1u << a;
            }
            pc += (uint32_t)sg_op_len(op);
        }
    }
    int kw = 0;
    for (int a = 0; a < GEN_MAXA; a++) G.chnAttrK[a] = -1;
    for (int a = 0; a < G.nattr[0]; a++) {
        if (!((want >> a) & 1u)) continue;
        const bool wide = G.attrType[0][a] == SG_T_LONG || G.attrType[0][a] == SG_T_DOUBLE;
        if (kw + (wide ? 2 : 1) > 2) return;
        G.chnAttrK[a] = kw;
        for (int h = 0; h < (wide ? 2 : 1); h++) {
            G.chnKeepW[kw] = G.absOff[a] + (uint32_t)h;
            G.chnKeepA[kw] = (uint32_t)a;
            kw++;
        }
    }
    G.chnKW = kw;
    G.chnN = n;
    const int RW = CHN_RW(n);
    G.chnWide = !getenv("SG_NO_CHN_WIDE") && G.L >= (uint32_t)RW && G.STCAP >= (uint32_t)RW + 1u &&
                (uint32_t)(RW * (n - 1)) <= std::min<uint32_t>(64u, G.SECAP);
    G.chnEvery = G.post[G.chnP[0]].nextEveryStatePre == G.chnP[0] ? 1 : 0;
    G.chnOk = getenv("SG_NO_CHN") ? 0 : 1;  // (SG_NO_CHN: A/B timing against the general kernels; same results)
}

// the absent-tail shape of abs_kernels.hip: `[every] e1=S[f0] -> not S[f1] for T [within W]` with the
// processors wired exactly as the kernels restate them (anything else stays on the general kernels)
// A filter program `operand [CVT] operand [CVT] CMP` (include/siddhi_gpu_ir.h encodings) as a JoFast, each
// operand an attribute or a constant ending in the compare domain; constants widened here as java_ops.h
// jo_cvt would widen them (JLS 5.1.2, round to nearest).  Any other program: on = 0 (the interpreter runs it).
static uint64_t jo_host_cvt(uint64_t b, uint32_t from, uint32_t to) {
    auto f32 = [](float f) { uint32_t u; memcpy(&u, &f, 4); return (uint64_t)u; };
    auto f64 = [](double d) { uint64_t u; memcpy(&u, &d, 8); return u; };
    if (from == to) return b;
    if (from == SG_T_INT) {
        const int32_t x = (int32_t)(uint32_t)b;
        if (to == SG_T_LONG) return (uint64_t)(int64_t)x;
        if (to == SG_T_FLOAT) return f32((float)x);
        if (to == SG_T_DOUBLE) return f64((double)x);
    } else if (from == SG_T_LONG) {
        const int64_t x = (int64_t)b;
        if (to == SG_T_FLOAT) return f32((float)x);
        if (to == SG_T_DOUBLE) return f64((double)x);
    } else if (from == SG_T_FLOAT && to == SG_T_DOUBLE) {
        float f;
        const uint32_t u = (uint32_t)b;
        memcpy(&f, &u, 4);
        return f64((double)f);
    }
    return b;
}
JoFast jo_fast_decode(const uint32_t* code, uint32_t pc, uint32_t n) {
    JoFast f{};
    if (n == 0) return f;
    const uint32_t end = pc + n;
    uint32_t fin[2] = {0, 0};
    for (int i = 0; i < 2; ++i) {
        if (pc + 3 > end) return JoFast{};
        const uint32_t w = code[pc], op = w & 0xffu, a = (w >> 8) & 0xffu, b = (w >> 16) & 0xffu;
        if (op == SG_OP_VAR) {
            f.isConst[i] = 0;
            f.from[i] = a;
            f.slot[i] = b;
            f.attr[i] = code[pc + 1];
            f.chain[i] = (int32_t)code[pc + 2];
        } else if (op == SG_OP_CONST) {
            f.isConst[i] = 1;
            f.from[i] = a;
            f.cbits[i] = (uint64_t)code[pc + 1] | ((uint64_t)code[pc + 2] << 32);
            f.cnull[i] = b != 0u;
        } else {
            return JoFast{};
        }
        pc += 3;
        fin[i] = f.from[i];
        if (pc < end && (code[pc] & 0xffu) == SG_OP_CVT) {
            if (((code[pc] >> 8) & 0xffu) != fin[i]) return JoFast{};
            fin[i] = (code[pc] >> 16) & 0xffu;
            pc += 1;
        }
    }
    if (pc + 1 != end) return JoFast{};
    const uint32_t op = code[pc] & 0xffu, dom = (code[pc] >> 8) & 0xffu;
    if (op < SG_OP_EQ || op > SG_OP_LE || fin[0] != dom || fin[1] != dom) return JoFast{};
    f.op = op;
    f.dom = dom;
    for (int i = 0; i < 2; ++i)
        if (f.isConst[i] && !f.cnull[i]) f.cbits[i] = jo_host_cvt(f.cbits[i], f.from[i], dom);
    f.on = 1;
    return f;
}

void abs_shape(GenProgram& G) {
    G.absOk = 0;
    if (G.qtype != SG_Q_PATTERN || !G.partitioned || !G.playback || G.nstreams != 1 || G.nprocs != 2 || G.nslots != 2)
        return;
    const GenPre &P0 = G.pre[0], &P1 = G.pre[1];
    const GenPost &Q0 = G.post[0], &Q1 = G.post[1];
    if (P0.kind != GK_STREAM || P0.absent || !P0.isStart || P1.kind != GK_STREAM || !P1.absent || P1.isStart) return;
    if (P1.waiting < 0 || P1.withinEvery != GEN_NONE || (P0.withinEvery != GEN_NONE && P0.withinEvery != 0)) return;
    if (Q0.nextStatePre != 1 || (Q0.nextEveryStatePre != GEN_NONE && Q0.nextEveryStatePre != 0) ||
        Q0.callbackPre != GEN_NONE || Q0.hasNext)
        return;
    if (Q1.nextStatePre != GEN_NONE || Q1.nextEveryStatePre != GEN_NONE || Q1.callbackPre != GEN_NONE || !Q1.hasNext)
        return;
    const GenRecv& R = G.recv[0];
    if (R.n != 2 || R.procs[0] != 0 || R.procs[1] != 1 || R.nStateProcs != 2 || R.stateProcs[0] != 0 ||
        R.stateProcs[1] != 1)
        return;
    if (G.nStartup != 1 || G.startup[0] != 1 || G.MC != 1 || P0.stateId == P1.stateId) return;
    if (G.slotStream[P0.stateId] != 0 || G.slotStream[P1.stateId] != 0) return;
    if (!shallow(G, P0) || !shallow(G, P1) || !reg_layout(G)) return;
    G.absP0 = 0;
    G.absP1 = 1;
    G.absEvery = Q0.nextEveryStatePre == 0 ? 1 : 0;
    G.absListener = 0;
    G.absOk = getenv("SG_NO_ABS") ? 0 : 1;  // (SG_NO_ABS: A/B timing against the general kernels; same results)
}

}  // namespace

GenProgram* gen_build_program(const uint32_t* w, size_t nw, uint32_t partialCap) {
    auto* G = new GenProgram();
    memset(G, 0, sizeof(*G));
    try {
        G->qtype = (int)w[2];
        G->nstreams = (int)w[3];
        G->nslots = (int)w[4];
        G->within = (int64_t)((uint64_t)w[5] | ((uint64_t)w[6] << 32));
        const uint32_t offS = w[7], offN = w[8], nN = w[9], offC = w[10], nC = w[11];
        G->partitioned = (w[12] & SG_IR_F_PARTITIONED) != 0;
        G->playback = (w[12] & SG_IR_F_PLAYBACK) != 0;
        if (G->nstreams > GEN_MAXS || G->nslots > GEN_MAXSLOT) throw std::runtime_error("query too large for the device engine");
        if (nC > GEN_MAXCODE) throw std::runtime_error("filters too long for the device engine");
        if (offN + nN > nw || offC + nC > nw) throw std::runtime_error("IR offsets out of range");
        size_t p = offS;
        uint32_t maxAttr = 1;
        for (int s = 0; s < G->nstreams; s++) {
            const uint32_t na = w[p++];
            if (na > GEN_MAXA) throw std::runtime_error("stream has too many attributes for the device engine");
            G->nattr[s] = (int)na;
            for (uint32_t a = 0; a < na; a++) G->attrType[s][a] = (int)w[p++];
            maxAttr = std::max(maxAttr, na);
        }
        G->ncode = nC;
        memcpy(G->code, w + offC, nC * 4);
        Builder B{*G, w + offN, nN};
        std::vector<int> preList;
        const int root = B.parse(-1, preList, true);
        if (B.pos != nN) throw std::runtime_error("IR node tree has trailing words");
        G->nAll = (int)preList.size();
        for (size_t i = 0; i < preList.size(); i++) G->allProcs[i] = preList[i];
        B.setQuerySelector(root);
        B.setup(root);
        B.initOrder(root);
        B.resetOrder(root);
        B.updateOrder(root);
        if (G->within != -1)
            for (int x : preList)
                if (G->pre[x].isStart) G->startIds[G->nStartIds++] = G->pre[x].stateId;
        G->rootFirst = B.rts[root].first;
        G->rootLast = B.rts[root].last;
        G->pre[G->rootFirst].thisLast = G->rootLast;
        for (int s = 0; s < G->nstreams; s++) G->recv[s].multi = G->recv[s].n > 1;
        // capacities and the per-key block layout
        uint32_t mc = 1;
        for (int x = 0; x < G->nprocs; x++)
            if (G->pre[x].kind == GK_COUNT) mc = std::max<uint32_t>(mc, G->pre[x].maxCount >= 0x7fffffff ? 48u : (uint32_t)G->pre[x].maxCount);
        for (int x = 0; x < G->nprocs; x++)
            if (G->pre[x].absent && G->pre[x].kind == GK_LOGICAL) mc = std::max<uint32_t>(mc, 2u);
        G->MC = std::min<uint32_t>(mc, 64u);  // output chain capacity (longer chains fail loudly)
        G->L = std::max<uint32_t>(4, partialCap);
        G->Q = 4 * G->L + 16;  // timer queues: one entry per notifyAt until it falls due
        G->STCAP = std::min<uint32_t>(2 * G->L + 16, 0xfff0u);
        G->SECAP = std::min<uint32_t>(G->STCAP * std::min<uint32_t>((uint32_t)G->nslots * mc, 8u), 0xfff0u);
        G->NA = maxAttr;
        G->DEF = G->L;
        G->ksWords = KS_LISTS + 2 * G->L + 2 * G->Q;
        G->stWords = ST_SLOTS + (uint32_t)G->nslots;
        G->seWords = SE_ATTR + 2 * G->NA;
        uint32_t off = 2;  // [0] key initialised, [1] scheduler order counter
        G->offKS = off;
        off += (uint32_t)G->nprocs * G->ksWords;
        G->offST = off;
        off += G->STCAP * G->stWords;
        G->offSTfree = off;
        off += ceil32(G->STCAP);
        G->offSE = off;
        off += G->SECAP * G->seWords;
        G->offSEfree = off;
        off += ceil32(G->SECAP);
        G->offDef = off;
        off += 1 + 2 * G->DEF;
        G->blockWords = (off + (1u << GEN_GRAN_LOG2) - 1u) & ~((1u << GEN_GRAN_LOG2) - 1u);  // whole granules
        for (int x = 0; x < G->nprocs; x++) G->pre[x].ff = jo_fast_decode(G->code, G->pre[x].fpc, G->pre[x].flen);
        abs_shape(*G);
        cnt_shape(*G);
        chn_shape(*G);
        return G;
    } catch (...) {
        delete G;
        throw;
    }
}

struct OutBufs {
    uint64_t* trig;
    uint64_t* slot;
    uint32_t* key;
    int64_t* ts;
    uint32_t* len;
    unsigned long long* count;
    uint64_t cap;
    uint32_t nslots, MC, recWords;
    uint32_t* err;
    uint64_t* pval;   // projection [projN][cap] value bits, [projN][cap] null flags
    uint8_t* pnull;
    uint32_t projN, projOff;
};

__device__ void write_out(const OutBufs& o, uint64_t d, const uint32_t* rec, bool timer) {
    if (d >= o.cap) { atomicOr(o.err, (uint32_t)GERR_MATCHCAP); return; }
    o.trig[d] = timer ? SG_TIMER_SEQ : ((uint64_t)rec[2] | ((uint64_t)rec[3] << 32));
    o.ts[d] = (int64_t)((uint64_t)rec[4] | ((uint64_t)rec[5] << 32));
    o.key[d] = rec[6];
    const uint32_t* lens = rec + 7;
    const uint32_t* seqs = lens + o.nslots;
    const bool packed = (rec[1] & GEN_REC_PACKED) != 0u;
    uint32_t at = 0;   // (packed: the slot's first entry)
    for (uint32_t s = 0; s < o.nslots; s++) {
        const uint32_t n = lens[s];
        o.len[d * o.nslots + s] = n;
        const uint32_t b = packed ? at : s * o.MC;
        for (uint32_t c = 0; c < o.MC; c++) {
            const uint64_t q = c < n ? ((uint64_t)seqs[2 * (b + c)] | ((uint64_t)seqs[2 * (b + c) + 1] << 32)) : SG_NULL_SEQ;
            o.slot[(d * o.nslots + s) * o.MC + c] = q;
        }
        at += n;
    }
    for (uint32_t i = 0; i < o.projN; i++) {  // the select list projected at emission (Lane::project)
        const uint32_t* pv = rec + o.projOff + 3 * i;
        o.pval[(size_t)i * o.cap + d] = (uint64_t)pv[0] | ((uint64_t)pv[1] << 32);
        o.pnull[(size_t)i * o.cap + d] = (uint8_t)pv[2];
    }
}

// batch matches: out_count + t_off[trigger] + rank (a grid-stride loop over the reserved raw slots); with
// `only_if` (the GEN_M_TFIRST ordering's t_multi flag) the launch does nothing unless the flag is set
__global__ void k_gen_scatter(const uint32_t* raw, const unsigned long long* raw_count, uint64_t seg_cap,
                              uint32_t nseg, const uint32_t* t_off, OutBufs o, const uint32_t* only_if,
                              const unsigned long long* obase) {
    if (only_if && *only_if == 0u) return;
    const unsigned long long base = *obase;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < seg_cap * nseg;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t sg = r / seg_cap;  // reservation segment (GenOut)
        const uint64_t n = raw_count[sg] < seg_cap ? raw_count[sg] : seg_cap;
        if (r - sg * seg_cap >= n) continue;
        const uint32_t* rec = raw + r * o.recWords;
        if (rec[0] >= 0xfffffffeu) continue;
        write_out(o, base + t_off[rec[0]] + (rec[1] & ~GEN_REC_PACKED), rec, false);
    }
}

// The batch ordering: output record of the r-th match of batch event t = the batch's base (the running count
// before the batch) + the exclusive prefix of the per-event counts + r, i.e. ascending trigger seq, then emission
// order (MultiProcessStreamReceiver.java:119-121).  Tiles of GEN_OT = 256 events: k_gen_tsum (tile totals),
// k_gen_tscan (one workgroup: the tiles' offsets, the batch's base, the running count moved past the batch),
// k_gen_order (a tile per workgroup: its events' offsets; the one-match-per-trigger gather; the counts reset for
// the next batch — only the nonzero ones are written), k_gen_scatter for the records the gather does not take.
#define GEN_OT 256u
#define GEN_OST 16u   // tiles per super tile (one k_gen_tsum workgroup): k_gen_tscan scans the super tiles
__global__ void __launch_bounds__(1024) k_gen_tsum(const uint32_t* __restrict__ t_cnt, uint32_t n,
                                                   uint32_t* __restrict__ tile_pre, uint32_t* __restrict__ sup_sum) {
    // a wave per tile (4 consecutive counts per lane), a workgroup per super tile: each tile's prefix inside its
    // super tile, the super tile's total
    __shared__ uint32_t ts[GEN_OST];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t tile = blockIdx.x * GEN_OST + w;
    const uint32_t i0 = tile * GEN_OT + lane * 4u;
    uint32_t c = 0;
    if (i0 + 3u < n) {
        const uint4 v = *reinterpret_cast<const uint4*>(t_cnt + i0);
        c = v.x + v.y + v.z + v.w;
    } else {
        for (uint32_t q = 0; q < 4u; ++q) c += i0 + q < n ? t_cnt[i0 + q] : 0u;
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if (lane == 0) ts[w] = c;
    __syncthreads();
    if (threadIdx.x < GEN_OST) {
        uint32_t pre = 0, all = 0;
        for (uint32_t q = 0; q < GEN_OST; ++q) {
            pre += q < threadIdx.x ? ts[q] : 0u;
            all += ts[q];
        }
        if ((blockIdx.x * GEN_OST + threadIdx.x) * GEN_OT < n) tile_pre[blockIdx.x * GEN_OST + threadIdx.x] = pre;
        if (threadIdx.x == 0) sup_sum[blockIdx.x] = all;
    }
}

// one workgroup of 1024 threads: sup_off = exclusive scan of the super tiles' totals; *obase = the running count;
// the count moves past the batch (every later launch of this batch reads *obase, never the count)
__global__ void __launch_bounds__(1024) k_gen_tscan(const uint32_t* __restrict__ sup_sum, uint32_t ns,
                                                    uint32_t* __restrict__ sup_off, unsigned long long* count,
                                                    unsigned long long* obase) {
    __shared__ uint32_t ws[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    constexpr uint32_t PER = 8;   // (<= 8192 super tiles: batches up to 2^25 events; checked on the host)
    uint32_t v[PER], s = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t j = tid * PER + q;
        v[q] = j < ns ? sup_sum[j] : 0u;
        s += v[q];
    }
    uint32_t incl = s;
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    uint32_t pre = 0, all = 0;
    for (uint32_t q = 0; q < 16; ++q) {
        pre += q < w ? ws[q] : 0u;
        all += ws[q];
    }
    uint32_t x = pre + incl - s;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t j = tid * PER + q;
        if (j < ns) sup_off[j] = x;
        x += v[q];
    }
    if (tid == 0) {
        const unsigned long long b = *count;
        *obase = b;
        *count = b + all;
    }
}

// a tile of 256 events per workgroup.  GATHER (GEN_M_TFIRST, no trigger with several matches): each wave's matches
// are consecutive output records (its counts are 0 / 1), so the slot chains ([n][n_slots][max_chain] u64: 192 B per
// match at C3_min1) and chain lengths are written by the whole wave over its contiguous output range — lane j stores
// element j, j + 64, ... of the range, reading the record word it needs (records found through an LDS table) —
// instead of one lane storing its match's 192 B with 64 lanes' stores 192 B apart.  Otherwise each event's offset
// goes to t_off for k_gen_scatter.
template <bool GATHER>
__global__ void __launch_bounds__(256) k_gen_order(const uint32_t* __restrict__ raw, uint32_t* __restrict__ t_cnt,
                                                   uint32_t* __restrict__ t_off, const uint32_t* __restrict__ t_first,
                                                   const uint32_t* __restrict__ tile_pre,
                                                   const uint32_t* __restrict__ sup_off, uint32_t n, OutBufs o,
                                                   const uint32_t* __restrict__ t_multi,
                                                   const unsigned long long* __restrict__ obase) {
    __shared__ uint32_t rb[4][64];   // per wave: the record index of its q-th match
    __shared__ uint32_t wsum[4];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t c = i < n ? t_cnt[i] : 0u;
    uint32_t incl = c;
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t pre = sup_off[blockIdx.x / GEN_OST] + tile_pre[blockIdx.x];
    for (uint32_t q = 0; q < w; ++q) pre += wsum[q];
    const uint32_t rel = pre + incl - c;   // this event's first record, relative to the batch's base
    if (c) t_cnt[i] = 0u;                  // (the counts are zero again for the next batch)
    if (!GATHER || *t_multi) {
        if (c) t_off[i] = rel;
        return;
    }
    const bool has = c != 0u;
    const uint64_t bm = __ballot(has);
    if (!bm) return;   // (wave-uniform)
    const uint32_t m = (uint32_t)__popcll(bm);
    const uint32_t first = (uint32_t)__ffsll((unsigned long long)bm) - 1u;
    const uint64_t d0 = *obase + __shfl(rel, (int)first, 64);
    if (d0 + m > o.cap) {   // (the capacity check of write_out, per wave)
        if (lane == 0) atomicOr(o.err, (uint32_t)GERR_MATCHCAP);
        return;
    }
    const uint32_t* rec = has ? raw + (uint64_t)t_first[i] * o.recWords : raw;
    if (has) {
        const uint32_t q = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
        rb[w][q] = t_first[i];
        const uint64_t d = d0 + q;
        o.trig[d] = (uint64_t)rec[2] | ((uint64_t)rec[3] << 32);
        o.ts[d] = (int64_t)((uint64_t)rec[4] | ((uint64_t)rec[5] << 32));
        o.key[d] = rec[6];
        for (uint32_t x = 0; x < o.projN; x++) {
            const uint32_t* pv = rec + o.projOff + 3 * x;
            o.pval[(size_t)x * o.cap + d] = (uint64_t)pv[0] | ((uint64_t)pv[1] << 32);
            o.pnull[(size_t)x * o.cap + d] = (uint8_t)pv[2];
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t ns = o.nslots, mc = o.MC, per = ns * mc;
    for (uint32_t x = lane; x < m * ns; x += 64) {   // chain lengths
        const uint32_t* r = raw + (uint64_t)rb[w][x / ns] * o.recWords;
        o.len[d0 * ns + x] = r[7 + x % ns];
    }
    for (uint32_t x = lane; x < m * per; x += 64) {  // slot chains
        const uint32_t q = x / per, y = x % per, sl = y / mc, cc = y % mc;
        const uint32_t* r = raw + (uint64_t)rb[w][q] * o.recWords;
        const uint32_t* seqs = r + 7 + ns;
        uint32_t b = sl * mc;
        if (r[1] & GEN_REC_PACKED) {   // (packed chains: after the lengths of the slots before this one)
            b = 0;
            for (uint32_t s2 = 0; s2 < sl; s2++) b += r[7 + s2];
        }
        o.slot[d0 * per + x] = cc < r[7 + sl] ? ((uint64_t)seqs[2 * (b + cc)] | ((uint64_t)seqs[2 * (b + cc) + 1] << 32))
                                              : SG_NULL_SEQ;
    }
}

// timer matches in sorted order
__global__ void k_gen_scatter_timers(const uint32_t* raw, const uint32_t* order, const unsigned long long* nvalid,
                                     OutBufs o) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= *nvalid) return;
    write_out(o, *o.count + r, raw + (uint64_t)order[r] * o.recWords, true);
}

// a poll's status (gen_poll): count, error word, largest count-kernel tile -> st (copied to the host); the count back to 0
// when the poll will hand the window out (no error of `fail_mask`, within the capacity)
__global__ void k_gen_status(unsigned long long* count, const uint32_t* err, const uint32_t* tile_max, uint64_t cap,
                             uint32_t fail_mask, unsigned long long* st) {
    if (threadIdx.x != 0) return;
    const unsigned long long c = *count;
    const uint32_t x = *err;
    st[0] = c;
    st[1] = x;
    st[2] = tile_max ? *tile_max : 0u;
    if ((x & fail_mask) == 0u && c <= cap) *count = 0ull;
}

__global__ void k_gen_bump(unsigned long long* count, const uint32_t* t_cnt, const uint32_t* t_off, uint32_t n,
                           const unsigned long long* nvalid) {
    if (nvalid) *count += *nvalid;
    else *count += (unsigned long long)t_off[n - 1] + t_cnt[n - 1];
}

// the per-batch / per-advance resets of the engine's counters and per-key bounds in one launch (a
// hipMemsetAsync each was a fill kernel of its own: ~26 per C4 step)
#define GEN_CLEAR_JOBS 8
struct GenClear {
    uint32_t n;
    uint32_t v[GEN_CLEAR_JOBS];      // the 32-bit fill value
    uint64_t words[GEN_CLEAR_JOBS];  // 32-bit words
    uint32_t* p[GEN_CLEAR_JOBS];     // 16-B aligned (device allocations)
};
__global__ void __launch_bounds__(256) k_gen_clear(const GenClear c) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
    for (uint32_t q = 0; q < c.n; ++q) {
        const uint32_t v = c.v[q];
        const uint64_t n4 = c.words[q] >> 2;
        uint4* p4 = (uint4*)c.p[q];
        for (uint64_t k = i; k < n4; k += st) p4[k] = make_uint4(v, v, v, v);
        for (uint64_t k = n4 * 4 + i; k < c.words[q]; k += st) c.p[q][k] = v;
    }
}
struct GenClearList {
    GenClear c{};
    uint64_t most = 0;
    void add(void* p, uint64_t bytes, uint32_t v = 0u) {
        c.p[c.n] = (uint32_t*)p;
        c.words[c.n] = bytes / 4;
        c.v[c.n++] = v;
        most = std::max<uint64_t>(most, bytes / 4);
    }
    hipError_t launch(hipStream_t s) const {
        if (!c.n) return hipSuccess;
        const uint64_t blocks = std::min<uint64_t>(std::max<uint64_t>((most / 4 + 255) / 256, 1), 2048);
        hipLaunchKernelGGL(k_gen_clear, dim3((unsigned)blocks), dim3(256), 0, s, c);
        return hipGetLastError();
    }
};

// the slots k_timer_prep filled in the due heads' hash set back to empty (instead of refilling the whole
// 2 K-slot table before every advance)
__global__ void k_ht_clear(const uint32_t* __restrict__ ins, const unsigned long long* __restrict__ ndue,
                           unsigned long long* __restrict__ ht) {
    const uint64_t n = *ndue;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (ins[i] != 0xffffffffu) ht[ins[i]] = ~0ull;
}

__global__ void k_gen_fill64(int64_t* x, uint64_t n, int64_t v) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = v;
}

// purged keys have no timers
__global__ void k_gen_nd_reset(const uint32_t* __restrict__ keys, uint32_t n, uint32_t K, int64_t* __restrict__ nd) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && keys[i] < K) nd[keys[i]] = GEN_NO_DEADLINE;
}

__global__ void k_gen_iota(uint32_t* x, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = (uint32_t)i;
}

// live partial matches (StateEvents holding an event) in every list of every processor; with seg_begin /
// seg_end, of the keys the batch touches only (sg_stats.live_at_batch_start, before the batch kernel)
__global__ void k_gen_live(const GenProgram* G, const uint32_t* S, uint32_t K, unsigned long long* out,
                           const uint32_t* rec, const uint32_t* seg_begin = nullptr, const uint32_t* seg_end = nullptr) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    if (seg_begin && seg_begin[k] >= seg_end[k]) return;
    unsigned long long live = 0;
    const uint32_t w0 = S[gen_at(K, G->blockWords, G->offST, k, 0)];
    if ((w0 & GEN_W0_REG) && rec) {   // the state in its record (GEN_W0_REG)
        const uint32_t h = rec[k];
        if (G->cntOk)   // the count partial: one StateEvent in each list it is in
            live = (h & 15u) ? ((h >> 4) & 1u) + ((h >> 5) & 1u) + 2u * ((h >> 6) & 1u) : 0u;
        else            // the absent shape: each partial holds its e1 (the seed holds no event)
            live = h & 15u;
        if (live) atomicAdd(out, live);
        return;
    }
    const bool deep = (w0 & GEN_W0_DEEP) != 0u;
    for (int p = 0; p < G->nprocs; p++) {
        const uint32_t ks = G->offKS + (uint32_t)p * G->ksWords;
        if (deep && p == G->absP1) {   // (the lists are in the deep store: every entry holds its e1)
            live += S[gen_at(K, G->blockWords, G->offST, k, ks + KS_PLEN)] +
                    S[gen_at(K, G->blockWords, G->offST, k, ks + KS_NLEN)];
            continue;
        }
        for (int which = 0; which < 2; which++) {
            const uint32_t n = S[gen_at(K, G->blockWords, G->offST, k, ks + KS_PLEN + which)];
            for (uint32_t i = 0; i < n; i++) {
                const uint32_t se = S[gen_at(K, G->blockWords, G->offST, k, ks + KS_LISTS + which * G->L + i)];
                for (int s = 0; s < G->nslots; s++)
                    if (S[gen_at(K, G->blockWords, G->offST, k, G->offST + se * G->stWords + ST_SLOTS + s)] != GEN_NIL) {
                        live++;
                        break;
                    }
            }
        }
    }
    if (live) atomicAdd(out, live);
}

// the smallest event seq any live partial still references: every StreamEvent a list's StateEvent reaches
// (count chains followed), over every initialised key (the multi-device engine trims its seq maps below it)
__global__ void k_gen_min_seq(const GenProgram* G, const uint32_t* S, uint32_t K, unsigned long long* out,
                              const uint32_t* rec) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long m = ~0ull;
    const uint32_t w0 = k < K ? S[gen_at(K, G->blockWords, G->offST, k, 0)] : 0u;
    if ((w0 & GEN_W0_REG) && rec) {   // the state in its record (GEN_W0_REG): the events of its partials
        const uint32_t n = rec[k] & 15u, ew = 5u + G->absNW;
        for (uint32_t j = 0; j < n && j < GEN_REC_R; j++) {
            const size_t o = (size_t)(GEN_REC_EV + j * ew) * K + k;
            const unsigned long long q = (unsigned long long)rec[o] | ((unsigned long long)rec[o + K] << 32);
            m = q < m ? q : m;
        }
    } else if (w0 & 1u) {
        auto W = [&](uint32_t w) { return S[gen_at(K, G->blockWords, G->offST, k, w)]; };
        for (int p = 0; p < G->nprocs; p++) {
            const uint32_t ks = G->offKS + (uint32_t)p * G->ksWords;
            for (int which = 0; which < 2; which++) {
                const uint32_t n = W(ks + KS_PLEN + which);
                for (uint32_t i = 0; i < n && i < G->L; i++) {
                    const uint32_t se = W(ks + KS_LISTS + which * G->L + i);
                    for (int sl = 0; sl < G->nslots; sl++) {
                        uint32_t ev = W(G->offST + se * G->stWords + ST_SLOTS + sl);
                        for (uint32_t guard = 0; ev != GEN_NIL && guard <= G->SECAP; guard++) {
                            const uint32_t b = G->offSE + ev * G->seWords;
                            const unsigned long long q = (unsigned long long)W(b + SE_SEQ) |
                                                         ((unsigned long long)W(b + SE_SEQ + 1) << 32);
                            m = q < m ? q : m;
                            ev = W(b + SE_NEXT);
                        }
                    }
                }
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, 64);
        m = o < m ? o : m;
    }
    if ((threadIdx.x & 63) == 0 && m != ~0ull) atomicMin(out, m);
}

// ---- timer matches ordered through the due keys (one listener: GenTimers.kcnt / dpair_kid) ----
// ctr: [0] largest sort key, [1] a lag that does not fit 32 bits, [2] keys with matches, [3] two due keys
// share a head time (the reference's collapse quirk)
#define GEN_TPREP_BLOCK 1024
__device__ __forceinline__ uint64_t gen_hmix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return x;
}
// per due slot: the head into an exact hash set (a second equal head = the A.10 collapse), and the keys
// that emitted matches into a compact list with their sort key 1 + (T - head) (descending = head order;
// the 64-bit head too, for lags beyond 32 bits).  One atomic per block for the list.
__global__ void __launch_bounds__(GEN_TPREP_BLOCK) k_timer_prep(
        const unsigned long long* __restrict__ dkey, const uint32_t* __restrict__ dkid,
        const unsigned long long* __restrict__ ndue, int64_t T, const uint32_t* __restrict__ kcnt,
        unsigned long long* __restrict__ ht, uint64_t htmask, uint32_t* __restrict__ ht_ins, uint32_t* __restrict__ rel_c,
        uint32_t* __restrict__ kid_c, unsigned long long* __restrict__ hkey_c, unsigned long long* __restrict__ ctr) {
    constexpr uint32_t NW = GEN_TPREP_BLOCK / 64;
    __shared__ uint32_t wcnt[NW];
    __shared__ unsigned long long bbase, bmax[NW];
    const int lane = threadIdx.x & 63;
    const uint32_t wv = threadIdx.x / 64;
    const uint64_t n = *ndue;
    unsigned long long mx = 0;
    for (uint64_t base = (uint64_t)blockIdx.x * GEN_TPREP_BLOCK; base < n; base += (uint64_t)gridDim.x * GEN_TPREP_BLOCK) {
        const uint64_t di = base + threadIdx.x;
        bool has = false;
        uint32_t r32 = 0, kid = GEN_PAIR_NONE;
        unsigned long long h = ~0ull;
        if (di < n) {
            h = dkey[di];
            kid = dkid[di];
            uint32_t ins = 0xffffffffu;   // the slot this entry filled (k_ht_clear empties it)
            if (h != ~0ull && kid != GEN_PAIR_NONE) {
                uint64_t p = gen_hmix(h) & htmask;
                for (uint64_t probe = 0; probe <= htmask; probe++) {
                    const unsigned long long prev = atomicCAS(&ht[p], ~0ull, h);
                    if (prev == ~0ull) { ins = (uint32_t)p; break; }
                    if (prev == h) { ctr[3] = 1ull; break; }
                    p = (p + 1) & htmask;
                }
                const int64_t head = (int64_t)(h ^ (1ull << 63));
                unsigned long long r = (unsigned long long)(T - head) + 1ull;
                if (T < head || r >= 0xffffffffull) { ctr[1] = 1ull; r = 0; }
                r32 = (uint32_t)r;
                mx = max(mx, r);
                has = (kcnt[kid] & ~GEN_KCNT_STAGED) != 0u;
            }
            ht_ins[di] = ins;
        }
        const unsigned long long m = __ballot(has);
        if (lane == 0) wcnt[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (uint32_t w = 0; w < NW; w++) t += wcnt[w];
            bbase = t ? atomicAdd(&ctr[2], (unsigned long long)t) : 0ull;
        }
        __syncthreads();
        if (has) {
            uint32_t before = 0;
            for (uint32_t w = 0; w < wv; w++) before += wcnt[w];
            const unsigned long long o = bbase + before + __popcll(m & ((1ull << lane) - 1ull));
            rel_c[o] = r32;
            kid_c[o] = kid;
            hkey_c[o] = h;
        }
        __syncthreads();
    }
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (unsigned long long)__shfl_xor(mx, off, 64));
    if (lane == 0) bmax[wv] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < NW; w++) t = max(t, bmax[w]);
        if (t) atomicMax(&ctr[0], t);
    }
}
// two due keys sharing a head time (adjacent after the sort): the reference's collapse quirk (A.10)
__global__ void k_timer_collapse(const uint32_t* __restrict__ srel, uint64_t n, uint32_t* __restrict__ err) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j == 0 || j >= n || srel[j] == 0u) return;
    if (srel[j] == srel[j - 1]) atomicOr(err, (uint32_t)GERR_COLLAPSE);
}
__global__ void k_timer_collapse64(const unsigned long long* __restrict__ skey, uint64_t n, uint32_t* __restrict__ err) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j == 0 || j >= n || skey[j] == ~0ull) return;
    if (skey[j] == skey[j - 1]) atomicOr(err, (uint32_t)GERR_COLLAPSE);
}
__global__ void k_timer_cnt(const uint32_t* __restrict__ skid, uint64_t n, const uint32_t* __restrict__ kcnt,
                            uint32_t* __restrict__ c) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) c[j] = skid[j] == GEN_PAIR_NONE ? 0u : (kcnt[skid[j]] & ~GEN_KCNT_STAGED);
}
// the matches k_abs_timers staged per key, to count + (the key's offset in head order) + rank
__global__ void k_timer_scatter_abs(const uint32_t* __restrict__ skid, uint64_t n, const uint32_t* __restrict__ kcnt,
                                    const uint32_t* __restrict__ koff, const unsigned long long* __restrict__ tstage,
                                    uint32_t K, uint32_t slot0, OutBufs o) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n || skid[j] == GEN_PAIR_NONE) return;
    const uint32_t key = skid[j];
    const uint32_t c = kcnt[key];
    if (!(c & GEN_KCNT_STAGED)) return;
    const uint64_t base = *o.count + koff[key];
    for (uint32_t r = 0; r < (c & ~GEN_KCNT_STAGED); r++) {
        const uint64_t d = base + r;
        if (d >= o.cap) { atomicOr(o.err, (uint32_t)GERR_MATCHCAP); return; }
        o.trig[d] = SG_TIMER_SEQ;
        o.ts[d] = (int64_t)tstage[(size_t)(ABS_R + r) * K + key];
        o.key[d] = key;
        for (uint32_t s = 0; s < o.nslots; s++) {
            o.len[d * o.nslots + s] = s == slot0 ? 1u : 0u;
            for (uint32_t q = 0; q < o.MC; q++)
                o.slot[(d * o.nslots + s) * o.MC + q] = (s == slot0 && q == 0) ? tstage[(size_t)r * K + key] : SG_NULL_SEQ;
        }
    }
}
__global__ void k_timer_bump(unsigned long long* count, const uint32_t* c, const uint32_t* off, uint64_t n) {
    *count += (unsigned long long)off[n - 1] + c[n - 1];
}
// the register-window kernels' per-wave counter rows into the engine counters (one block per counter)
__global__ void __launch_bounds__(256) k_gen_stats_reduce(const unsigned long long* __restrict__ w, uint32_t rows,
                                                          unsigned long long* __restrict__ stats) {
    __shared__ unsigned long long part[4];
    // block (c, y): counter c over rows y, y + gridDim.y, ... (a few loads per lane in flight instead of a
    // 64-deep dependent loop in one block per counter)
    const uint32_t c = blockIdx.x;
    unsigned long long x = 0;
    for (uint32_t r = blockIdx.y * blockDim.x + threadIdx.x; r < rows; r += gridDim.y * blockDim.x)
        x += w[(size_t)r * GST_N + c];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x / 64] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(&stats[c], t);
    }
}
__global__ void k_timer_off(const uint32_t* __restrict__ skid, uint64_t n, const uint32_t* __restrict__ off,
                            uint32_t* __restrict__ koff) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n && skid[j] != GEN_PAIR_NONE) koff[skid[j]] = off[j];
}
// each timer match to count + (its key's offset in head order) + (its rank in the key's sweep)
__global__ void k_timer_scatter(const uint32_t* raw, const unsigned long long* raw_count, const uint32_t* koff,
                                OutBufs o) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= *raw_count) return;
    const uint32_t* rec = raw + r * o.recWords;
    if (rec[0] != 0xfffffffeu) return;
    write_out(o, *o.count + koff[rec[6]] + rec[1], rec, true);
}

struct TimerLess {
    const uint32_t* k1;
    const int64_t* k2;
    const uint32_t* k3;
    __device__ bool operator()(uint32_t a, uint32_t b) const {
        if (k1[a] != k1[b]) return k1[a] < k1[b];
        if (k2[a] != k2[b]) return k2[a] < k2[b];
        if (k3[a] != k3[b]) return k3[a] < k3[b];
        return a < b;
    }
};

// ---------------------------------------------------------------------------------------------
// the engine
// ---------------------------------------------------------------------------------------------
struct GenEngine {
    // gen_keep_timer_heads: the last advance's emitting keys in head order and their heads (host copies)
    bool keep_heads = false;
    std::vector<uint32_t> head_keys;
    std::vector<int64_t> head_t;
    GenProgram host{};
    GenProgram* dprog = nullptr;
    hipStream_t stream = nullptr;
    uint32_t K = 1, maxb = 0;
    bool null_keys = false;  // SG_CFG_NULL_KEYS
    uint64_t mcap = 0, rawCap = 0;
    uint32_t recWords = 0;
    std::vector<void*> owned;
    uint32_t* state = nullptr;
    // batch staging
    int64_t* b_ts = nullptr;
    uint32_t* b_key = nullptr;
    std::vector<void*> b_cols;
    std::vector<uint8_t*> b_nulls;
    uint32_t *sidx = nullptr, *seg_begin = nullptr, *seg_end = nullptr;
    PartScratch pscr{};      // the grouping's and the timer sorts' scratch (part.h)
    // matches
    uint32_t* raw = nullptr;
    unsigned long long* raw_count = nullptr;
    uint32_t *t_cnt = nullptr, *t_first = nullptr, *t_off = nullptr;
    uint32_t *tile_pre = nullptr, *sup_sum = nullptr, *sup_off = nullptr;   // the batch ordering's tile prefixes
    unsigned long long* obase = nullptr;                  // the running match count before the batch
    PinnedVec<unsigned long long> h_stat;                 // gen_poll's status words (pinned: one DMA copy) and their device copy
    unsigned long long* d_stat = nullptr;
    uint32_t* t_multi = nullptr;          // GenOut.t_multi
    int64_t* tk2 = nullptr;
    uint32_t *tk1 = nullptr, *tk3 = nullptr, *order_in = nullptr, *order_out = nullptr;
    unsigned long long* nvalid = nullptr;
    void* msort_tmp = nullptr;
    size_t msort_tmp_bytes = 0;
    unsigned long long* stats = nullptr;
    // timers: per-key next deadline, the due-key list of an advance and its (due time, listener) pairs
    GenTimers tm{};
    uint64_t npairs_cap = 0;
    unsigned long long* pair_key_s = nullptr;
    uint32_t* pair_i_s = nullptr;
    unsigned long long* live = nullptr;  // k_gen_live's sum (diagnostics)
    unsigned long long* minseq = nullptr;  // k_gen_min_seq's result
    // keys the register-window kernels (abs_kernels.hip) hand to the general kernels
    uint32_t *fb_list = nullptr, *fb_start = nullptr;
    uint32_t *fb2_list = nullptr, *fb2_start = nullptr;  // the wave-per-key kernels' hand-over (absd_kernels.hip)
    uint32_t* deep = nullptr;                             // their deep store (GEN_W0_DEEP): deepWords per key
    uint32_t deepWords = 0;
    uint32_t* rec = nullptr;   // the register-window kernels' records (GEN_W0_REG): gen_rec_words rows per key
    bool absd_nochunk = false; // SG_NO_ABSD_CHUNK: the wave-per-key batch walk event by event
    bool abs_occ4 = true;      // the occupancy-4 absent kernels where they fit (SG_NO_ABS_OCC4: never)
    uint32_t ncu = 256;        // compute units of the device
    unsigned long long* fb2_n = nullptr;
    unsigned long long* fb_n = nullptr;
    uint32_t* pay = nullptr;   // the key-sorted payload of the register-window kernel (pack.h Pay<W>)
    bool cnt_fused = false;    // the count kernel's batches may take the fused tile grouping
    bool cnt_fused_last = false;
    bool cnt_skewed = false;   // a fused batch had a tile of more than 2^14 events: the sorted grouping from then on
    uint32_t* tile_max = nullptr;
    uint32_t* tpay = nullptr;  // fused: the batch grouped by 64-key tile (Pay<W>, key & 255 tagged), tile starts
    uint32_t* tile_lo = nullptr;
    unsigned long long* wstats = nullptr;  // its per-wave counter rows
    unsigned long long* tstage = nullptr;  // its staged timer matches
    // timer matches ordered through the due keys (keyorder: partitioned, playback, one listener)
    bool keyorder = false;
    uint32_t *rel = nullptr, *srel = nullptr, *skid = nullptr, *kc = nullptr, *koff_s = nullptr, *koff = nullptr;
    uint32_t* kid_c = nullptr;
    unsigned long long *hkey_c = nullptr, *hkey_s = nullptr;
    unsigned long long* ht = nullptr;   // the due heads' hash set (A.10 check), 2^k >= 2 K slots
    uint64_t htmask = 0;
    unsigned long long* ctr = nullptr;  // k_timer_prep's counters
    uint32_t* ht_ins = nullptr;         // [npairs_cap] the hash slot each due entry filled
    void* kscan_tmp = nullptr;
    size_t kscan_tmp_bytes = 0;
    uint32_t* err = nullptr;
    OutBufs out{};
    PinnedVec<uint64_t> h_trig, h_slot;
    PinnedVec<uint32_t> h_key, h_len;
    PinnedVec<int64_t> h_ts;
    bool held = false;
    uint64_t polled = 0;    // matches of the held poll (sg_get_projection)
    PinnedVec<uint64_t> h_pval;
    PinnedVec<uint8_t> h_pnull;
    int64_t now = 0;        // TimestampGenerator.currentTime() as last set by sg_advance_time
    int64_t lastEventTs = 0;
    bool advanced = false;
    sg_stats st{};
    // SG_CFG_TIMING: HIP events around the NFA kernels (batch + timer sweeps: advance_ns) and the
    // grouping (group_ns), resolved by gen_stats; the touched keys' live partials counted before each batch
    bool timing = false;
    unsigned long long* prof = nullptr;  // SG_GEN_PROF with a GENX_PROF build: walk-phase cycles, printed at destroy
    struct Span { hipEvent_t a, b; int which; };
    std::vector<Span> spans;
    hipEvent_t ev() {
        hipEvent_t x;
        GH_OK(hipEventCreate(&x));
        GH_OK(hipEventRecord(x, stream));
        return x;
    }

    template <class T> T* dalloc(size_t n) {
        void* p = nullptr;
        GH_OK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
        owned.push_back(p);
        return (T*)p;
    }
    ~GenEngine() {
        if (stream) (void)hipStreamSynchronize(stream);
        if (prof) {
            unsigned long long h[8] = {};
            if (hipMemcpy(h, prof, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess)
                fprintf(stderr, "gen prof (cycles summed over waves): start %llu stabilize %llu process %llu "
                        "project %llu end %llu timers %llu waves %llu\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
        }
        for (auto& x : spans) { (void)hipEventDestroy(x.a); (void)hipEventDestroy(x.b); }
        for (void* p : owned) (void)hipFree(p);
    }

    GenArgs args() const {
        GenArgs a{};
        a.G = dprog;
        a.state = state;
        a.K = K;
        a.o.raw = raw;
        a.o.raw_count = raw_count;
        a.o.raw_cap = rawCap;
        a.o.nseg = 1;
        a.o.seg_cap = rawCap;
        a.o.recWords = recWords;
        a.o.t_cnt = t_cnt;
        a.o.t_first = t_first;
        a.o.t_multi = t_multi;
        a.o.tk1 = tk1;
        a.o.tk2 = tk2;
        a.o.tk3 = tk3;
        a.o.nvalid = nvalid;
        a.o.stats = stats;
        a.o.wstats = wstats;
        a.o.err = err;
        a.o.prof = prof;
        a.t = tm;
        a.now = now;
        a.now0 = now;
        a.deep = deep;
        a.deepWords = deepWords;
        a.rec = rec;
        return a;
    }
};

GenEngine* gen_create(const uint32_t* ir, size_t nw, const sg_config& cfg, hipStream_t stream) {
    GenProgram* prog = gen_build_program(ir, nw, cfg.partial_capacity ? cfg.partial_capacity : 32);
    auto* e = new GenEngine();
    try {
        e->host = *prog;
        delete prog;
        e->stream = stream;
        e->K = e->host.partitioned ? (cfg.n_keys ? cfg.n_keys : 1) : 1;
        e->null_keys = (cfg.flags & SG_CFG_NULL_KEYS) != 0;
        e->timing = (cfg.flags & SG_CFG_TIMING) != 0;
        if (getenv("SG_GEN_PROF")) {
            e->prof = e->dalloc<unsigned long long>(8);
            GH_OK(hipMemsetAsync(e->prof, 0, 64, stream));
        }
        e->maxb = cfg.max_batch ? cfg.max_batch : (1u << 20);
        // (k_gen_tscan: one workgroup of 1024 threads x 8 super tiles of GEN_OT * GEN_OST events)
        if (e->maxb > 8192ull * GEN_OT * GEN_OST) throw std::runtime_error("max_batch above 2^25 events");
        e->mcap = cfg.match_capacity ? cfg.match_capacity : (uint64_t)e->maxb * 4;
        const GenProgram& G = e->host;
        e->recWords = 7 + (uint32_t)G.nslots + 2 * (uint32_t)G.nslots * G.MC;
        // lanes reserve GEN_RESCHUNK slots at a time in one of GEN_RAWSEG segments: slack for every
        // key's partly used chunks plus the segments' imbalance
        e->rawCap = (e->mcap + (uint64_t)e->K * 2 * GEN_RESCHUNK + GEN_RAWSEG * 4096ull) / GEN_RAWSEG * GEN_RAWSEG;
        const size_t K = e->K, B = e->maxb;
        e->dprog = e->dalloc<GenProgram>(1);
        GH_OK(hipMemcpy(e->dprog, &e->host, sizeof(GenProgram), hipMemcpyHostToDevice));
        e->state = e->dalloc<uint32_t>((size_t)G.blockWords * K);
        GH_OK(hipMemsetAsync(e->state, 0, (size_t)G.blockWords * K * 4, stream));
        e->b_ts = e->dalloc<int64_t>(B);
        e->b_key = e->dalloc<uint32_t>(B);
        int maxa = 1;
        for (int s = 0; s < G.nstreams; s++) maxa = std::max(maxa, G.nattr[s]);
        for (int a = 0; a < maxa; a++) {
            e->b_cols.push_back(e->dalloc<uint64_t>(B));
            e->b_nulls.push_back(e->dalloc<uint8_t>(B));
        }
        e->sidx = e->dalloc<uint32_t>(B);
        e->seg_begin = e->dalloc<uint32_t>(K);
        e->seg_end = e->dalloc<uint32_t>(K);
        e->raw = e->dalloc<uint32_t>(e->rawCap * e->recWords);
        e->raw_count = e->dalloc<unsigned long long>(GEN_RAWSEG);
        e->t_cnt = e->dalloc<uint32_t>(B);
        e->t_first = e->dalloc<uint32_t>(B);
        e->t_off = e->dalloc<uint32_t>(B);
        e->t_multi = e->dalloc<uint32_t>(1);
        GH_OK(hipMemsetAsync(e->t_cnt, 0, B * 4, stream));
        GH_OK(hipMemsetAsync(e->t_multi, 0, 4, stream));
        e->tk1 = e->dalloc<uint32_t>(e->rawCap);
        e->tk2 = e->dalloc<int64_t>(e->rawCap);
        e->tk3 = e->dalloc<uint32_t>(e->rawCap);
        e->order_in = e->dalloc<uint32_t>(e->rawCap);
        e->order_out = e->dalloc<uint32_t>(e->rawCap);
        e->nvalid = e->dalloc<unsigned long long>(1);
        e->tile_pre = e->dalloc<uint32_t>(B / GEN_OT + 1);
        e->sup_sum = e->dalloc<uint32_t>(B / (GEN_OT * GEN_OST) + 1);
        e->sup_off = e->dalloc<uint32_t>(B / (GEN_OT * GEN_OST) + 1);
        e->obase = e->dalloc<unsigned long long>(1);
        TimerLess lt{e->tk1, e->tk2, e->tk3};
        GH_OK(rocprim::merge_sort(nullptr, e->msort_tmp_bytes, e->order_in, e->order_out, (size_t)e->rawCap, lt, stream));
        e->msort_tmp = e->dalloc<uint8_t>(e->msort_tmp_bytes);
        e->stats = e->dalloc<unsigned long long>(GST_N);
        if (G.nStartup > 0) {
            e->tm.nd = e->dalloc<int64_t>(K);
            hipLaunchKernelGGL(k_gen_fill64, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, stream, e->tm.nd,
                               (uint64_t)K, (int64_t)GEN_NO_DEADLINE);
            e->tm.due = e->dalloc<uint32_t>(K);
            e->tm.ndue = e->dalloc<unsigned long long>(1);
            if (G.partitioned && G.playback) {
                e->npairs_cap = (uint64_t)K * (uint64_t)G.nStartup;
                e->tm.dpair_key = e->dalloc<unsigned long long>(e->npairs_cap);
                e->tm.dpair_i = e->dalloc<uint32_t>(e->npairs_cap);
                e->pair_key_s = e->dalloc<unsigned long long>(e->npairs_cap);
                e->pair_i_s = e->dalloc<uint32_t>(e->npairs_cap);
                if (G.nStartup == 1) {
                    e->keyorder = true;
                    e->tm.dpair_kid = e->dalloc<uint32_t>(K);
                    e->tm.kcnt = e->dalloc<uint32_t>(K);
                    e->rel = e->dalloc<uint32_t>(K);
                    e->srel = e->dalloc<uint32_t>(K);
                    e->skid = e->dalloc<uint32_t>(K);
                    e->kc = e->dalloc<uint32_t>(K);
                    e->koff_s = e->dalloc<uint32_t>(K);
                    e->koff = e->dalloc<uint32_t>(K);
                    e->ctr = e->dalloc<unsigned long long>(4);
                    e->kid_c = e->dalloc<uint32_t>(K);
                    e->hkey_c = e->dalloc<unsigned long long>(K);
                    e->hkey_s = e->dalloc<unsigned long long>(K);
                    uint64_t hs = 1024;
                    while (hs < 2 * (uint64_t)K) hs <<= 1;
                    e->ht = e->dalloc<unsigned long long>(hs);
                    e->htmask = hs - 1;
                    e->ht_ins = e->dalloc<uint32_t>(std::max<uint64_t>(e->npairs_cap, 1));
                    GH_OK(hipMemsetAsync(e->ht, 0xff, hs * 8, stream));   // empty; kept empty by k_ht_clear
                    GH_OK(rocprim::exclusive_scan(nullptr, e->kscan_tmp_bytes, e->kc, e->koff_s, 0u, (size_t)K,
                                                  rocprim::plus<uint32_t>(), stream));
                    e->kscan_tmp = e->dalloc<uint8_t>(e->kscan_tmp_bytes);
                }
            }
        }
        e->live = e->dalloc<unsigned long long>(1);
        if (G.absOk || G.cntOk || G.chnOk) {
            e->fb_list = e->dalloc<uint32_t>(K);
            e->fb_start = e->dalloc<uint32_t>(K);
            e->fb_n = e->dalloc<unsigned long long>(1);
            e->absd_nochunk = getenv("SG_NO_ABSD_CHUNK") != nullptr;
            e->abs_occ4 = getenv("SG_NO_ABS_OCC4") == nullptr;
            {
                int dev = 0, ncu = 0;
                GH_OK(hipGetDevice(&dev));
                GH_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
                if (ncu > 0) e->ncu = (uint32_t)ncu;
            }
            if (G.chnOk && G.chnWide) {   // (the wide chain kernel's hand-over list)
                e->fb2_list = e->dalloc<uint32_t>(K);
                e->fb2_start = e->dalloc<uint32_t>(K);
                e->fb2_n = e->dalloc<unsigned long long>(1);
            }
            if (G.absOk && !getenv("SG_NO_ABSD")) {
                e->fb2_list = e->dalloc<uint32_t>(K);
                e->fb2_start = e->dalloc<uint32_t>(K);
                e->fb2_n = e->dalloc<unsigned long long>(1);
                // the deep store: one contiguous record per key (lists + timer queue), so a deep key's one wave
                // reads and writes its state coalesced instead of one 4-B word per row of the interleaved block
                // (SG_NO_DEEP: the block only); capped at 64 GB of the HBM
                const GenDeepLayout dl = gen_deep_layout(G.L, G.Q, G.absNW);
                if (!getenv("SG_NO_DEEP") && (uint64_t)dl.words * 4 * K <= (64ull << 30)) {
                    e->deepWords = dl.words;
                    e->deep = e->dalloc<uint32_t>((size_t)dl.words * K);
                }
            }
            const uint64_t rw = gen_rec_words(G.absNW, G.cntOk ? 0u : G.Q);
            const bool regKernels = G.cntOk || (G.playback && G.partitioned && G.nStartup == 1 && e->keyorder);
            if (regKernels && !getenv("SG_NO_REC") && rw * 4 * K <= (64ull << 30)) {
                // the register-window kernels' records (GEN_W0_REG): a key's window coalesced across the wave's
                // keys, written back only where it changed (SG_NO_REC: the blocks, rewritten per touch)
                e->rec = e->dalloc<uint32_t>((size_t)rw * K);
            }
            e->pay = e->dalloc<uint32_t>(B * 6);  // Pay<4>: 6 words
            // the count kernel's fused grouping (by 64-key tile; the kernel splits its tile by key in LDS)
            e->cnt_fused = (regKernels || G.chnOk) && G.partitioned && sgd_fused_ok(K, B, 1, 6) && !getenv("SG_NO_FUSED");
            if (e->cnt_fused) {
                e->tpay = e->dalloc<uint32_t>(B * 6);
                e->tile_lo = e->dalloc<uint32_t>((K + 63) / 64 + 1);
                e->tile_max = e->dalloc<uint32_t>(1);
                GH_OK(hipMemsetAsync(e->tile_max, 0, 4, stream));
            }
            e->wstats = e->dalloc<unsigned long long>((size_t)((K + 63) / 64) * GST_N);
            if (G.playback && G.partitioned && G.nStartup == 1) {
                e->tstage = e->dalloc<unsigned long long>((size_t)K * ABS_R * 2);
                e->tm.tstage = e->tstage;
            }
        }
        {  // the grouping (B events) and the timer sorts (K keys, K x listeners due pairs)
            const uint64_t sn = std::max<uint64_t>({(uint64_t)B, (uint64_t)K, e->npairs_cap, 1});
            e->pscr = sgd_part_scratch(e->dalloc<uint8_t>(sgd_part_scratch_bytes(sn)), sn);
        }
        GH_OK(hipMemsetAsync(e->stats, 0, GST_N * 8, stream));
        e->err = e->dalloc<uint32_t>(1);
        GH_OK(hipMemsetAsync(e->err, 0, 4, stream));
        const uint64_t M = e->mcap;
        e->out.trig = e->dalloc<uint64_t>(M);
        e->out.slot = e->dalloc<uint64_t>(M * G.nslots * G.MC);
        e->out.key = e->dalloc<uint32_t>(M);
        e->out.ts = e->dalloc<int64_t>(M);
        e->out.len = e->dalloc<uint32_t>(M * G.nslots);
        e->out.count = e->dalloc<unsigned long long>(1);
        GH_OK(hipMemsetAsync(e->out.count, 0, 8, stream));
        e->out.cap = M;
        e->out.nslots = (uint32_t)G.nslots;
        e->out.MC = G.MC;
        e->out.recWords = e->recWords;
        e->out.err = e->err;
        GH_OK(hipStreamSynchronize(stream));  // the zeroed state and counters are in place before a push
        return e;
    } catch (...) {
        delete e;
        throw;
    }
}

void gen_destroy(GenEngine* e) { delete e; }

static size_t type_size(int t) {
    switch (t) {
    case SG_T_LONG: case SG_T_DOUBLE: return 8;
    case SG_T_BOOL: return 1;
    default: return 4;
    }
}

// the kernels take GenArgs (608 B) by value in their kernel arguments
enum { GEN_L_BATCH = 0, GEN_L_TIMERS = 1, GEN_L_DEADLINES = 2, GEN_L_ABS_BATCH = 3, GEN_L_ABS_TIMERS = 4, GEN_L_CNT_BATCH = 5,
       GEN_L_ABSD_BATCH = 6, GEN_L_ABSD_TIMERS = 7, GEN_L_CHN_BATCH = 8, GEN_L_CHN_WIDE = 9 };
// the general kernels over the keys a register-window kernel handed over: a fixed grid striding the list
#define GEN_FB_BLOCKS 1024u
// timer sweeps: a fixed grid of one-wave blocks striding over the due keys (their number is on the device)
#define GEN_TIMER_BLOCKS 4096u
// keys per lane of k_gen_batch: 1 (GEN_KPL=n, experiments: n keys per lane).  Measured on C3/C3_min1/C4 at
// 2^20 keys with 4 keys per lane (one resident wave per slot, a lane's runs averaging out): 2-7 % slower
// than one key per lane — the kernel is bound by its memory transactions, not by idle lanes
static uint32_t gen_kpl(uint32_t K) {
    (void)K;
    if (const char* x = getenv("GEN_KPL")) return std::max(1u, (uint32_t)strtoul(x, nullptr, 0));
    return 1u;
}

// the register-window kernels of abs_kernels.hip run this query (the shape, and no device projection: the
// selector items are evaluated by the general kernel's projectSelect)
static bool abs_on(const GenEngine* e) {
    return e->host.absOk && e->host.projN == 0 && e->fb_list && e->tstage && e->keyorder;
}
// the wave-per-key kernels of absd_kernels.hip take the keys the register window hands over (their LDS slice:
// one key's lists, partial_capacity entries of 20 + 4 NW bytes, within 64 KB); SG_NO_ABSD: A/B against the
// general kernels (same results)
static size_t absd_lds(const GenEngine* e) {   // the key's lists (+ the f1 keys of the FF kernels), its timer queue
    const size_t kb = ((size_t)e->host.L * (20u + 4u * e->host.absNW) + 7) & ~(size_t)7;
    return ((kb + 20 * (size_t)e->host.L + 7) & ~(size_t)7) + 8 * (size_t)e->host.Q;
}
static bool absd_on(const GenEngine* e) { return e->fb2_list && absd_lds(e) <= 65536; }

// the register-window kernel of cnt_kernels.hip runs this query (the shape, no device projection)
static bool cnt_on(const GenEngine* e) { return e->host.cntOk && e->host.projN == 0 && e->fb_list; }
// the chain kernel of chn_kernels.hip runs this query (the shape, no device projection)
static bool chn_on(const GenEngine* e) { return e->host.chnOk && e->host.projN == 0 && e->fb_list; }
static bool chn_wide_on(const GenEngine* e) { return chn_on(e) && e->host.chnWide && e->fb2_list; }
// the kernels that read the key-sorted payload with every attribute word of the event
static bool pay_on(const GenEngine* e) { return abs_on(e) || cnt_on(e) || chn_on(e); }

// both filters of the absent-tail shape are decoded compares (GenPre.ff): the kernel variants without the interpreter
static bool abs_ff(const GenEngine* e) {
    const GenPre& f0 = e->host.pre[e->host.absP0];
    const GenPre& f1 = e->host.pre[e->host.absP1];
    return (f0.flen == 0 || f0.ff.on) && (f1.flen == 0 || f1.ff.on);
}

static void launch_gen(GenEngine* e, GenArgs a, int which) {
    const uint32_t blocks = (e->K + 63) / 64;
    a.kpl = gen_kpl(e->K);
    const GenArgs& ap = a;   // (by value in the kernel arguments: no upload per launch)
    hipEvent_t t0 = (e->timing && which != GEN_L_DEADLINES) ? e->ev() : nullptr;
    const bool fb = (a.mode & (GEN_M_KEYLIST | GEN_M_NOPAIRS)) != 0;
    if (which == GEN_L_TIMERS)
        hipLaunchKernelGGL(k_gen_timers, dim3(fb ? GEN_FB_BLOCKS : e->host.partitioned ? std::min(blocks, GEN_TIMER_BLOCKS) : 1u),
                           dim3(64), 0, e->stream, ap);
    else if (which == GEN_L_DEADLINES) hipLaunchKernelGGL(k_gen_deadlines, dim3(blocks), dim3(64), 0, e->stream, ap);
    else if (which == GEN_L_ABSD_BATCH || which == GEN_L_ABSD_TIMERS) {
        // one wave per handed-over key (a fixed grid striding over the list, whose length is on the device); the
        // variant without the interpreter when both filters are decoded compares
        const bool ff = abs_ff(e);
        const AbsKernel k = which == GEN_L_ABSD_BATCH ? (ff ? kAbsdBatchF : kAbsdBatch)[e->host.absNW]
                                                       : (ff ? kAbsdTimersF : kAbsdTimers)[e->host.absNW];
        hipLaunchKernelGGL(k, dim3(GEN_FB_BLOCKS), dim3(64), (unsigned)absd_lds(e), e->stream, ap);
    }
    else if (which == GEN_L_CHN_BATCH) {   // one lane per key, then the waves' counter rows
        hipLaunchKernelGGL(kChnBatch[e->host.chnN - 2][e->host.chnKW], dim3(blocks), dim3(64), 0, e->stream, ap);
        hipLaunchKernelGGL(k_gen_stats_reduce, dim3(GST_N, std::min<uint32_t>((blocks + 1023) / 1024, 16u)), dim3(256),
                           0, e->stream, e->wstats, blocks, e->stats);
    }
    else if (which == GEN_L_CHN_WIDE) {   // a fixed grid striding the hand-over list (its length is on the device)
        const uint32_t wb = std::min<uint32_t>(GEN_FB_BLOCKS, blocks);
        hipLaunchKernelGGL(kChnWide[e->host.chnN - 2][e->host.chnKW], dim3(wb), dim3(64), 0, e->stream, ap);
        hipLaunchKernelGGL(k_gen_stats_reduce, dim3(GST_N, 1), dim3(256), 0, e->stream, e->wstats, wb, e->stats);
    }
    else if (which == GEN_L_ABS_BATCH || which == GEN_L_ABS_TIMERS || which == GEN_L_CNT_BATCH) {
        // one lane per key / possible due slot (the due count is on the device); then the waves' counter rows
        // (the absent kernel's variant for decoded-compare filters when both of its filters are; the occupancy-4
        // build when the launch's waves fit the chip at 4 per SIMD but not at 3)
        const bool ff = abs_ff(e);
        const uint32_t NW = e->host.absNW;
        const bool occ4 = e->abs_occ4 && NW <= 3 && blocks > 12u * e->ncu && blocks <= 16u * e->ncu;
        const unsigned lds = 0;
        hipLaunchKernelGGL(which == GEN_L_ABS_BATCH   ? (ff ? (occ4 ? kAbsBatchF4[NW] : kAbsBatchF[NW]) : kAbsBatch[NW])
                           : which == GEN_L_CNT_BATCH ? kCntBatch[NW]
                                                      : (occ4 ? kAbsTimers4[NW] : kAbsTimers[NW]),
                           dim3(blocks), dim3(64), lds, e->stream, ap);
        hipLaunchKernelGGL(k_gen_stats_reduce, dim3(GST_N, std::min<uint32_t>((blocks + 1023) / 1024, 16u)), dim3(256),
                           0, e->stream, e->wstats, blocks, e->stats);
    }
    else hipLaunchKernelGGL(k_gen_batch, dim3(fb ? GEN_FB_BLOCKS : (e->K + 64u * a.kpl - 1) / (64u * a.kpl)), dim3(64), 0,
                            e->stream, ap);
    GH_OK(hipGetLastError());
    if (t0) e->spans.push_back({t0, e->ev(), 1});
}

// largest key id of a host batch (branch-free, so it vectorises; range-checked after the H2D is queued)
static uint32_t sgd_max_key(const uint32_t* k, uint32_t n, bool skip_null) {
    uint32_t m = 0;
    if (skip_null)
        for (uint32_t i = 0; i < n; i++) m = (k[i] > m && k[i] != SG_KEY_NULL) ? k[i] : m;
    else
        for (uint32_t i = 0; i < n; i++) m = k[i] > m ? k[i] : m;
    return m;
}

int gen_push(GenEngine* e, const sg_batch* b, std::string& msg) {
    const GenProgram& G = e->host;
    (void)hipGetLastError();   // (a stale error of an unrelated earlier call on this thread: rocPRIM reads it)
    if (b->stream >= (uint32_t)G.nstreams) { msg = "stream index out of range"; return SG_ERR_INVALID; }
    if (b->n_cols != (uint32_t)G.nattr[b->stream]) { msg = "column count does not match the stream"; return SG_ERR_INVALID; }
    if (b->n == 0) return SG_OK;
    if (b->n > e->maxb) { msg = "batch larger than max_batch"; return SG_ERR_INVALID; }
    if (G.partitioned && !b->key) { msg = "partitioned query needs key ids"; return SG_ERR_INVALID; }
    if (e->held) { msg = "release the polled matches before pushing"; return SG_ERR_STATE; }
    const uint32_t n = (uint32_t)b->n;
    const bool dev = b->mem == SG_MEM_DEVICE;
    GenArgs a = e->args();
    a.b.n = n;
    a.b.stream = b->stream;
    a.b.seq_base = b->seq_base;
    a.b.ts = b->ts;
    if (!dev) {
        GH_OK(hipMemcpyAsync(e->b_ts, b->ts, (size_t)n * 8, hipMemcpyHostToDevice, e->stream));
        a.b.ts = e->b_ts;
    }
    for (uint32_t c = 0; c < b->n_cols; c++) {
        const int t = G.attrType[b->stream][c];
        if (dev) {
            a.b.col[c] = b->cols[c];
            a.b.nul[c] = b->nulls ? b->nulls[c] : nullptr;
        } else {
            GH_OK(hipMemcpyAsync(e->b_cols[c], b->cols[c], (size_t)n * type_size(t), hipMemcpyHostToDevice, e->stream));
            a.b.col[c] = e->b_cols[c];
            a.b.nul[c] = nullptr;
            if (b->nulls && b->nulls[c]) {
                GH_OK(hipMemcpyAsync(e->b_nulls[c], b->nulls[c], n, hipMemcpyHostToDevice, e->stream));
                a.b.nul[c] = e->b_nulls[c];
            }
        }
    }
    {   // per-key bounds, the raw-record counters and the hand-over lists' counts: one launch
        GenClearList cl;
        cl.add(e->seg_begin, (size_t)e->K * 4);
        cl.add(e->seg_end, (size_t)e->K * 4);
        cl.add(e->raw_count, 8 * GEN_RAWSEG);
        cl.add(e->t_multi, 4);
        if (pay_on(e)) cl.add(e->fb_n, 8);
        if ((abs_on(e) && absd_on(e)) || chn_wide_on(e)) cl.add(e->fb2_n, 8);
        GH_OK(cl.launch(e->stream));
    }
    if (G.partitioned) {
        const uint32_t* keys = b->key;
        if (!dev) {
            // the copy is queued first, so the host range check overlaps the DMA (pinned batches)
            GH_OK(hipMemcpyAsync(e->b_key, b->key, (size_t)n * 4, hipMemcpyHostToDevice, e->stream));
            keys = e->b_key;
            if (sgd_max_key(b->key, n, e->null_keys) >= e->K) {
                GH_OK(hipStreamSynchronize(e->stream));  // the queued copies read the caller's buffers
                msg = "key id outside [0, n_keys)";
                return SG_ERR_INVALID;
            }
        }
        hipEvent_t g0 = e->timing ? e->ev() : nullptr;
        // the register-window kernel's grouping carries the events' words through the sort (gathered in
        // arrival order in the first pass, so each key's events end up contiguous, instead of a random
        // gather per event in the walk); other engines sort batch positions
        PackSrc ps{};
        uint32_t W = 0;
        bool nul = false;
        if (pay_on(e)) {
            const int st = (int)b->stream;
            for (int c = 0; c < G.nattr[st] && W <= 4; c++) {
                const int t = G.attrType[st][c];
                const void* col = a.b.col[c];
                if (t == SG_T_LONG || t == SG_T_DOUBLE) {
                    if (W + 2 > 4) { W = 5; break; }
                    ps.p[W] = col; ps.kind[W++] = 1;
                    ps.p[W] = col; ps.kind[W++] = 2;
                } else {
                    if (W + 1 > 4) { W = 5; break; }
                    ps.p[W] = col;
                    ps.kind[W++] = t == SG_T_BOOL ? 3 : 0;
                }
                if (a.b.nul[c]) {
                    nul = true;
                    if (c < SGD_MAX_EVCOLS) ps.nul[c] = a.b.nul[c];
                    else W = 5;
                }
            }
            if (nul && W <= 4) {
                if (W + 1 > 4) W = 5;
                else { ps.p[W] = nullptr; ps.kind[W++] = 4; }
            }
            ps.ts = a.b.ts;
        }
        GroupArgs ga{};
        ga.n = n;
        ga.K = e->K;
        ga.drop_null = e->null_keys ? 1u : 0u;
        ga.keys = keys;
        ga.seg_begin = e->seg_begin;
        ga.seg_end = e->seg_end;
        ga.err = e->err;
        ga.s = e->pscr;
        // the register-window kernels' batches (count, absent): grouped by 64-key tile (two 7-bit passes), then split by key per tile
        // (k_cnt_split), instead of three 8-bit passes; while a batch has shown a tile of more than 2^14 events (one
        // wave splits a tile), the sorted grouping
        const bool fused = e->cnt_fused && !e->cnt_skewed && pay_on(e) && W >= 1 && W <= 4;
        e->cnt_fused_last = fused;
        if (fused) {
            ga.W = W;
            ga.src = ps;
            ga.out = e->tpay;
            ga.tile_bits = 6;
            GH_OK(sgd_group_tiles_fused(ga, e->tile_lo, e->stream));
            a.b.pay = e->pay;
            a.b.payStride = W + 2;
            a.b.payNull = nul ? 1u : 0u;
            a.b.sidx = e->pay;
            a.b.sidxStride = W + 2;
            a.b.tile_lo = e->tile_lo;
            a.b.tpay = e->tpay;
            a.b.tileMax = e->tile_max;
            a.b.seg_begin = e->seg_begin;
            a.b.seg_end = e->seg_end;
            hipLaunchKernelGGL(k_cnt_split, dim3(((e->K + 63) / 64 + 3) / 4), dim3(256), 0, e->stream, a);
            GH_OK(hipGetLastError());
            a.b.tile_lo = nullptr;
            a.b.tpay = nullptr;
            a.b.tileMax = nullptr;
        } else if (pay_on(e) && W >= 1 && W <= 4) {
            ga.W = W;
            ga.src = ps;
            ga.out = e->pay;
            GH_OK(sgd_group_sorted(ga, e->stream));
            a.b.pay = e->pay;
            a.b.payStride = W + 2;
            a.b.payNull = nul ? 1u : 0u;
            a.b.sidx = e->pay;  // (the general kernel over handed-over keys reads the positions from it)
            a.b.sidxStride = W + 2;
        } else {
            ga.W = 0;
            ga.out = e->sidx;
            GH_OK(sgd_group_sorted(ga, e->stream));
            a.b.sidx = e->sidx;
        }
        if (g0) e->spans.push_back({g0, e->ev(), 0});
    } else {
        GH_OK(hipMemcpyAsync(e->seg_end, &n, 4, hipMemcpyHostToDevice, e->stream));
        GH_OK(hipStreamSynchronize(e->stream));  // &n is a stack value
        a.b.sidx = nullptr;
    }
    a.b.seg_begin = e->seg_begin;
    a.b.seg_end = e->seg_end;
    a.o.nseg = GEN_RAWSEG;
    a.o.seg_cap = e->rawCap / GEN_RAWSEG;
    if (e->timing)  // sg_stats.live_at_batch_start (outside the batch kernel's span)
        hipLaunchKernelGGL(k_gen_live, dim3((e->K + 255) / 256), dim3(256), 0, e->stream, e->dprog, e->state, e->K,
                           e->stats + GST_LIVE0, (const uint32_t*)e->rec, e->seg_begin, e->seg_end);
    if (abs_on(e)) {
        // the register-window kernel, then the general kernel over the keys it handed over; this shape
        // emits nothing on events (an absent state's processAndReturn returns nothing; its matches come
        // from the timers), so there is no batch ordering
        a.fb_list = e->fb_list;
        a.fb_n = e->fb_n;
        a.fb_start = e->fb_start;
        launch_gen(e, a, GEN_L_ABS_BATCH);
        if (absd_on(e)) {  // the deep keys, one wave each; what they cannot hold goes on to the general kernel
            a.fb2_list = e->fb2_list;
            a.fb2_n = e->fb2_n;
            a.fb2_start = e->fb2_start;
            const uint32_t m0 = a.mode;
            if (e->absd_nochunk) a.mode |= GEN_M_NOCHUNK;   // (SG_NO_ABSD_CHUNK: the per-event walk only)
            launch_gen(e, a, GEN_L_ABSD_BATCH);
            a.mode = m0;
            a.fb_list = e->fb2_list;
            a.fb_n = e->fb2_n;
            a.fb_start = e->fb2_start;
        }
        a.mode = GEN_M_KEYLIST;
        launch_gen(e, a, GEN_L_BATCH);
        GH_OK(hipGetLastError());
        e->st.events += n;
        e->st.batches++;
        e->st.advance_launches++;
        if (!dev) GH_OK(hipStreamSynchronize(e->stream));
        return SG_OK;
    }
    if (cnt_on(e)) {
        // the register-window kernel, then the general kernel over the keys it handed over (whole runs);
        // both write raw records + per-trigger counts, ordered below
        a.fb_list = e->fb_list;
        a.fb_n = e->fb_n;
        a.fb_start = e->fb_start;
        a.mode = GEN_M_TFIRST;   // (this shape emits at most one match per event)
        launch_gen(e, a, GEN_L_CNT_BATCH);
        a.mode = GEN_M_KEYLIST | GEN_M_TFIRST;
    } else if (chn_on(e)) {
        // the chain kernel, then the general kernel over the keys it handed over (from the event where each stopped)
        a.fb_list = e->fb_list;
        a.fb_n = e->fb_n;
        a.fb_start = e->fb_start;
        launch_gen(e, a, GEN_L_CHN_BATCH);
        if (chn_wide_on(e)) {   // the keys it handed over, in the wide window; what that cannot hold goes on
            a.fb2_list = e->fb2_list;
            a.fb2_n = e->fb2_n;
            a.fb2_start = e->fb2_start;
            launch_gen(e, a, GEN_L_CHN_WIDE);
            a.fb_list = e->fb2_list;
            a.fb_n = e->fb2_n;
            a.fb_start = e->fb2_start;
        }
        a.mode = GEN_M_KEYLIST;
    }
    launch_gen(e, a, GEN_L_BATCH);
    // order: the batch's base + the exclusive prefix of the per-trigger counts + rank (k_gen_tsum / k_gen_tscan /
    // k_gen_order; the counts are reset by k_gen_order)
    const uint32_t nt = (n + GEN_OT - 1) / GEN_OT, nsup = (nt + GEN_OST - 1) / GEN_OST;
    hipLaunchKernelGGL(k_gen_tsum, dim3(nsup), dim3(1024), 0, e->stream, e->t_cnt, n, e->tile_pre, e->sup_sum);
    hipLaunchKernelGGL(k_gen_tscan, dim3(1), dim3(1024), 0, e->stream, e->sup_sum, nsup, e->sup_off, e->out.count, e->obase);
    const uint64_t maxRaw = e->rawCap;
    const unsigned scat_grid = (unsigned)std::min<uint64_t>((maxRaw + 255) / 256, 1024);
    if (a.mode & GEN_M_TFIRST) {
        // output-major gather of the one match per trigger; a trigger of a handed-over key that emitted several
        // (t_multi, set on the device) turns it off and every record is placed by (t_off, rank) instead
        hipLaunchKernelGGL(k_gen_order<true>, dim3(nt), dim3(256), 0, e->stream, e->raw, e->t_cnt, e->t_off, e->t_first,
                           e->tile_pre, e->sup_off, n, e->out, (const uint32_t*)e->t_multi,
                           (const unsigned long long*)e->obase);
        hipLaunchKernelGGL(k_gen_scatter, dim3(scat_grid), dim3(256), 0, e->stream, e->raw, e->raw_count,
                           e->rawCap / GEN_RAWSEG, (uint32_t)GEN_RAWSEG, e->t_off, e->out, (const uint32_t*)e->t_multi,
                           (const unsigned long long*)e->obase);
    } else {
        hipLaunchKernelGGL(k_gen_order<false>, dim3(nt), dim3(256), 0, e->stream, e->raw, e->t_cnt, e->t_off, e->t_first,
                           e->tile_pre, e->sup_off, n, e->out, (const uint32_t*)e->t_multi,
                           (const unsigned long long*)e->obase);
        hipLaunchKernelGGL(k_gen_scatter, dim3((unsigned)std::min<uint64_t>((maxRaw + 255) / 256, 4096)), dim3(256), 0,
                           e->stream, e->raw, e->raw_count, e->rawCap / GEN_RAWSEG, (uint32_t)GEN_RAWSEG, e->t_off, e->out,
                           (const uint32_t*)nullptr, (const unsigned long long*)e->obase);
    }
    GH_OK(hipGetLastError());
    e->st.events += n;
    e->st.batches++;
    e->st.advance_launches++;
    if (!dev) GH_OK(hipStreamSynchronize(e->stream));
    return SG_OK;
}

bool gen_keep_timer_heads(GenEngine* e, bool keep) {
    e->keep_heads = keep && e->keyorder;
    return e->keyorder;
}

void gen_timer_heads(const GenEngine* e, std::vector<uint32_t>& keys, std::vector<int64_t>& heads) {
    keys = e->head_keys;
    heads = e->head_t;
}

int gen_advance(GenEngine* e, int64_t t, std::string& msg) {
    const GenProgram& G = e->host;
    e->head_keys.clear();
    e->head_t.clear();
    if (G.playback) {
        // TimestampGeneratorImpl.setCurrentTimestamp ignores a time earlier than the last one
        if (e->advanced && t < e->lastEventTs) return SG_OK;
        e->lastEventTs = t;
    }
    if (G.nStartup == 0) {  // no absent state: the query has no timers, only the clock moves
        if (G.playback || !e->advanced || t > e->now) e->now = t;
        e->advanced = true;
        return SG_OK;
    }
    GenArgs a = e->args();
    a.now = t;         // the advance target (playback: the event clock)
    a.now0 = e->now;   // the clock before it (wall-clock callers run at their own times)
    {
        GenClearList cl;
        cl.add(e->raw_count, 8);
        cl.add(e->nvalid, 8);
        cl.add(e->tm.ndue, 8);
        if (abs_on(e)) cl.add(e->fb_n, 8);
        if (abs_on(e) && absd_on(e)) cl.add(e->fb2_n, 8);
        if (e->keyorder) cl.add(e->ctr, 32);
        GH_OK(cl.launch(e->stream));
    }
    if (G.partitioned) {  // the keys with a deadline <= t: one pass over nd[K]
        const uint32_t blocks = std::min<uint32_t>((e->K + 4095) / 4096, 1024u);
        hipLaunchKernelGGL(k_gen_due, dim3(blocks), dim3(256), 0, e->stream, e->tm.nd, e->K, t, e->tm.due, e->tm.ndue);
    }
    a.o.nseg = 1;
    a.o.seg_cap = e->rawCap;
    if (abs_on(e)) {  // the register-window sweep, then the general sweep over the keys it handed over
        a.fb_list = e->fb_list;
        a.fb_n = e->fb_n;
        a.fb_start = nullptr;
        launch_gen(e, a, GEN_L_ABS_TIMERS);
        a.mode = GEN_M_NOPAIRS;
        a.t.due = e->fb_list;
        a.t.ndue = e->fb_n;
        if (absd_on(e)) {
            a.fb2_list = e->fb2_list;
            a.fb2_n = e->fb2_n;
            a.fb2_start = nullptr;
            launch_gen(e, a, GEN_L_ABSD_TIMERS);
            a.t.due = e->fb2_list;
            a.t.ndue = e->fb2_n;
        }
        launch_gen(e, a, GEN_L_TIMERS);
    } else {
        launch_gen(e, a, GEN_L_TIMERS);
    }
    if (e->keyorder) {  // the A.10 check and the keys with matches, before the one host round trip
        const uint32_t blocks = std::min<uint32_t>((e->K + GEN_TPREP_BLOCK - 1) / GEN_TPREP_BLOCK, 1024u);
        hipLaunchKernelGGL(k_timer_prep, dim3(blocks), dim3(GEN_TPREP_BLOCK), 0, e->stream, e->tm.dpair_key,
                           e->tm.dpair_kid, e->tm.ndue, t, e->tm.kcnt, e->ht, e->htmask, e->ht_ins, e->rel, e->kid_c,
                           e->hkey_c, e->ctr);
        hipLaunchKernelGGL(k_ht_clear, dim3(blocks), dim3(GEN_TPREP_BLOCK), 0, e->stream, e->ht_ins, e->tm.ndue, e->ht);
    }
    unsigned long long nr = 0, ndue = 0, kctr[4] = {0, 0, 0, 0};
    GH_OK(hipMemcpyAsync(&nr, e->raw_count, 8, hipMemcpyDeviceToHost, e->stream));
    GH_OK(hipMemcpyAsync(&ndue, e->tm.ndue, 8, hipMemcpyDeviceToHost, e->stream));
    if (e->keyorder) GH_OK(hipMemcpyAsync(kctr, e->ctr, 32, hipMemcpyDeviceToHost, e->stream));
    GH_OK(hipStreamSynchronize(e->stream));
    bool check = false;
    bool collapse = false;
    if (e->keyorder) {
        // one listener: the keys that emitted sorted by queue head (TreeMultimap order of the listener's
        // collection, Scheduler.java:78-99) give the output order of their timer matches (each key's in
        // emission order).  Sort keys: 32-bit lags from the advance target when they fit (descending),
        // else the 64-bit heads.
        collapse = kctr[3] != 0;
        const size_t n = (size_t)kctr[2];
        if (n >= 1) {
            const dim3 g((unsigned)((n + 255) / 256));
            if (!kctr[1]) {
                int bits = 1;
                while (bits < 32 && (kctr[0] >> bits) != 0) bits++;
                GH_OK(sgd_sort_pairs(e->rel, e->srel, e->kid_c, e->skid, (uint32_t)n, (uint32_t)bits, false, true, e->pscr,
                                     e->stream));
            } else {
                GH_OK(sgd_sort_pairs(e->hkey_c, e->hkey_s, e->kid_c, e->skid, (uint32_t)n, 64, true, false, e->pscr,
                                     e->stream));
            }
            if (e->keep_heads) {  // (the sorted keys and their heads, for the multi-device merge)
                std::vector<uint32_t> rel(n);
                std::vector<unsigned long long> hk(n);
                e->head_keys.resize(n);
                GH_OK(hipMemcpyAsync(e->head_keys.data(), e->skid, n * 4, hipMemcpyDeviceToHost, e->stream));
                if (!kctr[1]) GH_OK(hipMemcpyAsync(rel.data(), e->srel, n * 4, hipMemcpyDeviceToHost, e->stream));
                else GH_OK(hipMemcpyAsync(hk.data(), e->hkey_s, n * 8, hipMemcpyDeviceToHost, e->stream));
                GH_OK(hipStreamSynchronize(e->stream));
                e->head_t.resize(n);
                for (size_t i = 0; i < n; i++)
                    e->head_t[i] = !kctr[1] ? t + 1 - (int64_t)rel[i] : (int64_t)(hk[i] ^ (1ull << 63));
            }
            hipLaunchKernelGGL(k_timer_cnt, g, dim3(256), 0, e->stream, e->skid, (uint64_t)n, e->tm.kcnt, e->kc);
            size_t st = e->kscan_tmp_bytes;
            GH_OK(rocprim::exclusive_scan(e->kscan_tmp, st, e->kc, e->koff_s, 0u, n, rocprim::plus<uint32_t>(), e->stream));
            hipLaunchKernelGGL(k_timer_off, g, dim3(256), 0, e->stream, e->skid, (uint64_t)n, e->koff_s, e->koff);
            if (nr > 0) {  // matches of the general kernels (raw records)
                const size_t m = (size_t)std::min<unsigned long long>(nr, e->rawCap);
                hipLaunchKernelGGL(k_timer_scatter, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, e->stream, e->raw,
                                   e->raw_count, e->koff, e->out);
            }
            if (e->tstage)  // matches k_abs_timers staged
                hipLaunchKernelGGL(k_timer_scatter_abs, g, dim3(256), 0, e->stream, e->skid, (uint64_t)n, e->tm.kcnt,
                                   e->koff, e->tstage, e->K, (uint32_t)G.pre[G.absP0].stateId, e->out);
            hipLaunchKernelGGL(k_timer_bump, dim3(1), dim3(1), 0, e->stream, e->out.count, e->kc, e->koff_s, (uint64_t)n);
            GH_OK(hipGetLastError());
        }
        nr = 0;  // ordered
    }
    if (!e->keyorder && G.partitioned && G.playback && ndue * (uint64_t)G.nStartup >= 2) {
        // the reference's listener collects the due (time, key) states in a
        // TreeMultimap whose value comparator is always 0 (Scheduler.java:78-89, 364-367), so of several
        // keys due at the same time only one (chosen by HashMap order) fires at this advance.  That
        // input has no defined result: detect it and fail instead of diverging silently.
        const size_t np = (size_t)(ndue * (uint64_t)G.nStartup);
        GH_OK(sgd_sort_pairs(e->tm.dpair_key, e->pair_key_s, e->tm.dpair_i, e->pair_i_s, (uint32_t)np, 64, true, false,
                             e->pscr, e->stream));
        hipLaunchKernelGGL(k_gen_collapse, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, e->stream, e->pair_key_s,
                           e->pair_i_s, (uint64_t)np, e->err);
        check = true;
    }
    if (nr > 0) {
        // the timer matches in the reference's order: playback by (listener, queue head), wall clock by
        // (run time, key); within one key in emission order
        const size_t n = (size_t)std::min<unsigned long long>(nr, e->rawCap);
        hipLaunchKernelGGL(k_gen_iota, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, e->order_in, (uint64_t)n);
        size_t tmp = e->msort_tmp_bytes;
        TimerLess lt{e->tk1, e->tk2, e->tk3};
        GH_OK(rocprim::merge_sort(e->msort_tmp, tmp, e->order_in, e->order_out, n, lt, e->stream));
        hipLaunchKernelGGL(k_gen_scatter_timers, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, e->raw,
                           e->order_out, e->nvalid, e->out);
        hipLaunchKernelGGL(k_gen_bump, dim3(1), dim3(1), 0, e->stream, e->out.count, e->t_cnt, e->t_off, 1u,
                           (const unsigned long long*)e->nvalid);
        GH_OK(hipGetLastError());
    }
    if (G.playback || !e->advanced || t > e->now) e->now = t;
    e->advanced = true;
    if (collapse) {
        msg = "two partition keys share a timer due time at one clock advance (reference Scheduler collapse "
              "quirk, SURVEY A.10): input not supported";
        return SG_ERR_UNSUPPORTED;
    }
    if (check) {
        uint32_t err = 0;
        GH_OK(hipMemcpyAsync(&err, e->err, 4, hipMemcpyDeviceToHost, e->stream));
        GH_OK(hipStreamSynchronize(e->stream));
        if (err & GERR_COLLAPSE) {
            const uint32_t rest = err & ~(uint32_t)GERR_COLLAPSE;
            GH_OK(hipMemcpy(e->err, &rest, 4, hipMemcpyHostToDevice));
            msg = "two partition keys share a timer due time at one clock advance (reference Scheduler collapse "
                  "quirk, SURVEY A.10): input not supported";
            return SG_ERR_UNSUPPORTED;
        }
    }
    return SG_OK;
}

int gen_poll(GenEngine* e, uint32_t mem, sg_match_batch* out, std::string& msg) {
    if (e->held) { msg = "previous matches not released"; return SG_ERR_STATE; }
    // the count, the error word and the largest tile gathered by one launch and copied to the host at once (three
    // copies were three blit launches); the count is reset there for the next window unless this poll fails
    if (!e->d_stat) e->d_stat = e->dalloc<unsigned long long>(4);
    hipLaunchKernelGGL(k_gen_status, dim3(1), dim3(64), 0, e->stream, e->out.count, (const uint32_t*)e->err,
                       (const uint32_t*)e->tile_max, e->out.cap,
                       (uint32_t)(GERR_KEY | GERR_CAP | GERR_MATCHCAP | GERR_CHAIN | GERR_REF), e->d_stat);
    GH_OK(hipGetLastError());
    e->h_stat.resize(4);
    GH_OK(hipMemcpyAsync(e->h_stat.data(), e->d_stat, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                         e->stream));
    GH_OK(hipStreamSynchronize(e->stream));
    const unsigned long long n = e->h_stat.data()[0];
    const uint32_t err = (uint32_t)e->h_stat.data()[1];
    const uint32_t tmax = (uint32_t)e->h_stat.data()[2];
    if (tmax > (1u << 14)) e->cnt_skewed = true;  // (one wave splits a tile: skewed streams take the sorted grouping)
    if (err & GERR_KEY) {
        // reported once: the events with valid keys were processed, the others dropped
        const uint32_t rest = err & ~(uint32_t)GERR_KEY;
        GH_OK(hipMemcpy(e->err, &rest, 4, hipMemcpyHostToDevice));
        msg = "a batch carried key ids outside [0, n_keys) (those events were dropped)";
        return SG_ERR_INVALID;
    }
    if (err & GERR_CAP) { msg = "a partition key exceeded the engine's per-key capacity (partial_capacity)"; return SG_ERR_CAPACITY; }
    if ((err & GERR_MATCHCAP) || n > e->mcap) { msg = "more matches than match_capacity between two polls"; return SG_ERR_CAPACITY; }
    if (err & GERR_CHAIN) { msg = "a count state chain is longer than the output chain capacity"; return SG_ERR_CAPACITY; }
    if (err & GERR_REF) { msg = "internal state error in the device engine"; return SG_ERR_STATE; }
    const GenProgram& G = e->host;
    const size_t ns = (size_t)G.nslots, mc = G.MC;
    out->n = n;
    out->n_slots = (uint32_t)ns;
    out->max_chain = (uint32_t)mc;
    out->reserved = 0;
    if (mem == SG_MEM_DEVICE) {
        out->trigger_seq = e->out.trig;
        out->slot_seq = e->out.slot;
        out->key = e->out.key;
        out->ts = e->out.ts;
        out->chain_len = e->out.len;
        out->mem = SG_MEM_DEVICE;
    } else {
        e->h_trig.resize(n);
        e->h_slot.resize(n * ns * mc);
        e->h_key.resize(n);
        e->h_ts.resize(n);
        e->h_len.resize(n * ns);
        if (n) {
            GH_OK(hipMemcpyAsync(e->h_trig.data(), e->out.trig, n * 8, hipMemcpyDeviceToHost, e->stream));
            GH_OK(hipMemcpyAsync(e->h_slot.data(), e->out.slot, n * ns * mc * 8, hipMemcpyDeviceToHost, e->stream));
            GH_OK(hipMemcpyAsync(e->h_key.data(), e->out.key, n * 4, hipMemcpyDeviceToHost, e->stream));
            GH_OK(hipMemcpyAsync(e->h_ts.data(), e->out.ts, n * 8, hipMemcpyDeviceToHost, e->stream));
            GH_OK(hipMemcpyAsync(e->h_len.data(), e->out.len, n * ns * 4, hipMemcpyDeviceToHost, e->stream));
            GH_OK(hipStreamSynchronize(e->stream));
        }
        out->trigger_seq = e->h_trig.data();
        out->slot_seq = e->h_slot.data();
        out->key = e->h_key.data();
        out->ts = e->h_ts.data();
        out->chain_len = e->h_len.data();
        out->mem = SG_MEM_HOST;
    }
    e->held = true;   // (the count was reset by k_gen_status)
    e->polled = n;
    return SG_OK;
}

int gen_set_projection(GenEngine* e, const uint32_t* code, uint32_t words, const uint32_t* pc, const uint32_t* len,
                       const uint32_t* types, uint32_t n, std::string& msg) {
    GenProgram& G = e->host;
    if (e->st.batches != 0 || e->held) { msg = "set the projection before the first push"; return SG_ERR_STATE; }
    if (G.projN) { msg = "the projection is already set"; return SG_ERR_STATE; }
    if (n > GEN_MAXPROJ) { msg = "too many select items for the device projection"; return SG_ERR_UNSUPPORTED; }
    if (G.ncode + words > GEN_MAXCODE) { msg = "select list too long for the device projection"; return SG_ERR_UNSUPPORTED; }
    // roles (siddhi_gpu_ir.h): aggregator arguments, then the select list, then at most one `having`
    uint32_t A = 0, S = 0, H = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (pc[i] + len[i] > words) { msg = "projection item outside its code"; return SG_ERR_INVALID; }
        if (types[i] & SG_PROJ_AGG_ITEM) {
            const uint32_t fn = (types[i] >> 8) & 0xffu;
            if (S || H || fn < SG_AGG_COUNT || fn > SG_AGG_MAX) { msg = "malformed aggregator item"; return SG_ERR_INVALID; }
            A++;
        } else if (types[i] & SG_PROJ_HAVING) {
            if (H) { msg = "more than one having item"; return SG_ERR_INVALID; }
            H = 1;
        } else {
            if (H) { msg = "select items after the having item"; return SG_ERR_INVALID; }
            S++;
        }
    }
    if (A > GEN_MAXAGG) { msg = "too many aggregators for the device projection"; return SG_ERR_UNSUPPORTED; }
    for (uint32_t i = 0; i < n; i++) {  // every opcode known, every slot in range
        for (uint32_t w = pc[i]; w < pc[i] + len[i];) {
            const uint32_t op = code[w] & 0xffu, b = (code[w] >> 16) & 0xffu;
            const bool known = op == SG_OP_VAR || op == SG_OP_CONST || op == SG_OP_CVT || op == SG_OP_ISNULL_EV ||
                               (op >= SG_OP_ADD && op <= SG_OP_MOD) || (op >= SG_OP_EQ && op <= SG_OP_LE) ||
                               (op >= SG_OP_AND && op <= SG_OP_ISNULL) || op == SG_OP_IFELSE;
            if (!known) { msg = "unknown opcode in the projection"; return SG_ERR_INVALID; }
            const uint32_t ow = (op == SG_OP_VAR || op == SG_OP_CONST) ? 3 : (op == SG_OP_ISNULL_EV ? 2 : 1);
            if (w + ow > pc[i] + len[i]) { msg = "projection item truncated"; return SG_ERR_INVALID; }
            if (op == SG_OP_VAR && (b == SG_PROJ_SLOT_AGG || b == SG_PROJ_SLOT_OUT)) {
                const uint32_t x = code[w + 1];
                if (b == SG_PROJ_SLOT_AGG ? (i < A || x >= A) : (!(H && i == n - 1) || x >= S)) {
                    msg = "projection reads an aggregator or output item it cannot see";
                    return SG_ERR_INVALID;
                }
            } else if ((op == SG_OP_VAR || op == SG_OP_ISNULL_EV) && b >= (uint32_t)G.nslots) {
                msg = "projection reads a slot the query does not have";
                return SG_ERR_INVALID;
            }
            w += ow;
        }
    }
    memcpy(G.code + G.ncode, code, (size_t)words * 4);
    for (uint32_t i = 0; i < n; i++) {
        G.projPc[i] = G.ncode + pc[i];
        G.projLen[i] = len[i];
        G.projType[i] = types[i];
    }
    G.ncode += words;
    G.projN = n;
    G.projAgg = A;
    G.projOff = e->recWords;
    e->recWords += 3 * (S + H);
    if (A) {  // the aggregators' per-key state joins the key blocks (no push yet: all zero)
        G.offAgg = G.blockWords;
        G.blockWords = (G.blockWords + 5 * A + (1u << GEN_GRAN_LOG2) - 1u) & ~((1u << GEN_GRAN_LOG2) - 1u);
        e->state = e->dalloc<uint32_t>((size_t)G.blockWords * e->K);
        GH_OK(hipMemsetAsync(e->state, 0, (size_t)G.blockWords * e->K * 4, e->stream));
    }
    e->raw = e->dalloc<uint32_t>(e->rawCap * e->recWords);  // (the smaller record buffer is freed at destroy)
    e->out.recWords = e->recWords;
    e->out.pval = e->dalloc<uint64_t>(e->mcap * (S + H));
    e->out.pnull = e->dalloc<uint8_t>(e->mcap * (S + H));
    e->out.projN = S + H;
    e->out.projOff = G.projOff;
    GH_OK(hipStreamSynchronize(e->stream));  // no kernel reads the program while it changes
    GH_OK(hipMemcpy(e->dprog, &G, sizeof(GenProgram), hipMemcpyHostToDevice));
    return SG_OK;
}

int gen_get_projection(GenEngine* e, uint32_t mem, sg_projection* out, std::string& msg) {
    if (!e->held) { msg = "poll the matches first"; return SG_ERR_STATE; }
    const uint32_t n = e->out.projN;   // output items: select list + having
    if (!e->host.projN) { msg = "no projection set"; return SG_ERR_STATE; }
    out->n = e->polled;
    out->n_items = n;
    if (mem == SG_MEM_DEVICE) {  // item i of match m at i * capacity + m
        if (e->polled && n > 1) { msg = "device projection rows are capacity-strided: poll to host"; return SG_ERR_INVALID; }
        out->value = e->out.pval;
        out->null = e->out.pnull;
        out->mem = SG_MEM_DEVICE;
        return SG_OK;
    }
    const size_t m = (size_t)e->polled;
    e->h_pval.resize(m * n);
    e->h_pnull.resize(m * n);
    for (uint32_t i = 0; i < n && m; i++) {
        GH_OK(hipMemcpyAsync(e->h_pval.data() + i * m, e->out.pval + (size_t)i * e->mcap, m * 8, hipMemcpyDeviceToHost,
                             e->stream));
        GH_OK(hipMemcpyAsync(e->h_pnull.data() + i * m, e->out.pnull + (size_t)i * e->mcap, m, hipMemcpyDeviceToHost,
                             e->stream));
    }
    GH_OK(hipStreamSynchronize(e->stream));
    out->value = e->h_pval.data();
    out->null = e->h_pnull.data();
    out->mem = SG_MEM_HOST;
    return SG_OK;
}

void gen_release(GenEngine* e) { e->held = false; }

void gen_stats(GenEngine* e, sg_stats* out) {
    unsigned long long s[GST_N];
    GH_OK(hipMemcpyAsync(s, e->stats, sizeof(s), hipMemcpyDeviceToHost, e->stream));
    unsigned long long* live = e->live;
    GH_OK(hipMemsetAsync(live, 0, 8, e->stream));
    hipLaunchKernelGGL(k_gen_live, dim3((e->K + 255) / 256), dim3(256), 0, e->stream, e->dprog, e->state, e->K, live,
                       (const uint32_t*)e->rec);
    unsigned long long lv = 0;
    GH_OK(hipMemcpyAsync(&lv, live, 8, hipMemcpyDeviceToHost, e->stream));
    GH_OK(hipStreamSynchronize(e->stream));
    for (auto& x : e->spans) {
        float ms = 0.f;
        GH_OK(hipEventElapsedTime(&ms, x.a, x.b));
        (x.which == 0 ? e->st.group_ns : e->st.advance_ns) += (uint64_t)((double)ms * 1e6);
        (void)hipEventDestroy(x.a);
        (void)hipEventDestroy(x.b);
    }
    e->spans.clear();
    *out = e->st;
    out->live_at_batch_start = s[GST_LIVE0];
    out->partials_scanned = s[GST_SCANNED];
    out->partials_created = s[GST_CREATED];
    out->matches = s[GST_MATCHES];
    out->keys_touched = s[GST_KEYS];
    out->window_spills = s[GST_SPILLS];
    out->partials_live = lv;
}

void gen_flush_deep(GenEngine* e, bool rec = true);

uint64_t gen_min_seq(GenEngine* e) {
    gen_flush_deep(e, false);   // (k_gen_min_seq reads the records in place)
    if (!e->minseq) e->minseq = e->dalloc<unsigned long long>(1);
    unsigned long long* m = e->minseq;
    unsigned long long h = ~0ull;
    GH_OK(hipMemcpyAsync(m, &h, 8, hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_gen_min_seq, dim3((e->K + 255) / 256), dim3(256), 0, e->stream, e->dprog, e->state, e->K, m,
                       (const uint32_t*)e->rec);
    GH_OK(hipMemcpyAsync(&h, m, 8, hipMemcpyDeviceToHost, e->stream));
    GH_OK(hipStreamSynchronize(e->stream));
    return h;
}

// the kernels a push and an advance dispatch (sg_engine_describe), in launch order
std::string gen_describe(const GenEngine* e) {
    const GenProgram& G = e->host;
    const std::string nw = std::to_string(G.absNW);
    std::string push, adv;
    if (abs_on(e)) {
        const GenPre& f0 = G.pre[G.absP0];
        const GenPre& f1 = G.pre[G.absP1];
        const bool ff = (f0.flen == 0 || f0.ff.on) && (f1.flen == 0 || f1.ff.on);
        const uint32_t blocks = (e->K + 63) / 64;
        const bool occ4 = e->abs_occ4 && G.absNW <= 3 && blocks > 12u * e->ncu && blocks <= 16u * e->ncu;
        push = (ff ? (occ4 ? "k_abs_batchf4_" : "k_abs_batchf_") : "k_abs_batch_") + nw + " (register window, lane per key)";
        adv = (occ4 ? "k_abs_timers4_" : "k_abs_timers_") + nw + " (register window)";
        if (absd_on(e)) {
            push += (ff ? " + k_absd_batchf_" : " + k_absd_batch_") + nw + " (deep keys, wave per key)";
            adv += (ff ? " + k_absd_timersf_" : " + k_absd_timers_") + nw + " (deep keys)";
        }
        push += " + k_gen_batch (keys handed over)";
        adv += " + k_gen_timers (keys handed over)";
    } else if (cnt_on(e)) {
        push = "k_cnt_batch_" + nw + " (register window, lane per key) + k_gen_batch (keys handed over)";
    } else if (chn_on(e)) {
        push = "k_chn_batch_" + std::to_string(G.chnN - 1) + "_" + std::to_string(G.chnKW) +
               " (chained states, register window, lane per key) + " +
               (chn_wide_on(e) ? "k_chn_wide_" + std::to_string(G.chnN - 1) + "_" + std::to_string(G.chnKW) +
                                     " (the keys handed over, wide window) + "
                               : std::string()) +
               "k_gen_batch (keys handed over)";
    } else {
        push = "k_gen_batch (general interpreter, lane per key)";
        if (G.nStartup > 0) adv = "k_gen_timers (general interpreter)";
    }
    if (e->cnt_fused_last)
        push = "k_part_hist + k_part_scan + k_part_scatter x2 + k_tile_bounds (grouping by 64-key tile) + k_cnt_split "
               "(key split per tile); " + push;
    return "push: " + push + (adv.empty() ? std::string() : "; advance: " + adv);
}

void gen_synchronize(GenEngine* e) { GH_OK(hipStreamSynchronize(e->stream)); }

// Persistence of the device NFA state (the reference snapshots every pre-state
// processor's pending / newAndEvery lists and absent-state flags per partition key,
// StreamPreStateProcessor.java:450-469, CountPreStateProcessor.java:206-219,
// AbsentStreamPreStateProcessor.java:328-341).  Here all of that, the per-key StateEvent/StreamEvent
// pools and the timer queues live in the key-interleaved state blocks, so the image is the blocks plus
// the engine clock.  Emitted matches are output, not state: both calls require that none are waiting
// to be polled (the reference delivers callbacks before a snapshot completes).
// one thread per (listed key, block word): word w of key k lives at gen_at(K, words, split, k, w)
__global__ void __launch_bounds__(256) k_gen_reset(const uint32_t* __restrict__ keys, uint32_t n, uint32_t words,
                                                   uint32_t split, uint32_t K, uint32_t* __restrict__ state) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)n * words) return;
    const uint32_t w = (uint32_t)(i / n), k = keys[i % n];
    if (k < K) state[gen_at(K, words, split, k, w)] = 0u;  // ids were range-checked by sg_reset_keys; never write outside
}

int gen_reset_keys(GenEngine* e, const uint32_t* keys, uint32_t n, std::string& msg) {
    (void)msg;
    if (n == 0 || !e->host.partitioned) return SG_OK;
    const uint64_t total = (uint64_t)n * e->host.blockWords;
    hipLaunchKernelGGL(k_gen_reset, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, e->stream, keys, n,
                       (uint32_t)e->host.blockWords, (uint32_t)e->host.offST, e->K, e->state);
    if (e->tm.nd)
        hipLaunchKernelGGL(k_gen_nd_reset, dim3((n + 255) / 256), dim3(256), 0, e->stream, keys, n, e->K, e->tm.nd);
    GH_OK(hipGetLastError());
    return SG_OK;
}

uint64_t gen_state_words(const GenEngine* e) { return (uint64_t)e->host.blockWords * e->K; }

static bool gen_outputs_pending(GenEngine* e) {
    unsigned long long n = 0;
    GH_OK(hipMemcpyAsync(&n, e->out.count, 8, hipMemcpyDeviceToHost, e->stream));
    GH_OK(hipStreamSynchronize(e->stream));
    return n != 0;
}

// every key whose lists live in the deep store (GEN_W0_DEEP) written back to its block: before anything reads
// the blocks' lists on the host or in a kernel that does not know the deep store
void gen_flush_deep(GenEngine* e, bool rec) {
    if (e->rec && rec) {   // the register-window kernels' records
        GenArgs a = e->args();
        const GenArgs& ap = a;
        hipLaunchKernelGGL(e->host.cntOk ? kCntFlush[e->host.absNW] : kAbsFlush[e->host.absNW], dim3((e->K + 63) / 64),
                           dim3(64), 0, e->stream, ap);
        GH_OK(hipGetLastError());
    }
    if (!e->deep || !absd_on(e)) return;
    GenArgs a = e->args();
    const GenArgs& ap = a;
    hipLaunchKernelGGL(kAbsdFlush[e->host.absNW], dim3(std::min<uint32_t>(e->K, 4096u)), dim3(64),
                       (unsigned)absd_lds(e), e->stream, ap);
    GH_OK(hipGetLastError());
}

int gen_snapshot(GenEngine* e, uint32_t* words, GenClock* clk, std::string& msg) {
    if (e->held) { msg = "release the polled matches before a snapshot"; return SG_ERR_STATE; }
    if (gen_outputs_pending(e)) { msg = "poll the emitted matches before a snapshot"; return SG_ERR_STATE; }
    gen_flush_deep(e);
    GH_OK(hipMemcpyAsync(words, e->state, gen_state_words(e) * 4, hipMemcpyDeviceToHost, e->stream));
    GH_OK(hipStreamSynchronize(e->stream));
    clk->now = e->now;
    clk->last_event_ts = e->lastEventTs;
    clk->advanced = e->advanced ? 1u : 0u;
    clk->pad = 0;
    return SG_OK;
}

int gen_restore(GenEngine* e, const uint32_t* words, const GenClock& clk, std::string& msg) {
    if (e->held) { msg = "release the polled matches before a restore"; return SG_ERR_STATE; }
    if (gen_outputs_pending(e)) { msg = "poll the emitted matches before a restore"; return SG_ERR_STATE; }
    GH_OK(hipMemcpyAsync(e->state, words, gen_state_words(e) * 4, hipMemcpyHostToDevice, e->stream));
    if (e->tm.nd) launch_gen(e, e->args(), GEN_L_DEADLINES);  // the timers' due index from the restored state
    GH_OK(hipStreamSynchronize(e->stream));
    e->now = clk.now;
    e->lastEventTs = clk.last_event_ts;
    e->advanced = clk.advanced != 0;
    return SG_OK;
}

// ---- the per-key state in the reference's per-state-processor form (state_doc.h) -----------------------
// Decoded from / encoded into the interleaved state blocks on the host (word w of key k at w * K + k):
// every initialised key's processors (flags, absent-state times, pending / newAndEvery lists, timer queue,
// wall-clock caller) with the StateEvents and StreamEvents the lists reach.  Import replaces the whole
// state (keys absent from the document become never-seen) and recomputes the refcounts and free bitmaps
// from the references the document holds.
int gen_state_export(GenEngine* e, SdDoc& d, std::string& msg) {
    const GenProgram& G = e->host;
    const uint64_t K = e->K;
    std::vector<uint32_t> S(gen_state_words(e));
    GenClock clk{};
    const int rc = gen_snapshot(e, S.data(), &clk, msg);
    if (rc != SG_OK) return rc;
    auto W = [&](uint32_t k, uint32_t w) -> uint32_t { return S[gen_il(K, k, w)]; };
    auto R64 = [&](uint32_t k, uint32_t w) -> int64_t {
        return (int64_t)((uint64_t)W(k, w) | ((uint64_t)W(k, w + 1) << 32));
    };
    d.n_procs = (uint32_t)G.nprocs;
    d.n_slots = (uint32_t)G.nslots;
    for (int p = 0; p < G.nprocs; p++)
        d.desc.push_back(SdProcDesc{(uint32_t)G.pre[p].kind, G.pre[p].absent ? 1u : 0u, (uint32_t)G.pre[p].stateId});
    d.now = clk.now;
    d.last_event_ts = clk.last_event_ts;
    d.clock_flags = clk.advanced ? 1u : 0u;
    for (uint32_t k = 0; k < K; k++) {
        if (!(W(k, 0) & 1u)) continue;
        SdKeyBuilder<uint32_t, uint32_t> B;
        B.k.key = k;
        std::function<uint32_t(uint32_t, int)> visit_ev = [&](uint32_t ev, int slot) -> uint32_t {
            bool fresh;
            const uint32_t i = B.stream(ev, fresh);
            if (!fresh) return i;
            const uint32_t base = G.offSE + ev * G.seWords;
            SdStream x;
            x.seq = (uint64_t)R64(k, base + SE_SEQ);
            x.ts = R64(k, base + SE_TS);
            x.null_bits = W(k, base + SE_NULL);
            if (x.null_bits != 0xffffffffu) {
                const int st = G.slotStream[slot];
                const int na = G.nattr[st];
                for (int a = 0; a < na; a++) {  // (32-bit types: the low word; the kernel leaves the high one)
                    const int32_t t = G.attrType[st][a];
                    const uint32_t w = base + SE_ATTR + 2 * (uint32_t)a;
                    x.attr.push_back((t == SG_T_LONG || t == SG_T_DOUBLE) ? (uint64_t)R64(k, w) : (uint64_t)W(k, w));
                }
                x.present = na >= 32 ? 0xffffffffu : ((1u << na) - 1u);
                x.null_bits &= x.present;
            }
            B.k.streams[i] = x;
            return i;
        };
        auto visit_st = [&](uint32_t st) -> uint32_t {
            bool fresh;
            const uint32_t i = B.state(st, fresh);
            if (!fresh) return i;
            const uint32_t base = G.offST + st * G.stWords;
            SdState x;
            x.ts = R64(k, base + ST_TS);
            x.type = W(k, base + ST_TYPE);
            x.chains.resize(G.nslots);
            for (int sl = 0; sl < G.nslots; sl++) {
                uint32_t ev = W(k, base + ST_SLOTS + (uint32_t)sl);
                for (uint32_t guard = 0; ev != GEN_NIL && guard <= G.SECAP; guard++) {
                    x.chains[sl].push_back(visit_ev(ev, sl));
                    ev = W(k, G.offSE + ev * G.seWords + SE_NEXT);
                }
            }
            B.k.states[i] = x;
            return i;
        };
        for (int p = 0; p < G.nprocs; p++) {
            const uint32_t ks = G.offKS + (uint32_t)p * G.ksWords;
            const uint32_t f = W(k, ks + KS_FLAGS);
            SdProc P;
            P.flags = ((f & GF_INIT) ? (uint32_t)SD_INITIALIZED : 0u) | ((f & GF_STARTED) ? (uint32_t)SD_STARTED : 0u) |
                      ((f & GF_SUCCESS) ? (uint32_t)SD_SUCCESS : 0u) | ((f & GF_SSRESET) ? (uint32_t)SD_SSRESET : 0u) |
                      ((f & GF_INACTIVE) ? 0u : (uint32_t)SD_ACTIVE);
            P.last_scheduled = R64(k, ks + KS_LST);
            P.last_arrival = R64(k, ks + KS_LAT);
            for (int which = 0; which < 2; which++) {
                const uint32_t n = W(k, ks + KS_PLEN + (uint32_t)which);
                for (uint32_t i = 0; i < n && i < G.L; i++) {
                    const uint32_t st = visit_st(W(k, ks + KS_LISTS + (uint32_t)which * G.L + i));
                    (which ? P.newev : P.pending).push_back(st);
                }
            }
            const uint32_t h = W(k, ks + KS_QHEAD), q = W(k, ks + KS_QLEN);
            for (uint32_t i = 0; i < q && i < G.Q; i++) P.queue.push_back(R64(k, ks + KS_LISTS + 2 * G.L + 2 * ((h + i) % G.Q)));
            P.running = (f & GF_RUNNING) ? 1u : 0u;
            P.fire_at = P.running ? R64(k, ks + KS_FIRE) : 0;
            P.order = W(k, ks + KS_ORDER);
            B.k.procs.push_back(P);
        }
        sd_rank_orders(B.k);
        d.keys.push_back(std::move(B.k));
    }
    return SG_OK;
}

int gen_state_import(GenEngine* e, const SdDoc& d, std::string& msg) {
    const GenProgram& G = e->host;
    const uint64_t K = e->K;
    bool same = d.n_procs == (uint32_t)G.nprocs && d.n_slots == (uint32_t)G.nslots;
    for (int p = 0; same && p < G.nprocs; p++)
        same = d.desc[p] == SdProcDesc{(uint32_t)G.pre[p].kind, G.pre[p].absent ? 1u : 0u, (uint32_t)G.pre[p].stateId};
    if (!same) {
        msg = "state document of a different query shape";
        return SG_ERR_INVALID;
    }
    std::vector<uint32_t> S(gen_state_words(e), 0u);
    auto W = [&](uint32_t k, uint32_t w) -> uint32_t& { return S[gen_il(K, k, w)]; };
    if (G.projAgg) {
        // the device aggregators' running values (QuerySelector state, not pattern state: the document
        // does not carry them) stay as they are, as the two-state engine's import leaves its aggregators
        std::vector<uint32_t> cur(gen_state_words(e));
        GenClock c0{};
        const int rc = gen_snapshot(e, cur.data(), &c0, msg);
        if (rc != SG_OK) return rc;
        for (uint32_t w = G.offAgg; w < G.offAgg + 5 * G.projAgg; w++)
            for (uint64_t k = 0; k < K; k++) S[gen_il(K, (uint32_t)k, w)] = cur[gen_il(K, (uint32_t)k, w)];
    }
    auto W64 = [&](uint32_t k, uint32_t w, int64_t v) {
        W(k, w) = (uint32_t)(uint64_t)v;
        W(k, w + 1) = (uint32_t)((uint64_t)v >> 32);
    };
    for (const SdKey& x : d.keys) {
        if (x.key >= K) { msg = "state document key id outside [0, n_keys)"; return SG_ERR_INVALID; }
        if (x.states.size() > G.STCAP || x.streams.size() > G.SECAP) {
            msg = "state document holds more partial matches per key than partial_capacity allows";
            return SG_ERR_CAPACITY;
        }
        const uint32_t k = x.key;
        W(k, 0) = 1u;
        // references: a StateEvent is held by each list entry; a StreamEvent by each slot head and by the
        // event before it in a count chain
        std::vector<uint32_t> st_rc(x.states.size(), 0), ev_rc(x.streams.size(), 0);
        std::vector<uint32_t> next(x.streams.size(), GEN_NIL);
        std::vector<uint8_t> linked(x.streams.size(), 0);
        for (const SdState& st : x.states)
            for (const auto& c : st.chains) {
                if (c.empty()) continue;
                ev_rc[c[0]]++;
                for (size_t i = 0; i + 1 < c.size(); i++) {
                    if (next[c[i]] == GEN_NIL) next[c[i]] = c[i + 1];
                    else if (next[c[i]] != c[i + 1]) { msg = "state document chains disagree"; return SG_ERR_INVALID; }
                    if (!linked[c[i + 1]]) { linked[c[i + 1]] = 1; ev_rc[c[i + 1]]++; }
                }
            }
        uint32_t maxOrder = 0;
        for (int p = 0; p < G.nprocs; p++) {
            const SdProc& P = x.procs[p];
            const uint32_t ks = G.offKS + (uint32_t)p * G.ksWords;
            if (P.pending.size() > G.L || P.newev.size() > G.L || P.queue.size() > G.Q) {
                msg = "state document list longer than this engine's capacity";
                return SG_ERR_CAPACITY;
            }
            uint32_t f = 0;
            if (P.flags & SD_INITIALIZED) f |= GF_INIT;
            if (P.flags & SD_STARTED) f |= GF_STARTED;
            if (P.flags & SD_SUCCESS) f |= GF_SUCCESS;
            if (P.flags & SD_SSRESET) f |= GF_SSRESET;
            if (!(P.flags & SD_ACTIVE)) f |= GF_INACTIVE;
            if (P.running) f |= GF_RUNNING;
            W(k, ks + KS_FLAGS) = f;
            W64(k, ks + KS_LST, P.last_scheduled);
            W64(k, ks + KS_LAT, P.last_arrival);
            W64(k, ks + KS_FIRE, P.running ? P.fire_at : 0);
            W(k, ks + KS_ORDER) = (uint32_t)P.order;
            maxOrder = std::max(maxOrder, (uint32_t)P.order);
            W(k, ks + KS_QHEAD) = 0;
            W(k, ks + KS_QLEN) = (uint32_t)P.queue.size();
            for (size_t i = 0; i < P.queue.size(); i++) W64(k, ks + KS_LISTS + 2 * G.L + 2 * (uint32_t)i, P.queue[i]);
            for (int which = 0; which < 2; which++) {
                const auto& l = which ? P.newev : P.pending;
                W(k, ks + KS_PLEN + (uint32_t)which) = (uint32_t)l.size();
                for (size_t i = 0; i < l.size(); i++) {
                    W(k, ks + KS_LISTS + (uint32_t)which * G.L + (uint32_t)i) = l[i];
                    st_rc[l[i]]++;
                }
            }
        }
        W(k, 1) = maxOrder;  // the key's scheduler order counter
        for (size_t i = 0; i < x.states.size(); i++) {
            const SdState& st = x.states[i];
            const uint32_t base = G.offST + (uint32_t)i * G.stWords;
            W64(k, base + ST_TS, st.ts);
            W(k, base + ST_TYPE) = st.type;
            W(k, base + ST_RC) = st_rc[i];
            for (int sl = 0; sl < G.nslots; sl++)
                W(k, base + ST_SLOTS + (uint32_t)sl) = st.chains[sl].empty() ? GEN_NIL : st.chains[sl][0];
            W(k, G.offSTfree + (uint32_t)i / 32) |= 1u << (i % 32);
        }
        for (size_t i = 0; i < x.streams.size(); i++) {
            const SdStream& ev = x.streams[i];
            const uint32_t base = G.offSE + (uint32_t)i * G.seWords;
            W64(k, base + SE_SEQ, (int64_t)ev.seq);
            W64(k, base + SE_TS, ev.ts);
            W(k, base + SE_NEXT) = next[i];
            W(k, base + SE_RC) = ev_rc[i];
            W(k, base + SE_NULL) = ev.null_bits;
            for (size_t a = 0; a < ev.attr.size() && a < G.NA; a++) W64(k, base + SE_ATTR + 2 * (uint32_t)a, (int64_t)ev.attr[a]);
            W(k, G.offSEfree + (uint32_t)i / 32) |= 1u << (i % 32);
        }
    }
    GenClock clk{d.now, d.last_event_ts, (uint32_t)(d.clock_flags & 1u), 0};
    return gen_restore(e, S.data(), clk, msg);
}
