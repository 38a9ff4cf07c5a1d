// gen_kernels.hip — device side of the general NFA engine (see gen_engine.h).
//
// One lane owns one partition key and runs the key's processor graph exactly as the reference does
// for that key, over the key's events of the micro-batch in arrival order.  The processors are the
// flat tables of GenProgram; their per-key state lives in HBM (interleaved by key).  Restated from
// (paths under /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/):
//   StreamPreStateProcessor.java:118-403     isExpired, init, addState, addEveryState, resetState,
//                                            updateState, expireEvents, processAndReturn
//   StreamPostStateProcessor.java:64-83      post processing of a passed filter
//   CountPre/PostStateProcessor.java         `<m:n>` (chains appended to the SAME StateEvent objects)
//   LogicalPre/PostStateProcessor.java       `and` / `or`
//   Absent{Stream,Logical}{Pre,Post}StateProcessor.java   `not S for T` and its timers
//   util/Scheduler.java:65-298               per-key FIFO timer queues
//   query/input/*ProcessStreamReceiver.java  stabilize + reverse state order + deferred projection
//   executor/condition/**, executor/math/**  filters with Java numerics (null, int wrap, /0 -> null)
#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu.h"
#include "../../include/siddhi_gpu_ir.h"
#include "gen_engine.h"
#include "java_ops.h"

// GENX_PROF=1 (experiment builds only): s_memtime per walk phase of each wave, summed into A.o.prof:
// 0 key start (bounds, initKey), 1 stabilize, 2 processAndReturn, 3 projection / deferral,
// 4 key end (flush, reservations, deadline), 5 timer sweeps, 6 waves
#ifndef GENX_PROF
#define GENX_PROF 0
#endif
#if GENX_PROF
#define GENX_T(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); prof[i] += t_ - prof_t; prof_t = t_; } while (0)
#else
#define GENX_T(i) do { } while (0)
#endif

namespace {

// Address spaces made explicit: the per-key state and the batch columns are global memory
// (address_space 1: global_load/store, whose waits are counted per kind, instead of flat accesses
// that every wait must drain completely); the program tables are constant memory (address_space 4:
// scalar loads wherever the index is wave-uniform).
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(4))) const GenProgram cGenProgram;
template <class T> __device__ __forceinline__ __attribute__((address_space(1))) T* gp(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

struct Lane {
    const cGenProgram& G;
    const GenArgs& A;
    gu32* S;
    gu32* pool;             // this key's pool words (gen_at)
    uint32_t split;
    uint32_t K, k;
    int64_t now;
    uint64_t trigSeq;       // seq of the event being processed (SG_TIMER_SEQ in a timer sweep)
    uint32_t trigIdx;       // its batch position
    uint32_t trigRank;      // matches emitted so far for this trigger
    int64_t tk2;            // timer sort keys of the matches emitted now
    uint32_t tk1;
    uint32_t retm;          // StreamPostStateProcessor.isEventReturned per post processor (transient bits)
    unsigned long long scanned, created, matches;
    uint32_t err;
    unsigned long long resBase;  // this lane's reserved raw match slots
    unsigned long long resEnd;   // end of its reservation segment
    uint32_t resLeft;
#if GENX_PROF
    uint64_t prof[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t prof_t = __builtin_amdgcn_s_memtime();
#endif

    __device__ Lane(const GenArgs& a, uint32_t key)
        : G(*(cGenProgram*)a.G), A(a), S(gp(a.state)), K(a.K), k(key), now(a.now), trigSeq(SG_TIMER_SEQ), trigIdx(0), trigRank(0),
          tk2(0), tk1(0), scanned(0), created(0), matches(0), err(0), resBase(0), resEnd(0), resLeft(0) {
        retm = 0;
        split = G.offST;
        pool = S + (size_t)split * K + (size_t)k * (G.blockWords - split);
    }
    // the next key of this lane (k_gen_batch walks several keys per lane; the work counters, the error
    // bits and the raw-slot reservation carry over)
    __device__ void retarget(uint32_t key) __restrict__ {
        k = key;
        pool = S + (size_t)split * K + (size_t)k * (G.blockWords - split);
        trigSeq = SG_TIMER_SEQ;
        trigIdx = 0;
        trigRank = 0;
        retm = 0;
    }

    // ---- HBM words of this key ----
    // (gen_engine.h gen_at: KeyState words interleaved across keys, pool words contiguous per key)
    __device__ __forceinline__ gu32& W(uint32_t w) const {
        if (!GEN_SPLIT || w < split) return S[gen_il(K, k, w)];
        return pool[w - split];
    }
    __device__ __forceinline__ int64_t R64(uint32_t w) const __restrict__ {
        return (int64_t)((uint64_t)W(w) | ((uint64_t)W(w + 1) << 32));
    }
    __device__ __forceinline__ void W64(uint32_t w, int64_t v) const __restrict__ {
        W(w) = (uint32_t)(uint64_t)v;
        W(w + 1) = (uint32_t)((uint64_t)v >> 32);
    }

    // ---- KeyState of processor p ----
    __device__ __forceinline__ uint32_t ks(int p) const { return G.offKS + (uint32_t)p * G.ksWords; }
    __device__ __forceinline__ uint32_t flags(int p) const { return W(ks(p) + KS_FLAGS); }
    __device__ __forceinline__ bool flag(int p, uint32_t f) const { return (flags(p) & f) != 0; }
    __device__ __forceinline__ void setFlag(int p, uint32_t f, bool on) const __restrict__ {
        gu32& x = W(ks(p) + KS_FLAGS);
        x = on ? (x | f) : (x & ~f);
    }
    // lists: which 0 = pending, 1 = newAndEvery
    __device__ __forceinline__ gu32& len(int p, int which) const { return W(ks(p) + KS_PLEN + which); }
    __device__ __forceinline__ gu32& at(int p, int which, uint32_t i) const __restrict__ {
        return W(ks(p) + KS_LISTS + (uint32_t)which * G.L + i);
    }

    // ---- StateEvent pool ----
    __device__ __forceinline__ uint32_t stw(uint32_t se, uint32_t f) const { return G.offST + se * G.stWords + f; }
    __device__ __forceinline__ int64_t stTs(uint32_t se) const { return R64(stw(se, ST_TS)); }
    __device__ __forceinline__ void setStTs(uint32_t se, int64_t t) const { W64(stw(se, ST_TS), t); }
    __device__ __forceinline__ uint32_t slot(uint32_t se, int s) const { return W(stw(se, ST_SLOTS + (uint32_t)s)); }
    // ---- StreamEvent pool ----
    __device__ __forceinline__ uint32_t sew(uint32_t e, uint32_t f) const { return G.offSE + e * G.seWords + f; }
    __device__ __forceinline__ int64_t evTs(uint32_t e) const { return R64(sew(e, SE_TS)); }
    __device__ __forceinline__ uint64_t evSeq(uint32_t e) const { return (uint64_t)R64(sew(e, SE_SEQ)); }
    __device__ __forceinline__ uint32_t evNext(uint32_t e) const { return W(sew(e, SE_NEXT)); }
    // attribute `attr` of StreamEvent e, an event of slot `slot`'s stream (32-bit types: the low word only)
    __device__ __forceinline__ uint64_t attrWord(uint32_t e, uint32_t slot, uint32_t attr) const {
        const uint32_t w = sew(e, SE_ATTR + 2 * attr);
        const int32_t t = G.attrType[G.slotStream[slot]][attr];
        return (t == SG_T_LONG || t == SG_T_DOUBLE) ? (uint64_t)R64(w) : (uint64_t)W(w);
    }

    __device__ uint32_t alloc(uint32_t freeOff, uint32_t cap) __restrict__ {
        const uint32_t nw = (cap + 31) / 32;
        for (uint32_t w = 0; w < nw; w++) {
            uint32_t x = W(freeOff + w);
            if (x != 0xffffffffu) {
                const uint32_t b = __ffs(~x) - 1;
                const uint32_t idx = w * 32 + b;
                if (idx >= cap) break;
                W(freeOff + w) = x | (1u << b);
                return idx;
            }
        }
        err |= GERR_CAP;
        return GEN_NIL;
    }
    __device__ void freeBit(uint32_t freeOff, uint32_t idx) const __restrict__ {
        gu32& x = W(freeOff + idx / 32);
        x &= ~(1u << (idx % 32));
    }

    __device__ void evIncref(uint32_t e) const __restrict__ {
        if (e != GEN_NIL) W(sew(e, SE_RC)) += 1;
    }
    __device__ void evDecref(uint32_t e) __restrict__ {
        while (e != GEN_NIL) {
            gu32& rc = W(sew(e, SE_RC));
            if (rc == 0) { err |= GERR_REF; return; }
            if (--rc != 0) return;
            const uint32_t nx = evNext(e);
            freeBit(G.offSEfree, e);
            e = nx;
        }
    }
    __device__ uint32_t newEv(uint64_t seq, int64_t ts, uint32_t batchPos, bool blank) __restrict__ {
        const uint32_t e = alloc(G.offSEfree, G.SECAP);
        if (e == GEN_NIL) return e;
        W64(sew(e, SE_SEQ), (int64_t)seq);
        W64(sew(e, SE_TS), ts);
        W(sew(e, SE_NEXT)) = GEN_NIL;
        W(sew(e, SE_RC)) = 0;
        uint32_t nb = 0;
        if (!blank) {  // capture the event's attributes (the StreamEvent's data)
            const int s = (int)A.b.stream;
            const int na = G.nattr[s];
            for (int a = 0; a < na; a++) {
                // two words per attribute; the high word is written (and read, attrWord) only for long/double
                const void* c = A.b.col[a];
                const uint32_t w = sew(e, SE_ATTR + 2 * (uint32_t)a);
                switch (G.attrType[s][a]) {
                case SG_T_LONG: case SG_T_DOUBLE: W64(w, (int64_t)gp((const uint64_t*)c)[batchPos]); break;
                case SG_T_BOOL: W(w) = gp((const uint8_t*)c)[batchPos] ? 1u : 0u; break;
                default: W(w) = gp((const uint32_t*)c)[batchPos];
                }
                if (A.b.nul[a] && gp(A.b.nul[a])[batchPos]) nb |= 1u << a;
            }
        } else {
            nb = 0xffffffffu;  // StreamEventFactory.newInstance(): no data
        }
        W(sew(e, SE_NULL)) = nb;
        return e;
    }

    __device__ void stIncref(uint32_t se) const __restrict__ {
        if (se != GEN_NIL) W(stw(se, ST_RC)) += 1;
    }
    __device__ void stDecref(uint32_t se) __restrict__ {
        if (se == GEN_NIL) return;
        gu32& rc = W(stw(se, ST_RC));
        if (rc == 0) { err |= GERR_REF; return; }
        if (--rc != 0) return;
        for (int s = 0; s < G.nslots; s++) evDecref(slot(se, s));
        freeBit(G.offSTfree, se);
    }
    __device__ uint32_t newSt() __restrict__ {
        const uint32_t se = alloc(G.offSTfree, G.STCAP);
        if (se == GEN_NIL) return se;
        W64(stw(se, ST_TS), -1);
        W(stw(se, ST_TYPE)) = 0;
        W(stw(se, ST_RC)) = 0;
        for (int s = 0; s < G.nslots; s++) W(stw(se, ST_SLOTS + (uint32_t)s)) = GEN_NIL;
        return se;
    }
    __device__ void setSlot(uint32_t se, int s, uint32_t e) __restrict__ {
        evIncref(e);
        gu32& w = W(stw(se, ST_SLOTS + (uint32_t)s));
        const uint32_t old = w;
        w = e;
        evDecref(old);
    }
    // StateEventCloner.copyStateEvent: shallow copy of the slot references (StateEventCloner.java:48-60)
    __device__ uint32_t cloneSt(uint32_t se) __restrict__ {
        const uint32_t c = newSt();
        if (c == GEN_NIL) return c;
        for (int s = 0; s < G.nslots; s++) setSlot(c, s, slot(se, s));
        W(stw(c, ST_TYPE)) = W(stw(se, ST_TYPE));
        setStTs(c, stTs(se));
        return c;
    }
    // StateEvent.getStreamEvent(int[]) for (slot, index-in-chain) (StateEvent.java:138-182)
    __device__ uint32_t chainAt(uint32_t se, int s, int idx) const __restrict__ {
        uint32_t e = slot(se, s);
        if (e == GEN_NIL) return GEN_NIL;
        if (idx >= 0) {
            for (int i = 1; i <= idx; i++) {
                e = evNext(e);
                if (e == GEN_NIL) return GEN_NIL;
            }
            return e;
        }
        if (idx == -1) {
            while (evNext(e) != GEN_NIL) e = evNext(e);
            return e;
        }
        if (idx == -2) {
            if (evNext(e) == GEN_NIL) return GEN_NIL;
            while (evNext(evNext(e)) != GEN_NIL) e = evNext(e);
            return e;
        }
        int n = 0;
        for (uint32_t x = e; x != GEN_NIL; x = evNext(x)) n++;
        const int index = n + idx;
        if (index < 0) return GEN_NIL;
        for (int i = 0; i < index; i++) e = evNext(e);
        return e;
    }
    // StateEvent.addEvent / removeLastEvent (StateEvent.java:212-236)
    __device__ void addEvent(uint32_t se, int s, uint32_t e) __restrict__ {
        uint32_t x = slot(se, s);
        if (x == GEN_NIL) { setSlot(se, s, e); return; }
        while (evNext(x) != GEN_NIL) x = evNext(x);
        evIncref(e);
        W(sew(x, SE_NEXT)) = e;
    }
    __device__ void removeLastEvent(uint32_t se, int s) __restrict__ {
        uint32_t x = slot(se, s);
        if (x == GEN_NIL) return;
        while (evNext(x) != GEN_NIL) {
            const uint32_t nx = evNext(x);
            if (evNext(nx) == GEN_NIL) {
                W(sew(x, SE_NEXT)) = GEN_NIL;
                evDecref(nx);
                return;
            }
            x = nx;
        }
        setSlot(se, s, GEN_NIL);
    }

    // ---- lists of StateEvents ----
    __device__ void push(int p, int which, uint32_t se) __restrict__ {
        gu32& n = len(p, which);
        if (n >= G.L) { err |= GERR_CAP; return; }
        stIncref(se);
        at(p, which, n) = se;
        n++;
    }
    __device__ void erase(int p, int which, uint32_t i) __restrict__ {
        gu32& n = len(p, which);
        const uint32_t se = at(p, which, i);
        for (uint32_t j = i + 1; j < n; j++) at(p, which, j - 1) = at(p, which, j);
        n--;
        stDecref(se);
    }
    __device__ void clearList(int p, int which) __restrict__ {
        gu32& n = len(p, which);
        const uint32_t m = n;
        n = 0;
        for (uint32_t j = 0; j < m; j++) stDecref(at(p, which, j));
    }
    __device__ bool removeValue(int p, int which, uint32_t se) __restrict__ {
        const uint32_t n = len(p, which);
        for (uint32_t j = 0; j < n; j++)
            if (at(p, which, j) == se) { erase(p, which, j); return true; }
        return false;
    }
    // eventTimeComparator (StreamPreStateProcessor.java:66-80): ts -1 last; List.sort is stable
    __device__ bool tsBefore(uint32_t a, uint32_t b) const __restrict__ {
        const int64_t ta = stTs(a), tb = stTs(b);
        if (ta == -1) return false;
        if (tb == -1) return true;
        return ta < tb;
    }
    // newAndEvery sorted by ts, appended to pending, cleared
    __device__ void promote(int p) __restrict__ {
        const uint32_t n = len(p, 1);
        for (uint32_t i = 1; i < n; i++) {  // stable insertion sort
            const uint32_t x = at(p, 1, i);
            uint32_t j = i;
            while (j > 0 && tsBefore(x, at(p, 1, j - 1))) { at(p, 1, j) = at(p, 1, j - 1); j--; }
            at(p, 1, j) = x;
        }
        gu32& pn = len(p, 0);
        for (uint32_t i = 0; i < n; i++) {
            if (pn >= G.L) { err |= GERR_CAP; break; }
            at(p, 0, pn++) = at(p, 1, i);  // the reference moves: no count change
        }
        len(p, 1) = 0;
    }

    // ---- timers (Scheduler) ----
    __device__ uint32_t qlen(int p) const { return W(ks(p) + KS_QLEN); }
    __device__ int64_t qhead(int p) const __restrict__ {
        const uint32_t h = W(ks(p) + KS_QHEAD);
        return R64(ks(p) + KS_LISTS + 2 * G.L + 2 * h);
    }
    __device__ void qpop(int p) const __restrict__ {
        gu32& h = W(ks(p) + KS_QHEAD);
        h = (h + 1) % G.Q;
        W(ks(p) + KS_QLEN) -= 1;
    }
    // this key's next timer deadline (GenTimers): the earliest queue head of its absent processors
    // (playback listener, Scheduler.java:73-104) or the earliest fire time of its running callers
    // (wall clock, Scheduler.EventCaller, Scheduler.java:238-298)
    __device__ int64_t nextDeadline() const __restrict__ {
        int64_t best = GEN_NO_DEADLINE;
        for (int i = 0; i < G.nStartup; i++) {
            const int p = G.startup[i];
            int64_t t = GEN_NO_DEADLINE;
            if (G.playback) {
                if (qlen(p) != 0) t = qhead(p);
            } else if (flag(p, GF_RUNNING)) {
                t = R64(ks(p) + KS_FIRE);
            }
            best = t < best ? t : best;
        }
        return best;
    }

    __device__ void notifyAt(int p, int64_t t) __restrict__ {  // Scheduler.notifyAt + schedule (Scheduler.java:114-156)
        gu32& n = W(ks(p) + KS_QLEN);
        if (n >= G.Q) { err |= GERR_CAP; return; }
        const uint32_t pos = (W(ks(p) + KS_QHEAD) + n) % G.Q;
        W64(ks(p) + KS_LISTS + 2 * G.L + 2 * pos, t);
        n++;
        if (!G.playback && !flag(p, GF_RUNNING) && n == 1) {
            setFlag(p, GF_RUNNING, true);
            W64(ks(p) + KS_FIRE, t > now ? t : now);
            W(ks(p) + KS_ORDER) = ++W(1);
        }
    }

    // ---- filters (java_ops.h: Java value semantics of the expression bytecode) ----
    // a value of the expression program: VAR reads slot s's event at chain index c (its captured attribute)
    template <class CodePtr> __device__ GVal evalv(uint32_t se, CodePtr code, uint32_t pc, uint32_t n) __restrict__ {
        return jo_eval(code, pc, n, err,
                       [&](uint32_t slot, uint32_t attr, int32_t chain) -> GVal {
                           const uint32_t e = chainAt(se, (int)slot, chain);
                           if (e == GEN_NIL) return GVal{0, true};
                           return GVal{attrWord(e, slot, attr), ((W(sew(e, SE_NULL)) >> attr) & 1u) != 0};
                       },
                       [&](uint32_t slot, int32_t chain) -> bool { return chainAt(se, (int)slot, chain) == GEN_NIL; });
    }
    // FilterProcessor.process: pass iff the condition is a non-null true (FilterProcessor.java:48-60)
    __device__ bool eval(uint32_t se, uint32_t pc, uint32_t n) __restrict__ {
        const GVal v = evalv(se, G.code, pc, n);
        return !v.null && (v.b & 1);
    }

    // a filter decoded on the host into one compare (gen_engine.h JoFast): the same reads, no interpreter
    template <class F> __device__ bool evalFast(uint32_t se, const F& f) __restrict__ {
        return jo_fast(f, [&](uint32_t slot, uint32_t attr, int32_t chain) -> GVal {
            const uint32_t e = chainAt(se, (int)slot, chain);
            if (e == GEN_NIL) return GVal{0, true};
            return GVal{attrWord(e, slot, attr), ((W(sew(e, SE_NULL)) >> attr) & 1u) != 0};
        });
    }

    // QuerySelector.processNoGroupBy (QuerySelector.java:162-206) at emission, in this key's output order:
    // each aggregator's processAdd over its argument (java_ops.h jo_agg, per-key state in the block), then
    // the select list (reading the aggregators' values) and `having` (reading the output row), 3 words per
    // output item (value lo, hi, null)
    __device__ __noinline__ void projectSelect(uint32_t se, gu32* pv) __restrict__ {
        GVal aggres[GEN_MAXAGG];
        for (uint32_t a = 0; a < G.projAgg; a++) {
            const GVal arg = G.projLen[a] ? evalv(se, G.code, G.projPc[a], G.projLen[a]) : GVal{0, true};
            const uint32_t base = G.offAgg + 5 * a;
            int64_t n = R64(base);
            uint64_t v = (uint64_t)R64(base + 2);
            bool has = W(base + 4) != 0;
            aggres[a] = jo_agg((G.projType[a] >> 8) & 0xffu, (int)(G.projType[a] & 0xffu), arg, n, v, has);
            W64(base, n);
            W64(base + 2, (int64_t)v);
            W(base + 4) = has ? 1u : 0u;
        }
        for (uint32_t i = G.projAgg; i < G.projN; i++) {
            const GVal v = jo_eval(G.code, G.projPc[i], G.projLen[i], err,
                                   [&](uint32_t slot, uint32_t attr, int32_t chain) -> GVal {
                                       if (slot == SG_PROJ_SLOT_AGG) return attr < GEN_MAXAGG ? aggres[attr] : GVal{0, true};
                                       if (slot == SG_PROJ_SLOT_OUT)
                                           return GVal{(uint64_t)pv[3 * attr] | ((uint64_t)pv[3 * attr + 1] << 32),
                                                       pv[3 * attr + 2] != 0};
                                       const uint32_t e = chainAt(se, (int)slot, chain);
                                       if (e == GEN_NIL) return GVal{0, true};
                                       return GVal{attrWord(e, slot, attr), ((W(sew(e, SE_NULL)) >> attr) & 1u) != 0};
                                   },
                                   [&](uint32_t slot, int32_t chain) -> bool { return chainAt(se, (int)slot, chain) == GEN_NIL; });
            const uint32_t j = i - G.projAgg;
            pv[3 * j] = (uint32_t)v.b;
            pv[3 * j + 1] = (uint32_t)(v.b >> 32);
            pv[3 * j + 2] = v.null ? 1u : 0u;
        }
    }

    // ---- match output (QuerySelector input) ----
    __device__ void project(uint32_t se) __restrict__ {
        if (resLeft == 0) {
            const uint32_t sg = blockIdx.x % A.o.nseg;  // one wave per block
            resBase = (unsigned long long)sg * A.o.seg_cap + atomicAdd(&A.o.raw_count[sg], (unsigned long long)GEN_RESCHUNK);
            resEnd = (unsigned long long)(sg + 1) * A.o.seg_cap;
            resLeft = GEN_RESCHUNK;
        }
        const unsigned long long r = resBase++;
        resLeft--;
        matches++;
        if (r >= resEnd) { err |= GERR_MATCHCAP; return; }
        gu32* rec = gp(A.o.raw) + r * A.o.recWords;
        const bool timer = trigSeq == SG_TIMER_SEQ;
        rec[0] = timer ? 0xfffffffeu : trigIdx;
        rec[1] = trigRank++;  // a timer match: its rank in this key's sweep (gen_host.hip timer ordering)
        rec[2] = (uint32_t)trigSeq;
        rec[3] = (uint32_t)(trigSeq >> 32);
        const int64_t ts = stTs(se);
        rec[4] = (uint32_t)(uint64_t)ts;
        rec[5] = (uint32_t)((uint64_t)ts >> 32);
        rec[6] = k;
        gu32* lens = rec + 7;
        gu32* seqs = lens + G.nslots;
        for (int s = 0; s < G.nslots; s++) {
            uint32_t n = 0;
            for (uint32_t e = slot(se, s); e != GEN_NIL; e = evNext(e)) {
                if (n >= G.MC) { err |= GERR_CHAIN; break; }
                const uint64_t q = evSeq(e);
                seqs[2 * (s * G.MC + n)] = (uint32_t)q;
                seqs[2 * (s * G.MC + n) + 1] = (uint32_t)(q >> 32);
                n++;
            }
            lens[s] = n;
        }
        if (G.projN) projectSelect(se, rec + G.projOff);
        if (timer) {  // (nvalid: the timers kernel adds its waves' match counts)
            gp(A.o.tk1)[r] = tk1;
            gp(A.o.tk2)[r] = tk2;
            gp(A.o.tk3)[r] = k;
        } else {
            const uint32_t c0 = gp(A.o.t_cnt)[trigIdx];
            gp(A.o.t_cnt)[trigIdx] = c0 + 1u;
            if (A.mode & GEN_M_TFIRST) {
                gp(A.o.t_first)[trigIdx] = (uint32_t)r;
                // a second match of one trigger (a key handed over in a non-canonical state, e.g. imported,
                // can hold several partials): t_first keeps one record only, so the ordering must place
                // every record by (t_off, rank) instead (gen_host.hip: k_gen_scatter when t_multi is set)
                if (c0) *gp(A.o.t_multi) = 1u;
            }
        }
    }

    // ---- StreamPreStateProcessor & co (per processor p, this key) ----
    __device__ bool isExpired(uint32_t se, int64_t t) const __restrict__ {  // StreamPreStateProcessor.java:118-129
        if (G.within == -1) return false;
        for (int i = 0; i < G.nStartIds; i++) {
            const uint32_t e = slot(se, G.startIds[i]);
            if (e != GEN_NIL) {
                const int64_t d = evTs(e) - t;
                if ((d < 0 ? -d : d) > G.within) return true;
            }
        }
        return false;
    }

    __device__ void init(int p) __restrict__ {  // StreamPreStateProcessor.java:178-194
        const auto& P = G.pre[p];
        const auto& Q = G.post[P.thisPost];
        if (P.isStart && (!flag(p, GF_INIT) || Q.nextEveryStatePre != GEN_NONE ||
                          (G.qtype == SG_Q_SEQUENCE && Q.nextStatePre != GEN_NONE && G.pre[Q.nextStatePre].absent))) {
            const uint32_t se = newSt();
            if (se == GEN_NIL) return;
            stIncref(se);
            addState(p, se);
            stDecref(se);
            setFlag(p, GF_INIT, true);
        }
    }

    // addState with CountPreStateProcessor's min-count-0 forwarding (:129-136 -> processMinCountReached ->
    // the next state's addState, and so on down a chain of <0:n> states) run as a loop over the chain:
    // the continuations of processMinCountReached (its addEveryState and the reference drop) run after
    // the innermost addState returns, innermost first, as the recursive calls would.  Keeping the call
    // graph acyclic lets the compiler inline the whole processor graph (no call stack in scratch).
    __device__ void addState(int p, uint32_t se) __restrict__ {
        int pend[GEN_MAXP];
        int np = 0;
        for (;;) {
            if (addStateOne(p, se)) break;
            const int q = G.pre[p].countPost;  // processMinCountReached(q, se), up to its addState
            const auto& Q = G.post[q];
            if (Q.hasNext) {
                setFlag(Q.thisPre, GF_CHANGED, true);
                retm |= 1u << q;
            }
            stIncref(se);
            if (np >= GEN_MAXP) { err |= GERR_REF; stDecref(se); break; }
            pend[np++] = q;
            if (Q.nextStatePre == GEN_NONE) break;
            p = Q.nextStatePre;
        }
        while (np > 0) {
            const auto& Q = G.post[pend[--np]];
            if (Q.nextEveryStatePre != GEN_NONE) addEveryState(Q.nextEveryStatePre, se);
            stDecref(se);
        }
    }

    // one StreamPre/CountPre/Logical/Absent addState; true when done, false when a count state with
    // min 0 and an empty slot forwards the partial (processMinCountReached)
    __device__ bool addStateOne(int p, uint32_t se) __restrict__ {
        const auto& P = G.pre[p];
        if (P.absent && flag(p, GF_INACTIVE)) return true;
        if (P.absent && P.kind == GK_STREAM) {  // AbsentStreamPreStateProcessor.java:83-103
            if (G.qtype == SG_Q_SEQUENCE) clearList(p, 1);
            push(p, 1, se);
            if (!P.isStart) {
                const int64_t t = stTs(se) + P.waiting;
                W64(ks(p) + KS_LST, t);
                notifyAt(p, t);
            }
            return true;
        }
        if (P.kind == GK_LOGICAL) {  // LogicalPreStateProcessor.java:43-62
            if (P.isStart || G.qtype == SG_Q_SEQUENCE) {
                if (len(p, 1) == 0) push(p, 1, se);
                if (P.partner != GEN_NONE && len(P.partner, 1) == 0) push(P.partner, 1, se);
            } else {
                push(p, 1, se);
                if (P.partner != GEN_NONE) push(P.partner, 1, se);
            }
            if (P.absent && !P.isStart && P.waiting != -1) {  // AbsentLogicalPreStateProcessor.java:77-97
                notifyAt(p, stTs(se) + P.waiting);
                if (G.pre[P.partner].absent) notifyAt(P.partner, stTs(se) + G.pre[P.partner].waiting);
            }
            return true;
        }
        // StreamPreStateProcessor.java:214-227, CountPreStateProcessor.java:114-128
        if (G.qtype == SG_Q_SEQUENCE) {
            if (len(p, 1) == 0) push(p, 1, se);
        } else {
            push(p, 1, se);
        }
        return !(P.kind == GK_COUNT && P.minCount == 0 && slot(se, P.stateId) == GEN_NIL);  // :129-136
    }

    __device__ void addEveryState(int p, uint32_t se) __restrict__ {
        const auto& P = G.pre[p];
        const uint32_t c = cloneSt(se);
        if (c == GEN_NIL) return;
        stIncref(c);
        W(stw(c, ST_TYPE)) = 0;  // CURRENT
        created++;
        if (P.absent && P.kind == GK_LOGICAL) {  // AbsentLogicalPreStateProcessor.java:99-118
            const uint32_t own = slot(c, P.stateId);
            if (own != GEN_NIL) setStTs(c, evTs(own));
            setSlot(c, P.stateId, GEN_NIL);
            setSlot(c, G.pre[P.partner].stateId, GEN_NIL);
            push(p, 1, c);
            push(P.partner, 1, c);
        } else if (P.absent) {  // AbsentStreamPreStateProcessor.java:105-123
            for (int i = P.stateId; i < G.nslots; i++) setSlot(c, i, GEN_NIL);
            push(p, 1, c);
            const int64_t t = stTs(se) + P.waiting;
            W64(ks(p) + KS_LST, t);
            notifyAt(p, t);
        } else if (P.kind == GK_LOGICAL) {  // LogicalPreStateProcessor.java:64-84
            for (int i = P.stateId; i < G.nslots; i++) setSlot(c, i, GEN_NIL);
            push(p, 1, c);
            if (P.partner != GEN_NONE) {
                setSlot(c, G.pre[P.partner].stateId, GEN_NIL);
                push(P.partner, 1, c);
            }
        } else {  // StreamPreStateProcessor.java:229-247
            for (int i = P.stateId; i < G.nslots; i++) setSlot(c, i, GEN_NIL);
            push(p, 1, c);
        }
        stDecref(c);
    }

    __device__ bool seqHold(int p) const __restrict__ {  // SEQUENCE, no every, the next state still has pending partials
        const auto& Q = G.post[G.pre[p].thisPost];
        return G.qtype == SG_Q_SEQUENCE && Q.nextEveryStatePre == GEN_NONE && Q.nextStatePre != GEN_NONE &&
               len(Q.nextStatePre, 0) != 0;
    }

    __device__ void resetState(int p) __restrict__ {
        const auto& P = G.pre[p];
        if (P.kind == GK_LOGICAL) {  // LogicalPreStateProcessor.java:86-108
            if (P.logicalType == SG_L_OR || len(p, 0) == len(P.partner, 0)) {
                clearList(p, 0);
                clearList(P.partner, 0);
                if (P.isStart && len(p, 1) == 0) {
                    if (seqHold(p)) return;
                    init(p);
                }
            }
            return;
        }
        clearList(p, 0);  // StreamPreStateProcessor.java:287-305
        if (P.isStart && len(p, 1) == 0) {
            if (seqHold(p)) return;
            init(p);
        }
    }

    __device__ void updateState(int p) __restrict__ {
        const auto& P = G.pre[p];
        if (P.kind == GK_COUNT && flag(p, GF_SSRESET)) {  // CountPreStateProcessor.java:168-180
            setFlag(p, GF_SSRESET, false);
            init(p);
        }
        promote(p);
        if (P.kind == GK_LOGICAL) promote(P.partner);  // LogicalPreStateProcessor.java:110-122
    }

    // One pass per list: the expired entries are dropped (their references released in list order, as
    // the reference's iterator.remove() calls do) and the survivors moved down once (no per-erase shift).
    __device__ void expireEvents(int p, int64_t t) __restrict__ {  // StreamPreStateProcessor.java:325-361
        uint32_t expired = GEN_NIL;
        const uint32_t n0 = len(p, 0);
        uint32_t i = 0;
        for (; i < n0; i++) {  // a prefix of the pending list (:331-343)
            const uint32_t se = at(p, 0, i);
            if (!isExpired(se, t)) break;
            if (W(stw(se, ST_TYPE)) != 1) {
                W(stw(se, ST_TYPE)) = 1;
                stIncref(se);
                stDecref(expired);
                expired = se;
            }
            stDecref(se);
        }
        if (i > 0) {
            for (uint32_t j = i; j < n0; j++) at(p, 0, j - i) = at(p, 0, j);
            len(p, 0) = n0 - i;
        }
        const uint32_t n1 = len(p, 1);
        uint32_t w = 0;
        for (i = 0; i < n1; i++) {  // any entry of newAndEvery (:345-357)
            const uint32_t se = at(p, 1, i);
            if (isExpired(se, t)) {
                if (W(stw(se, ST_TYPE)) != 1) {
                    W(stw(se, ST_TYPE)) = 1;
                    stIncref(se);
                    stDecref(expired);
                    expired = se;
                }
                stDecref(se);
            } else {
                if (w != i) at(p, 1, w) = se;
                w++;
            }
        }
        if (w != n1) len(p, 1) = w;
        const int we = G.pre[p].withinEvery;
        if (expired != GEN_NIL && we != GEN_NONE) {
            addEveryState(we, expired);
            updateState(we);
        }
        stDecref(expired);
    }

    __device__ void startStateReset(int p) __restrict__ {  // CountPreStateProcessor.java:155-166
        for (int depth = 0; depth < 2 * GEN_MAXP; depth++) {
            setFlag(p, GF_SSRESET, true);
            const auto& P = G.pre[p];
            if (G.post[P.thisPost].callbackPre == GEN_NONE) return;
            p = G.post[P.countPost].thisPre;
        }
        err |= GERR_REF;  // the reference overflows its stack here
    }

    __device__ void runChain(int p, uint32_t se) __restrict__ {  // StreamPreStateProcessor.process(StateEvent) :131-142
        setFlag(p, GF_CHANGED, false);
        const auto& P = G.pre[p];
        if (P.flen == 0 || (P.ff.on ? evalFast(se, P.ff) : eval(se, P.fpc, P.flen))) postProcess(P.thisPost, se);
    }

    // ---- post processors ----
    __device__ void streamProcess(int q, uint32_t se) __restrict__ {  // StreamPostStateProcessor.java:64-83
        const auto& Q = G.post[q];
        setFlag(Q.thisPre, GF_CHANGED, true);
        setStTs(se, evTs(slot(se, Q.stateId)));
        if (Q.hasNext) retm |= 1u << q;
        stIncref(se);
        if (Q.nextStatePre != GEN_NONE) addState(Q.nextStatePre, se);
        if (Q.nextEveryStatePre != GEN_NONE) addEveryState(Q.nextEveryStatePre, se);
        if (Q.callbackPre != GEN_NONE) startStateReset(Q.callbackPre);
        stDecref(se);
    }
    __device__ void processMinCountReached(int q, uint32_t se) __restrict__ {  // CountPostStateProcessor.java:68-80
        const auto& Q = G.post[q];
        if (Q.hasNext) {
            setFlag(Q.thisPre, GF_CHANGED, true);
            retm |= 1u << q;
        }
        stIncref(se);
        if (Q.nextStatePre != GEN_NONE) addState(Q.nextStatePre, se);
        if (Q.nextEveryStatePre != GEN_NONE) addEveryState(Q.nextEveryStatePre, se);
        stDecref(se);
    }
    __device__ void postProcess(int q, uint32_t se) __restrict__ {
        const auto& Q = G.post[q];
        if (Q.absent) {  // Absent{Stream,Logical}PostStateProcessor
            const uint32_t ev = slot(se, Q.stateId);
            setFlag(Q.thisPre, GF_CHANGED, true);
            retm |= 1u << q;
            if (Q.kind == GK_STREAM) {
                setStTs(se, evTs(ev));
                if (G.pre[Q.thisPre].isStart && Q.nextEveryStatePre == Q.thisPre) addEveryState(Q.thisPre, se);
            }
            updateLastArrivalTime(Q.thisPre, evTs(ev));
            return;
        }
        if (Q.kind == GK_COUNT) {  // CountPostStateProcessor.java:39-66
            uint32_t e = slot(se, Q.stateId);
            int n = 1;
            while (evNext(e) != GEN_NIL) { n++; e = evNext(e); }
            setFlag(Q.thisPre, GF_SUCCESS, true);
            setStTs(se, evTs(e));
            if (n >= Q.minCount) {
                if (G.qtype == SG_Q_SEQUENCE) {
                    stIncref(se);
                    if (Q.nextStatePre != GEN_NONE) addState(Q.nextStatePre, se);
                    if (n != Q.maxCount) addState(Q.thisPre, se);
                    stDecref(se);
                } else if (n == Q.minCount) {
                    processMinCountReached(q, se);
                }
                if (n == Q.maxCount) setFlag(Q.thisPre, GF_CHANGED, true);
            }
            return;
        }
        if (Q.kind == GK_LOGICAL) {  // LogicalPostStateProcessor.java:59-83
            if (Q.logicalType == SG_L_AND) {
                const auto& PP = G.pre[Q.partnerPre];
                const bool go = PP.absent ? partnerCanProceed(Q.partnerPre, se) : slot(se, PP.stateId) != GEN_NIL;
                if (go) streamProcess(q, se);
                else setFlag(Q.thisPre, GF_CHANGED, true);
            } else {
                streamProcess(q, se);
                if (G.post[Q.partnerPost].hasNext && G.pre[Q.thisPre].thisLast == Q.partnerPost) retm |= 1u << Q.partnerPost;
            }
            return;
        }
        streamProcess(q, se);
    }

    // ---- absent states ----
    __device__ void updateLastArrivalTime(int p, int64_t ts) __restrict__ {
        if (G.pre[p].kind == GK_LOGICAL) {  // AbsentLogicalPreStateProcessor.java:65-74
            W64(ks(p) + KS_LAT, ts);
            return;
        }
        const int64_t t = ts + G.pre[p].waiting;  // AbsentStreamPreStateProcessor.java:70-81
        W64(ks(p) + KS_LST, t);
        notifyAt(p, t);
    }
    __device__ void partitionCreated(int p) __restrict__ {  // AbsentStreamPreStateProcessor.java:290-308 (+ logical)
        if (flag(p, GF_STARTED)) return;
        setFlag(p, GF_STARTED, true);
        const auto& P = G.pre[p];
        if (P.isStart && P.waiting != -1 && !flag(p, GF_INACTIVE)) {
            if (P.kind == GK_STREAM) W64(ks(p) + KS_LST, now + P.waiting);
            notifyAt(p, now + P.waiting);
        }
    }
    __device__ bool partnerCanProceed(int p, uint32_t se) __restrict__ {  // AbsentLogicalPreStateProcessor.java:391-422
        const auto& P = G.pre[p];
        const auto& Q = G.post[P.thisPost];
        const int64_t lat = R64(ks(p) + KS_LAT);
        if (G.qtype == SG_Q_SEQUENCE && Q.nextEveryStatePre == GEN_NONE && lat > 0) return false;
        if (P.waiting == -1) {
            if (Q.nextEveryStatePre == GEN_NONE) return slot(se, P.stateId) == GEN_NIL;
            if (lat > 0) {
                W64(ks(p) + KS_LAT, 0);
                init(p);
                return false;
            }
            return true;
        }
        return slot(se, P.stateId) != GEN_NIL;
    }
    __device__ void sendAbsentEvent(int p, uint32_t se) __restrict__ {  // Absent*PreStateProcessor.sendEvent
        const auto& P = G.pre[p];
        const auto& Q = G.post[P.thisPost];
        if (Q.hasNext) project(se);
        if (Q.nextStatePre != GEN_NONE) addState(Q.nextStatePre, se);
        if (Q.nextEveryStatePre != GEN_NONE) {
            addEveryState(Q.nextEveryStatePre, se);
        } else if (P.isStart) {
            setFlag(p, GF_INACTIVE, true);
            if (P.kind == GK_LOGICAL && P.logicalType == SG_L_OR && G.pre[P.partner].absent)
                setFlag(P.partner, GF_INACTIVE, true);
        }
        if (Q.callbackPre != GEN_NONE) startStateReset(Q.callbackPre);
    }

    // the TIMER event of processor p for this key at currentTime (Absent*PreStateProcessor.process)
    __device__ void processTimer(int p, int64_t currentTime) __restrict__ {
        const auto& P = G.pre[p];
        const auto& Q = G.post[P.thisPost];
        if (flag(p, GF_INACTIVE)) return;
        uint32_t rl[64];
        uint32_t nr = 0;
        if (P.kind == GK_STREAM) {  // AbsentStreamPreStateProcessor.java:151-227
            bool initialize = P.isStart && len(p, 1) == 0 && len(p, 0) == 0;
            if (initialize && G.qtype == SG_Q_SEQUENCE && Q.nextEveryStatePre == GEN_NONE && R64(ks(p) + KS_LST) > 0)
                initialize = false;
            if (initialize) {
                const uint32_t se = newSt();
                if (se != GEN_NIL) { stIncref(se); addState(p, se); stDecref(se); }
            } else if (G.qtype == SG_Q_SEQUENCE && len(p, 1) != 0) {
                resetState(p);
            }
            updateState(p);
            uint32_t i = 0;
            while (i < len(p, 0)) {
                const uint32_t se = at(p, 0, i);
                scanned++;
                if (isExpired(se, currentTime)) {
                    stIncref(se);
                    erase(p, 0, i);
                    if (P.withinEvery != GEN_NONE && Q.nextEveryStatePre != p) {
                        if (Q.nextEveryStatePre == GEN_NONE) err |= GERR_REF;
                        else addEveryState(Q.nextEveryStatePre, se);
                    }
                    stDecref(se);
                    continue;
                }
                const int64_t ts = stTs(se);
                if ((ts == -1 && currentTime >= R64(ks(p) + KS_LST)) || (ts != -1 && currentTime >= ts + P.waiting)) {
                    stIncref(se);
                    erase(p, 0, i);
                    setStTs(se, currentTime);
                    if (nr < 64) rl[nr++] = se; else { err |= GERR_CAP; stDecref(se); }
                    continue;
                }
                i++;
            }
            if (P.withinEvery != GEN_NONE) updateState(P.withinEvery);
            const bool notProcessed = nr == 0;
            for (uint32_t j = 0; j < nr; j++) { sendAbsentEvent(p, rl[j]); stDecref(rl[j]); }
            if (now > P.waiting + currentTime) W64(ks(p) + KS_LST, now + P.waiting);
            if (notProcessed && R64(ks(p) + KS_LST) < currentTime) {
                W64(ks(p) + KS_LST, currentTime + P.waiting);
                notifyAt(p, currentTime + P.waiting);
            }
            return;
        }
        // AbsentLogicalPreStateProcessor.java:121-209
        bool notProcessed = true;
        if (currentTime >= R64(ks(p) + KS_LAT) + P.waiting) {
            if (P.isStart && G.qtype == SG_Q_SEQUENCE && len(p, 1) == 0 && len(p, 0) == 0) {
                const uint32_t se = newSt();
                if (se != GEN_NIL) { stIncref(se); addState(p, se); stDecref(se); }
            } else if (G.qtype == SG_Q_SEQUENCE && len(p, 1) != 0) {
                resetState(p);
            }
            updateState(p);
            uint32_t expired = GEN_NIL;
            uint32_t i = 0;
            const int ps = G.pre[P.partner].stateId;
            while (i < len(p, 0)) {
                const uint32_t se = at(p, 0, i);
                scanned++;
                if (isExpired(se, currentTime)) {
                    stIncref(se);
                    stDecref(expired);
                    expired = se;
                    erase(p, 0, i);
                    continue;
                }
                const uint32_t own = slot(se, P.stateId);
                const bool passed = own != GEN_NIL ? currentTime >= evTs(own) + P.waiting : currentTime >= stTs(se) + P.waiting;
                if (passed) {
                    stIncref(se);
                    erase(p, 0, i);
                    const bool partnerIn = slot(se, ps) != GEN_NIL;
                    bool keep = false;
                    if (P.logicalType == SG_L_OR && !partnerIn) {
                        const uint32_t b = newEv(SG_BLANK_SEQ, -1, 0, true);
                        if (b != GEN_NIL) addEvent(se, P.stateId, b);
                        keep = true;
                    } else if (P.logicalType == SG_L_AND && partnerIn) {
                        keep = true;
                    } else if (P.logicalType == SG_L_AND && !partnerIn) {
                        const uint32_t b = newEv(SG_BLANK_SEQ, -1, 0, true);
                        if (b != GEN_NIL) addEvent(se, P.stateId, b);
                    }
                    if (keep && nr < 64) rl[nr++] = se;
                    else { if (keep) err |= GERR_CAP; stDecref(se); }
                    continue;
                }
                i++;
            }
            if (expired != GEN_NIL && P.withinEvery != GEN_NONE) {
                addEveryState(P.withinEvery, expired);
                updateState(P.withinEvery);
            }
            stDecref(expired);
            notProcessed = nr == 0;
            for (uint32_t j = 0; j < nr; j++) {
                setStTs(rl[j], currentTime);
                sendAbsentEvent(p, rl[j]);
                stDecref(rl[j]);
            }
            W64(ks(p) + KS_LAT, 0);
        }
        if (Q.nextEveryStatePre != GEN_NONE || (notProcessed && P.isStart)) {
            const int64_t lat = R64(ks(p) + KS_LAT);
            notifyAt(p, lat == 0 ? now + P.waiting : lat + P.waiting);
        }
    }

    // Scheduler.sendTimerEvents (Scheduler.java:172-210)
    __device__ void sendTimerEvents(int p) __restrict__ {
        for (int guard = 0; guard < (1 << 20); guard++) {
            if (qlen(p) == 0) return;
            const int64_t t = qhead(p);
            if (t > now) return;
            qpop(p);
            processTimer(p, t);
        }
        err |= GERR_CAP;
    }

    // ---- processAndReturn ----
    __device__ void processAndReturnAbsentLogical(int p, uint64_t seq, int64_t ts, uint32_t pos) __restrict__ {
        const auto& P = G.pre[p];
        const auto& Q = G.post[P.thisPost];
        uint32_t i = 0;
        while (i < len(p, 0)) {
            const uint32_t se = at(p, 0, i);
            scanned++;
            if (P.logicalType == SG_L_OR && slot(se, G.pre[P.partner].stateId) != GEN_NIL) {
                erase(p, 0, i);
                continue;
            }
            stIncref(se);
            const uint32_t cur = slot(se, P.stateId);
            evIncref(cur);
            const uint32_t e = newEv(seq, ts, pos, false);
            setSlot(se, P.stateId, e);
            runChain(p, se);
            if (P.waiting != -1 ||
                (G.qtype == SG_Q_SEQUENCE && P.logicalType == SG_L_AND && Q.nextEveryStatePre != GEN_NONE))
                setSlot(se, P.stateId, cur);
            bool removed = false;
            if ((retm >> P.thisLast) & 1u) {
                retm &= ~(1u << P.thisLast);
                erase(p, 0, i);
                removed = true;
                if (G.qtype == SG_Q_SEQUENCE) removeValue(P.partner, 0, se);
            }
            if (!flag(p, GF_CHANGED)) {
                setSlot(se, P.stateId, cur);
                if (G.qtype == SG_Q_SEQUENCE) {
                    if (removed) err |= GERR_REF;
                    else { erase(p, 0, i); removed = true; }
                }
            }
            evDecref(cur);
            stDecref(se);
            if (!removed) i++;
        }
    }

    // matches returned to the receiver are appended to `outList` (state event refs held)
    // (outList holds at most OUTCAP entries)
    static constexpr uint32_t OUTCAP = 64;
    __device__ void processAndReturn(int p, uint64_t seq, int64_t ts, uint32_t pos, uint32_t* outList, uint32_t& nOut) __restrict__ {
        const auto& P = G.pre[p];
        if (P.absent) {
            if (flag(p, GF_INACTIVE)) return;
            if (P.kind == GK_LOGICAL) { processAndReturnAbsentLogical(p, seq, ts, pos); return; }
        }
        const uint32_t out0 = nOut;
        // The reference clones the event into a fresh StreamEvent per pending partial
        // (StreamPreStateProcessor.java:373).  A stream or logical state's slot event is never appended
        // to (only count chains and absent-logical slots are), so one reference-counted copy per
        // (event, processor) is indistinguishable and saves a record write per partial.
        uint32_t shared = GEN_NIL;
        // one pass over the pending list: a dropped entry's reference is released where the reference's
        // iterator.remove() runs, the survivors move down once (nothing else touches this list meanwhile:
        // the processors the chain reaches append to newAndEvery lists only)
        const uint32_t n0 = len(p, 0);
        uint32_t w = 0;
        for (uint32_t i = 0; i < n0; i++) {
            const uint32_t se = at(p, 0, i);
            scanned++;
            bool removed = false;
            if (P.kind == GK_COUNT) {  // CountPreStateProcessor.java:53-95
                if ((G.nslots > P.stateId + 1 && slot(se, P.stateId + 1) != GEN_NIL) ||
                    (G.nslots > P.stateId + 2 && slot(se, P.stateId + 2) != GEN_NIL)) {
                    stDecref(se);
                    continue;
                }
                stIncref(se);
                const uint32_t e = newEv(seq, ts, pos, false);
                if (e != GEN_NIL) addEvent(se, P.stateId, e);
                setFlag(p, GF_SUCCESS, false);
                runChain(p, se);
                if ((retm >> P.thisLast) & 1u) {
                    retm &= ~(1u << P.thisLast);
                    if (nOut < OUTCAP) { stIncref(se); outList[nOut++] = se; } else err |= GERR_CAP;
                }
                if (flag(p, GF_CHANGED)) { stDecref(se); removed = true; }
                if (!flag(p, GF_SUCCESS)) {
                    removeLastEvent(se, P.stateId);
                    if (G.qtype == SG_Q_SEQUENCE && !removed) { stDecref(se); removed = true; }
                }
                stDecref(se);
                if (!removed) { if (w != i) at(p, 0, w) = se; w++; }
                continue;
            }
            if (P.kind == GK_LOGICAL && P.logicalType == SG_L_OR && slot(se, G.pre[P.partner].stateId) != GEN_NIL) {
                stDecref(se);  // LogicalPreStateProcessor.java:153-157
                continue;
            }
            // StreamPreStateProcessor.java:371-397
            stIncref(se);
            if (shared == GEN_NIL) {
                shared = newEv(seq, ts, pos, false);
                evIncref(shared);  // held until the loop ends
            }
            setSlot(se, P.stateId, shared);
            runChain(p, se);
            if ((retm >> P.thisLast) & 1u) {
                retm &= ~(1u << P.thisLast);
                // (an absent state returns nothing, :265-283: its partials are not collected at all, so
                // one event may kill any number of them)
                if (!P.absent) {
                    if (nOut < OUTCAP) { stIncref(se); outList[nOut++] = se; } else err |= GERR_CAP;
                }
            }
            if (flag(p, GF_CHANGED)) {
                stDecref(se);
                removed = true;
            } else {
                setSlot(se, P.stateId, GEN_NIL);
                if (G.qtype == SG_Q_SEQUENCE) {
                    if (!(P.kind == GK_STREAM && P.absent)) { stDecref(se); removed = true; }
                    if (P.kind == GK_STREAM && G.post[P.thisPost].callbackPre != GEN_NONE)
                        startStateReset(G.post[P.thisPost].callbackPre);
                }
            }
            stDecref(se);
            if (!removed) { if (w != i) at(p, 0, w) = se; w++; }
        }
        if (w != n0) len(p, 0) = w;
        evDecref(shared);
        if (P.absent) {  // AbsentStreamPreStateProcessor.processAndReturn returns nothing (:265-283)
            for (uint32_t j = out0; j < nOut; j++) stDecref(outList[j]);
            nOut = out0;
        }
    }

    // ---- receivers ----
    __device__ void stabilize(const __attribute__((address_space(4))) GenRecv& r, int64_t ts) __restrict__ {
        for (int i = 0; i < G.nAll; i++) expireEvents(G.allProcs[i], ts);
        if (G.qtype == SG_Q_SEQUENCE) {  // Sequence*ProcessStreamReceiver.stabilizeStates -> resetAndUpdate
            for (int i = 0; i < G.nReset; i++) resetState(G.resetOrder[i]);
            for (int i = 0; i < G.nUpdate; i++) updateState(G.updateOrder[i]);
        } else if (r.multi) {  // PatternMultiProcessStreamReceiver.java:42-51
            for (int i = 0; i < r.nStateProcs; i++) updateState(r.stateProcs[i]);
        } else if (r.nStateProcs > 0) {  // PatternSingleProcessStreamReceiver.java:34-41
            updateState(r.stateProcs[0]);
        }
    }

    __device__ void initKey() __restrict__ {  // PartitionRuntimeImpl.initPartition -> StateStreamRuntime.initPartition
        const uint32_t w0 = W(0);
        if (w0 & 1u) {
            // (this kernel's allocations do not keep abs_kernels' pool words, nor chn_kernels' layout)
            if (w0 & (GEN_W0_POOLC | GEN_W0_CHN)) W(0) = 1u;
            return;
        }
        W(0) = 1u;
        for (int i = 0; i < G.nInit; i++) init(G.initOrder[i]);
        for (int i = 0; i < G.nStartup; i++) partitionCreated(G.startup[i]);
    }

    __device__ uint32_t defBase() const { return G.offDef; }

    // one event of this key (MultiProcessStreamReceiver / SingleProcessStreamReceiver semantics)
    __device__ void processEvent(const __attribute__((address_space(4))) GenRecv& r, uint32_t pos, bool chunkEnd) __restrict__ {
        const uint64_t seq = A.b.seq_base + pos;
        const int64_t ts = gp(A.b.ts)[pos];
        GENX_T(4);
        stabilize(r, ts);
        GENX_T(1);
        gu32& nd = W(defBase());
        if (r.multi) {
            trigSeq = seq;
            trigIdx = pos;
            trigRank = 0;
            for (int j = r.n - 1; j >= 0; j--) {  // reverse declaration order, projected at once
                uint32_t outl[64];
                uint32_t no = 0;
                processAndReturn(r.procs[j], seq, ts, pos, outl, no);
                GENX_T(2);
                for (uint32_t x = 0; x < no; x++) { project(outl[x]); stDecref(outl[x]); }
                GENX_T(3);
            }
        } else {
            // deferred until the end of the chunk (consecutive events of this key in the batch)
            uint32_t outl[64];
            uint32_t no = 0;
            processAndReturn(r.procs[0], seq, ts, pos, outl, no);
            GENX_T(2);
            for (uint32_t x = 0; x < no; x++) {
                if (nd >= G.DEF) { err |= GERR_CAP; stDecref(outl[x]); continue; }
                W(defBase() + 1 + 2 * nd) = outl[x];
                W(defBase() + 2 + 2 * nd) = pos;
                nd++;
            }
            if (chunkEnd) flushDeferred();
            GENX_T(3);
        }
    }
    __device__ void flushDeferred() __restrict__ {
        gu32& nd = W(defBase());
        uint32_t lastPos = 0xffffffffu;
        for (uint32_t x = 0; x < nd; x++) {
            const uint32_t se = W(defBase() + 1 + 2 * x), pos = W(defBase() + 2 + 2 * x);
            if (pos != lastPos) { trigRank = 0; lastPos = pos; }
            trigIdx = pos;
            trigSeq = A.b.seq_base + pos;
            project(se);
            stDecref(se);
        }
        nd = 0;
    }
};

// the lanes' work counters, reduced over the wave (all 64 lanes call this): one atomic per wave
__device__ void gen_wave_stats(const GenArgs& a, unsigned long long sc, unsigned long long cr, unsigned long long ma,
                               unsigned long long ky, uint32_t er) {
    for (int off = 32; off > 0; off >>= 1) {
        sc += __shfl_xor(sc, off, 64);
        cr += __shfl_xor(cr, off, 64);
        ma += __shfl_xor(ma, off, 64);
        ky += __shfl_xor(ky, off, 64);
        er |= (uint32_t)__shfl_xor((int)er, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (er) atomicOr(a.o.err, er);
        if (sc) atomicAdd(&a.o.stats[GST_SCANNED], sc);
        if (cr) atomicAdd(&a.o.stats[GST_CREATED], cr);
        if (ma) atomicAdd(&a.o.stats[GST_MATCHES], ma);
        if (ky) atomicAdd(&a.o.stats[GST_KEYS], ky);
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// batch: one lane per key walks its key-sorted events
// ------------------------------------------------------------------------------------------------
// Occupancy: GEN_WAVES waves/SIMD (above) for this latency-bound kernel.
// The arguments live in device memory (written by the host before the launch): the lanes hold a
// reference to them, and a reference to a by-value kernel argument would force a private copy of the
// whole struct into every lane's scratch.
// occupancy (waves per SIMD): measured C3_min1 / C4 / C4_deep at 2, 3, 4, 6, 8: 4 best (fewer spills
// at 128 VGPRs outweigh the waves lost)
#ifndef GEN_WAVES
#define GEN_WAVES 4
#endif
// Several keys per lane (a.kpl, sized by the host so that the grid is about one resident wave per slot):
// lane l of block b walks keys (b*kpl + j)*64 + l for j = 0..kpl-1, one flat loop whose every step is
// either one event or the switch to the lane's next key, so a wave runs for the longest SUM of its lanes'
// runs instead of the sum over j of the longest run (Poisson runs of a few events per key: one key per
// lane leaves half of every wave's lane-steps idle).  A wave's 64 lanes still touch 64
// consecutive keys of one row of the interleaved state at each j.
// The kernels below read their GenArgs through the kernarg segment pointer instead of the by-value parameter:
// the interpreter indexes its arrays (columns, null flags) at run time, and taking the parameter's address
// made the compiler copy all ~600 B of it into scratch at kernel entry — 40 MB of writes per 1,024-wave
// launch, even when every wave then left at once.
__device__ __forceinline__ const GenArgs& gen_kernarg() {
    return *(const GenArgs*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
}
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GEN_WAVES, 8))) k_gen_batch(const GenArgs ap) {
    const GenArgs& a = gen_kernarg();
    // a hand-over launch (a fixed grid over a list whose length only the device knows) whose waves have no
    // key leave before the lane object exists: building it (it lives in scratch) wrote ~50 MB per empty launch
    if ((a.mode & GEN_M_KEYLIST) && (unsigned long long)blockIdx.x * 64u >= *a.fb_n) return;
    const uint32_t kpl = a.kpl ? a.kpl : 1u;
    const uint32_t k0 = blockIdx.x * kpl * 64u + threadIdx.x;
    const auto& r = ((const cGenProgram*)a.G)->recv[a.b.stream];
    Lane L(a, k0);
    uint32_t j = 0, i = 0, e = 0;
    bool open = false, any = false;
    unsigned long long ky = 0;
    for (;;) {
        if (!open) {
            uint32_t key = 0;
            if (a.mode & GEN_M_KEYLIST) {  // the keys the register-window kernel handed over, from their resume index
                // (a fixed grid striding over the list: the list length is known on the device only)
                const unsigned long long li = ((unsigned long long)j * gridDim.x + blockIdx.x) * 64u + threadIdx.x;
                if (li >= *a.fb_n) break;
                key = gp(a.fb_list)[li];
                i = gp(a.fb_start)[key];
                e = gp(a.b.seg_end)[key];
            } else {
                for (; j < kpl; j++) {  // the lane's next key with events in this batch
                    key = k0 + j * 64u;
                    if (key < a.K && gp(a.b.seg_begin)[key] < gp(a.b.seg_end)[key]) break;
                }
                if (j >= kpl) break;
                i = gp(a.b.seg_begin)[key];
                e = gp(a.b.seg_end)[key];
            }
            L.retarget(key);
            L.initKey();
            open = true;
            any = true;
#if GENX_PROF
            { const uint64_t t_ = __builtin_amdgcn_s_memtime(); L.prof[0] += t_ - L.prof_t; L.prof_t = t_; }
#endif
            if (r.n == 0) i = e;
        }
        if (i < e) {
            const size_t ss = a.b.sidxStride ? a.b.sidxStride : 1u;
            const uint32_t pos = a.b.sidx ? gp(a.b.sidx)[i * ss] : i;
            const uint32_t nxt = (i + 1 < e) ? (a.b.sidx ? gp(a.b.sidx)[(i + 1) * ss] : i + 1) : 0xffffffffu;
            L.processEvent(r, pos, nxt != pos + 1);
            i++;
        }
        if (i >= e) {  // the key's run is done
            if (a.G->nStartup > 0) gp(a.t.nd)[L.k] = L.nextDeadline();
            ky++;
            open = false;
            j++;
        }
    }
    if (any) {
        // unused reserved raw slots are marked empty
        for (uint32_t x = 0; x < L.resLeft; x++) {
            const unsigned long long rr = L.resBase + x;
            if (rr < L.resEnd) {
                gp(a.o.raw)[rr * a.o.recWords] = 0xffffffffu;
                gp(a.o.tk1)[rr] = 0xffffffffu;  // sorts after every real timer match
            }
        }
#if GENX_PROF
        { const uint64_t t_ = __builtin_amdgcn_s_memtime(); L.prof[4] += t_ - L.prof_t; L.prof_t = t_; }
        if (a.o.prof && (threadIdx.x & 63) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63))
            for (int q = 0; q < 5; q++) atomicAdd(&a.o.prof[q], (unsigned long long)L.prof[q]);
#endif
    }
#if GENX_PROF
    if (a.o.prof && (threadIdx.x & 63) == 0) atomicAdd(&a.o.prof[6], 1ull);
#endif
    gen_wave_stats(a, L.scanned, L.created, L.matches, ky, L.err);
}

// ------------------------------------------------------------------------------------------------
// timer sweep to a.now (sg_advance_time): every key with due timers runs them in the reference order
// ------------------------------------------------------------------------------------------------
namespace {
__device__ __forceinline__ unsigned long long gen_ord64(int64_t t) { return (unsigned long long)t ^ (1ull << 63); }

__device__ void gen_timers_key(const GenArgs& a, uint32_t key, uint64_t di, unsigned long long& sc,
                               unsigned long long& cr, unsigned long long& ma, uint32_t& er) {
    Lane L(a, key);
    const cGenProgram& G = *(cGenProgram*)a.G;
    if (!(L.W(0) & 1u)) {
        if (G.partitioned) {  // a key is created by its first event (not due: nd had no deadline)
            if (G.playback && !(a.mode & GEN_M_NOPAIRS))
                for (int i = 0; i < G.nStartup; i++) {
                    a.t.dpair_key[di * (uint64_t)G.nStartup + (uint64_t)i] = ~0ull;
                    a.t.dpair_i[di * (uint64_t)G.nStartup + (uint64_t)i] = GEN_PAIR_NONE;
                    if (a.t.dpair_kid) a.t.dpair_kid[di * (uint64_t)G.nStartup + (uint64_t)i] = GEN_PAIR_NONE;
                }
            a.t.nd[key] = GEN_NO_DEADLINE;
            return;
        }
        // unpartitioned: QueryRuntimeImpl.start seeds the query at the clock of start()
        L.now = G.playback ? a.now0 : a.now;
        L.initKey();
    } else if (L.W(0) & GEN_W0_POOLC) {
        L.W(0) = 1u;  // (see initKey)
    }
    const int64_t T = a.now;
    if (G.playback) {
        // each Scheduler's time-change listener, in registration order (Scheduler.java:73-104); the
        // listener's TreeMultimap orders the keys by their queue head at collection
        L.now = T;
        for (int i = 0; i < G.nStartup; i++) {
            const int p = G.startup[i];
            const bool due = L.qlen(p) != 0 && L.qhead(p) <= T;
            if (G.partitioned && !(a.mode & GEN_M_NOPAIRS)) {  // the listener's collection of (due time, key): the A.10 check
                const uint64_t slot = di * (uint64_t)G.nStartup + (uint64_t)i;
                a.t.dpair_key[slot] = due ? gen_ord64(L.qhead(p)) : ~0ull;
                a.t.dpair_i[slot] = due ? (uint32_t)i : GEN_PAIR_NONE;
                if (a.t.dpair_kid) a.t.dpair_kid[slot] = due ? key : GEN_PAIR_NONE;
            }
            if (!due) continue;
            L.tk1 = (uint32_t)i;
            L.tk2 = L.qhead(p);
            L.sendTimerEvents(p);
        }
    } else {
        L.now = a.now0;  // the engine clock before this advance
        // EventCallers of this key in time order (Scheduler.EventCaller.run, Scheduler.java:264-298)
        for (int guard = 0; guard < (1 << 20); guard++) {
            int best = -1;
            int64_t bf = 0;
            uint32_t bo = 0;
            for (int i = 0; i < G.nStartup; i++) {
                const int p = G.startup[i];
                if (!L.flag(p, GF_RUNNING)) continue;
                const int64_t f = L.R64(L.ks(p) + KS_FIRE);
                const uint32_t o = L.W(L.ks(p) + KS_ORDER);
                if (f <= T && (best < 0 || f < bf || (f == bf && o < bo))) { best = G.startup[i]; bf = f; bo = o; }
            }
            if (best < 0) break;
            if (bf > L.now) L.now = bf;
            L.tk1 = 0;
            L.tk2 = bf;  // callers of different keys due together run in key order
            L.sendTimerEvents(best);
            if (L.qlen(best) != 0) {
                const int64_t h = L.qhead(best);
                L.W64(L.ks(best) + KS_FIRE, h > L.now ? h : L.now);
                L.W(L.ks(best) + KS_ORDER) = ++L.W(1);
            } else {
                L.setFlag(best, GF_RUNNING, false);
            }
        }
    }
    a.t.nd[key] = L.nextDeadline();
    if (a.t.kcnt) a.t.kcnt[key] = (uint32_t)L.matches;
    sc += L.scanned;
    cr += L.created;
    ma += L.matches;
    er |= L.err;
    for (uint32_t x = 0; x < L.resLeft; x++) {
        const unsigned long long rr = L.resBase + x;
        if (rr < L.resEnd) {
            gp(a.o.raw)[rr * a.o.recWords] = 0xffffffffu;
            gp(a.o.tk1)[rr] = 0xffffffffu;  // sorts after every real timer match
        }
    }
}
}  // namespace

// next deadline of every key from its state (after a restore)
extern "C" __global__ void __launch_bounds__(64) k_gen_deadlines(const GenArgs ap) {
    const GenArgs& a = ap;
    const uint32_t key = blockIdx.x * blockDim.x + threadIdx.x;
    if (key >= a.K) return;
    Lane L(a, key);
    a.t.nd[key] = (L.W(0) & 1u) ? L.nextDeadline() : GEN_NO_DEADLINE;
}

// the keys due at this advance (nd <= now), compacted into t.due: each block takes a contiguous range of
// keys, counts its due keys (wave ballots combined in LDS) and reserves its output range with ONE atomic
// (one atomic per wave serialised ~16K atomics on one counter at 2^20 keys: 150-200 us)
#define GEN_DUE_BLOCK 256
extern "C" __global__ void __launch_bounds__(GEN_DUE_BLOCK) k_gen_due(const int64_t* __restrict__ nd, uint32_t K,
                                                                      int64_t now, uint32_t* __restrict__ due,
                                                                      unsigned long long* __restrict__ ndue) {
    constexpr uint32_t NW = GEN_DUE_BLOCK / 64;
    __shared__ uint32_t wcnt[NW];
    __shared__ unsigned long long bbase;
    const int lane = threadIdx.x & 63;
    const uint32_t wv = threadIdx.x / 64;
    const uint32_t per = (K + gridDim.x - 1) / gridDim.x;              // keys of this block
    const uint32_t lo = min(K, blockIdx.x * per), hi = min(K, lo + per);
    const uint32_t step = GEN_DUE_BLOCK;
    // pass 1: count
    uint32_t mine = 0;
    for (uint32_t k = lo + threadIdx.x; k < hi; k += step) mine += nd[k] <= now ? 1u : 0u;
    for (int off = 32; off > 0; off >>= 1) mine += (uint32_t)__shfl_xor((int)mine, off, 64);
    if (lane == 0) wcnt[wv] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < NW; w++) t += wcnt[w];
        bbase = t ? atomicAdd(ndue, (unsigned long long)t) : 0ull;
    }
    __syncthreads();
    // pass 2: write, in key order inside the block (ballot prefix per wave row, a running offset per row)
    unsigned long long pos = bbase;
    for (uint32_t base = lo; base < hi; base += step) {
        const uint32_t k = base + threadIdx.x;
        const bool d = k < hi && nd[k] <= now;
        const unsigned long long m = __ballot(d);
        if (lane == 0) wcnt[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, row = 0;
        for (uint32_t w = 0; w < NW; w++) {
            before += w < wv ? wcnt[w] : 0u;
            row += wcnt[w];
        }
        if (d) due[pos + before + __popcll(m & ((1ull << lane) - 1ull))] = k;
        pos += row;
        __syncthreads();
    }
}

// sorted (due time, listener) pairs of one advance: two equal ones = two keys share a due time (A.10)
extern "C" __global__ void __launch_bounds__(256) k_gen_collapse(const unsigned long long* __restrict__ key,
                                                                 const uint32_t* __restrict__ li, uint64_t n,
                                                                 uint32_t* __restrict__ err) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j == 0 || j >= n || li[j] == GEN_PAIR_NONE || key[j] != key[j - 1]) return;
    for (uint64_t m = j; m-- > 0 && key[m] == key[j];)
        if (li[m] == li[j]) { atomicOr(err, (uint32_t)GERR_COLLAPSE); return; }
}

// timer sweep over the due keys (every key when unpartitioned: key 0, seeded at start())
// occupancy of the timer sweep (waves per SIMD), separate from the batch kernel's
#ifndef GEN_TWAVES
#define GEN_TWAVES GEN_WAVES
#endif
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GEN_TWAVES, 8))) k_gen_timers(const GenArgs ap) {
    const GenArgs& a = gen_kernarg();
#if GENX_PROF
    const uint64_t t0_ = __builtin_amdgcn_s_memtime();
#endif
    const uint64_t n = a.G->partitioned ? *a.t.ndue : 1ull;
    if ((uint64_t)blockIdx.x * blockDim.x >= n) return;   // (waves with no due key: nothing to count)
    unsigned long long sc = 0, cr = 0, ma = 0;
    uint32_t er = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        gen_timers_key(a, a.G->partitioned ? a.t.due[i] : 0u, i, sc, cr, ma, er);
#if GENX_PROF
    if (a.o.prof && (threadIdx.x & 63) == 0) atomicAdd(&a.o.prof[5], (unsigned long long)(__builtin_amdgcn_s_memtime() - t0_));
#endif
    unsigned long long mw = ma;
    for (int off = 32; off > 0; off >>= 1) mw += __shfl_xor(mw, off, 64);
    if ((threadIdx.x & 63) == 0 && mw) atomicAdd(a.o.nvalid, mw);  // timer matches of this wave
    gen_wave_stats(a, sc, cr, ma, 0, er);
}
