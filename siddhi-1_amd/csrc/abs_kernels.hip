// abs_kernels.hip — register-window kernels for the absent-tail pattern
//
//     [every] e1=S[f0] -> not S[f1(e1)] for T [within W]      (PATTERN, partitioned, @app:playback)
//
// (BASELINE configs[3], "C4").  The general kernels (gen_kernels.hip) interpret the processor graph with
// every partial match in the key-interleaved state blocks of HBM: each partial a key creates costs ~40
// word stores to the StateEvent / StreamEvent pools even when it dies a few events later.  These kernels
// run the same two processors on the same state with one lane per key, but hold the key's lists in
// registers for the whole walk:
//   start processor p0   its seed (pending or staged: at most one), the seed's timestamp
//   absent processor p1  a window of ABS_R partials {e1 ts, e1 seq, e1's attribute words, null bits}
//                        in list order (pending slots, then staged), lastScheduledTime, the timer queue's
//                        head / length (entries appended straight to the HBM ring)
// and write the lists back once per key into the general blocks: StateEvent 0 = the seed, and each partial
// keeps the pool entry it was created in (StreamEvent e, StateEvent 1 + e) for its whole life, so a
// write-back stores the list words, the header, word 0 of the free bitmaps and only the records of the
// partials created in this walk (a key loaded in another layout is rewritten whole, partial j at entry j).
// The state stays the general
// engine's state: snapshots, state documents, purge and the general kernels read it unchanged.  A key this
// path cannot hold (a shared or foreign-shaped list, more than ABS_R partials, a queue about to fill) is
// handed to the general kernel from the event where it stops (k_gen_batch GEN_M_KEYLIST) or for its whole
// timer sweep (k_gen_timers over the list), so the results stay exactly the general engine's.
//
// Semantics restated from (paths under /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/):
//   query/input/stream/state/StreamPreStateProcessor.java:118-129 isExpired, :214-247 addState /
//       addEveryState, :308-323 updateState (stable sort by ts, -1 last), :325-361 expireEvents,
//       :364-403 processAndReturn
//   query/input/stream/state/StreamPostStateProcessor.java:64-83 (the start state's post processing)
//   query/input/stream/state/AbsentStreamPreStateProcessor.java:80-103 addState (schedules ts + T),
//       :150-227 process (the TIMER event), :256-274 processAndReturn (returns nothing)
//   query/input/stream/state/AbsentStreamPostStateProcessor.java:36-56 (a matching event kills the partial
//       and reschedules at its ts + T)
//   query/input/stream/state/receiver/PatternMultiProcessStreamReceiver.java:31-51 (stabilize, then the
//       later state first)
//   util/Scheduler.java:114-128 notifyAt, :172-210 sendTimerEvents
#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu.h"
#include "../../include/siddhi_gpu_ir.h"
#include "gen_engine.h"
#include "java_ops.h"
#include "sg_engine.h"
#include "reg_common.h"

namespace {

// one key's absent-tail state during a walk (see the file comment); TM: the timer sweep, which also keeps
// the first ABS_QP entries of the timer queue in registers (the pops of one sweep need no dependent loads)
#define ABS_QP 4
// FF: the filters are decoded compares (GenPre.ff; a kernel variant of its own, so the interpreter's registers
// are not allocated beside them)
template <int NW, bool TM, bool FF = false> struct AbsKey {
    const cGenProgram& G;
    gu32* S;
    uint32_t K, k;
    uint32_t ks0, ks1;  // KeyState word offsets of p0 / p1
    int stream, slot0, slot1;
    // window: slots [0, n) live, [0, np) pending, [np, n) staged (newAndEvery)
    int64_t ts[ABS_R];
    uint64_t seq[ABS_R];
    uint32_t w[ABS_R][NW];
    uint32_t nb[ABS_R];
    uint32_t n, np;
    uint32_t px[ABS_R];   // slot j's pool entry: StreamEvent px[j], StateEvent 1 + px[j]
    uint32_t used;        // the pool entries in use (bit e)
    uint32_t dpool;       // the pool entries whose records this walk wrote into registers (stored)
    bool canon;           // loaded in this layout: only the new records and bitmap word 0 need storing
    uint32_t hw0;         // pool entries [0, hw0) hold their constant words (GEN_W0_POOLC, as loaded)
    uint32_t used0;       // the entries of the partials as loaded (checked: their constant words are in place)
    bool seed0;           // a seed was loaded (at StateEvent 0), with timestamp seedTs0
    int64_t seedTs0;
    uint32_t h0[8];       // the header words as loaded (canon: only the changed ones are stored)
    bool sbad;            // the staged slots may be out of ts order (promotion sorts them)
    uint32_t seedPend, seedStg;
    int64_t seedPendTs, seedStgTs;
    uint32_t f0, f1;      // the processors' flag words
    int64_t lst;          // p1 lastScheduledTime
    uint32_t qh, ql;      // p1 timer queue head index / length
    int64_t qhv;          // the head entry (valid while ql > 0)
    int64_t qbuf[ABS_QP]; // TM: queue entries [qh, qh + qb)
    uint32_t qb;
    uint32_t err;
    unsigned long long scanned, created, matches;
    // the register-native record (GEN_W0_REG; nullptr: the block only).  In record mode the window is stored
    // in list order (slot j at record entry j: slots [dmin, n) differ from the record) and the timer queue is
    // linear (entries [qh, qh + ql) of its rows; stored from row 0)
    gu32* R;
    bool wasRec;
    uint32_t dmin;

    __device__ AbsKey(const GenProgram* g, uint32_t* state, uint32_t K_, uint32_t key, uint32_t* rec = nullptr)
        : G(*(cGenProgram*)g), S(gp(state)), K(K_), k(key), n(0), np(0), used(0), dpool(0), canon(false),
          hw0(0), used0(0), seed0(false), seedTs0(0), sbad(false), seedPend(0), seedStg(0),
          seedPendTs(-1), seedStgTs(-1), f0(0), f1(0), lst(0), qh(0), ql(0), qhv(0), qb(0), err(0), scanned(0), created(0),
          matches(0), R(rec ? gp(rec) : nullptr), wasRec(false), dmin(0) {
        ks0 = G.offKS + (uint32_t)G.absP0 * G.ksWords;
        ks1 = G.offKS + (uint32_t)G.absP1 * G.ksWords;
        stream = G.slotStream[G.pre[G.absP0].stateId];
        slot0 = G.pre[G.absP0].stateId;
        slot1 = G.pre[G.absP1].stateId;
    }

    __device__ __forceinline__ gu32& W(uint32_t w_) const { return S[gen_il(K, k, w_)]; }
    __device__ __forceinline__ int64_t R64(uint32_t w_) const {
        return (int64_t)((uint64_t)W(w_) | ((uint64_t)W(w_ + 1) << 32));
    }
    __device__ __forceinline__ void W64(uint32_t w_, int64_t v) const {
        W(w_) = (uint32_t)(uint64_t)v;
        W(w_ + 1) = (uint32_t)((uint64_t)v >> 32);
    }
    __device__ __forceinline__ uint32_t qword(uint32_t i) const { return ks1 + KS_LISTS + 2 * G.L + 2 * i; }
    // the record: header rows, window entry rows, the queue's 64-bit rows
    __device__ __forceinline__ gu32& RW(uint32_t w_) const { return R[(size_t)w_ * K + k]; }
    __device__ __forceinline__ uint32_t rev(uint32_t j, uint32_t f) const { return GEN_REC_EV + j * (5u + NW) + f; }
    __device__ __forceinline__ __attribute__((address_space(1))) unsigned long long& Q64(uint32_t i) const {
        return ((__attribute__((address_space(1))) unsigned long long*)(R + (size_t)gen_rec_q(NW) * K))[(size_t)i * K + k];
    }
    // queue entry at position p of the walk (record: linear rows; block: the ring)
    __device__ __forceinline__ int64_t qget(uint32_t p) const {
        if (R) return (int64_t)Q64(p);
        return R64(qword(p >= G.Q ? p - G.Q : p));
    }

    // ---- the record (GEN_W0_REG): header row 0 = n | np << 4 | seedPend << 8 | seedStg << 9 | sbad << 10 |
    // f0 << 16 | f1 << 24, rows 1-2 the seed's ts, 3-4 lastScheduledTime, 5 the queue length (head at row 0)
    __device__ void loadRec() {
        const uint32_t h = RW(0);
        n = h & 15u;
        np = (h >> 4) & 15u;
        seedPend = (h >> 8) & 1u;
        seedStg = (h >> 9) & 1u;
        sbad = (h >> 10) & 1u;
        f0 = (h >> 16) & 0xffu;
        f1 = h >> 24;
        seedPendTs = seedStgTs = (int64_t)((uint64_t)RW(1) | ((uint64_t)RW(2) << 32));
        lst = (int64_t)((uint64_t)RW(3) | ((uint64_t)RW(4) << 32));
        ql = RW(5);
        qh = 0;
#pragma unroll
        for (int j = 0; j < ABS_R; ++j) {
            // (every element loaded and assigned unconditionally — a slot past n reads the header row, a cache
            // hit — because conditional assignments to the window's elements keep the key object in scratch)
            const bool live = (uint32_t)j < n;
            uint32_t x[5 + NW];
#pragma unroll
            for (int f = 0; f < 5 + NW; ++f) {
                const uint32_t v = RW(live ? rev(j, (uint32_t)f) : 0u);
                x[f] = live ? v : 0u;
            }
            seq[j] = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
            ts[j] = (int64_t)((uint64_t)x[2] | ((uint64_t)x[3] << 32));
            nb[j] = x[4];
#pragma unroll
            for (int q = 0; q < NW; ++q) w[j][q] = x[5 + q];
        }
        wasRec = true;
        dmin = n;
    }
    // the header, the window entries [dmin, n), the queue moved to row 0 when its head advanced
    __device__ void storeRec() const {
        if (!wasRec) W(0) = 1u | GEN_W0_REG;
        const int64_t sts = seedPend ? seedPendTs : seedStgTs;
        RW(0) = n | (np << 4) | (seedPend << 8) | (seedStg << 9) | (sbad ? 1024u : 0u) | (f0 << 16) | (f1 << 24);
        RW(1) = (uint32_t)(uint64_t)sts;
        RW(2) = (uint32_t)((uint64_t)sts >> 32);
        RW(3) = (uint32_t)(uint64_t)lst;
        RW(4) = (uint32_t)((uint64_t)lst >> 32);
        RW(5) = ql;
        for (uint32_t j = dmin; j < n; j++) {   // (slot j's registers picked by selects: no dynamic indexing)
            uint32_t pn = 0, pw[NW];
            int64_t t = 0;
            uint64_t q = 0;
#pragma unroll
            for (int x = 0; x < NW; ++x) pw[x] = 0;
#pragma unroll
            for (int y = 0; y < ABS_R; ++y) {
                if ((uint32_t)y == j) {
                    t = ts[y]; q = seq[y]; pn = nb[y];
#pragma unroll
                    for (int x = 0; x < NW; ++x) pw[x] = w[y][x];
                }
            }
            RW(rev(j, 0)) = (uint32_t)q;
            RW(rev(j, 1)) = (uint32_t)(q >> 32);
            RW(rev(j, 2)) = (uint32_t)(uint64_t)t;
            RW(rev(j, 3)) = (uint32_t)((uint64_t)t >> 32);
            RW(rev(j, 4)) = pn;
#pragma unroll
            for (int x = 0; x < NW; ++x) RW(rev(j, 5u + (uint32_t)x)) = pw[x];
        }
        if constexpr (TM) {   // (only a sweep pops)
            if (qh)
                for (uint32_t i = 0; i < ql; i++) Q64(i) = Q64(qh + i);
        }
    }
    // the general layout from the registers (a hand-over to the general / wave-per-key kernels, a flush): the
    // queue back into the block's ring from position 0, then every record (word 0 loses GEN_W0_REG)
    __device__ __forceinline__ void store_general() const { store(true); }

    // ---- load: false = this key's lists are not of the shape the window holds (the general kernel takes it)
    __device__ __forceinline__ bool load() {
#pragma unroll
        for (int j = 0; j < ABS_R; ++j) px[j] = (uint32_t)j;
        const uint32_t w0 = W(0);
        if (!(w0 & 1u)) {  // PartitionRuntimeImpl.initPartition: p0.init() stages one seed; p1.partitionCreated()
            seedStg = 1;
            seedStgTs = -1;
            f0 = GF_INIT;
            f1 = GF_STARTED;
            return true;     // (canon = false: the zeroed block is written whole)
        }
        if (w0 & GEN_W0_DEEP) return false;   // (the lists are in the deep store: the wave-per-key kernels take it)
        if ((w0 & GEN_W0_REG) && R) {
            loadRec();
            if constexpr (TM) qfill();
            else qhv = ql ? (int64_t)Q64(0) : 0;
            return true;
        }
        canon = true;
        f0 = W(ks0 + KS_FLAGS);
        f1 = W(ks1 + KS_FLAGS);
        if ((f0 | f1) & (GF_INACTIVE | GF_RUNNING)) return false;
        const uint32_t p0n = W(ks0 + KS_PLEN), s0n = W(ks0 + KS_NLEN);
        if (p0n + s0n > 1u) return false;
        if (p0n + s0n == 1u) {
            const uint32_t st = W(ks0 + KS_LISTS + (p0n ? 0u : G.L));
            if (st >= G.STCAP) return false;
            const uint32_t b = G.offST + st * G.stWords;
            if (W(b + ST_TYPE) != 0u || W(b + ST_RC) != 1u) return false;
            for (int s = 0; s < G.nslots; s++)
                if (W(b + ST_SLOTS + (uint32_t)s) != GEN_NIL) return false;
            const int64_t t = R64(b + ST_TS);
            if (p0n) { seedPend = 1; seedPendTs = t; } else { seedStg = 1; seedStgTs = t; }
            canon = canon && st == 0u;
            seed0 = true;
            seedTs0 = t;
        }
        np = W(ks1 + KS_PLEN);
        const uint32_t ns = W(ks1 + KS_NLEN);
        if (np + ns > (uint32_t)ABS_R) return false;
        const uint32_t lim = pool_lim();
        n = np + ns;
        bool ok = true;
        int64_t prev = 0;
#pragma unroll
        for (int j = 0; j < ABS_R; ++j) {
            ts[j] = 0;
            seq[j] = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) w[j][q] = 0;
            nb[j] = 0;
            if ((uint32_t)j < n) {
                const uint32_t st = W(ks1 + KS_LISTS + ((uint32_t)j < np ? (uint32_t)j : G.L + (uint32_t)j - np));
                ok = ok && st < G.STCAP;
                const uint32_t b = G.offST + (st < G.STCAP ? st : 0u) * G.stWords;
                const uint32_t e = W(b + ST_SLOTS + (uint32_t)slot0);
                ok = ok && W(b + ST_TYPE) == 0u && W(b + ST_RC) == 1u && e < G.SECAP &&
                     W(b + ST_SLOTS + (uint32_t)slot1) == GEN_NIL;
                const uint32_t eb = G.offSE + (e < G.SECAP ? e : 0u) * G.seWords;
                const int64_t t = R64(b + ST_TS);
                ok = ok && W(eb + SE_NEXT) == GEN_NIL && W(eb + SE_RC) == 1u && R64(eb + SE_TS) == t;
                ts[j] = t;
                canon = canon && st == 1u + e && e < lim;
                px[j] = e < G.SECAP ? e : 0u;
                used |= e < 32u ? 1u << e : 0u;
                if ((uint32_t)j > np && ts_before(t, prev)) sbad = true;
                prev = t;
            }
        }
        if (!ok) return false;
        // the partials' payload: the timer sweep of a key in this layout reads none of it (a timer tests
        // timestamps; an emitted partial's seq is read when it fires, and no record is rewritten)
        if (!TM || !canon || R) {   // (record mode: the key's window is rewritten into the record)
#pragma unroll
            for (int j = 0; j < ABS_R; ++j) {
                if ((uint32_t)j < n) {
                    const uint32_t eb = G.offSE + px[j] * G.seWords;
                    seq[j] = (uint64_t)R64(eb + SE_SEQ);
                    nb[j] = W(eb + SE_NULL);
                    const int na = G.nattr[stream];
                    for (int a = 0; a < na; a++) {
                        const int ty = G.attrType[stream][a];
                        const bool wide = ty == SG_T_LONG || ty == SG_T_DOUBLE;
                        const uint32_t o = G.absOff[a];
                        const uint32_t lo = W(eb + SE_ATTR + 2 * (uint32_t)a);
                        const uint32_t hi = wide ? W(eb + SE_ATTR + 2 * (uint32_t)a + 1) : 0u;
#pragma unroll
                        for (int q = 0; q < NW; ++q) {
                            if ((uint32_t)q == o) w[j][q] = lo;
                            if (wide && (uint32_t)q == o + 1) w[j][q] = hi;
                        }
                    }
                }
            }
        }
        if (R) canon = false;   // (record mode: no pool entries; a hand-over writes partial j at entry j)
        hw0 = (canon && (w0 & GEN_W0_POOLC)) ? (w0 >> 2) & 63u : 0u;
        used0 = used;
        if (!canon) {  // rewritten whole at the store, partial j at entry j
#pragma unroll
            for (int j = 0; j < ABS_R; ++j) px[j] = (uint32_t)j;
        }
        lst = R64(ks1 + KS_LST);
        qh = W(ks1 + KS_QHEAD);
        ql = W(ks1 + KS_QLEN);
        if (qh >= G.Q || ql > G.Q) return false;
        if (R) {   // record mode: the queue's entries from the ring to the record's rows [0, ql)
            for (uint32_t i = 0; i < ql; i++) {
                const uint32_t p = qh + i;
                Q64(i) = (unsigned long long)R64(qword(p >= G.Q ? p - G.Q : p));
            }
            qh = 0;
        }
        hdr(h0);
        if constexpr (TM) {
            qfill();
        } else {
            if (ql) qhv = R64(qword(qh));
        }
        return true;
    }
    // TM: (re)load the buffered queue entries (independent loads, all in flight together)
    __device__ __forceinline__ void qfill() {
        qb = ql < (uint32_t)ABS_QP ? ql : (uint32_t)ABS_QP;
#pragma unroll
        for (int i = 0; i < ABS_QP; ++i) qbuf[i] = (uint32_t)i < qb ? qget(qh + (uint32_t)i) : 0;
        qhv = qbuf[0];
    }

    // the pool entries a partial may take: e < 31 (StateEvent 1 + e in bitmap word 0) and inside both pools
    __device__ __forceinline__ uint32_t pool_lim() const {
        uint32_t l = 31u;
        l = G.SECAP < l ? G.SECAP : l;
        l = G.STCAP - 1u < l ? G.STCAP - 1u : l;
        return l;
    }
    // the partials the window may hold: its slots, and pool entries for all of them
    __device__ __forceinline__ uint32_t cap_n() const {
        const uint32_t l = pool_lim();
        return l < (uint32_t)ABS_R ? l : (uint32_t)ABS_R;
    }
    // a pool entry for a new partial (the lowest free one: n < cap_n() <= pool_lim entries are in use)
    __device__ __forceinline__ uint32_t alloc() {
        const uint32_t lim = pool_lim();
        const uint32_t fr = ~used & (lim >= 32u ? 0xffffffffu : ((1u << lim) - 1u));
        // (branch-free: a branch that updates one member or another becomes a select of member addresses,
        // which puts the struct in scratch)
        const uint32_t e = fr ? (uint32_t)__ffs(fr) - 1u : 0u;
        const uint32_t bit = fr ? 1u << e : 0u;
        err |= fr ? 0u : (uint32_t)GERR_REF;
        used |= bit;
        dpool |= bit;
        return e;
    }

    // ---- store: the header, the list words, the records of the partials this walk created (every record
    // when the key was loaded in another layout), the free bitmaps (word 0; all words then)
    // (general: the general layout even in record mode — one call site of store_all, whose second inlined copy
    // would keep the key object in scratch)
    __device__ __forceinline__ void store(bool general = false) const {
        if (R && !general) {
            storeRec();
            return;
        }
        if (R)   // the record's linear queue back into the block's ring from position 0
            for (uint32_t i = 0; i < ql; i++) W64(qword(i), (int64_t)Q64(qh + i));
        if (!canon || R) {
            store_all(R ? 0u : qh);
            return;
        }
        uint32_t h[8];
        hdr(h);
        const uint32_t at[8] = {ks0 + KS_FLAGS, ks0 + KS_PLEN, ks0 + KS_NLEN, ks1 + KS_FLAGS, ks1 + KS_LST,
                                ks1 + KS_LST + 1, ks1 + KS_QHEAD, ks1 + KS_QLEN};
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (h[i] != h0[i]) W(at[i]) = h[i];
        if (seedPend && !h0[1]) W(ks0 + KS_LISTS) = 0u;
        if (seedStg && !h0[2]) W(ks0 + KS_LISTS + G.L) = 0u;
        uint32_t cw = 0;   // entries whose records (constant words included) this store writes
        const int64_t sts = seedPend ? seedPendTs : seedStgTs;
        if ((seedPend | seedStg) && (!seed0 || sts != seedTs0)) {
            const uint32_t b = G.offST;
            W64(b + ST_TS, sts);
            if (!seed0) {
                W(b + ST_TYPE) = 0u;
                W(b + ST_RC) = 1u;
                for (int s = 0; s < G.nslots; s++) W(b + ST_SLOTS + (uint32_t)s) = GEN_NIL;
            }
        }
        W(ks1 + KS_PLEN) = np;
        W(ks1 + KS_NLEN) = n - np;
        for (uint32_t j = 0; j < n; j++) {   // (slot j's registers picked by selects: no dynamic indexing)
            uint32_t e = 0, pn = 0, pw[NW];
            int64_t t = 0;
            uint64_t q = 0;
#pragma unroll
            for (int x = 0; x < NW; ++x) pw[x] = 0;
#pragma unroll
            for (int y = 0; y < ABS_R; ++y) {
                if ((uint32_t)y == j) {
                    e = px[y]; t = ts[y]; q = seq[y]; pn = nb[y];
#pragma unroll
                    for (int x = 0; x < NW; ++x) pw[x] = w[y][x];
                }
            }
            W(ks1 + KS_LISTS + (j < np ? j : G.L + j - np)) = 1u + e;
            if ((dpool >> e) & 1u) {
                put_record(e, t, q, pn, pw);
                cw |= 1u << e;
            }
        }
        // the entries whose constant words are now known in place: below hw0, the partials loaded, the records
        // just written; the new mark is the run of them from entry 0
        const uint32_t V = (hw0 >= 32u ? 0xffffffffu : ((1u << hw0) - 1u)) | used0 | cw;
        const uint32_t hw = ~V ? (uint32_t)__ffs(~V) - 1u : 32u;
        if (hw != hw0) W(0) = 1u | GEN_W0_POOLC | (hw << 2);
        W(G.offSTfree) = ((seedPend | seedStg) ? 1u : 0u) | (used << 1);
        W(G.offSEfree) = used;
    }
    // pool entry e's constant words (a partial of this shape: StateEvent 1 + e of type 0 holding StreamEvent e
    // in slot0, both referenced once, no chain)
    __device__ __forceinline__ void put_consts(uint32_t e) const {
        const uint32_t b = G.offST + (1u + e) * G.stWords;
        const uint32_t eb = G.offSE + e * G.seWords;
        W(b + ST_TYPE) = 0u;
        W(b + ST_RC) = 1u;
        for (int s = 0; s < G.nslots; s++) W(b + ST_SLOTS + (uint32_t)s) = s == slot0 ? e : GEN_NIL;
        W(eb + SE_NEXT) = GEN_NIL;
        W(eb + SE_RC) = 1u;
    }
    // the header words store() compares: p0 flags / pending / staged seed counts, p1 flags, lastScheduledTime,
    // the timer queue's head and length
    __device__ __forceinline__ void hdr(uint32_t (&h)[8]) const {
        h[0] = f0; h[1] = seedPend; h[2] = seedStg; h[3] = f1;
        h[4] = (uint32_t)(uint64_t)lst; h[5] = (uint32_t)((uint64_t)lst >> 32); h[6] = qh; h[7] = ql;
    }
    // a partial's StateEvent / StreamEvent records at its pool entry e
    __device__ __forceinline__ void put_record(uint32_t e, int64_t t, uint64_t q, uint32_t pn,
                                               const uint32_t (&pw)[NW]) const {
        const uint32_t b = G.offST + (1u + e) * G.stWords;
        const uint32_t eb = G.offSE + e * G.seWords;
        W64(b + ST_TS, t);
        if (e >= hw0) put_consts(e);
        W64(eb + SE_SEQ, (int64_t)q);
        W64(eb + SE_TS, t);
        W(eb + SE_NULL) = pn;
        const int na = G.nattr[stream];
        for (int a = 0; a < na; a++) {
            const int ty = G.attrType[stream][a];
            const bool wide = ty == SG_T_LONG || ty == SG_T_DOUBLE;
            const uint32_t o = G.absOff[a];
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (int x = 0; x < NW; ++x) {
                if ((uint32_t)x == o) lo = pw[x];
                if ((uint32_t)x == o + 1) hi = pw[x];
            }
            W(eb + SE_ATTR + 2 * (uint32_t)a) = lo;
            if (wide) W(eb + SE_ATTR + 2 * (uint32_t)a + 1) = hi;
        }
    }
    // a key loaded in another layout (or created here): every record, partial j at entry j (px[j] = j: the
    // window's entries were assigned in slot order), the constant words of the free entries, every bitmap word
    __device__ __forceinline__ void store_all(uint32_t qhead) const {
        W(0) = 1u | GEN_W0_POOLC | (n << 2);  // (entries [0, n) written below)
        W(ks0 + KS_FLAGS) = f0;
        W(ks0 + KS_PLEN) = seedPend;
        W(ks0 + KS_NLEN) = seedStg;
        if (seedPend) W(ks0 + KS_LISTS) = 0u;
        if (seedStg) W(ks0 + KS_LISTS + G.L) = 0u;
        if (seedPend | seedStg) {
            const uint32_t b = G.offST;
            W64(b + ST_TS, seedPend ? seedPendTs : seedStgTs);
            W(b + ST_TYPE) = 0u;
            W(b + ST_RC) = 1u;
            for (int s = 0; s < G.nslots; s++) W(b + ST_SLOTS + (uint32_t)s) = GEN_NIL;
        }
        W(ks1 + KS_FLAGS) = f1;
        W64(ks1 + KS_LST, lst);
        W(ks1 + KS_QHEAD) = qhead;
        W(ks1 + KS_QLEN) = ql;
        W(ks1 + KS_PLEN) = np;
        W(ks1 + KS_NLEN) = n - np;
        const int na = G.nattr[stream];
#pragma unroll
        for (int j = 0; j < ABS_R; ++j) {
            if ((uint32_t)j < n) {
                W(ks1 + KS_LISTS + ((uint32_t)j < np ? (uint32_t)j : G.L + (uint32_t)j - np)) = 1u + (uint32_t)j;
                const uint32_t b = G.offST + (1u + (uint32_t)j) * G.stWords;
                W64(b + ST_TS, ts[j]);
                W(b + ST_TYPE) = 0u;
                W(b + ST_RC) = 1u;
                for (int s = 0; s < G.nslots; s++) W(b + ST_SLOTS + (uint32_t)s) = s == slot0 ? (uint32_t)j : GEN_NIL;
                const uint32_t eb = G.offSE + (uint32_t)j * G.seWords;
                W64(eb + SE_SEQ, (int64_t)seq[j]);
                W64(eb + SE_TS, ts[j]);
                W(eb + SE_NEXT) = GEN_NIL;
                W(eb + SE_RC) = 1u;
                W(eb + SE_NULL) = nb[j];
                for (int a = 0; a < na; a++) {
                    const int ty = G.attrType[stream][a];
                    const bool wide = ty == SG_T_LONG || ty == SG_T_DOUBLE;
                    const uint32_t o = G.absOff[a];
                    uint32_t lo = 0, hi = 0;
#pragma unroll
                    for (int q = 0; q < NW; ++q) {
                        if ((uint32_t)q == o) lo = w[j][q];
                        if ((uint32_t)q == o + 1) hi = w[j][q];
                    }
                    W(eb + SE_ATTR + 2 * (uint32_t)a) = lo;
                    if (wide) W(eb + SE_ATTR + 2 * (uint32_t)a + 1) = hi;
                }
            }
        }
        // free bitmaps: StateEvents {0 if a seed} + [1, 1 + n), StreamEvents [0, n)
        const uint32_t stBits = (seedPend | seedStg) ? 1u : 0u;
        for (uint32_t x = 0; x < (G.STCAP + 31) / 32; x++) {
            uint32_t m = 0;
            if (x == 0) m = stBits | (n >= 31u ? 0xfffffffeu : (((1u << n) - 1u) << 1));
            else if (n + 1 > 32 * x) m = (n + 1 >= 32 * (x + 1)) ? 0xffffffffu : ((1u << (n + 1 - 32 * x)) - 1u);
            W(G.offSTfree + x) = m;
        }
        for (uint32_t x = 0; x < (G.SECAP + 31) / 32; x++) {
            uint32_t m = 0;
            if (n > 32 * x) m = (n >= 32 * (x + 1)) ? 0xffffffffu : ((1u << (n - 32 * x)) - 1u);
            W(G.offSEfree + x) = m;
        }
    }

    __device__ __forceinline__ int64_t deadline() const { return ql ? qhv : GEN_NO_DEADLINE; }

    // Scheduler.notifyAt under playback (Scheduler.java:114-128): append to the key's queue
    __device__ __forceinline__ void notifyAt(int64_t t) {
        if (ql >= G.Q || (R && qh + ql >= G.Q)) { err |= GERR_CAP; return; }
        if (R) Q64(qh + ql) = (unsigned long long)t;   // (rows: a sweep pops before it appends, so qh + ql < Q)
        else W64(qword((qh + ql) % G.Q), t);  // (TM: the buffer stays a prefix of the queue; a pop past it reloads)
        if (ql == 0) qhv = t;
        ql++;
    }
    __device__ __forceinline__ void qpop() {
        if constexpr (TM) {
            if (qb == 0) qfill();
            qh = R ? qh + 1 : (qh + 1) % G.Q;
            ql--;
#pragma unroll
            for (int i = 0; i + 1 < ABS_QP; ++i) qbuf[i] = qbuf[i + 1];
            qb--;
            if (qb == 0 && ql) qfill();
            if (ql) qhv = qbuf[0];
        } else {
            qh = R ? qh + 1 : (qh + 1) % G.Q;
            ql--;
            if (ql) qhv = qget(qh);
        }
    }

    // ---- the window ----
    __device__ __forceinline__ void copy_slot(int d, int s) {
        px[d] = px[s];
        ts[d] = ts[s];
        seq[d] = seq[s];
#pragma unroll
        for (int q = 0; q < NW; ++q) w[d][q] = w[s][q];
        nb[d] = nb[s];
    }
    // drop the slots whose bit is set in `drop`, keeping the order of the rest: every kept slot moves down
    // by the number of dropped slots below it, in log2(ABS_R) collision-free steps (static register indices)
    __device__ __forceinline__ void remove(uint32_t drop) {
        drop &= (n >= 32u ? 0xffffffffu : ((1u << n) - 1u));
        if (!drop) return;
        const uint32_t keep = ((n >= 32u ? 0xffffffffu : ((1u << n) - 1u))) & ~drop;
        const uint32_t lo = (uint32_t)__ffs(drop) - 1u;   // the slots from the lowest dropped one move
        dmin = lo < dmin ? lo : dmin;
        if (canon) {  // the dropped partials' pool entries are free again
#pragma unroll
            for (int j = 0; j < ABS_R; ++j)
                if ((drop >> j) & 1u) used &= ~(1u << px[j]);
        }
        uint32_t d[ABS_R];
#pragma unroll
        for (int j = 0; j < ABS_R; ++j) d[j] = __popc(drop & ((1u << j) - 1u));
        uint32_t cur = keep;
#pragma unroll
        for (int s = 0; (1 << s) < ABS_R; ++s) {
            const int sh = 1 << s;
#pragma unroll
            for (int j = sh; j < ABS_R; ++j) {
                if (((cur >> j) & 1u) && ((d[j] >> s) & 1u)) {
                    copy_slot(j - sh, j);
                    d[j - sh] = d[j];
                    cur = (cur & ~(1u << j)) | (1u << (j - sh));
                }
            }
        }
        const uint32_t lowMask = np >= 32u ? 0xffffffffu : ((1u << np) - 1u);
        np -= __popc(drop & lowMask);
        n -= __popc(drop);
    }
    // updateState: the staged slots join the pending list, stable-sorted by ts (eventTimeComparator)
    __device__ __forceinline__ void promote() {
        if (n > np && sbad) {
            dmin = np < dmin ? np : dmin;
#pragma unroll
            for (int pass = 0; pass < ABS_R - 1; ++pass) {
#pragma unroll
                for (int j = 0; j + 1 < ABS_R; ++j) {
                    if ((uint32_t)j >= np && (uint32_t)(j + 1) < n && ts_before(ts[j + 1], ts[j])) {
                        int64_t t = ts[j]; ts[j] = ts[j + 1]; ts[j + 1] = t;
                        uint64_t q = seq[j]; seq[j] = seq[j + 1]; seq[j + 1] = q;
#pragma unroll
                        for (int x = 0; x < NW; ++x) { uint32_t c = w[j][x]; w[j][x] = w[j + 1][x]; w[j + 1][x] = c; }
                        uint32_t c = nb[j]; nb[j] = nb[j + 1]; nb[j + 1] = c;
                        c = px[j]; px[j] = px[j + 1]; px[j + 1] = c;
                    }
                }
            }
        }
        np = n;
        sbad = false;
    }
    // StreamPreStateProcessor.expireEvents on p1: the expired prefix of pending, any expired staged slot
    // (p0's seed holds no event and never expires; p1 has no withinEvery processor: gen_host abs_shape)
    __device__ __forceinline__ void expire(int64_t now) {
        if (G.within == -1 || n == 0) return;
        uint32_t X = 0;
#pragma unroll
        for (int j = 0; j < ABS_R; ++j) {
            const int64_t dd = ts[j] - now;
            if ((uint32_t)j < n && (dd < 0 ? -dd : dd) > G.within) X |= 1u << j;
        }
        if (!X) return;
        const uint32_t P = np >= 32u ? 0xffffffffu : ((1u << np) - 1u);
        const uint32_t f = P & ~X;  // the first pending partial that survives ends the prefix
        const uint32_t pre = f ? (P & X & ((f & (0u - f)) - 1u)) : (P & X);
        remove(pre | (X & ~P));
    }

    // ---- values for the filters (java_ops.h jo_eval) ----
    __device__ __forceinline__ GVal attr(const uint32_t (&ww)[NW], uint32_t nbits, uint32_t a) const {
        const int ty = G.attrType[stream][a];
        const uint32_t o = G.absOff[a];
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            if ((uint32_t)q == o) lo = ww[q];
            if ((uint32_t)q == o + 1) hi = ww[q];
        }
        const uint64_t b = (ty == SG_T_LONG || ty == SG_T_DOUBLE) ? ((uint64_t)lo | ((uint64_t)hi << 32)) : (uint64_t)lo;
        return GVal{b, ((nbits >> a) & 1u) != 0};
    }
    // f0 on the seed: slot0 = the event, every other slot empty
    __device__ __forceinline__ bool evalF0(const AbsEv<NW>& ev) {
        const auto& P = G.pre[G.absP0];
        if (P.flen == 0) return true;
        auto var_ = [&](uint32_t s, uint32_t a, int32_t c) -> GVal {
                                   if ((int)s == slot0 && (c == 0 || c == -1)) return attr(ev.w, ev.nb, a);
                                   return GVal{0, true};
                               };
        if constexpr (FF) return jo_fast(P.ff, var_);   // (gen_engine.h JoFast)
        const GVal v = jo_eval<false>(G.code, P.fpc, P.flen, err, var_,
                                      [&](uint32_t s, int32_t c) -> bool { return !((int)s == slot0 && (c == 0 || c == -1)); });
        return !v.null && (v.b & 1);
    }
    // f1 on a partial whose e1 words are `pw` / `pn`: slot0 = its e1, slot1 = the event
    __device__ __forceinline__ bool evalF1(const AbsEv<NW>& ev, const uint32_t (&pw)[NW], uint32_t pn) {
        const auto& P = G.pre[G.absP1];
        if (P.flen == 0) return true;
        auto var_ = [&](uint32_t s, uint32_t a, int32_t c) -> GVal {
                                          if (c != 0 && c != -1) return GVal{0, true};
                                          if ((int)s == slot1) return attr(ev.w, ev.nb, a);
                                          if ((int)s == slot0) return attr(pw, pn, a);
                                          return GVal{0, true};
                                      };
        if constexpr (FF) return jo_fast(P.ff, var_);   // (gen_engine.h JoFast)
        const GVal v = jo_eval<false>(G.code, P.fpc, P.flen, err, var_,
                                      [&](uint32_t s, int32_t c) -> bool {
                                          return !(((int)s == slot0 || (int)s == slot1) && (c == 0 || c == -1));
                                      });
        return !v.null && (v.b & 1);
    }
    // p1.processAndReturn: f1 over the pending partials in list order; the ones it passes die (one
    // interpreted evaluation per partial: slot j's words are selected into registers first)
    __device__ __forceinline__ uint32_t killScan(const AbsEv<NW>& ev) {
        uint32_t kill = 0;
        for (uint32_t j = 0; j < np; j++) {
            uint32_t pw[NW], pn = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) pw[q] = 0;
#pragma unroll
            for (int x = 0; x < ABS_R; ++x) {
                if ((uint32_t)x == j) {
#pragma unroll
                    for (int q = 0; q < NW; ++q) pw[q] = w[x][q];
                    pn = nb[x];
                }
            }
            scanned++;
            if (evalF1(ev, pw, pn)) {  // AbsentStreamPostStateProcessor.process: the partial dies
                kill |= 1u << j;
                lst = ev.ts + G.pre[G.absP1].waiting;  // updateLastArrivalTime
                notifyAt(lst);
            }
        }
        return kill;
    }

    // one event of this key (PatternMultiProcessStreamReceiver: stabilize, then p1, then p0)
    __device__ __forceinline__ void event(const AbsEv<NW>& ev) {
        expire(ev.ts);
        seedPend += seedStg;  // updateState(p0): the seed moves to pending
        if (seedStg) seedPendTs = seedStgTs;
        seedStg = 0;
        promote();            // updateState(p1)
        // p1.processAndReturn: a partial whose f1 passes is removed (and reschedules), the rest stay
        remove(killScan(ev));
        // p0.processAndReturn over its seed
        if (seedPend) {
            scanned++;
            if (evalF0(ev)) {
                // StreamPostStateProcessor: the seed becomes the partial (ts = e1.ts) -> p1.addState
                // (staged; schedules e1.ts + T); `every`: p0.addEveryState (a new seed, staged, same ts)
                const uint32_t t = n;
                const uint32_t e = canon ? alloc() : t;   // (store_all writes partial j at entry j)
                dmin = t < dmin ? t : dmin;
#pragma unroll
                for (int j = 0; j < ABS_R; ++j) {
                    if ((uint32_t)j == t) {
                        px[j] = e;
                        ts[j] = ev.ts;
                        seq[j] = ev.seq;
#pragma unroll
                        for (int q = 0; q < NW; ++q) w[j][q] = ev.w[q];
                        nb[j] = ev.nb;
                    }
                }
                if (n > np) {  // a staged append out of ts order: promotion sorts
                    int64_t last = 0;
#pragma unroll
                    for (int j = 0; j < ABS_R; ++j) if ((uint32_t)j + 1 == t) last = ts[j];
                    if (ts_before(ev.ts, last)) sbad = true;
                }
                n++;
                lst = ev.ts + G.pre[G.absP1].waiting;
                notifyAt(lst);
                seedPend = 0;
                if (G.absEvery) {
                    seedStg = 1;
                    seedStgTs = ev.ts;
                    created++;
                }
            }
        }
    }

    // AbsentStreamPreStateProcessor.process for the TIMER event at currentTime = t (the clock is `now`)
    __device__ __forceinline__ void timer(int64_t t, int64_t now, const GenArgs& a) {
        promote();  // this.updateState()
        const int64_t waiting = G.pre[G.absP1].waiting;
        uint32_t drop = 0, emit = 0;
#pragma unroll
        for (int j = 0; j < ABS_R; ++j) {
            if ((uint32_t)j < np) {
                scanned++;
                const int64_t dd = ts[j] - t;
                if (G.within != -1 && (dd < 0 ? -dd : dd) > G.within) {
                    drop |= 1u << j;
                } else if ((ts[j] == -1 && t >= lst) || (ts[j] != -1 && t >= ts[j] + waiting)) {
                    drop |= 1u << j;
                    emit |= 1u << j;
                }
            }
        }
        // sendEvent in list order: the selector gets each (slot0 = e1, ts = currentTime)
        for (uint32_t m = emit; m; m &= m - 1u) {
            const uint32_t j = (uint32_t)__ffs(m) - 1u;
            uint64_t q = 0;
            uint32_t e = 0;
#pragma unroll
            for (int x = 0; x < ABS_R; ++x)
                if ((uint32_t)x == j) { q = seq[x]; e = px[x]; }
            if (TM && canon) q = (uint64_t)R64(G.offSE + e * G.seWords + SE_SEQ);  // (not loaded: see load)
            project(q, t, a);
        }
        remove(drop);
        if (now > waiting + t) lst = now + waiting;
        if (emit == 0 && lst < t) {
            lst = t + waiting;
            notifyAt(t + waiting);
        }
    }

    // a timer match (QuerySelector input: slot0 = e1, ts = the fire time) staged at its rank in this key's
    // sweep (gen_host.hip k_timer_scatter_abs writes it out in the due keys' head order): no atomics
    __device__ __forceinline__ void project(uint64_t e1seq, int64_t t, const GenArgs& a) {
        const uint32_t rank = (uint32_t)matches++;
        if (rank >= (uint32_t)ABS_R) { err |= GERR_REF; return; }  // (a sweep emits only partials it loaded)
        auto st = gp(a.t.tstage);
        st[(size_t)rank * K + k] = e1seq;
        st[(size_t)(ABS_R + rank) * K + k] = (unsigned long long)t;
    }
};

// ---- batch: one lane per key walks its events of the key-sorted batch ----
template <int NW, bool FF> __device__ void abs_batch(const GenArgs& a) {
    const cGenProgram& G = *(cGenProgram*)a.G;
    const uint32_t key = blockIdx.x * 64u + threadIdx.x;
    uint32_t b = 0, e = 0;
    if (key < a.K) {
        b = gp(a.b.seg_begin)[key];
        e = gp(a.b.seg_end)[key];
    }
    AbsKey<NW, false, FF> L(a.G, a.state, a.K, key < a.K ? key : 0u, a.rec);
    bool walk = b < e;
    bool fb = false;
    uint32_t stop = b;
    if (walk && !L.load()) {  // not this path's shape: the general kernel walks the whole run
        fb = true;
        walk = false;
    }

    unsigned long long ky = 0;
    const int64_t tbase = a.b.pay ? gp(a.b.ts)[0] : 0;  // the payload's ts offsets are from the batch's first ts
    if (walk) {
        uint32_t i = b;
        for (; i < e; i++) {
            // at most n + 1 appends to the queue and one new partial per event: stop before an event that
            // could overflow the window or the queue (the general kernel continues from it)
            if (L.n + 1u > L.cap_n() || L.ql + L.n + 1u > G.Q) break;
            AbsEv<NW> ev;
            if (a.b.pay) {
                abs_pay<NW>(a, i, tbase, ev);   // (a prefetch of event i + 1 here puts the key object in scratch)
            } else {
                const uint32_t pos = a.b.sidx ? gp(a.b.sidx)[i] : i;
                ev.ts = gp(a.b.ts)[pos];
                ev.seq = a.b.seq_base + pos;
                abs_gather<NW>(a, G, pos, ev);
            }
            L.event(ev);
        }
        L.store(i < e);   // (a hand-over: the general / wave-per-key kernels continue from the block)
        if (i < e) {
            fb = true;
            stop = i;
        } else {
            gp(a.t.nd)[key] = L.deadline();
            ky = 1;
        }
    }
    abs_fallback(a, fb, key, stop);
    abs_wave_stats(a, L.scanned, L.created, 0ull, ky, L.err, fb ? 1ull : 0ull);
}

__device__ __forceinline__ unsigned long long abs_ord64(int64_t t) { return (unsigned long long)t ^ (1ull << 63); }

// ---- timer sweep to a.now over the due keys (k_gen_due) ----
template <int NW> __device__ void abs_timers(const GenArgs& a) {
    const cGenProgram& G = *(cGenProgram*)a.G;
    const uint64_t nd = *a.t.ndue;
    unsigned long long sc = 0, cr = 0, ma = 0, nfb = 0;
    uint32_t er = 0;
    const uint32_t li = (uint32_t)G.absListener;
    // (one lane per due slot: the grid covers every key, each wave at most one pass)
    for (uint64_t base = (uint64_t)blockIdx.x * 64u; base < nd; base += (uint64_t)gridDim.x * 64u) {
        const uint64_t di = base + threadIdx.x;
        const bool act = di < nd;
        const uint32_t key = act ? gp(a.t.due)[di] : 0u;
        AbsKey<NW, true> L(a.G, a.state, a.K, key, a.rec);
        bool fb = false;
        if (act) {
            const uint32_t w0 = L.W(0);
            if (!(w0 & 1u)) {  // a key is created by its first event (not due)
                gp(a.t.dpair_key)[di] = ~0ull;
                gp(a.t.dpair_i)[di] = GEN_PAIR_NONE;
                if (a.t.dpair_kid) gp(a.t.dpair_kid)[di] = GEN_PAIR_NONE;
                gp(a.t.nd)[key] = GEN_NO_DEADLINE;
            } else {
                // the listener's collection of (due time, key) from the queue head (the A.10 check)
                const bool rec = (w0 & GEN_W0_REG) && L.R;
                const uint32_t qh = rec ? 0u : L.W(L.ks1 + KS_QHEAD), ql = rec ? L.RW(5) : L.W(L.ks1 + KS_QLEN);
                int64_t h = 0;
                if (ql && rec) {   // (the queue in the record, its head at row 0)
                    h = (int64_t)L.Q64(0);
                } else if (ql && (w0 & GEN_W0_DEEP) && a.deep) {   // (the queue in the deep store, normalised)
                    const gu32* D = gp(a.deep) + (size_t)key * a.deepWords +
                                    gen_deep_layout(G.L, G.Q, (uint32_t)NW).oQ;
                    h = (int64_t)((uint64_t)D[0] | ((uint64_t)D[1] << 32));
                } else if (ql) {
                    h = L.R64(L.qword(qh < G.Q ? qh : 0u));
                }
                const bool due = ql != 0 && h <= a.now;
                gp(a.t.dpair_key)[di] = due ? abs_ord64(h) : ~0ull;
                gp(a.t.dpair_i)[di] = due ? li : GEN_PAIR_NONE;
                if (a.t.dpair_kid) gp(a.t.dpair_kid)[di] = due ? key : GEN_PAIR_NONE;
                if (!L.load()) {
                    fb = true;
                } else {
                    for (int guard = 0; guard < (1 << 20); guard++) {  // Scheduler.sendTimerEvents
                        if (L.ql == 0 || L.qhv > a.now) break;
                        const int64_t t = L.qhv;
                        L.qpop();
                        L.timer(t, a.now, a);
                    }
                    L.store();
                    gp(a.t.nd)[key] = L.deadline();
                    gp(a.t.kcnt)[key] = (uint32_t)L.matches | GEN_KCNT_STAGED;
                }
            }
        }
        abs_fallback(a, fb, key, 0u);
        nfb += fb ? 1ull : 0ull;
        sc += L.scanned;
        cr += L.created;
        ma += L.matches;
        er |= L.err;
    }
    abs_wave_stats(a, sc, cr, ma, 0ull, er, nfb);
}

// ---- the records written back to the blocks in the general layout (before a snapshot, ...) ----
template <int NW> __device__ void abs_flush(const GenArgs& a) {
    const uint32_t key = blockIdx.x * 64u + threadIdx.x;
    if (key >= a.K || !a.rec) return;
    AbsKey<NW, false> L(a.G, a.state, a.K, key, a.rec);
    if (!(L.W(0) & GEN_W0_REG)) return;
    L.load();
    L.store_general();
}

}  // namespace

// One kernel per captured-word count (NW = the stream's attributes as 32-bit words, long / double 2 each).
// The batch and timer kernels' occupancy floor (waves per SIMD): 3 brings the timer sweep from 177 VGPRs (2 waves)
// under 170 with no spill; measured per 4.19M-event batch C4 0.387 -> 0.366 ms, C4_deep 2.08 -> 1.99 ms of kernel
// time (4: 128 VGPRs, 96-168 B spilled, C4 0.409 ms; profiles/r04f/abs_waves.log)
#ifndef SG_ABS_WAVES
#define SG_ABS_WAVES 3
#endif
#define ABS_OCC(NW) __attribute__((amdgpu_waves_per_eu((NW) <= 3 ? SG_ABS_WAVES : 1, 8)))   // (wider events: no floor)
#define ABS_KERNELS(NW)                                                                                             \
    extern "C" __global__ void __launch_bounds__(64) ABS_OCC(NW) k_abs_batch_##NW(const GenArgs ap) {   \
        abs_batch<NW, false>(ap);                                                                                  \
    }                                                                                                               \
    extern "C" __global__ void __launch_bounds__(64) ABS_OCC(NW) k_abs_batchf_##NW(const GenArgs ap) {  \
        abs_batch<NW, true>(ap);                                                                                   \
    }                                                                                                               \
    extern "C" __global__ void __launch_bounds__(64) ABS_OCC(NW) k_abs_timers_##NW(const GenArgs ap) {  \
        abs_timers<NW>(ap);                                                                                        \
    }                                                                                                               \
    extern "C" __global__ void __launch_bounds__(64) k_abs_flush_##NW(const GenArgs ap) { abs_flush<NW>(ap); }
// (narrow events) the same batch / timer kernels at an occupancy floor of 4 (128 VGPRs, ~100 B spilled): the host
// takes them when a launch has more waves than fit the chip at 3 per SIMD but not more than at 4 (C4_deep's
// 262,144 keys: 4,096 waves run in one round instead of 1.33, gen_host.hip abs_occ4)
#define ABS_KERNELS4(NW)                                                                                            \
    extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 8)))                    \
    k_abs_batchf4_##NW(const GenArgs ap) { abs_batch<NW, true>(ap); }                                              \
    extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 8)))                    \
    k_abs_timers4_##NW(const GenArgs ap) { abs_timers<NW>(ap); }
ABS_KERNELS4(1)
ABS_KERNELS4(2)
ABS_KERNELS4(3)
ABS_KERNELS(1)
ABS_KERNELS(2)
ABS_KERNELS(3)
ABS_KERNELS(4)
ABS_KERNELS(5)
ABS_KERNELS(6)
ABS_KERNELS(7)
ABS_KERNELS(8)
