// absd_kernels.hip — wave-per-key kernels for the absent-tail shape with deep per-key state
//
//     [every] e1=S[f0] -> not S[f1] for T [within W]          (PATTERN, partitioned, @app:playback)
//
// (BASELINE configs[3], "deep partial-match state in HBM").  The register-window kernels (abs_kernels.hip) hold
// at most ABS_R partials per key in one lane's registers and hand a key with more to the next stage.  With
// hundreds of live partials per key, one lane per key leaves the GPU idle (a few thousand lanes) and walks each
// key's list serially; here ONE WAVE owns a key: its pending / newAndEvery lists live in the wave's LDS slice
// (list order, SoA: ts, e1 seq, null bits, the event's attribute words), and every list operation is
// data-parallel over the 64 lanes — the `within` expiry of the pending prefix and of any staged partial, the
// kill scan of `not S[f1]` over every pending partial, the timer's expiry / emission test — each followed by an
// order-preserving compaction (wave ballot + prefix count, chunk by chunk in place).  The key's scalar state
// (start seed, flag words, lastScheduledTime, timer queue head / length) is wave-uniform.  State is read from
// and written back to the general engine's blocks in the canonical layout of abs_kernels.hip (StateEvent 0 =
// the seed, 1 + j / StreamEvent j = partial j), so every other component reads it unchanged; a key whose lists
// are not of that shape, or whose next event could overflow the lists or the timer queue, goes on to the
// general kernels (k_gen_batch / k_gen_timers over the second hand-over list).
//
// The keys come from the register-window kernels' hand-over list (those whose lists outgrew ABS_R or were not
// canonical); a fixed grid of one-wave work-groups strides over it.
//
// Semantics restated from (paths under /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/):
//   query/input/stream/state/StreamPreStateProcessor.java:118-129 isExpired, :308-323 updateState (stable sort
//       by ts, -1 last), :325-361 expireEvents (the expired prefix of pending, any staged)
//   query/input/stream/state/AbsentStreamPreStateProcessor.java:80-103 addState (schedules ts + T), :150-227
//       process (the TIMER event: expired partials dropped, due ones sent in list order), :256-274
//       processAndReturn (returns nothing)
//   query/input/stream/state/AbsentStreamPostStateProcessor.java:36-56 (a matching event kills the partial and
//       reschedules at its ts + T)
//   util/Scheduler.java:114-128 notifyAt, :172-210 sendTimerEvents
#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu.h"
#include "../../include/siddhi_gpu_ir.h"
#include "gen_engine.h"
#include "java_ops.h"
#include "sg_engine.h"
#include "reg_common.h"

#ifndef ABSD_PROF
#define ABSD_PROF 0
#endif

namespace {

template <int NW> struct DEnt {
    int64_t ts;
    uint64_t seq;
    uint32_t nb;
    uint32_t w[NW];
    // (FF kernels) f1's operands read from the partial's e1, converted to the compare domain once, when the entry
    // enters the LDS list (not per event and partial); kn bit i = operand i null
    uint64_t k[2];
    uint32_t kn;
};

// one key's absent-tail state, one wave (every member is wave-uniform except where noted)
// A decoded compare (GenPre.ff) hoisted out of a scan: its fields as values, each operand's source (0 constant,
// 1 the event, 2 the partial's e1, 3 null), word offset, width and null bit.  Built once per list scan and kept in
// registers, so the scan's evaluations read no program word (every read of the constant program inside the scan
// was a scalar load the wave waited on: a few thousand cycles per 64 partials)
struct HoistF {
    uint32_t op, dom;
    uint32_t src[2], o[2], wide[2], a[2], from[2], cn[2];
    uint64_t cb[2];
};
__device__ __forceinline__ HoistF hoist_f(const __attribute__((address_space(4))) GenProgram& G, int p, bool isF1,
                                          int slot0, int slot1) {
    const auto& P = G.pre[p];
    HoistF f;
    f.op = P.ff.op;
    f.dom = P.ff.dom;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t at = P.ff.attr[i] < GEN_MAXA ? P.ff.attr[i] : 0u;
        const int32_t c = P.ff.chain[i];
        const int sl = (int)P.ff.slot[i];
        const int ty = G.attrType[0][at];
        f.a[i] = at;
        f.o[i] = G.absOff[at];
        f.wide[i] = (ty == SG_T_LONG || ty == SG_T_DOUBLE) ? 1u : 0u;
        f.from[i] = P.ff.from[i];
        f.cb[i] = P.ff.cbits[i];
        f.cn[i] = P.ff.cnull[i];
        if (P.ff.isConst[i]) f.src[i] = 0u;
        else if (c != 0 && c != -1) f.src[i] = 3u;
        else if (isF1 ? sl == slot1 : sl == slot0) f.src[i] = 1u;
        else if (isF1 && sl == slot0) f.src[i] = 2u;
        else f.src[i] = 3u;
    }
    return f;
}
template <int NW>
__device__ __forceinline__ bool hoisted_eval(const HoistF& f, const uint32_t (&ew)[NW], uint32_t enb,
                                             const uint32_t (&xw)[NW], uint32_t xnb) {
    GVal v[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if (f.src[i] == 0u) {
            v[i] = GVal{f.cb[i], f.cn[i] != 0u};   // (constants are already in the compare domain)
        } else if (f.src[i] == 3u) {
            v[i] = jo_cvt(GVal{0, true}, (int)f.from[i], (int)f.dom);
        } else {
            const bool e = f.src[i] == 1u;
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                const uint32_t w = e ? ew[q] : xw[q];
                lo = (uint32_t)q == f.o[i] ? w : lo;
                hi = (uint32_t)q == f.o[i] + 1u ? w : hi;
            }
            const uint64_t b = f.wide[i] ? ((uint64_t)lo | ((uint64_t)hi << 32)) : (uint64_t)lo;
            v[i] = jo_cvt(GVal{b, (((e ? enb : xnb) >> f.a[i]) & 1u) != 0u}, (int)f.from[i], (int)f.dom);
        }
    }
    return jo_compare((int)f.op, (int)f.dom, v[0], v[1]);
}

// FF: both filters are decoded compares (GenPre.ff): the kernel variant carries no interpreter (its registers and
// scalar pressure made every evaluation of the kill scan a few thousand cycles of reloaded program words)
template <int NW, bool FF = false> struct DeepKey {
    const cGenProgram& G;
    const GenArgs& A;
    gu32* S;
    uint32_t K, k, C;
    uint32_t ks0, ks1;
    int slot0, slot1;
    int lane;
    // the lists in LDS: entries [0, n) in list order, [0, np) pending, [np, n) staged; the timer queue in LDS
    // (a ring of Q entries from qh)
    int64_t* lts;
    uint64_t* lseq;
    uint32_t* lnb;
    uint32_t* lw;    // [NW][C]
    uint64_t* lk;    // [2][C] (FF) f1's partial-side operands in the compare domain
    uint32_t* lkn;   // [C]
    int64_t* lq;     // [Q]
    uint32_t Q;
    gu32* D;         // this key's deep-store record (GEN_W0_DEEP), or nullptr (no deep store)
    GenDeepLayout dl;
    uint32_t n, np;
    bool sbad;
    uint32_t seedPend, seedStg;
    int64_t seedPendTs, seedStgTs;
    uint32_t f0, f1;
    int64_t lst;
    uint32_t qh, ql;
    uint32_t err;
    unsigned long long scanned, created, matches;
    uint32_t rank;   // timer matches of this key's sweep so far
    HoistF hf0, hf1;   // (FF) the filters, hoisted once per key
#if ABSD_PROF
    unsigned long long* pf = nullptr;   // (ABSD_PROF builds) the phase counters of absd_batch
    uint64_t pt = 0;
    __device__ __forceinline__ void stamp(int i) {
        const uint64_t t_ = __builtin_amdgcn_s_memtime();
        if (pf) pf[i] += t_ - pt;
        pt = t_;
    }
#else
    __device__ __forceinline__ void stamp(int) {}
#endif
    // the program's values the walk reads per event, copied once per key (each read of the constant program is a
    // scalar load the wave waits on: per event they were ~70 loads of a few hundred cycles each)
    int64_t within, waiting;
    bool every;

    __device__ DeepKey(const GenArgs& a, uint8_t* smem, uint32_t key)
        : G(*(cGenProgram*)a.G), A(a), S(gp(a.state)), K(a.K), k(key), n(0), np(0), sbad(false), seedPend(0),
          seedStg(0), seedPendTs(-1), seedStgTs(-1), f0(0), f1(0), lst(0), qh(0), ql(0), err(0), scanned(0),
          created(0), matches(0), rank(0) {
        C = G.L;
        ks0 = G.offKS + (uint32_t)G.absP0 * G.ksWords;
        ks1 = G.offKS + (uint32_t)G.absP1 * G.ksWords;
        slot0 = G.pre[G.absP0].stateId;
        slot1 = G.pre[G.absP1].stateId;
        lane = (int)(threadIdx.x & 63);
        lts = (int64_t*)smem;
        lseq = (uint64_t*)(smem + 8 * (size_t)C);
        lnb = (uint32_t*)(smem + 16 * (size_t)C);
        lw = (uint32_t*)(smem + 20 * (size_t)C);
        const size_t kb = ((20 + 4 * (size_t)NW) * C + 7) & ~(size_t)7;
        lk = (uint64_t*)(smem + kb);
        lkn = (uint32_t*)(smem + kb + 16 * (size_t)C);
        lq = (int64_t*)(smem + ((kb + 20 * (size_t)C + 7) & ~(size_t)7));
        Q = G.Q;
        dl = gen_deep_layout(G.L, G.Q, (uint32_t)NW);
        D = a.deep ? gp(a.deep) + (size_t)key * a.deepWords : nullptr;
        within = G.within;
        waiting = G.pre[G.absP1].waiting;
        every = G.absEvery != 0;
        if constexpr (FF) {
            hf0 = hoist_f(G, G.absP0, false, slot0, slot1);
            hf1 = hoist_f(G, G.absP1, true, slot0, slot1);
        }
    }
    __device__ __forceinline__ int64_t D64(uint32_t w_) const {
        return (int64_t)((uint64_t)D[w_] | ((uint64_t)D[w_ + 1] << 32));
    }
    __device__ __forceinline__ void DW64(uint32_t w_, int64_t v) const {
        D[w_] = (uint32_t)(uint64_t)v;
        D[w_ + 1] = (uint32_t)((uint64_t)v >> 32);
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
    __device__ __forceinline__ bool wany(bool x) const { return __ballot(x) != 0ull; }

    __device__ __forceinline__ void get(uint32_t i, DEnt<NW>& e) const {
        e.ts = lts[i];
        e.seq = lseq[i];
        e.nb = lnb[i];
#pragma unroll
        for (int q = 0; q < NW; ++q) e.w[q] = lw[(size_t)q * C + i];
        if constexpr (FF) {
            e.k[0] = lk[i];
            e.k[1] = lk[C + i];
            e.kn = lkn[i];
        }
    }
    __device__ __forceinline__ void put(uint32_t i, const DEnt<NW>& e) const {
        lts[i] = e.ts;
        lseq[i] = e.seq;
        lnb[i] = e.nb;
#pragma unroll
        for (int q = 0; q < NW; ++q) lw[(size_t)q * C + i] = e.w[q];
        if constexpr (FF) {
            lk[i] = e.k[0];
            lk[C + i] = e.k[1];
            lkn[i] = e.kn;
        }
    }
    // (FF) f1's partial-side operands of entry x, converted to the compare domain
    __device__ __forceinline__ void keys(const HoistF& h, DEnt<NW>& x) const {
        x.kn = 0;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            x.k[i] = 0;
            if (h.src[i] == 2u) {
                uint32_t lo = 0, hi = 0;
#pragma unroll
                for (int q = 0; q < NW; ++q) {
                    lo = (uint32_t)q == h.o[i] ? x.w[q] : lo;
                    hi = (uint32_t)q == h.o[i] + 1u ? x.w[q] : hi;
                }
                const uint64_t b = h.wide[i] ? ((uint64_t)lo | ((uint64_t)hi << 32)) : (uint64_t)lo;
                const GVal v = jo_cvt(GVal{b, ((x.nb >> h.a[i]) & 1u) != 0u}, (int)h.from[i], (int)h.dom);
                x.k[i] = v.b;
                x.kn |= (v.null ? 1u : 0u) << i;
            }
        }
    }
    // (FF) f1's operand i when it does not come from the partial (a constant, the event, null): once per event
    __device__ __forceinline__ GVal evOperand(const HoistF& h, int i, const AbsEv<NW>& ev) const {
        if (h.src[i] == 0u) return GVal{h.cb[i], h.cn[i] != 0u};
        if (h.src[i] != 1u) return jo_cvt(GVal{0, true}, (int)h.from[i], (int)h.dom);
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            lo = (uint32_t)q == h.o[i] ? ev.w[q] : lo;
            hi = (uint32_t)q == h.o[i] + 1u ? ev.w[q] : hi;
        }
        const uint64_t b = h.wide[i] ? ((uint64_t)lo | ((uint64_t)hi << 32)) : (uint64_t)lo;
        return jo_cvt(GVal{b, ((ev.nb >> h.a[i]) & 1u) != 0u}, (int)h.from[i], (int)h.dom);
    }
    __device__ __forceinline__ bool killTest(const HoistF& h, const GVal& e0, const GVal& e1, const DEnt<NW>& x) const {
        const GVal l = h.src[0] == 2u ? GVal{x.k[0], (x.kn & 1u) != 0u} : e0;
        const GVal r = h.src[1] == 2u ? GVal{x.k[1], (x.kn & 2u) != 0u} : e1;
        return jo_compare((int)h.op, (int)h.dom, l, r);
    }

    // ---- load: false = not this kernel's shape (the general kernels take the key)
    __device__ bool load() {
        if (!(W(0) & 1u)) {
            seedStg = 1;
            seedStgTs = -1;
            f0 = GF_INIT;
            f1 = GF_STARTED;
            return true;
        }
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
        }
        np = W(ks1 + KS_PLEN);
        const uint32_t ns = W(ks1 + KS_NLEN);
        if (np > G.L || ns > G.L || np + ns > C) return false;
        n = np + ns;
        lst = R64(ks1 + KS_LST);
        const uint32_t qh0 = W(ks1 + KS_QHEAD);
        ql = W(ks1 + KS_QLEN);
        if (qh0 >= Q || ql > Q) return false;
        qh = 0;   // (the LDS ring starts normalised)
        bool ok = true, bad = false;
        if (W(0) & GEN_W0_DEEP) {
            // the record: contiguous per field, one coalesced access per 64 entries
            if (!D) return false;
            for (uint32_t c = 0; c < n; c += 64) {
                const uint32_t i = c + (uint32_t)lane;
                if (i < n) {
                    DEnt<NW> x;
                    x.ts = D64(dl.oTs + 2 * i);
                    x.seq = (uint64_t)D64(dl.oSeq + 2 * i);
                    x.nb = D[dl.oNb + i];
#pragma unroll
                    for (int q = 0; q < NW; ++q) x.w[q] = D[dl.oW + (uint32_t)q * G.L + i];
                    put(i, x);
                }
            }
            for (uint32_t c = 0; c < ql; c += 64) {
                const uint32_t i = c + (uint32_t)lane;
                if (i < ql) lq[i] = D64(dl.oQ + 2 * i);
            }
        } else {
            for (uint32_t c = 0; c < n; c += 64) {
                const uint32_t i = c + (uint32_t)lane;
                if (i < n) {
                    const uint32_t st = W(ks1 + KS_LISTS + (i < np ? i : G.L + i - np));
                    ok = ok && st < G.STCAP;
                    const uint32_t b = G.offST + (st < G.STCAP ? st : 0u) * G.stWords;
                    const uint32_t e = W(b + ST_SLOTS + (uint32_t)slot0);
                    ok = ok && W(b + ST_TYPE) == 0u && W(b + ST_RC) == 1u && e < G.SECAP &&
                         W(b + ST_SLOTS + (uint32_t)slot1) == GEN_NIL;
                    const uint32_t eb = G.offSE + (e < G.SECAP ? e : 0u) * G.seWords;
                    const int64_t t = R64(b + ST_TS);
                    ok = ok && W(eb + SE_NEXT) == GEN_NIL && W(eb + SE_RC) == 1u && R64(eb + SE_TS) == t;
                    DEnt<NW> x;
                    x.ts = t;
                    x.seq = (uint64_t)R64(eb + SE_SEQ);
                    x.nb = W(eb + SE_NULL);
#pragma unroll
                    for (int q = 0; q < NW; ++q) x.w[q] = W(eb + G.absWordAt[q]);
                    put(i, x);
                }
            }
            for (uint32_t c = 0; c < ql; c += 64) {
                const uint32_t i = c + (uint32_t)lane;
                if (i < ql) {
                    uint32_t pos = qh0 + i;
                    if (pos >= Q) pos -= Q;
                    lq[i] = R64(qword(pos));
                }
            }
        }
        if (wany(!ok)) return false;
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        if constexpr (FF) {   // the entries' f1 keys (the lists come without them)
            for (uint32_t c = 0; c < n; c += 64) {
                const uint32_t i = c + (uint32_t)lane;
                if (i < n) {
                    DEnt<NW> x;
                    get(i, x);
                    keys(hf1, x);
                    lk[i] = x.k[0];
                    lk[C + i] = x.k[1];
                    lkn[i] = x.kn;
                }
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
        }
        // staged partials out of ts order (promotion sorts them)
        for (uint32_t c = np + 1; c < n; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            if (i < n && ts_before(lts[i], lts[i - 1])) bad = true;
        }
        sbad = wany(bad);
        return true;
    }

    // the key's header words in the block (flags, the seed, list lengths, lastScheduledTime, queue length):
    // lane 0; the queue is written normalised (head 0)
    __device__ void store_header(uint32_t w0) const {
        if (lane == 0) {
            W(0) = w0;
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
            W(ks1 + KS_QHEAD) = 0u;
            W(ks1 + KS_QLEN) = ql;
            W(ks1 + KS_PLEN) = np;
            W(ks1 + KS_NLEN) = n - np;
        }
    }

    // ---- store into the deep-store record (GEN_W0_DEEP): the lists and the queue contiguous, the header in
    // the block; falls back to the block's canonical layout without a deep store
    __device__ void store() const {
        if (!D) {
            store_general();
            return;
        }
        for (uint32_t c = 0; c < n; c += 64) {
            const uint32_t j = c + (uint32_t)lane;
            if (j < n) {
                DEnt<NW> x;
                get(j, x);
                DW64(dl.oTs + 2 * j, x.ts);
                DW64(dl.oSeq + 2 * j, (int64_t)x.seq);
                D[dl.oNb + j] = x.nb;
#pragma unroll
                for (int q = 0; q < NW; ++q) D[dl.oW + (uint32_t)q * G.L + j] = x.w[q];
            }
        }
        for (uint32_t c = 0; c < ql; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            if (i < ql) {
                uint32_t pos = qh + i;
                if (pos >= Q) pos -= Q;
                DW64(dl.oQ + 2 * i, lq[pos]);
            }
        }
        store_header(1u | GEN_W0_DEEP);
    }

    // ---- store into the block, the canonical layout (StateEvent 0 = the seed, 1 + j = partial j over StreamEvent
    // j; the queue normalised): what the general kernels and every host reader take
    __device__ void store_general() const {
        for (uint32_t c = 0; c < n; c += 64) {
            const uint32_t j = c + (uint32_t)lane;
            if (j < n) {
                DEnt<NW> x;
                get(j, x);
                W(ks1 + KS_LISTS + (j < np ? j : G.L + j - np)) = 1u + j;
                const uint32_t b = G.offST + (1u + j) * G.stWords;
                W64(b + ST_TS, x.ts);
                W(b + ST_TYPE) = 0u;
                W(b + ST_RC) = 1u;
                for (int s = 0; s < G.nslots; s++) W(b + ST_SLOTS + (uint32_t)s) = s == slot0 ? j : GEN_NIL;
                const uint32_t eb = G.offSE + j * G.seWords;
                W64(eb + SE_SEQ, (int64_t)x.seq);
                W64(eb + SE_TS, x.ts);
                W(eb + SE_NEXT) = GEN_NIL;
                W(eb + SE_RC) = 1u;
                W(eb + SE_NULL) = x.nb;
#pragma unroll
                for (int q = 0; q < NW; ++q) W(eb + G.absWordAt[q]) = x.w[q];
            }
        }
        // free bitmaps: StateEvents {0 if a seed} + [1, 1 + n), StreamEvents [0, n)
        const uint32_t stBits = (seedPend | seedStg) ? 1u : 0u;
        for (uint32_t x = (uint32_t)lane; x < (G.STCAP + 31) / 32; x += 64) {
            uint32_t m = 0;
            const uint32_t lo = 32 * x;  // StateEvent bits lo..lo+31: index s set when s == 0 && seed, or 1 <= s <= n
            for (int bit = 0; bit < 32; bit++) {
                const uint32_t sidx = lo + (uint32_t)bit;
                if ((sidx == 0 && stBits) || (sidx >= 1 && sidx <= n)) m |= 1u << bit;
            }
            W(G.offSTfree + x) = m;
        }
        for (uint32_t x = (uint32_t)lane; x < (G.SECAP + 31) / 32; x += 64) {
            uint32_t m = 0;
            if (n > 32 * x) m = (n >= 32 * (x + 1)) ? 0xffffffffu : ((1u << (n - 32 * x)) - 1u);
            W(G.offSEfree + x) = m;
        }
        for (uint32_t c = 0; c < ql; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            if (i < ql) {
                uint32_t pos = qh + i;
                if (pos >= Q) pos -= Q;
                W64(qword(i), lq[pos]);
            }
        }
        store_header(1u);
    }

    // the timer queue in LDS (lanes append entries; a wave barrier before they are read)
    __device__ __forceinline__ int64_t qread(uint32_t i) const { return lq[i]; }
    __device__ __forceinline__ int64_t deadline() const { return ql ? lq[qh] : GEN_NO_DEADLINE; }

    // Scheduler.notifyAt under playback, `cnt` times at t (lanes [0, cnt) write one entry each)
    __device__ __forceinline__ void notifyAt(int64_t t, uint32_t cnt) {
        if (ql + cnt > Q) { err |= GERR_CAP; return; }
        for (uint32_t c = 0; c < cnt; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            if (i < cnt) {
                uint32_t pos = qh + ql + i;
                while (pos >= Q) pos -= Q;
                lq[pos] = t;
            }
        }
        ql += cnt;
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
    }

    // ---- values for the filters ----
    __device__ __forceinline__ GVal attr(const uint32_t (&ww)[NW], uint32_t nbits, uint32_t a) const {
        const int ty = G.attrType[0][a];
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
    __device__ bool evalF0(const AbsEv<NW>& ev) {
        const auto& P = G.pre[G.absP0];
        if (P.flen == 0) return true;
        auto var_ = [&](uint32_t s, uint32_t a, int32_t c) -> GVal {
                                          if ((int)s == slot0 && (c == 0 || c == -1)) return attr(ev.w, ev.nb, a);
                                          return GVal{0, true};
                                      };
        if constexpr (FF) return jo_fast(P.ff, var_);   // (gen_engine.h JoFast)
        if (P.ff.on) return jo_fast(P.ff, var_);
        const GVal v = jo_eval<false>(G.code, P.fpc, P.flen, err, var_,
                                      [&](uint32_t s, int32_t c) -> bool { return !((int)s == slot0 && (c == 0 || c == -1)); });
        return !v.null && (v.b & 1);
    }
    __device__ bool evalF1(const AbsEv<NW>& ev, const DEnt<NW>& x) {
        const auto& P = G.pre[G.absP1];
        if (P.flen == 0) return true;
        auto var_ = [&](uint32_t s, uint32_t a, int32_t c) -> GVal {
                                          if (c != 0 && c != -1) return GVal{0, true};
                                          if ((int)s == slot1) return attr(ev.w, ev.nb, a);
                                          if ((int)s == slot0) return attr(x.w, x.nb, a);
                                          return GVal{0, true};
                                      };
        if constexpr (FF) return jo_fast(P.ff, var_);   // (gen_engine.h JoFast)
        if (P.ff.on) return jo_fast(P.ff, var_);
        const GVal v = jo_eval<false>(G.code, P.fpc, P.flen, err, var_,
                                      [&](uint32_t s, int32_t c) -> bool {
                                          return !(((int)s == slot0 || (int)s == slot1) && (c == 0 || c == -1));
                                      });
        return !v.null && (v.b & 1);
    }

    // ---- the order-preserving compaction: decide(i, entry) -> keep, chunk by chunk in place (a kept entry
    // only moves down, below every entry not yet read); np becomes the kept count of [0, np)
    template <class F> __device__ __forceinline__ void compact(F decide) {
        uint32_t w = 0, keptPend = 0;
        const unsigned long long below = (1ull << lane) - 1ull;
        for (uint32_t c = 0; c < n; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            DEnt<NW> x{};
            bool keep = false;
            if (i < n) {
                get(i, x);
                keep = decide(i, x);
            }
            const unsigned long long m = __ballot(keep);
            const unsigned long long mp = __ballot(keep && i < np);
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            if (keep) put(w + (uint32_t)__popcll(m & below), x);
            w += (uint32_t)__popcll(m);
            keptPend += (uint32_t)__popcll(mp);
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
        }
        n = w;
        np = keptPend;
    }

    // updateState: the staged entries join the pending list stable-sorted by ts (eventTimeComparator); an
    // out-of-order append is rare: lane 0 sorts the staged range in LDS
    __device__ void promote() {
        if (n > np && sbad) {
            if (lane == 0) {
                for (uint32_t i = np + 1; i < n; i++) {
                    DEnt<NW> x;
                    get(i, x);
                    uint32_t j = i;
                    while (j > np) {
                        DEnt<NW> y;
                        get(j - 1, y);
                        if (!ts_before(x.ts, y.ts)) break;
                        put(j, y);
                        j--;
                    }
                    put(j, x);
                }
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
        }
        np = n;
        sbad = false;
    }

    __device__ __forceinline__ bool expiredAt(int64_t ts, int64_t now) const {
        const int64_t d = ts - now;
        return (d < 0 ? -d : d) > within;
    }

    // StreamPreStateProcessor.expireEvents on p1: the expired prefix of pending, any expired staged entry
    __device__ void expire(int64_t now) {
        if (within == -1 || n == 0) return;
        // the first pending entry that survives ends the prefix
        uint32_t f = np;
        for (uint32_t c = 0; c < np; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            const unsigned long long m = __ballot(i < np && !expiredAt(lts[i], now));
            if (m) {
                f = c + (uint32_t)(__ffsll((long long)m) - 1);
                break;
            }
        }
        bool anyStaged = false;
        for (uint32_t c = np; c < n; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            anyStaged = anyStaged || (i < n && expiredAt(lts[i], now));
        }
        if (f == 0 && !wany(anyStaged)) return;
        compact([&](uint32_t i, const DEnt<NW>& x) { return i < np ? i >= f : !expiredAt(x.ts, now); });
    }

    // one event of this key (PatternMultiProcessStreamReceiver: stabilize, then p1, then p0)
    __device__ void event(const AbsEv<NW>& ev) {
        stamp(1);
        expire(ev.ts);
        seedPend += seedStg;
        if (seedStg) seedPendTs = seedStgTs;
        seedStg = 0;
        promote();
        stamp(2);
        // p1.processAndReturn: every pending partial whose f1 passes dies and reschedules (each kill sets
        // lastScheduledTime = ev.ts + T and notifies at it, AbsentStreamPostStateProcessor.java:36-56)
        scanned += np;
        uint32_t kills = 0;
        const bool f1any = G.pre[G.absP1].flen != 0;
        GVal e0{0, true}, e1{0, true};
        if constexpr (FF) {
            e0 = evOperand(hf1, 0, ev);
            e1 = evOperand(hf1, 1, ev);
        }
        for (uint32_t c = 0; c < np; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            bool kl = false;
            if (i < np) {
                DEnt<NW> x;
                get(i, x);
                if constexpr (FF) kl = !f1any || killTest(hf1, e0, e1, x);
                else kl = evalF1(ev, x);
            }
            kills += (uint32_t)__popcll(__ballot(kl));
        }
        if (kills) {
            const int64_t t = ev.ts + waiting;
            lst = t;
            notifyAt(t, kills);
            if constexpr (FF)
                compact([&](uint32_t i, const DEnt<NW>& x) { return !(i < np && (!f1any || killTest(hf1, e0, e1, x))); });
            else
                compact([&](uint32_t i, const DEnt<NW>& x) { return !(i < np && evalF1(ev, x)); });
        }
        stamp(3);
        // p0.processAndReturn over its seed
        if (seedPend) {
            scanned++;
            bool f0 = true;
            if constexpr (FF) f0 = G.pre[G.absP0].flen == 0 || hoisted_eval<NW>(hf0, ev.w, ev.nb, ev.w, ev.nb);
            else f0 = evalF0(ev);
            if (f0) {
                if (lane == 0) {
                    DEnt<NW> x;
                    x.ts = ev.ts;
                    x.seq = ev.seq;
                    x.nb = ev.nb;
#pragma unroll
                    for (int q = 0; q < NW; ++q) x.w[q] = ev.w[q];
                    if constexpr (FF) keys(hf1, x);
                    put(n, x);
                }
                if (n > np && n > 0 && ts_before(ev.ts, lts[n - 1])) sbad = true;
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_wave_barrier();
                n++;
                lst = ev.ts + waiting;
                notifyAt(lst, 1u);
                seedPend = 0;
                if (every) {
                    seedStg = 1;
                    seedStgTs = ev.ts;
                    created++;
                }
            }
        }
        stamp(4);
    }

    // ---- m <= 64 consecutive events at once (lane j holds event j: `mine`).  Under the preconditions of
    // chunkOk — the events' timestamps nondecreasing, the list sorted by ts and none of it later than the first
    // event, room for every partial the chunk could create and every timer it could schedule — the per-event walk
    // reduces to one decision per partial: it dies at the first later event that expires it (ts_j - ts > within:
    // with sorted timestamps the expired entries are always a prefix, as expireEvents takes them) or whose f1
    // passes (a kill), whichever comes first (expiry is tested before the kill scan of the same event).  So every
    // partial, old or created in the chunk, is tested against the chunk's events lane-parallel, the survivors
    // are compacted once, and each event's timer entries (its kills, then its new partial, all at ts_j + T) are
    // written at once.  The start seed is a scalar chain over the events (f0 tested lane-parallel first).  The
    // result — lists, seed, lastScheduledTime, queue, work counters — is the per-event walk's.
    __device__ __forceinline__ int64_t rl64(int64_t x, uint32_t j) const {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)x, (int)j);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), (int)j);
        return (int64_t)(((uint64_t)hi << 32) | lo);
    }
    __device__ bool chunkOk(const AbsEv<NW>& mine, uint32_t m) const {
        if (m < 2 || n + m > C || ql + n + 2u * m > Q) return false;
        const bool act = (uint32_t)lane < m;
        const int64_t t0 = rl64(mine.ts, 0);
        const uint32_t pl = (uint32_t)(lane > 0 ? lane - 1 : 0);
        const uint32_t plo = (uint32_t)__shfl((int)(uint32_t)(uint64_t)mine.ts, (int)pl, 64);
        const uint32_t phi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)mine.ts >> 32), (int)pl, 64);
        const int64_t pts = (int64_t)(((uint64_t)phi << 32) | plo);
        bool bad = act && (mine.ts == -1 || (lane > 0 && mine.ts < pts));
        for (uint32_t c = 0; c < n; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            if (i < n) {
                const int64_t t = lts[i];
                bad = bad || t == -1 || t > t0 || (i + 1 < n && lts[i + 1] < t);
            }
        }
        return !wany(bad);
    }
    // the first event (>= start) that expires / kills partial x: m when none
    __device__ __forceinline__ void fate(const DEnt<NW>& x, uint32_t start, uint32_t m, const AbsEv<NW>& mine,
                                         const GVal& me0, const GVal& me1, uint32_t& Kx, uint32_t& Ex) {
        unsigned long long km = 0, em = 0;
        const bool f1any = G.pre[G.absP1].flen != 0;
        for (uint32_t j = 0; j < m; j++) {
            const int64_t tj = rl64(mine.ts, j);
            if (within != -1 && tj - x.ts > within) em |= 1ull << j;
            bool kl;
            if constexpr (FF) {
                const GVal a0{(uint64_t)rl64((int64_t)me0.b, j), __builtin_amdgcn_readlane(me0.null ? 1 : 0, (int)j) != 0};
                const GVal a1{(uint64_t)rl64((int64_t)me1.b, j), __builtin_amdgcn_readlane(me1.null ? 1 : 0, (int)j) != 0};
                kl = !f1any || killTest(hf1, a0, a1, x);
            } else {
                AbsEv<NW> ev;
                ev.ts = tj;
                ev.seq = (uint64_t)rl64((int64_t)mine.seq, j);
                ev.nb = (uint32_t)__builtin_amdgcn_readlane((int)mine.nb, (int)j);
#pragma unroll
                for (int q = 0; q < NW; ++q) ev.w[q] = (uint32_t)__builtin_amdgcn_readlane((int)mine.w[q], (int)j);
                kl = evalF1(ev, x);
            }
            if (kl) km |= 1ull << j;
        }
        const unsigned long long keep = start >= 64u ? 0ull : ~((1ull << start) - 1ull);
        km &= keep;
        em &= keep;
        Kx = km ? (uint32_t)(__ffsll((long long)km) - 1) : m;
        Ex = em ? (uint32_t)(__ffsll((long long)em) - 1) : m;
    }
    __device__ void chunk(const AbsEv<NW>& mine, uint32_t m) {
        const bool act = (uint32_t)lane < m;
        // f0 on every event, then the seed in event order (updateState moves a staged seed to pending)
        bool f0j = false;
        if (act) {
            if constexpr (FF) f0j = G.pre[G.absP0].flen == 0 || hoisted_eval<NW>(hf0, mine.w, mine.nb, mine.w, mine.nb);
            else f0j = evalF0(mine);
        }
        const unsigned long long f0m = __ballot(f0j);
        unsigned long long cm = 0;   // the events that create a partial
        uint32_t sp = seedPend, ss = seedStg, seedScans = 0, made = 0;
        int64_t spTs = seedPendTs, ssTs = seedStgTs;
        for (uint32_t j = 0; j < m; j++) {
            sp += ss;
            if (ss) spTs = ssTs;
            ss = 0;
            if (sp) {
                seedScans++;
                if ((f0m >> j) & 1ull) {
                    cm |= 1ull << j;
                    sp = 0;
                    if (every) {
                        ss = 1;
                        ssTs = rl64(mine.ts, j);
                        made++;
                    }
                }
            }
        }
        // f1's event-side operands, once per event (lane j)
        GVal me0{0, true}, me1{0, true};
        if constexpr (FF) {
            if (act) {
                me0 = evOperand(hf1, 0, mine);
                me1 = evOperand(hf1, 1, mine);
            }
        }
        unsigned long long scans = 0;
        uint32_t kc = 0;   // lane j: the partials event j kills
        auto count_kills = [&](uint32_t kat) {
            for (uint32_t j = 0; j < m; j++) {
                const uint32_t c = (uint32_t)__popcll(__ballot(kat == j));
                if ((uint32_t)lane == j) kc += c;
            }
        };
        const unsigned long long below = (1ull << lane) - 1ull;
        // the list's partials (pending from event 0 on): fates, then compacted in place (a kept entry only moves
        // down, below every entry not yet read)
        uint32_t wpos = 0;
        for (uint32_t c = 0; c < n; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            DEnt<NW> x{};
            uint32_t Kx = m, Ex = m;
            const bool valid = i < n;
            if (valid) {
                get(i, x);
                fate(x, 0u, m, mine, me0, me1, Kx, Ex);
            }
            const bool dead = valid && (Ex < m || Kx < m);
            const uint32_t kat = (valid && Kx < m && Kx < Ex) ? Kx : 64u;
            if (valid) scans += (unsigned long long)min(min(Ex, Kx + 1u), m);
            const bool keep = valid && !dead;
            const unsigned long long km = __ballot(keep);
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            if (keep) put(wpos + (uint32_t)__popcll(km & below), x);
            wpos += (uint32_t)__popcll(km);
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            if (__ballot(kat < 64u)) count_kills(kat);
        }
        // the chunk's new partials (lane j: created at event j, pending from event j + 1 on), appended in order
        {
            const bool valid = act && ((cm >> lane) & 1ull);
            DEnt<NW> x{};
            uint32_t Kx = m, Ex = m;
            if (valid) {
                x.ts = mine.ts;
                x.seq = mine.seq;
                x.nb = mine.nb;
#pragma unroll
                for (int q = 0; q < NW; ++q) x.w[q] = mine.w[q];
                if constexpr (FF) keys(hf1, x);
            }
            if (__ballot(valid)) fate(x, (uint32_t)lane + 1u, m, mine, me0, me1, Kx, Ex);
            const bool dead = valid && (Ex < m || Kx < m);
            const uint32_t kat = (valid && Kx < m && Kx < Ex) ? Kx : 64u;
            if (valid) {
                const uint32_t last = min(min(Ex, Kx + 1u), m);
                scans += last > (uint32_t)lane + 1u ? (unsigned long long)(last - (uint32_t)lane - 1u) : 0ull;
            }
            const bool keep = valid && !dead;
            const unsigned long long km = __ballot(keep);
            if (keep) put(wpos + (uint32_t)__popcll(km & below), x);
            wpos += (uint32_t)__popcll(km);
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            if (__ballot(kat < 64u)) count_kills(kat);
        }
        n = wpos;
        np = n - (uint32_t)((cm >> (m - 1u)) & 1ull);   // (created at the last event: still staged)
        sbad = false;
        seedPend = sp;
        seedStg = ss;
        seedPendTs = spTs;
        seedStgTs = ssTs;
        // the timer queue: event j's kills, then its new partial, each at ts_j + T, in event order
        const uint32_t cnt = act ? kc + (uint32_t)((cm >> lane) & 1ull) : 0u;
        uint32_t off = cnt;
        for (int d = 1; d < 64; d <<= 1) {   // inclusive prefix over the lanes
            const uint32_t o = (uint32_t)__shfl_up((int)off, d, 64);
            if (lane >= d) off += o;
        }
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)off, 63);
        off -= cnt;
        const int64_t t = mine.ts + waiting;
        for (uint32_t x = 0; x < cnt; x++) {
            uint32_t pos = qh + ql + off + x;
            while (pos >= Q) pos -= Q;
            lq[pos] = t;
        }
        ql += total;
        const unsigned long long any = __ballot(cnt > 0u);
        if (any) lst = rl64(t, (uint32_t)(63 - __builtin_clzll(any)));
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        // work counters: each pending partial once per event's kill scan, the seed once per event it is pending
        for (int d = 32; d > 0; d >>= 1) scans += __shfl_xor(scans, d, 64);
        scanned += scans + seedScans;
        created += made;
    }

    // a timer match: a raw record of the general engine (trigger = timer, rank within this key's sweep)
    __device__ void project(uint64_t base, uint32_t r, uint64_t e1seq, int64_t t) {
        const unsigned long long slot = base + r;
        if (slot >= A.o.seg_cap) { err |= GERR_MATCHCAP; return; }
        gu32* rec = gp(A.o.raw) + slot * A.o.recWords;
        rec[0] = 0xfffffffeu;
        rec[1] = rank + r;
        rec[2] = 0xffffffffu;
        rec[3] = 0xffffffffu;
        rec[4] = (uint32_t)(uint64_t)t;
        rec[5] = (uint32_t)((uint64_t)t >> 32);
        rec[6] = k;
        gu32* lens = rec + 7;
        gu32* seqs = lens + G.nslots;
        for (int s = 0; s < G.nslots; s++) lens[s] = s == slot0 ? 1u : 0u;
        seqs[2 * (slot0 * G.MC)] = (uint32_t)e1seq;
        seqs[2 * (slot0 * G.MC) + 1] = (uint32_t)(e1seq >> 32);
        gp(A.o.tk1)[slot] = (uint32_t)G.absListener;
        gp(A.o.tk2)[slot] = t;
        gp(A.o.tk3)[slot] = k;
    }

    // AbsentStreamPreStateProcessor.process for the TIMER event at currentTime = t (the clock is `now`)
    __device__ void timer(int64_t t, int64_t now) {
        promote();
        scanned += np;
        auto due = [&](const DEnt<NW>& x) {
            return (x.ts == -1 && t >= lst) || (x.ts != -1 && t >= x.ts + waiting);
        };
        auto gone = [&](const DEnt<NW>& x) { return within != -1 && expiredAt(x.ts, t); };
        // the emitted partials in list order (sendEvent per partial: slot0 = e1, ts = currentTime)
        uint32_t emits = 0, drops = 0;
        for (uint32_t c = 0; c < np; c += 64) {
            const uint32_t i = c + (uint32_t)lane;
            bool em = false, dr = false;
            if (i < np) {
                DEnt<NW> x;
                get(i, x);
                dr = gone(x);
                em = !dr && due(x);
            }
            emits += (uint32_t)__popcll(__ballot(em));
            drops += (uint32_t)__popcll(__ballot(dr || em));
        }
        if (emits) {
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(&A.o.raw_count[0], (unsigned long long)emits);
            base = __shfl(base, 0, 64);
            uint32_t r = 0;
            const unsigned long long below = (1ull << lane) - 1ull;
            for (uint32_t c = 0; c < np; c += 64) {
                const uint32_t i = c + (uint32_t)lane;
                bool em = false;
                DEnt<NW> x{};
                if (i < np) {
                    get(i, x);
                    em = !gone(x) && due(x);
                }
                const unsigned long long m = __ballot(em);
                if (em) project(base, r + (uint32_t)__popcll(m & below), x.seq, t);
                r += (uint32_t)__popcll(m);
            }
            rank += emits;
            matches += emits;
        }
        if (drops) compact([&](uint32_t i, const DEnt<NW>& x) { return !(i < np && (gone(x) || due(x))); });
        if (now > waiting + t) lst = now + waiting;
        if (emits == 0 && lst < t) {
            lst = t + waiting;
            notifyAt(t + waiting, 1u);
        }
    }
};

// a wave-aggregated append to the second hand-over list (the general kernels take these keys)
__device__ __forceinline__ void absd_handover(const GenArgs& a, uint32_t key, uint32_t start) {
    if ((threadIdx.x & 63) == 0) {
        const unsigned long long i = atomicAdd(a.fb2_n, 1ull);
        gp(a.fb2_list)[i] = key;
        if (a.fb2_start) gp(a.fb2_start)[key] = start;
    }
}

__device__ void absd_stats(const GenArgs& a, unsigned long long sc, unsigned long long cr, unsigned long long ma,
                           unsigned long long ky, uint32_t er, unsigned long long fb) {
    if ((threadIdx.x & 63) == 0) {  // (a few waves: device-wide atomics are cheap here)
        if (er) atomicOr(a.o.err, er);
        if (sc) atomicAdd(&a.o.stats[GST_SCANNED], sc);
        if (cr) atomicAdd(&a.o.stats[GST_CREATED], cr);
        if (ma) atomicAdd(&a.o.stats[GST_MATCHES], ma);
        if (ky) atomicAdd(&a.o.stats[GST_KEYS], ky);
        if (fb) atomicAdd(&a.o.stats[GST_SPILLS], fb);
    }
}

// ---- batch: one wave per handed-over key walks its events from where the register window stopped ----
// ABSD_PROF=1 (experiment builds): shader-clock cycles per phase (load, event fetch, expire + promote, kill scan,
// seed, store) summed into GenOut.prof slots 0..5, events and loaded entries in 6, 7 (SG_GEN_PROF=1; printed when
// the engine is destroyed)
template <int NW, bool FF> __device__ void absd_batch(const GenArgs& a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const cGenProgram& G = *(cGenProgram*)a.G;
#if ABSD_PROF
    unsigned long long pf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    unsigned long long sc = 0, cr = 0, ky = 0, fb = 0;
    uint32_t er = 0;
    const uint64_t nfb = *a.fb_n;
    const int64_t tbase = a.b.pay ? gp(a.b.ts)[0] : 0;
    const bool noChunk = (a.mode & GEN_M_NOCHUNK) != 0u;
    for (uint64_t li = blockIdx.x; li < nfb; li += gridDim.x) {
        const uint32_t key = __builtin_amdgcn_readfirstlane(gp(a.fb_list)[li]);
        const uint32_t b = __builtin_amdgcn_readfirstlane(gp(a.fb_start)[key]);
        const uint32_t e = __builtin_amdgcn_readfirstlane(gp(a.b.seg_end)[key]);
        DeepKey<NW, FF> L(a, smem, key);
#if ABSD_PROF
        L.pf = pf;
        L.pt = __builtin_amdgcn_s_memtime();
#endif
        if (!L.load()) {
            absd_handover(a, key, b);
            fb++;
            continue;
        }
        L.stamp(0);
#if ABSD_PROF
        pf[6] += e - b;
        pf[7] += L.n;
#endif
        uint32_t i = b;
        // the key's events, 64 at a time: lane j loads event i0 + j's payload words (one coalesced load per word),
        // each event is then read out of the lanes (readlane) instead of a dependent global load per event
        constexpr int MW = NW + 3;
        uint32_t pw[MW];
        const uint32_t st = a.b.payStride;
        for (; i < e; i++) {
            // at most one new partial and n + 1 queue entries per event: stop before an event that could overflow
            if (L.n + 1u > L.C || L.ql + L.n + 1u > G.Q) break;
            AbsEv<NW> ev;
            if (a.b.pay) {
                // payload words x of one event -> the event
                auto decode = [&](const uint32_t (&x)[MW], AbsEv<NW>& o) {
                    const uint32_t pos = x[0];
#pragma unroll
                    for (int q = 0; q < NW; ++q) o.w[q] = x[1 + q];
                    uint32_t toff = 0, nb = 0;
#pragma unroll
                    for (int q = 1; q < MW; ++q) {
                        if ((uint32_t)q == st - 1) toff = x[q];
                        if (a.b.payNull && (uint32_t)q == st - 2) nb = x[q];
                    }
                    o.nb = nb;
                    o.ts = (int32_t)toff == SGD_TS_FAR ? gp(a.b.ts)[pos] : tbase + (int64_t)(int32_t)toff;
                    o.seq = a.b.seq_base + pos;
                };
                const uint32_t j = (i - b) & 63u;
                if (j == 0u) {
                    const uint32_t my = i + (uint32_t)(threadIdx.x & 63);
                    const gu32* pp = gp(a.b.pay) + (size_t)my * st;
#pragma unroll
                    for (int q = 0; q < MW; ++q) pw[q] = (my < e && (uint32_t)q < st) ? pp[q] : 0u;
                    // the next (up to) 64 events at once when their order and the key's list allow it (chunk)
                    const uint32_t m = e - i < 64u ? e - i : 64u;
                    // (the decoded-compare variant only: the interpreter's evaluations per partial and event
                    // put the interpreting kernel's key object in scratch)
                    if (FF && !noChunk && m > 1u) {
                        AbsEv<NW> mine{};
                        if ((uint32_t)(threadIdx.x & 63) < m) decode(pw, mine);
                        if (L.chunkOk(mine, m)) {
                            L.chunk(mine, m);
                            L.stamp(3);
                            i += m - 1u;
                            continue;
                        }
                    }
                }
                uint32_t x[MW];
#pragma unroll
                for (int q = 0; q < MW; ++q) x[q] = (uint32_t)__builtin_amdgcn_readlane((int)pw[q], (int)j);
                decode(x, ev);
            } else {
                const uint32_t pos = a.b.sidx ? gp(a.b.sidx)[i] : i;
                ev.ts = gp(a.b.ts)[pos];
                ev.seq = a.b.seq_base + pos;
                abs_gather<NW>(a, G, pos, ev);
            }
            L.event(ev);
        }
        L.stamp(1);
        if (i < e) {   // the general kernels continue from event i: the block holds the key's lists again
            L.store_general();
            absd_handover(a, key, i);
            fb++;
        } else {
            L.store();
            if ((threadIdx.x & 63) == 0) gp(a.t.nd)[key] = L.deadline();
            ky++;
        }
        L.stamp(5);
        sc += L.scanned;
        cr += L.created;
        er |= L.err;
    }
#if ABSD_PROF
    if ((threadIdx.x & 63) == 0 && a.o.prof)
        for (int q = 0; q < 8; q++) atomicAdd(&a.o.prof[q], pf[q]);
#endif
    absd_stats(a, sc, cr, 0ull, ky, er, fb);
}

// ---- timer sweep: one wave per handed-over due key ----
template <int NW, bool FF> __device__ void absd_timers(const GenArgs& a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const cGenProgram& G = *(cGenProgram*)a.G;
    unsigned long long sc = 0, cr = 0, ma = 0, fb = 0;
    uint32_t er = 0;
    const uint64_t nfb = *a.fb_n;
    for (uint64_t li = blockIdx.x; li < nfb; li += gridDim.x) {
        const uint32_t key = __builtin_amdgcn_readfirstlane(gp(a.fb_list)[li]);
        DeepKey<NW, FF> L(a, smem, key);
        if (!L.load()) {
            absd_handover(a, key, 0u);
            fb++;
            continue;
        }
        for (int guard = 0; guard < (1 << 20); guard++) {  // Scheduler.sendTimerEvents
            if (L.ql == 0) break;
            const int64_t t = L.qread(L.qh);
            if (t > a.now) break;
            L.qh = L.qh + 1u == G.Q ? 0u : L.qh + 1u;
            L.ql--;
            L.timer(t, a.now);
        }
        L.store();
        if ((threadIdx.x & 63) == 0) {
            gp(a.t.nd)[key] = L.deadline();
            if (a.t.kcnt) gp(a.t.kcnt)[key] = L.rank;
        }
        sc += L.scanned;
        ma += L.matches;
        er |= L.err;
    }
    if ((threadIdx.x & 63) == 0 && ma) atomicAdd(a.o.nvalid, ma);
    absd_stats(a, sc, cr, ma, 0ull, er, fb);
}

// ---- flush: every key whose lists live in the deep store written back to its block (the canonical layout), for
// the readers of the blocks (snapshots, state documents, the fan-out's seq-map trim); a fixed grid of one-wave
// work-groups strides over the keys ----
template <int NW> __device__ void absd_flush(const GenArgs& a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t er = 0;
    for (uint32_t key = blockIdx.x; key < a.K; key += gridDim.x) {
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(gp(a.state)[gen_il(a.K, key, 0)]);
        if (!(w0 & GEN_W0_DEEP)) continue;
        DeepKey<NW> L(a, smem, key);
        if (L.load()) L.store_general();
        else er |= GERR_REF;   // (a deep record whose header does not validate: never written so)
    }
    if ((threadIdx.x & 63) == 0 && er) atomicOr(a.o.err, er);
}

}  // namespace

// One kernel per captured-word count (NW), one wave per work-group, dynamic LDS = the key's lists.
#define ABSD_KERNELS(NW)                                                                                            \
    extern "C" __global__ void __launch_bounds__(64) k_absd_batch_##NW(const GenArgs ap) {          \
        absd_batch<NW, false>(ap);                                                                                 \
    }                                                                                                               \
    extern "C" __global__ void __launch_bounds__(64) k_absd_timers_##NW(const GenArgs ap) {         \
        absd_timers<NW, false>(ap);                                                                                \
    }                                                                                                               \
    extern "C" __global__ void __launch_bounds__(64) k_absd_batchf_##NW(const GenArgs ap) {         \
        absd_batch<NW, true>(ap);                                                                                  \
    }                                                                                                               \
    extern "C" __global__ void __launch_bounds__(64) k_absd_timersf_##NW(const GenArgs ap) {        \
        absd_timers<NW, true>(ap);                                                                                 \
    }                                                                                                               \
    extern "C" __global__ void __launch_bounds__(64) k_absd_flush_##NW(const GenArgs ap) {          \
        absd_flush<NW>(ap);                                                                                        \
    }
ABSD_KERNELS(1)
ABSD_KERNELS(2)
ABSD_KERNELS(3)
ABSD_KERNELS(4)
ABSD_KERNELS(5)
ABSD_KERNELS(6)
ABSD_KERNELS(7)
ABSD_KERNELS(8)
