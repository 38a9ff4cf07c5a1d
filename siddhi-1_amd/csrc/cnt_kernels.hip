// cnt_kernels.hip — register-window kernel for the counting sequence shape
//
//     every e1=S[f0]<m:n>, e2=S[fA] or e3=S[fB] [within W]          (SEQUENCE, partitioned, 1 <= m, n <= CNT_R)
//
// (BASELINE configs[2], "C3" / "C3_min1").  The general kernel (gen_kernels.hip) runs this query through the
// processor graph with every StateEvent / StreamEvent in the key-interleaved pools of HBM: a count partial
// that grows by one event costs ~25 word accesses to distinct rows (pool bitmaps, records, list entries,
// refcounts) per processor visit.  Under SEQUENCE semantics a key of this shape holds at most ONE partial
// between events (StateStreamRuntime.resetAndUpdate clears every pending list before each event, and the
// SEQUENCE addState keeps at most one staged entry per processor), so one lane per key keeps that partial —
// the count chain e1 (up to CNT_R events: seq, ts, attribute words, null bits), its list memberships and the
// three processors' flag words — in registers for the key's whole run of the batch, and writes the lists back
// once, in a canonical layout of the general blocks (StateEvent 0 = the partial over StreamEvents 0..len-1
// linked by `next`, StateEvent 1 = a staged start seed, free bitmaps rebuilt).  The state stays the general
// engine's: snapshots, state documents, purge and the general kernel read it unchanged; a key whose stored
// lists are not of this canonical shape (e.g. imported from a document of another shape's history) is handed
// to the general kernel for its whole run (k_gen_batch GEN_M_KEYLIST), so the results stay exactly the
// general engine's.
//
// What one event of a key does (restated from the reference, paths under
// /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/query/input/stream/state/):
//   receiver/SequenceMultiProcessStreamReceiver.java:39-50 stabilizeStates -> StateStreamRuntime.java:81-88
//       resetAndUpdate, then the states in reverse order (pA, pB, p0), each projected at once
//   StreamPreStateProcessor.java:118-129 isExpired, :325-361 expireEvents (+ :354-357 withinEvery clone),
//       :287-305 resetState (+ :178-194 init: `every` stages a fresh seed), :308-323 updateState
//   LogicalPreStateProcessor.java:43-62 addState (SEQUENCE: one entry, both partners), :96-124 resetState,
//       :126-140 updateState, :143-180 processAndReturn (a partial whose partner slot is filled is dropped)
//   LogicalPostStateProcessor.java:59-83 (OR: StreamPostStateProcessor + the partner's event-returned flag)
//   CountPreStateProcessor.java:53-95 processAndReturn (a partial whose e2 / e3 slot is filled is dropped;
//       the event appended to the chain, removed again when the filter fails; SEQUENCE drops a failed one)
//   CountPostStateProcessor.java:39-66 (SEQUENCE: n >= m -> next state's addState; n != max -> own addState;
//       n == max -> stateChanged)
#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu.h"
#include "../../include/siddhi_gpu_ir.h"
#include "gen_engine.h"
#include "java_ops.h"
#include "sg_engine.h"
#include "reg_common.h"

namespace {

template <int NW> struct CntKey {
    const cGenProgram& G;
    const GenArgs& A;
    gu32* S;
    uint32_t K, k;
    int p0, pA, pB;           // processors (an event visits pA, pB, p0)
    int s0, sA, sB;           // their slots
    uint32_t ks0, ksA, ksB;   // KeyState word offsets
    int32_t mn, mx;           // count bounds
    // the partial X: e1's chain [0, n) (n = 0: no partial), X's timestamp and its list memberships
    int64_t ts[CNT_R];
    uint64_t seq[CNT_R];
    uint32_t w[CNT_R][NW];
    uint32_t nb[CNT_R];
    uint32_t n;
    int64_t xts;
    bool inP0p, inP0n, inL;   // X in p0.pending / p0.newAndEvery / both logical newAndEvery lists
    bool seedN;               // a blank start seed staged in p0.newAndEvery
    uint32_t f0, fA, fB;      // the processors' flag words
    uint32_t err;
    unsigned long long scanned, created, matches;
    uint32_t trigRank;
    // the register-native record (GEN_W0_REG; nullptr: the block only): chain events [dirty, n) differ from it
    gu32* R;
    uint32_t dirty;
    bool wasRec;

    __device__ CntKey(const GenArgs& a, uint32_t key)
        : G(*(cGenProgram*)a.G), A(a), S(gp(a.state)), K(a.K), k(key), n(0), xts(-1), inP0p(false), inP0n(false),
          inL(false), seedN(false), f0(0), fA(0), fB(0), err(0), scanned(0), created(0), matches(0), trigRank(0), R(a.rec ? gp(a.rec) : nullptr), dirty(0), wasRec(false) {
        p0 = G.cntP0;
        pA = G.cntPA;
        pB = G.cntPB;
        s0 = G.pre[p0].stateId;
        sA = G.pre[pA].stateId;
        sB = G.pre[pB].stateId;
        ks0 = G.offKS + (uint32_t)p0 * G.ksWords;
        ksA = G.offKS + (uint32_t)pA * G.ksWords;
        ksB = G.offKS + (uint32_t)pB * G.ksWords;
        mn = G.pre[p0].minCount;
        mx = G.pre[p0].maxCount;
    }

    __device__ __forceinline__ gu32& W(uint32_t w_) const { return S[gen_il(K, k, w_)]; }
    __device__ __forceinline__ int64_t R64(uint32_t w_) const {
        return (int64_t)((uint64_t)W(w_) | ((uint64_t)W(w_ + 1) << 32));
    }
    __device__ __forceinline__ void W64(uint32_t w_, int64_t v) const {
        W(w_) = (uint32_t)(uint64_t)v;
        W(w_ + 1) = (uint32_t)((uint64_t)v >> 32);
    }
    __device__ __forceinline__ uint32_t stw(uint32_t se, uint32_t f) const { return G.offST + se * G.stWords + f; }
    __device__ __forceinline__ uint32_t sew(uint32_t e, uint32_t f) const { return G.offSE + e * G.seWords + f; }

    // ---- the register-native record (GEN_W0_REG): header word = n | inP0p << 4 | inP0n << 5 | inL << 6 |
    // seedN << 7 | f0 << 8 | fA << 16 | fB << 24, the partial's ts, then per chain event seq, ts, null bits, words
    __device__ __forceinline__ gu32& RW(uint32_t w_) const { return R[(size_t)w_ * K + k]; }
    __device__ __forceinline__ uint32_t rev(uint32_t j, uint32_t f) const { return GEN_REC_EV + j * (5u + NW) + f; }
    __device__ void loadRec() {
        const uint32_t h = RW(0);
        xts = (int64_t)((uint64_t)RW(1) | ((uint64_t)RW(2) << 32));
        n = h & 15u;
        inP0p = (h >> 4) & 1u;
        inP0n = (h >> 5) & 1u;
        inL = (h >> 6) & 1u;
        seedN = (h >> 7) & 1u;
        f0 = (h >> 8) & 0xffu;
        fA = (h >> 16) & 0xffu;
        fB = h >> 24;
#pragma unroll
        for (int j = 0; j < CNT_R; ++j) {
            ts[j] = 0;
            seq[j] = 0;
            nb[j] = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) w[j][q] = 0;
            if ((uint32_t)j < n) {
                seq[j] = (uint64_t)RW(rev(j, 0)) | ((uint64_t)RW(rev(j, 1)) << 32);
                ts[j] = (int64_t)((uint64_t)RW(rev(j, 2)) | ((uint64_t)RW(rev(j, 3)) << 32));
                nb[j] = RW(rev(j, 4));
#pragma unroll
                for (int q = 0; q < NW; ++q) w[j][q] = RW(rev(j, 5u + (uint32_t)q));
            }
        }
        dirty = n;
        wasRec = true;
    }
    // the header, the timestamp and the chain events appended since the load (a chain only grows at its end
    // or restarts: the events below `dirty` are the record's already)
    __device__ void storeRec() const {
        if (!wasRec) W(0) = 1u | GEN_W0_REG;
        RW(0) = n | (inP0p ? 16u : 0u) | (inP0n ? 32u : 0u) | (inL ? 64u : 0u) | (seedN ? 128u : 0u) | (f0 << 8) |
                (fA << 16) | (fB << 24);
        RW(1) = (uint32_t)(uint64_t)xts;
        RW(2) = (uint32_t)((uint64_t)xts >> 32);
#pragma unroll
        for (int j = 0; j < CNT_R; ++j) {
            if ((uint32_t)j >= dirty && (uint32_t)j < n) {
                RW(rev(j, 0)) = (uint32_t)seq[j];
                RW(rev(j, 1)) = (uint32_t)(seq[j] >> 32);
                RW(rev(j, 2)) = (uint32_t)(uint64_t)ts[j];
                RW(rev(j, 3)) = (uint32_t)((uint64_t)ts[j] >> 32);
                RW(rev(j, 4)) = nb[j];
#pragma unroll
                for (int q = 0; q < NW; ++q) RW(rev(j, 5u + (uint32_t)q)) = w[j][q];
            }
        }
    }

    // ---- load: false = the stored lists are not of this kernel's canonical shape (the general kernel
    // takes the key's run)
    __device__ bool load() {
        const uint32_t w0 = W(0);
        if (w0 & GEN_W0_REG) {
            loadRec();
            return true;
        }
        if (!(w0 & 1u)) {  // PartitionRuntimeImpl.initPartition: p0.init() stages one seed
            seedN = true;
            f0 = GF_INIT;
            return true;
        }
        f0 = W(ks0 + KS_FLAGS);
        fA = W(ksA + KS_FLAGS);
        fB = W(ksB + KS_FLAGS);
        const uint32_t p0p = W(ks0 + KS_PLEN), p0n = W(ks0 + KS_NLEN);
        const uint32_t Ap = W(ksA + KS_PLEN), An = W(ksA + KS_NLEN), Bp = W(ksB + KS_PLEN), Bn = W(ksB + KS_NLEN);
        if (Ap != 0u || Bp != 0u || p0p > 1u || p0n > 1u || An > 1u || An != Bn) return false;
        // (memberships computed as values and assigned once: branches that store to different members
        // make the compiler select a member address, which keeps the whole key object in scratch)
        uint32_t xi = GEN_NIL;
        const bool l = An != 0u;
        if (l) {
            xi = W(ksA + KS_LISTS + G.L);
            if (W(ksB + KS_LISTS + G.L) != xi) return false;
        }
        const bool pp = p0p != 0u;
        if (pp) {
            const uint32_t y = W(ks0 + KS_LISTS);
            if (xi != GEN_NIL && y != xi) return false;
            xi = y;
        }
        bool pn = false, sd = false;
        if (p0n) {
            const uint32_t y = W(ks0 + KS_LISTS + G.L);
            const bool blank = y < G.STCAP && W(stw(y, ST_TYPE)) == 0u && W(stw(y, ST_RC)) == 1u &&
                               R64(stw(y, ST_TS)) == -1 && W(stw(y, ST_SLOTS + (uint32_t)s0)) == GEN_NIL &&
                               W(stw(y, ST_SLOTS + (uint32_t)sA)) == GEN_NIL && W(stw(y, ST_SLOTS + (uint32_t)sB)) == GEN_NIL;
            sd = y != xi && blank && !pp;  // (a staged seed: only before the key's first event)
            pn = !sd;
            if (pn && xi != GEN_NIL && y != xi) return false;
            xi = pn ? y : xi;
        }
        inL = l;
        inP0p = pp;
        inP0n = pn;
        seedN = sd;
        if (xi == GEN_NIL) return true;
        if (xi >= G.STCAP) return false;
        const uint32_t rc = (inP0p ? 1u : 0u) + (inP0n ? 1u : 0u) + (inL ? 2u : 0u);
        if (W(stw(xi, ST_TYPE)) != 0u || W(stw(xi, ST_RC)) != rc) return false;
        if (W(stw(xi, ST_SLOTS + (uint32_t)sA)) != GEN_NIL || W(stw(xi, ST_SLOTS + (uint32_t)sB)) != GEN_NIL) return false;
        xts = R64(stw(xi, ST_TS));
        uint32_t e = W(stw(xi, ST_SLOTS + (uint32_t)s0));
#pragma unroll
        for (int j = 0; j < CNT_R; ++j) {
            ts[j] = 0;
            seq[j] = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) w[j][q] = 0;
            nb[j] = 0;
        }
        uint32_t len = 0;
        while (e != GEN_NIL) {
            if (e >= G.SECAP || len >= (uint32_t)mx || len >= (uint32_t)CNT_R || W(sew(e, SE_RC)) != 1u) return false;
            const int64_t t = R64(sew(e, SE_TS));
            const uint64_t q = (uint64_t)R64(sew(e, SE_SEQ));
            const uint32_t nbits = W(sew(e, SE_NULL));
            uint32_t ww[NW];
#pragma unroll
            for (int x = 0; x < NW; ++x) ww[x] = W(sew(e, G.absWordAt[x]));
#pragma unroll
            for (int j = 0; j < CNT_R; ++j) {  // (selects: a conditional store at j == len becomes an indexed one)
                const bool here = (uint32_t)j == len;
                ts[j] = here ? t : ts[j];
                seq[j] = here ? q : seq[j];
                nb[j] = here ? nbits : nb[j];
#pragma unroll
                for (int x = 0; x < NW; ++x) w[j][x] = here ? ww[x] : w[j][x];
            }
            len++;
            e = W(sew(e, SE_NEXT));
        }
        if (len == 0u) return false;
        n = len;
        return true;
    }

    // ---- store: the lists in the canonical layout, free bitmaps rebuilt
    __device__ void store() const {
        W(0) = 1u;
        W(ks0 + KS_FLAGS) = f0;
        W(ksA + KS_FLAGS) = fA;
        W(ksB + KS_FLAGS) = fB;
        const bool x = n > 0u;
        const uint32_t seedIdx = x ? 1u : 0u;
        W(ks0 + KS_PLEN) = (x && inP0p) ? 1u : 0u;
        W(ks0 + KS_NLEN) = ((x && inP0n) || seedN) ? 1u : 0u;
        if (x && inP0p) W(ks0 + KS_LISTS) = 0u;
        if (x && inP0n) W(ks0 + KS_LISTS + G.L) = 0u;
        else if (seedN) W(ks0 + KS_LISTS + G.L) = seedIdx;
        W(ksA + KS_PLEN) = 0u;
        W(ksB + KS_PLEN) = 0u;
        W(ksA + KS_NLEN) = (x && inL) ? 1u : 0u;
        W(ksB + KS_NLEN) = (x && inL) ? 1u : 0u;
        if (x && inL) {
            W(ksA + KS_LISTS + G.L) = 0u;
            W(ksB + KS_LISTS + G.L) = 0u;
        }
        if (x) {
            const uint32_t b = G.offST;
            W64(b + ST_TS, xts);
            W(b + ST_TYPE) = 0u;
            W(b + ST_RC) = (inP0p ? 1u : 0u) + (inP0n ? 1u : 0u) + (inL ? 2u : 0u);
            for (int s = 0; s < G.nslots; s++) W(b + ST_SLOTS + (uint32_t)s) = s == s0 ? 0u : GEN_NIL;
#pragma unroll
            for (int j = 0; j < CNT_R; ++j) {
                if ((uint32_t)j < n) {
                    const uint32_t eb = G.offSE + (uint32_t)j * G.seWords;
                    W64(eb + SE_SEQ, (int64_t)seq[j]);
                    W64(eb + SE_TS, ts[j]);
                    W(eb + SE_NEXT) = (uint32_t)j + 1u < n ? (uint32_t)j + 1u : GEN_NIL;
                    W(eb + SE_RC) = 1u;
                    W(eb + SE_NULL) = nb[j];
#pragma unroll
                    for (int q = 0; q < NW; ++q) W(eb + G.absWordAt[q]) = w[j][q];
                }
            }
        }
        if (seedN) {
            const uint32_t b = G.offST + seedIdx * G.stWords;
            W64(b + ST_TS, -1);
            W(b + ST_TYPE) = 0u;
            W(b + ST_RC) = 1u;
            for (int s = 0; s < G.nslots; s++) W(b + ST_SLOTS + (uint32_t)s) = GEN_NIL;
        }
        // free bitmaps: StateEvents [0, x + seed), StreamEvents [0, n)
        const uint32_t nst = (x ? 1u : 0u) + (seedN ? 1u : 0u);
        for (uint32_t q = 0; q < (G.STCAP + 31) / 32; q++) W(G.offSTfree + q) = q == 0 ? ((1u << nst) - 1u) : 0u;
        for (uint32_t q = 0; q < (G.SECAP + 31) / 32; q++) {
            uint32_t m = 0;
            if (n > 32 * q) m = (n >= 32 * (q + 1)) ? 0xffffffffu : ((1u << (n - 32 * q)) - 1u);
            W(G.offSEfree + q) = m;
        }
        W(G.offDef) = 0u;
    }

    // ---- filter values (java_ops.h jo_eval): e1's chain at index c (StateEvent.getStreamEvent, the general
    // kernel's chainAt: c >= 0 the c-th, -1 the last, -2 the one before it, else len + c)
    __device__ __forceinline__ int chainIdx(int32_t c, uint32_t len) const {
        if (c >= 0) return c < (int32_t)len ? c : -1;
        if (c == -1) return len ? (int)len - 1 : -1;
        if (c == -2) return len >= 2u ? (int)len - 2 : -1;
        const int i = (int)len + c;
        return i >= 0 ? i : -1;
    }
    __device__ __forceinline__ GVal word(const uint32_t (&ww)[NW], uint32_t nbits, uint32_t a) const {
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
    __device__ __forceinline__ GVal chainAttr(int idx, uint32_t a) const {
        // the word of attribute a of chain entry idx, selected without indexing the register arrays
        const int ty = G.attrType[0][a];
        const uint32_t o = G.absOff[a];
        uint32_t lo = 0, hi = 0, nbits = 0;
#pragma unroll
        for (int j = 0; j < CNT_R; ++j) {
            const bool here = j == idx;
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                lo = (here && (uint32_t)q == o) ? w[j][q] : lo;
                hi = (here && (uint32_t)q == o + 1) ? w[j][q] : hi;
            }
            nbits = here ? nb[j] : nbits;
        }
        const uint64_t b = (ty == SG_T_LONG || ty == SG_T_DOUBLE) ? ((uint64_t)lo | ((uint64_t)hi << 32)) : (uint64_t)lo;
        return GVal{b, ((nbits >> a) & 1u) != 0};
    }
    // filter of processor p on X: slot s0 = the chain [0, len), slots `evSlot` and `evSlot2` (the AND pair's
    // partner slot, already filled by this event; -1: none) = the event alone
    __device__ bool evalOn(int p, uint32_t len, int evSlot, const AbsEv<NW>& ev, int evSlot2 = -1) {
        const auto& P = G.pre[p];
        if (P.flen == 0) return true;
        auto var_ = [&](uint32_t s, uint32_t a, int32_t c) -> GVal {
                if ((int)s == s0) {
                    const int i = chainIdx(c, len);
                    return i < 0 ? GVal{0, true} : chainAttr(i, a);
                }
                if (((int)s == evSlot || (int)s == evSlot2) && chainIdx(c, 1u) == 0) return word(ev.w, ev.nb, a);
                return GVal{0, true};
            };
        if (P.ff.on) return jo_fast(P.ff, var_);   // (gen_engine.h JoFast)
        const GVal v = jo_eval<false>(G.code, P.fpc, P.flen, err, var_,
                                      [&](uint32_t s, int32_t c) -> bool {
                if ((int)s == s0) return chainIdx(c, len) < 0;
                if ((int)s == evSlot || (int)s == evSlot2) return chainIdx(c, 1u) != 0;
                return true;
            });
        return !v.null && (v.b & 1);
    }

    // ---- a match (QuerySelector input): X with e1's chain and the event in `evSlot` (and, for the AND pair, in
    // `evSlot2` too) (Lane::project's record)
    __device__ void project(const AbsEv<NW>& ev, uint32_t pos, int evSlot, int evSlot2 = -1) {
        // one raw slot per match, reserved at once for the lanes of the wave that match here (one atomic per wave
        // and call site; per-lane chunks left ~2.5 unused slots per matching key, each marked empty by a
        // scattered store)
        const unsigned long long act = __ballot(true);
        const int leader = __ffsll((long long)act) - 1;
        const uint32_t sg = blockIdx.x % A.o.nseg;
        unsigned long long base = 0;
        if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(&A.o.raw_count[sg], (unsigned long long)__popcll(act));
        base = __shfl(base, leader, 64);
        const unsigned long long r = (unsigned long long)sg * A.o.seg_cap + base +
                                     __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
        const unsigned long long resEnd = (unsigned long long)(sg + 1) * A.o.seg_cap;
        matches++;
        if (r >= resEnd) { err |= GERR_MATCHCAP; return; }
        gu32* rec = gp(A.o.raw) + r * A.o.recWords;
        rec[0] = pos;
        rec[1] = (trigRank++) | GEN_REC_PACKED;   // (the chains packed: the used words contiguous)
        rec[2] = (uint32_t)ev.seq;
        rec[3] = (uint32_t)(ev.seq >> 32);
        rec[4] = (uint32_t)(uint64_t)xts;
        rec[5] = (uint32_t)((uint64_t)xts >> 32);
        rec[6] = k;
        gu32* lens = rec + 7;
        gu32* seqs = lens + G.nslots;
        for (int s = 0; s < G.nslots; s++) lens[s] = s == s0 ? n : ((s == evSlot || s == evSlot2) ? 1u : 0u);
        // packed in slot order: e1's chain (slot s0), then the e2 / e3 event (its slots are s0 + 1 and s0 + 2)
#pragma unroll
        for (int j = 0; j < CNT_R; ++j) {
            if ((uint32_t)j < n) {
                seqs[2 * j] = (uint32_t)seq[j];
                seqs[2 * j + 1] = (uint32_t)(seq[j] >> 32);
            }
        }
        seqs[2 * n] = (uint32_t)ev.seq;
        seqs[2 * n + 1] = (uint32_t)(ev.seq >> 32);
        if (evSlot2 >= 0) {
            seqs[2 * n + 2] = (uint32_t)ev.seq;
            seqs[2 * n + 3] = (uint32_t)(ev.seq >> 32);
        }
        gp(A.o.t_cnt)[pos] += 1;
        if (A.mode & GEN_M_TFIRST) gp(A.o.t_first)[pos] = (uint32_t)r;
    }

    // ---- one event of this key (SequenceMultiProcessStreamReceiver: stabilize, then pA, pB, p0)
    __device__ void event(const AbsEv<NW>& ev, uint32_t pos) {
        trigRank = 0;
        // expireEvents over p0, pA, pB: X expires as a whole (one isExpired per StateEvent); found in p0's
        // lists first, it is cloned into p0.newAndEvery by withinEvery and promoted — a clone the reset below
        // drops again (only the creation counter sees it)
        if (G.within != -1 && n > 0u) {
            const int64_t d = ts[0] - ev.ts;
            if ((d < 0 ? -d : d) > G.within) {
                if ((inP0p || inP0n) && G.cntWE) created++;
                n = 0;
                inP0p = inP0n = inL = false;
            }
        }
        // resetAndUpdate: the logical pair's pending lists clear (empty between events), p0's pending clears;
        // p0 with nothing staged inits (`every`: a fresh seed); then p0's and the pair's staged entries are promoted
        inP0p = false;
        if (!(inP0n && n > 0u) && !seedN) {
            seedN = true;
            f0 |= GF_INIT;
        }
        const bool xP0 = inP0n && n > 0u, sP0 = seedN && !xP0, xL = inL && n > 0u;
        inP0n = false;
        seedN = false;
        inL = false;
        if (!xP0 && !xL) n = 0;  // a partial only p0's pending held dies at the reset
        // pA, then pB: X in both pending lists.  OR (LogicalPreStateProcessor.java:143-180,
        // LogicalPostStateProcessor.java:59-83): a pass of pA matches and fills e2, and the filled partner slot
        // drops X from pB unseen; else pB's pass matches.  AND: pA's pass fills e2 and, without e3, only changes
        // state (X leaves pA's pending, the slot kept); pB then tests X with e2 already this event and matches
        // when both passed.  Either way X leaves both lists, and a filled slot makes the count state drop it
        // below — so an AND match needs fA and fB on the same event.  (One call site per filter and one for the
        // match: each inlined evaluation carries the interpreter, and more copies put the key object in scratch.)
        bool matched = false;
        if (xL) {
            const bool both = G.cntAnd != 0;
            scanned += 2;
            fA &= ~(uint32_t)GF_CHANGED;
            const bool a = evalOn(pA, n, sA, ev);
            if (a) fA |= GF_CHANGED;
            bool bp = false;
            if (both || !a) {
                fB &= ~(uint32_t)GF_CHANGED;
                bp = evalOn(pB, n, sB, ev, (both && a) ? sA : -1);
                if (bp) fB |= GF_CHANGED;
            }
            if (both ? (a && bp) : (a || bp)) {
                xts = ev.ts;
                const int lo = sA < sB ? sA : sB, hi = sA < sB ? sB : sA;
                project(ev, pos, both ? lo : (a ? sA : sB), both ? hi : -1);
            }
            matched = a || bp;
        }
        // p0: X (its e2 / e3 slot filled: dropped; else the event joins the chain) or the seed
        if (xP0 || sP0) {
            scanned++;
            if (xP0 && matched) {
                n = 0;
            } else {
                if (sP0) n = 0;  // X (if any) was the pair's alone and has left it: the seed starts a chain
                if (n >= (uint32_t)CNT_R) { err |= GERR_CHAIN; return; }
                dirty = n < dirty ? n : dirty;
#pragma unroll
                for (int j = 0; j < CNT_R; ++j) {
                    const bool here = (uint32_t)j == n;
                    ts[j] = here ? ev.ts : ts[j];
                    seq[j] = here ? ev.seq : seq[j];
                    nb[j] = here ? ev.nb : nb[j];
#pragma unroll
                    for (int q = 0; q < NW; ++q) w[j][q] = here ? ev.w[q] : w[j][q];
                }
                const uint32_t len = n + 1u;
                f0 &= ~(uint32_t)(GF_SUCCESS | GF_CHANGED);
                if (evalOn(p0, len, -1, ev)) {  // CountPostStateProcessor
                    f0 |= GF_SUCCESS;
                    xts = ev.ts;
                    n = len;
                    if ((int32_t)len >= mn) {
                        inL = true;
                        if ((int32_t)len != mx) inP0n = true;
                    }
                    if ((int32_t)len == mx) f0 |= GF_CHANGED;
                    inP0p = (f0 & GF_CHANGED) == 0u;
                } else {
                    // removeLastEvent, and SEQUENCE drops the partial from pending (a seed goes with it)
                    if (sP0) n = 0;
                }
            }
        } else if (matched) {
            n = 0;
        }
        if (!inP0p && !inP0n && !inL) n = 0;
    }
};

// ---- the fused grouping: a workgroup per 64-key tile splits it by key ----
// (gen_host.hip groups the batch by tile = key >> 6 only, two 7-bit passes instead of three 8-bit ones; this kernel
// then splits each tile by key into the key-sorted payload, one read and one write of the tile instead of a third
// radix pass with its histogram and scan; PartitionStreamReceiver.java:175-260's per-key runs in arrival order are
// what the split builds.  Splitting inside k_cnt_batch instead (the tile in LDS) was measured: the split's code in
// the walk kernel costs it 1.1 KB of scratch per lane at its 128-VGPR cap, 10x slower.)
__device__ __forceinline__ uint32_t cnt_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t cnt_match6(uint32_t v, uint64_t act) {  // lanes holding the same 6-bit value
    uint64_t m = act;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
        const bool x = (v >> b) & 1u;
        const uint64_t bb = __ballot(x);
        m &= x ? bb : ~bb;
    }
    return m;
}
__device__ __forceinline__ uint32_t cnt_excl_scan(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t v = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, off, 64);
        if (lane >= (uint32_t)off) v += t;
    }
    return v - x;
}
constexpr uint32_t CNT_MAXST = 6;  // payload words per element (W <= 4, + position and ts offset)

// One wave per 64-key tile (tile = blockIdx.x, lane = key & 63): the tile's elements (arrival order, key & 255 tagged
// in the position's top byte) counted per key, then placed into the key-sorted payload at the tile's range (arrival
// order within a key, the tag cleared), with every key's [begin, end).
// A tile of at most 64 * CNT_SPLIT_R events (the usual case) is loaded into registers at once, so the split waits for
// memory once; larger tiles are read twice in 64-event rounds.
constexpr uint32_t CNT_SPLIT_R = 8;
#define CNT_WSYNC() do { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); __builtin_amdgcn_wave_barrier(); } while (0)
extern "C" __global__ void __launch_bounds__(256) k_cnt_split(const GenArgs a) {
    // four tiles per workgroup, a wave each (waves sync among themselves only: LDS ops of one wave run in order)
    __shared__ uint32_t s_cnt[4][64];
    __shared__ uint32_t s_el[4][64 * CNT_SPLIT_R * 4];  // a small tile's elements, key-sorted (<= 4 words each)
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.x * 4u + w;
    const uint32_t ntiles = (a.K + 63u) / 64u;
    if (tile >= ntiles) return;
    uint32_t* cnt = s_cnt[w];
    const uint32_t key = tile * 64u + lane;
    const uint32_t st = a.b.payStride;
    const uint32_t lo = gp(a.b.tile_lo)[tile], nt = gp(a.b.tile_lo)[tile + 1] - lo;
    const gu32* src = gp(a.b.tpay) + (size_t)lo * st;
    gu32* dst = (gu32*)gp(a.b.pay) + (size_t)lo * st;
    cnt[lane] = 0u;
    // the host's skew check: only tiles past its threshold report (one device-wide counter hit by every workgroup
    // serialises at the memory side: 16K atomics cost ~0.2 ms)
    if (lane == 0 && nt > (1u << 14) && a.b.tileMax) atomicMax((uint32_t*)gp(a.b.tileMax), nt);
    CNT_WSYNC();
    uint32_t c = 0, kb = 0;
    if (nt <= 64u * CNT_SPLIT_R) {
        uint32_t el[CNT_SPLIT_R][CNT_MAXST];
#pragma unroll
        for (uint32_t r = 0; r < CNT_SPLIT_R; ++r) {
            const uint32_t j = r * 64u + lane;
#pragma unroll
            for (uint32_t u = 0; u < CNT_MAXST; ++u) el[r][u] = (j < nt && u < st) ? src[(size_t)j * st + u] : 0u;
        }
        uint64_t mm[CNT_SPLIT_R];
#pragma unroll
        for (uint32_t r = 0; r < CNT_SPLIT_R; ++r) {  // (one wave: LDS ops in program order)
            mm[r] = 0;
            if (r * 64u < nt) {
                const bool v = r * 64u + lane < nt;
                const uint32_t kl = (el[r][0] >> 24) & 63u;
                mm[r] = cnt_match6(kl, __ballot(v));
                if (v && cnt_rank(mm[r]) == 0u) cnt[kl] += (uint32_t)__popcll(mm[r]);
                CNT_WSYNC();
            }
        }
        c = cnt[lane];
        kb = cnt_excl_scan(c);
        CNT_WSYNC();
        cnt[lane] = kb;
        CNT_WSYNC();
#pragma unroll
        for (uint32_t r = 0; r < CNT_SPLIT_R; ++r) {
            if (r * 64u < nt) {
                const bool v = r * 64u + lane < nt;
                const uint32_t kl = (el[r][0] >> 24) & 63u;
                uint32_t pos = 0;
                if (v) {
                    const uint32_t rk = cnt_rank(mm[r]), base = cnt[kl];
                    pos = base + rk;
                    if (rk == 0u) cnt[kl] = base + (uint32_t)__popcll(mm[r]);
                }
                CNT_WSYNC();
                if (v) {
                    el[r][0] &= 0xffffffu;
                    if (st <= 4u) {  // placed in LDS, written out contiguously below
#pragma unroll
                        for (uint32_t u = 0; u < 4u; ++u)
                            if (u < st) s_el[w][pos * st + u] = el[r][u];
                    } else {
#pragma unroll
                        for (uint32_t u = 0; u < CNT_MAXST; ++u)
                            if (u < st) dst[(size_t)pos * st + u] = el[r][u];
                    }
                }
            }
        }
        if (st <= 4u) {  // the key-sorted tile, coalesced
            CNT_WSYNC();
            for (uint32_t x = lane; x < nt * st; x += 64u) dst[x] = s_el[w][x];
        }
    } else {
        for (uint32_t r0 = 0; r0 < nt; r0 += 64u) {
            const uint32_t j = r0 + lane;
            const bool v = j < nt;
            const uint32_t kl = v ? (src[(size_t)j * st] >> 24) & 63u : 0u;
            const uint64_t m = cnt_match6(kl, __ballot(v));
            if (v && cnt_rank(m) == 0u) cnt[kl] += (uint32_t)__popcll(m);
            CNT_WSYNC();
        }
        c = cnt[lane];
        kb = cnt_excl_scan(c);
        CNT_WSYNC();
        cnt[lane] = kb;
        CNT_WSYNC();
        for (uint32_t r0 = 0; r0 < nt; r0 += 64u) {
            const uint32_t j = r0 + lane;
            const bool v = j < nt;
            uint32_t el[CNT_MAXST];
#pragma unroll
            for (uint32_t u = 0; u < CNT_MAXST; ++u) el[u] = (v && u < st) ? src[(size_t)j * st + u] : 0u;
            const uint32_t kl = (el[0] >> 24) & 63u;
            const uint64_t m = cnt_match6(kl, __ballot(v));
            uint32_t pos = 0;
            if (v) {
                const uint32_t rk = cnt_rank(m), base = cnt[kl];
                pos = base + rk;
                if (rk == 0u) cnt[kl] = base + (uint32_t)__popcll(m);
            }
            CNT_WSYNC();
            if (v) {
                el[0] &= 0xffffffu;
#pragma unroll
                for (uint32_t u = 0; u < CNT_MAXST; ++u)
                    if (u < st) dst[(size_t)pos * st + u] = el[u];
            }
        }
    }
    if (key < a.K) {
        ((gu32*)gp(a.b.seg_begin))[key] = lo + kb;
        ((gu32*)gp(a.b.seg_end))[key] = lo + kb + c;
    }
}

// ---- batch: one lane per key walks its events of the key-sorted batch ----
template <int NW> __device__ void cnt_batch(const GenArgs& a) {
    const uint32_t key = blockIdx.x * 64u + threadIdx.x;
    uint32_t b = 0, e = 0;
    if (key < a.K) {
        b = gp(a.b.seg_begin)[key];
        e = gp(a.b.seg_end)[key];
    }
    CntKey<NW> L(a, key < a.K ? key : 0u);
    bool walk = b < e;
    bool fb = false;
    if (walk && !L.load()) {  // not this kernel's canonical state: the general kernel walks the whole run
        fb = true;
        walk = false;
    }
    unsigned long long ky = 0;
    const int64_t tbase = a.b.pay ? gp(a.b.ts)[0] : 0;  // the payload's ts offsets are from the batch's first ts
    if (walk) {
        PayAhead<NW> ahead;
        ahead.first(a, b, e);
        for (uint32_t i = b; i < e; i++) {
            AbsEv<NW> ev;
            uint32_t pos;
            if (a.b.pay) {
                ahead.next(a, i, e, tbase, ev);
                pos = (uint32_t)(ev.seq - a.b.seq_base);
            } else {
                pos = a.b.sidx ? gp(a.b.sidx)[i] : i;
                ev.ts = gp(a.b.ts)[pos];
                ev.seq = a.b.seq_base + pos;
                abs_gather<NW>(a, *(cGenProgram*)a.G, pos, ev);
            }
            L.event(ev, pos);
        }
        if (L.R) L.storeRec();
        else L.store();
        ky = 1;
    }
    abs_fallback(a, fb, key, b);
    abs_wave_stats(a, L.scanned, L.created, L.matches, ky, L.err, fb ? 1ull : 0ull);
}

// ---- the records written back to the blocks in the canonical layout (before a snapshot, min-seq scan, ...) ----
template <int NW> __device__ void cnt_flush(const GenArgs& a) {
    const uint32_t key = blockIdx.x * 64u + threadIdx.x;
    if (key >= a.K || !a.rec) return;
    CntKey<NW> L(a, key);
    if (!(L.W(0) & GEN_W0_REG)) return;
    L.loadRec();
    L.store();   // (word 0 = 1: the block is the key's state again)
}

}  // namespace

// One kernel per captured-word count (NW = the stream's attributes as 32-bit words, long / double 2 each).
// The batch kernel's occupancy floor (waves per SIMD): 4 caps it at 128 VGPRs (150 uncapped: 3 waves), which spills
// 96 B per lane but hides more of the walk's latency — measured C3 0.165 -> 0.146 ms, C3_min1 0.414 -> 0.386 ms per
// 4.19M-event batch; 5 (96 VGPRs, 228 B spilled) is 2.7x slower (profiles/r04f/cnt_waves.log)
#ifndef SG_CNT_WAVES
#define SG_CNT_WAVES 4
#endif
#define CNT_OCC(NW) __attribute__((amdgpu_waves_per_eu((NW) <= 3 ? SG_CNT_WAVES : 1, 8)))   // (wider events: no floor)
#define CNT_KERNELS(NW)                                                                                             \
    extern "C" __global__ void __launch_bounds__(64) CNT_OCC(NW) k_cnt_batch_##NW(const GenArgs ap) {   \
        cnt_batch<NW>(ap);                                                                                         \
    }                                                                                                              \
    extern "C" __global__ void __launch_bounds__(64) k_cnt_flush_##NW(const GenArgs ap) { cnt_flush<NW>(ap); }
CNT_KERNELS(1)
CNT_KERNELS(2)
CNT_KERNELS(3)
CNT_KERNELS(4)
CNT_KERNELS(5)
CNT_KERNELS(6)
CNT_KERNELS(7)
CNT_KERNELS(8)
