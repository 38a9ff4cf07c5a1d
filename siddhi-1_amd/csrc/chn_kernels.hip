// chn_kernels.hip — register-window kernel for chained stream states
//
//     [every] e1=S[f0] -> e2=S[f1] -> ... -> en=S[f(n-1)] [within W]      (PATTERN, partitioned, one stream, n = 2..4)
//
// (the "P3" leg of the bench is the 3-state chain of BASELINE configs[1]'s query).  The general kernel
// (gen_kernels.hip) runs this shape through the processor graph with every StateEvent / StreamEvent in the
// key-interleaved pools of HBM: each partial a key moves costs tens of word accesses to distinct rows, and the
// interpreter's per-lane output lists live in scratch (~10 KB of HBM traffic per event).  Here one lane per key
// holds the key's partials in registers for its whole run of the batch:
//   - a window of CHN_R(n) partials; per partial its state s (1 .. n-1: it has e1 .. es and waits in processor
//     p_s), the seqs of e1 .. es (32-bit offsets from the batch's seq base), e1's timestamp (32-bit offset from
//     the batch's first timestamp: the `within` test, StreamPreStateProcessor.java:118-129, reads only the start
//     state's event), the attribute words later filters read of each captured event, and the pool entries of
//     the events captured in earlier batches;
//   - list order by an order stamp: a partial appended to any list takes the next stamp, so each processor's
//     pending list is its partials of that state in stamp order, its newAndEvery list the staged ones after them
//     (no partial moves in the registers when it changes state);
//   - the start state's seed (pending or staged, its StateEvent timestamp) and every processor's flag word.
// and writes the lists back once in the general engine's block layout: partial j = StateEvent j, the seed =
// StateEvent R, the events it captured in this batch at free pool entries below min(64, SECAP) (the events carried in
// stay where they are), the block marked GEN_W0_CHN so that the next batch reads it back without the shape checks,
// each partial into the slot of its StateEvent (an unchanged partial is then not rewritten; the cold fields — the
// events' seqs and pool entries — live in LDS).  The state stays the general engine's: snapshots, state documents,
// purge, the live / min-seq scans and the general kernel read it unchanged.  A key whose stored lists do not fit this
// (another shape's history, an import, more partials than the window) is handed to the general kernel for its whole
// run (k_gen_batch GEN_M_KEYLIST); a key whose window could overflow at its next event (or whose next timestamp is
// outside the 32-bit offsets) is stored there and handed over from that event, so the results stay exactly the
// general engine's.
//
// One event of a key (restated from the reference, paths under
// /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/query/input/stream/state/):
//   receiver/PatternMultiProcessStreamReceiver.java:42-51 stabilizeStates: every processor's expireEvents
//       (StreamPreStateProcessor.java:325-361: the expired PREFIX of pending — the first surviving partial ends
//       it — and every expired newAndEvery entry), then every processor's updateState (:308-323: newAndEvery
//       sorted by timestamp, appended to pending; within one event every staged partial of a list has the same
//       timestamp, so the sort keeps their order);
//   PatternMultiProcessStreamReceiver.java:31-40: the processors in reverse order, p(n-1) .. p0;
//   StreamPreStateProcessor.java:364-403 processAndReturn: each pending partial (list order) with the event in its
//       slot through the filter (FilterProcessor.java:48-60); passing -> StreamPostStateProcessor.java:64-83: the
//       StateEvent's timestamp becomes the event's, it moves to the next processor's newAndEvery (addState,
//       :214-227), or, for the last state, is returned (a match) — either way it leaves the pending list; failing
//       -> it stays (PATTERN);
//   p0's seed: passing makes it the new partial and `every` stages a blank clone (addEveryState :229-247, the
//       `partials_created` counter); without `every` the start state is spent.
#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu.h"
#include "../../include/siddhi_gpu_ir.h"
#include "gen_engine.h"
#include "java_ops.h"
#include "sg_engine.h"
#include "reg_common.h"

namespace {

// CHN_ABL (experiment builds only, wrong results): 1 = no store, 2 = no event walked, 3 = every key loaded as fresh,
// 4 = captured events' pool entries not written
#ifndef CHN_ABL
#define CHN_ABL 0
#endif
#ifndef CHN_DEFER
#define CHN_DEFER 1   // captured events written at the store, slot by slot (0: as they are captured)
#endif
constexpr int CHN_NW = CHN_MAXNW;   // attribute words of an event (pack.h Pay<W>, W <= 4; chn_shape checks absNW)
constexpr uint32_t CHN_ORD_MASK = 0xffffffu;   // order stamp: low 24 bits of ord[]; the kept words' null bits above

template <int NE, int KW, int RR> struct ChnKey {
    static constexpr int R = RR;
    static constexpr int XW = (NE + 1) / 2;   // 16-bit pool entries, two per word
    const cGenProgram& G;
    const GenArgs& A;
    gu32* S;
    uint32_t K, k;
    int64_t tbase;
    uint64_t sbase;
    // the window
    uint32_t live, stg, pl0, pl1;   // slot masks: holds a partial, staged (in its processor's newAndEvery), state - 1 (2 bits)
    uint32_t ord[R];                // order stamp | kept-word null bits << 24
    int32_t t1[R];                  // e1 ts - tbase
    uint32_t kw[R][NE][KW > 0 ? KW : 1];
    // the fields only matches and the store read, in LDS (this lane's column of the wave's block): per slot the seq
    // offsets of e1 .. e(NE) (seq - sbase) and the pool entries of the events carried in (16 bits each, 0xffff:
    // captured in this batch)
    uint32_t* cold;
    uint32_t lane;
    uint32_t runB, cur;             // the key's run start and the payload index of the event being walked
    uint32_t stamp;                 // the next order stamp
    bool seedP, seedN;              // p0's seed in pending / newAndEvery
    int64_t seedTs;
    uint32_t fl[NE + 1];            // the processors' flag words
    uint32_t dirty;                 // slots whose StateEvent the store rewrites (new partials, moved ones, any untrusted load)
    uint32_t whole;                 // of those, the ones rewritten whole (new partials, untrusted loads); a moved partial
                                    // only gets its new event's slot word and its timestamp
    bool stHigh, outside;           // loaded with a StateEvent past the first bitmap word / an event past CHN_PA: the store
                                    // rewrites those bitmap words too
    bool canonOK;                   // the block was fresh or canonical: every dead slot's canonical entries are free, so
                                    // a captured event is written to its entry (and its StateEvent updated) as it is
                                    // captured, from the event's registers; else the store places and copies it
    uint32_t err;
    uint32_t scanned, created, matches;   // (this key's run: < 2^32)

    __device__ __forceinline__ ChnKey(const GenArgs& a, uint32_t key)
        : G(*(cGenProgram*)a.G), A(a), S(gp(a.state)), K(a.K), k(key), live(0), stg(0), pl0(0), pl1(0), runB(0), cur(0), stamp(0),
          seedP(false), seedN(false), seedTs(-1), dirty(0), whole(0), stHigh(false), outside(false),
          canonOK(false), err(0), scanned(0), created(0),
          matches(0) {
        tbase = a.b.pay ? gp(a.b.ts)[0] : 0;
        sbase = a.b.seq_base;
        lane = threadIdx.x & 63u;
#pragma unroll
        for (int i = 0; i <= NE; ++i) fl[i] = 0;
    }

    __device__ __forceinline__ gu32& W(uint32_t w_) const { return S[gen_il(K, k, w_)]; }
    __device__ __forceinline__ int64_t R64(uint32_t w_) const {
        return (int64_t)((uint64_t)W(w_) | ((uint64_t)W(w_ + 1) << 32));
    }
    __device__ __forceinline__ void W64(uint32_t w_, int64_t v) const {
        W(w_) = (uint32_t)(uint64_t)v;
        W(w_ + 1) = (uint32_t)((uint64_t)v >> 32);
    }
    __device__ __forceinline__ int proc(int i) const { return G.chnP[i]; }
    __device__ __forceinline__ uint32_t ks(int i) const { return G.offKS + (uint32_t)G.chnP[i] * G.ksWords; }
    __device__ __forceinline__ uint32_t stw(uint32_t se, uint32_t f) const { return G.offST + se * G.stWords + f; }
    __device__ __forceinline__ uint32_t sew(uint32_t e, uint32_t f) const { return G.offSE + e * G.seWords + f; }
    __device__ __forceinline__ uint32_t sid(int i) const { return (uint32_t)G.pre[G.chnP[i]].stateId; }
    // the partials of state s (1 .. NE)
    __device__ __forceinline__ uint32_t smask(int s) const {
        const uint32_t v = (uint32_t)(s - 1);
        return live & ((v & 1u) ? pl0 : ~pl0) & ((v & 2u) ? pl1 : ~pl1);
    }
    // new events take pool entries below PA (the window's R * NE events always fit there, chn_shape)
    __device__ __forceinline__ uint32_t poolArea() const { return G.SECAP < 64u ? G.SECAP : 64u; }
    // the canonical pool entry of event i of the partial in slot j (a partial owns its events: `every` only on p0, so
    // no clone shares them).  A block stored with every event at its canonical entry is marked GEN_W0_CHN and read
    // back slot by slot: all lanes of the wave at slot j read the same words of their keys, adjacent in the
    // key-interleaved block — coalesced, where a walk in list order reads a different entry per lane (one 64-B
    // sector per 4-B word: ~4.6 KB per key per batch at P3)
    static __device__ __forceinline__ uint32_t canon(int j, int i) { return (uint32_t)(j * NE + i); }
    __device__ __forceinline__ uint32_t& sqw(int j, int i) const { return cold[((uint32_t)i * R + (uint32_t)j) * 64u + lane]; }
    __device__ __forceinline__ uint32_t& ixw(int j, int h) const {
        return cold[((uint32_t)(NE + h) * R + (uint32_t)j) * 64u + lane];
    }
    __device__ __forceinline__ uint32_t getIx(int j, int i) const { return (ixw(j, i >> 1) >> ((i & 1) * 16)) & 0xffffu; }

    // ---- load: false = the stored lists are not this kernel's (the general kernel takes the key's whole run).  A
    // block this kernel stored (GEN_W0_CHN; the general kernel clears the mark when it takes the key) is read without
    // the shape checks, each partial back into the slot of its StateEvent (so an unchanged partial is not rewritten)
    __device__ __forceinline__ bool load() {
        const uint32_t w0 = W(0);
        if (!(w0 & 1u)) {   // PartitionRuntimeImpl.initPartition: p0.init() stages one seed (StreamPreStateProcessor.java:178-194)
            seedN = true;
            seedTs = -1;
            fl[0] = GF_INIT;
            canonOK = true;
            return true;     // (a fresh or purged key's block is zero)
        }
        const bool trusted = w0 == (1u | GEN_W0_CHN);
        if (!trusted && w0 != 1u) return false;   // (another register kernel's record or mark: not this shape's)
#pragma unroll
        for (int i = 0; i <= NE; ++i) fl[i] = W(ks(i) + KS_FLAGS);
        {
            const uint32_t pl = W(ks(0) + KS_PLEN), nl = W(ks(0) + KS_NLEN);
            if (pl + nl > 1u) return false;
            if (pl + nl == 1u) {
                const uint32_t x = W(ks(0) + KS_LISTS + (pl ? 0u : G.L));
                if (!trusted) {
                    if (x >= G.STCAP || W(stw(x, ST_TYPE)) != 0u || W(stw(x, ST_RC)) != 1u) return false;
                    for (int q = 0; q < G.nslots; q++)
                        if (W(stw(x, ST_SLOTS + (uint32_t)q)) != GEN_NIL) return false;
                    stHigh |= x >= 32u;
                }
                seedTs = R64(stw(x, ST_TS));
                seedP = pl != 0u;
                seedN = nl != 0u;
            }
        }
        if (trusted) return canonOK = loadCanonical();
        // every partial of every list, in list order (its order stamp), pending before newAndEvery
        const uint32_t PA = poolArea();
        for (int s = 1; s <= NE; ++s) {
            for (uint32_t which = 0; which < 2u; ++which) {
                const uint32_t n = W(ks(s) + KS_PLEN + which);
                int64_t prev = INT64_MIN;
                for (uint32_t e = 0; e < n; ++e) {
                    if (stamp >= (uint32_t)R) return false;
                    const uint32_t x = W(ks(s) + KS_LISTS + which * G.L + e);
                    int64_t xts = 0;
                    if (!trusted) {
                        if (x >= G.STCAP || W(stw(x, ST_TYPE)) != 0u || W(stw(x, ST_RC)) != 1u) return false;
                        xts = R64(stw(x, ST_TS));
                        stHigh |= x >= 32u;
                        if (which) {   // newAndEvery: already in timestamp order (its promotion sort keeps it)
                            if (xts == -1 || xts < prev) return false;
                            prev = xts;
                        }
                        for (int q = 0; q < G.nslots; q++) {
                            const uint32_t v = W(stw(x, ST_SLOTS + (uint32_t)q));
                            bool want = false;
#pragma unroll
                            for (int i = 0; i < NE; ++i) want |= (i < s && (uint32_t)q == sid(i));
                            if ((v != GEN_NIL) != want) return false;
                        }
                    }
                    int32_t q_[NE];
                    uint32_t x_[NE];
                    uint32_t w_[NE][KW > 0 ? KW : 1];
                    uint32_t nbits = 0;
                    int32_t e1t = 0;
#pragma unroll
                    for (int i = 0; i < NE; ++i) {
                        q_[i] = 0;
                        x_[i] = 0xffffu;
#pragma unroll
                        for (int c = 0; c < (KW > 0 ? KW : 1); ++c) w_[i][c] = 0;
                        if (i < s) {
                            const uint32_t ev = W(stw(x, ST_SLOTS + sid(i)));
                            if (!trusted && (ev >= G.SECAP || W(sew(ev, SE_NEXT)) != GEN_NIL)) return false;
                            const int64_t d = R64(sew(ev, SE_SEQ)) - (int64_t)sbase;
                            if (d < INT32_MIN || d > INT32_MAX) return false;
                            q_[i] = (int32_t)d;
                            x_[i] = ev;
                            outside |= ev >= PA;
                            if (i == 0 || (!trusted && i == s - 1)) {
                                const int64_t t = R64(sew(ev, SE_TS));
                                if (!trusted && i == s - 1 && t != xts) return false;   // (its ts is its last event's)
                                if (i == 0) {
                                    const int64_t o = t - tbase;
                                    if (t == -1 || o <= -SGD_TS_LIM || o >= SGD_TS_LIM) return false;
                                    e1t = (int32_t)o;
                                }
                            }
                            if (KW > 0) {
                                const uint32_t nb = W(sew(ev, SE_NULL));
#pragma unroll
                                for (int c = 0; c < KW; ++c) {
                                    w_[i][c] = W(sew(ev, G.absWordAt[G.chnKeepW[c]]));
                                    nbits |= ((nb >> G.chnKeepA[c]) & 1u) << (i * KW + c);
                                }
                            }
                        }
                    }
                    // the slot: its StateEvent's (this kernel's layout), else the next free one (rewritten at the store)
                    const uint32_t j = trusted ? x : stamp;
                    if (j >= (uint32_t)R || ((live >> j) & 1u)) return false;
#pragma unroll
                    for (int jj = 0; jj < R; ++jj) {   // (selects: a conditional store to a window element would put
                        const bool here = (uint32_t)jj == j;   //  the whole key object in scratch)
                        ord[jj] = here ? (stamp | (nbits << 24)) : ord[jj];
                        t1[jj] = here ? e1t : t1[jj];
#pragma unroll
                        for (int i = 0; i < NE; ++i)
#pragma unroll
                            for (int c = 0; c < (KW > 0 ? KW : 1); ++c) kw[jj][i][c] = here ? w_[i][c] : kw[jj][i][c];
                    }
#pragma unroll
                    for (int i = 0; i < NE; ++i) sqw((int)j, i) = (uint32_t)q_[i];
#pragma unroll
                    for (int h = 0; h < XW; ++h) ixw((int)j, h) = x_[2 * h] | ((2 * h + 1 < NE ? x_[2 * h + 1] : 0xffffu) << 16);
                    live |= 1u << j;
                    if (which) stg |= 1u << j;
                    if ((uint32_t)(s - 1) & 1u) pl0 |= 1u << j;
                    if ((uint32_t)(s - 1) & 2u) pl1 |= 1u << j;
                    stamp++;
                }
            }
        }
        if (!trusted) dirty = whole = live;
        return true;
    }

    // a block this kernel stored in the canonical layout: the lists give each slot's state, staging and order stamp
    // (list entry = StateEvent = slot; the list rows are read at the same position by every lane), then slot by slot
    // the captured events at their canonical entries
    __device__ __forceinline__ bool loadCanonical() {
        for (int s = 1; s <= NE; ++s) {
            for (uint32_t which = 0; which < 2u; ++which) {
                const uint32_t n = W(ks(s) + KS_PLEN + which);
                for (uint32_t e = 0; e < n; ++e) {
                    const uint32_t j = W(ks(s) + KS_LISTS + which * G.L + e);
                    if (stamp >= (uint32_t)R || j >= (uint32_t)R || ((live >> j) & 1u)) return false;
#pragma unroll
                    for (int jj = 0; jj < R; ++jj) ord[jj] = (uint32_t)jj == j ? stamp : ord[jj];
                    live |= 1u << j;
                    if (which) stg |= 1u << j;
                    if ((uint32_t)(s - 1) & 1u) pl0 |= 1u << j;
                    if ((uint32_t)(s - 1) & 2u) pl1 |= 1u << j;
                    stamp++;
                }
            }
        }
        bool ok = true;
#pragma unroll
        for (int jj = 0; jj < R; ++jj) {
            if (!((live >> jj) & 1u)) continue;
            const int s = (int)(((pl0 >> jj) & 1u) | (((pl1 >> jj) & 1u) << 1)) + 1;
            uint32_t nbits = 0;
#pragma unroll
            for (int i = 0; i < NE; ++i) {
                if (i >= s) continue;
                const uint32_t ev = canon(jj, i);
                const int64_t d = R64(sew(ev, SE_SEQ)) - (int64_t)sbase;
                ok &= d >= INT32_MIN && d <= INT32_MAX;
                sqw(jj, i) = (uint32_t)(int32_t)d;
                if (i == 0) {
                    const int64_t t = R64(sew(ev, SE_TS));
                    const int64_t o = t - tbase;
                    ok &= t != -1 && o > -SGD_TS_LIM && o < SGD_TS_LIM;
                    t1[jj] = (int32_t)o;
                }
                if (KW > 0) {
                    const uint32_t nb = W(sew(ev, SE_NULL));
#pragma unroll
                    for (int c = 0; c < KW; ++c) {
                        kw[jj][i][c] = W(sew(ev, G.absWordAt[G.chnKeepW[c]]));
                        nbits |= ((nb >> G.chnKeepA[c]) & 1u) << (i * KW + c);
                    }
                }
            }
            ord[jj] |= nbits << 24;
#pragma unroll
            for (int h = 0; h < XW; ++h)
                ixw(jj, h) = canon(jj, 2 * h) | ((2 * h + 1 < NE ? canon(jj, 2 * h + 1) : 0xffffu) << 16);
        }
        return ok;
    }

    // the kept words and their null bits of the partial in slot j (j at run time: selects over the static slots, so
    // the window stays in registers — indexing it at run time would move it to scratch)
    struct View {
        uint32_t w[NE][KW > 0 ? KW : 1];
        uint32_t nb;
    };
    __device__ __forceinline__ View view(int j) const {
        View v;
        v.nb = 0;
#pragma unroll
        for (int i = 0; i < NE; ++i)
#pragma unroll
            for (int c = 0; c < (KW > 0 ? KW : 1); ++c) v.w[i][c] = 0;
#pragma unroll
        for (int jj = 0; jj < R; ++jj) {
            const bool here = jj == j;
            v.nb = here ? ord[jj] >> 24 : v.nb;
#pragma unroll
            for (int i = 0; i < NE; ++i)
#pragma unroll
                for (int c = 0; c < KW; ++c) v.w[i][c] = here ? kw[jj][i][c] : v.w[i][c];
        }
        return v;
    }

    // ---- filter of processor p_t (t = 0: the seed, no events) on a partial's captured events (its kept words) with
    // the event in p_t's slot
    __device__ __forceinline__ bool evalOn(int t, const View& pv, const AbsEv<CHN_NW>& ev) {
        const auto& P = G.pre[proc(t)];
        if (P.flen == 0) return true;
        const uint32_t evSlot = sid(t);
        auto var_ = [&](uint32_t s, uint32_t a, int32_t c) -> GVal {
            if (c != 0 && c != -1) return GVal{0, true};   // a single event per slot
            const int ty = G.attrType[0][a];
            const bool wide = ty == SG_T_LONG || ty == SG_T_DOUBLE;
            uint32_t lo = 0, hi = 0, nb = 0;
            if (s == evSlot) {
                const uint32_t o = G.absOff[a];
#pragma unroll
                for (int q = 0; q < CHN_NW; ++q) {
                    lo = (uint32_t)q == o ? ev.w[q] : lo;
                    hi = (uint32_t)q == o + 1 ? ev.w[q] : hi;
                }
                nb = (ev.nb >> a) & 1u;
            } else {
                const int i = G.chnSlotEv[s];   // the captured event in slot s (e(i+1)), or -1
                if (i < 0 || i >= t) return GVal{0, true};
                const int c0 = G.chnAttrK[a];    // its first kept word
#pragma unroll
                for (int ii = 0; ii < NE; ++ii) {
#pragma unroll
                    for (int cc = 0; cc < KW; ++cc) {
                        lo = (ii == i && cc == c0) ? pv.w[ii][cc] : lo;
                        hi = (ii == i && cc == c0 + 1) ? pv.w[ii][cc] : hi;
                        nb = (ii == i && cc == c0) ? ((pv.nb >> (ii * KW + cc)) & 1u) : nb;
                    }
                }
            }
            return GVal{wide ? ((uint64_t)lo | ((uint64_t)hi << 32)) : (uint64_t)lo, nb != 0u};
        };
        if (P.ff.on) return jo_fast(P.ff, var_);
        const GVal v = jo_eval<false>(G.code, P.fpc, P.flen, err, var_, [&](uint32_t s, int32_t c) -> bool {
            if (s == evSlot) return !(c == 0 || c == -1);
            const int i = G.chnSlotEv[s];
            return i < 0 || i >= t || !(c == 0 || c == -1);
        });
        return !v.null && (v.b & 1);
    }
    // the filter of p_t over the partials of P: the hit mask (one evaluation site, slots walked at run time)
    __device__ __forceinline__ uint32_t hits(int t, uint32_t P, const AbsEv<CHN_NW>& ev) {
        uint32_t H = 0;
        for (uint32_t m = P; m; m &= m - 1u) {
            const int j = __ffs(m) - 1;
            if (evalOn(t, view(j), ev)) H |= 1u << j;
        }
        return H;
    }

    // the slot of the lowest order stamp among the slots of m (m != 0)
    __device__ __forceinline__ int firstOf(uint32_t m) const {
        uint32_t best = 0xffffffffu;
        int bj = 0;
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t o = ord[j] & CHN_ORD_MASK;
            const bool take = ((m >> j) & 1u) && o < best;
            best = take ? o : best;
            bj = take ? j : bj;
        }
        return bj;
    }
    __device__ __forceinline__ uint32_t minStamp(uint32_t m) const {   // the lowest order stamp among the slots of m
        uint32_t best = 0xffffffffu;
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t o = ord[j] & CHN_ORD_MASK;
            best = (((m >> j) & 1u) && o < best) ? o : best;
        }
        return best;
    }
    __device__ __forceinline__ int lastOf(uint32_t m) const {
        uint32_t best = 0;
        int bj = 0;
        bool any = false;
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t o = ord[j] & CHN_ORD_MASK;
            const bool take = ((m >> j) & 1u) && (!any || o > best);
            best = take ? o : best;
            bj = take ? j : bj;
            any |= ((m >> j) & 1u) != 0u;
        }
        return bj;
    }
    // order stamps renumbered from 0 in order (before they would leave 24 bits; at most once per ~1M events of a key)
    __device__ __forceinline__ void renumber() {
        uint32_t n = 0;
        for (uint32_t m = live; m;) {
            const int j = firstOf(m);
            m &= ~(1u << j);
#pragma unroll
            for (int jj = 0; jj < R; ++jj) ord[jj] = jj == j ? ((ord[jj] & ~CHN_ORD_MASK) | n) : ord[jj];
            n++;
        }
        stamp = n;
    }

    // ---- the matches of the last state's partials `H` on this event: one raw record each, in list order
    __device__ __forceinline__ void emit(uint32_t H, const AbsEv<CHN_NW>& ev, uint32_t pos) {
        const uint32_t c = __popc(H);
        uint32_t rank = 0;
        // one record per round for every lane with a match left (one atomic per wave and round)
        for (uint32_t m = H; m;) {
            const int j = firstOf(m);
            m &= ~(1u << j);
            const unsigned long long act = __ballot(true);
            const int leader = __ffsll((long long)act) - 1;
            const uint32_t sg = blockIdx.x % A.o.nseg;
            unsigned long long base = 0;
            if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(&A.o.raw_count[sg], (unsigned long long)__popcll(act));
            base = __shfl(base, leader, 64);
            const unsigned long long r = (unsigned long long)sg * A.o.seg_cap + base +
                                         __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
            const unsigned long long resEnd = (unsigned long long)(sg + 1) * A.o.seg_cap;
            if (r >= resEnd) { err |= GERR_MATCHCAP; rank++; continue; }
            gu32* rec = gp(A.o.raw) + r * A.o.recWords;
            rec[0] = pos;
            rec[1] = rank++;
            rec[2] = (uint32_t)ev.seq;
            rec[3] = (uint32_t)(ev.seq >> 32);
            rec[4] = (uint32_t)(uint64_t)ev.ts;   // StreamPostStateProcessor.java:68: the match's ts is the event's
            rec[5] = (uint32_t)((uint64_t)ev.ts >> 32);
            rec[6] = k;
            gu32* lens = rec + 7;
            gu32* seqs = lens + G.nslots;
            for (int q = 0; q < G.nslots; q++) lens[q] = 1u;
#pragma unroll
            for (int i = 0; i < NE; ++i) {
                const uint64_t q = sbase + (uint64_t)(int64_t)(int32_t)sqw(j, i);
                seqs[2 * sid(i)] = (uint32_t)q;
                seqs[2 * sid(i) + 1] = (uint32_t)(q >> 32);
            }
            seqs[2 * sid(NE)] = (uint32_t)ev.seq;
            seqs[2 * sid(NE) + 1] = (uint32_t)(ev.seq >> 32);
        }
        matches += c;
        gp(A.o.t_cnt)[pos] = c;
    }

    // ---- a captured event written where it is captured (canonOK): its StreamEvent at the canonical entry from the
    // event's registers (every attribute word is in ev.w: reg_layout), the StateEvent's slot word and timestamp
    __device__ __forceinline__ void putEvent(uint32_t to, const AbsEv<CHN_NW>& ev) const {
        W64(sew(to, SE_SEQ), (int64_t)ev.seq);
        W64(sew(to, SE_TS), ev.ts);
        W(sew(to, SE_NEXT)) = GEN_NIL;
        W(sew(to, SE_RC)) = 1u;
#pragma unroll
        for (int q = 0; q < CHN_NW; ++q)
            if ((uint32_t)q < G.absNW) W(sew(to, G.absWordAt[q])) = ev.w[q];
        W(sew(to, SE_NULL)) = ev.nb;
    }
    // canonOK: a captured event's 16-bit entry in the LDS column — deferred (0x8000 | its index in the key's run:
    // written at the store, slot by slot, if its partial is still alive, from the key-sorted payload), or, without a
    // payload or past 0x7fff events into the run, its canonical pool entry written now
    __device__ __forceinline__ uint32_t capture(int j, int i, const AbsEv<CHN_NW>& ev, bool fresh) const {
        const uint32_t d = cur - runB;
        if (CHN_DEFER && A.b.pay && d < 0x7fffu) return 0x8000u | d;
        captured(j, i, ev, fresh);
        return canon(j, i);
    }
    __device__ __forceinline__ void captured(int j, int i, const AbsEv<CHN_NW>& ev, bool fresh) const {
        const uint32_t e = canon(j, i), sb = G.offST + (uint32_t)j * G.stWords;
        if (CHN_ABL != 4) putEvent(e, ev);
        if (fresh) {
            for (int q = 0; q < G.nslots; q++) W(sb + ST_SLOTS + (uint32_t)q) = GEN_NIL;
            W(sb + ST_TYPE) = 0u;
            W(sb + ST_RC) = 1u;
        }
        W(sb + ST_SLOTS + sid(i)) = e;
        W64(sb + ST_TS, ev.ts);
    }

    // ---- one event of this key; false: stopped before it (the window could overflow, or the timestamp is
    // outside the 32-bit offsets), the general kernel continues from it
    __device__ __forceinline__ bool event(const AbsEv<CHN_NW>& ev, uint32_t pos) {
        const int64_t nowo = ev.ts - tbase;
        if (ev.ts == -1 || nowo <= -SGD_TS_LIM || nowo >= SGD_TS_LIM) return false;
        if ((seedP || seedN) && __popc(live) >= (uint32_t)R) return false;
        if (stamp + (uint32_t)R + 1u > CHN_ORD_MASK) renumber();
        const int32_t now = (int32_t)nowo;
        // stabilize: expireEvents of every processor (p0's seed holds no event: never expired), then updateState
        if (G.within != -1 && live) {
            uint32_t X = 0;
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const int64_t d = (int64_t)t1[j] - (int64_t)now;
                X |= (((d < 0 ? -d : d) > G.within) ? 1u : 0u) << j;
            }
            X &= live;
            if (X) {
                uint32_t kill = 0;
#pragma unroll
                for (int s = 1; s <= NE; ++s) {
                    const uint32_t M = smask(s), P = M & ~stg;
                    const uint32_t NX = P & ~X;
                    uint32_t pre = P & X;
                    if (NX) {   // the prefix before the first surviving pending partial
                        const uint32_t mo = minStamp(NX);
                        uint32_t below = 0;
#pragma unroll
                        for (int j = 0; j < R; ++j) below |= ((ord[j] & CHN_ORD_MASK) < mo ? 1u : 0u) << j;
                        pre &= below;
                    }
                    kill |= pre | (M & stg & X);
                }
                live &= ~kill;
                stg &= ~kill;
            }
        }
        stg = 0;   // updateState: the staged partials join their pending lists (same timestamps: order kept)
        if (seedN) {
            seedP = true;
            seedN = false;
        }
        // the processors in reverse order: the last state's partials match
        {
            const uint32_t P = smask(NE);
            const uint32_t H = P ? hits(NE, P, ev) : 0u;
            scanned += __popc(P);
            // GF_CHANGED: the last partial's result (StreamPreStateProcessor.process clears it per partial)
            const uint32_t fc = ((H >> lastOf(P)) & 1u) ? (fl[NE] | GF_CHANGED) : (fl[NE] & ~(uint32_t)GF_CHANGED);
            fl[NE] = P ? fc : fl[NE];
            if (H) {
                emit(H, ev, pos);
                live &= ~H;
            }
        }
        // the middle states: a passing partial takes the event in its next slot and moves on, staged
#pragma unroll
        for (int s = NE - 1; s >= 1; --s) {
            const uint32_t P = smask(s);
            const uint32_t H = P ? hits(s, P, ev) : 0u;
            scanned += __popc(P);
            const uint32_t fc = ((H >> lastOf(P)) & 1u) ? (fl[s] | GF_CHANGED) : (fl[s] & ~(uint32_t)GF_CHANGED);
            fl[s] = P ? fc : fl[s];
            // newAndEvery of p(s+1) in p(s)'s list order: new stamps in the old ones' order
            uint32_t wv[KW > 0 ? KW : 1], nbn = 0;
#pragma unroll
            for (int c = 0; c < KW; ++c) {
                uint32_t x = 0;
#pragma unroll
                for (int q = 0; q < CHN_NW; ++q) x = (uint32_t)q == G.chnKeepW[c] ? ev.w[q] : x;
                wv[c] = x;
                nbn |= ((ev.nb >> G.chnKeepA[c]) & 1u) << (s * KW + c);
            }
            const int32_t qn = (int32_t)(ev.seq - sbase);
            // newAndEvery of p(s+1) in p(s)'s list order: the hits take new stamps in their old stamps' order
            for (uint32_t m = H; m;) {
                const int j = firstOf(m);
                m &= ~(1u << j);
#pragma unroll
                for (int jj = 0; jj < R; ++jj) {
                    const bool here = jj == j;
#pragma unroll
                    for (int c = 0; c < KW; ++c) kw[jj][s][c] = here ? wv[c] : kw[jj][s][c];
                    ord[jj] = here ? (stamp | (((ord[jj] >> 24) | nbn) << 24)) : ord[jj];
                }
                stamp++;
                sqw(j, s) = (uint32_t)qn;   // the event's seq (LDS)
                if (canonOK) {              // its canonical pool entry, written now or at the store
                    const uint32_t sh = (uint32_t)(s & 1) * 16u;
                    ixw(j, s >> 1) = (ixw(j, s >> 1) & ~(0xffffu << sh)) | (capture(j, s, ev, false) << sh);
                } else {                    // no pool entry yet: the store places it
                    ixw(j, s >> 1) |= 0xffffu << ((s & 1) * 16);
                }
            }
            dirty |= H;
            const uint32_t ns = (uint32_t)s;   // new state s + 1: (s) in the planes
            pl0 = (pl0 & ~H) | ((ns & 1u) ? H : 0u);
            pl1 = (pl1 & ~H) | ((ns & 2u) ? H : 0u);
            stg |= H;
        }
        // p0: the seed
        if (seedP) {
            scanned++;
            View none;
            none.nb = 0;
#pragma unroll
            for (int i = 0; i < NE; ++i)
#pragma unroll
                for (int c = 0; c < (KW > 0 ? KW : 1); ++c) none.w[i][c] = 0;
            const bool hit = evalOn(0, none, ev);
            fl[0] = hit ? (fl[0] | GF_CHANGED) : (fl[0] & ~(uint32_t)GF_CHANGED);
            if (hit) {
                const uint32_t fr = ~live & (R >= 32 ? 0xffffffffu : ((1u << (R & 31)) - 1u));
                const int j = __ffs(fr) - 1;   // (the window had room: checked above)
                uint32_t nb = 0;
                uint32_t wk[KW > 0 ? KW : 1];
#pragma unroll
                for (int c = 0; c < KW; ++c) {
                    uint32_t wv = 0;
#pragma unroll
                    for (int q = 0; q < CHN_NW; ++q) wv = (uint32_t)q == G.chnKeepW[c] ? ev.w[q] : wv;
                    wk[c] = wv;
                    nb |= ((ev.nb >> G.chnKeepA[c]) & 1u) << c;
                }
                const int32_t qn = (int32_t)(ev.seq - sbase);
#pragma unroll
                for (int jj = 0; jj < R; ++jj) {
                    const bool here = jj == j;
                    ord[jj] = here ? (stamp | (nb << 24)) : ord[jj];
                    t1[jj] = here ? now : t1[jj];
#pragma unroll
                    for (int c = 0; c < KW; ++c) kw[jj][0][c] = here ? wk[c] : kw[jj][0][c];
                }
                sqw(j, 0) = (uint32_t)qn;
#pragma unroll
                for (int h = 0; h < XW; ++h) ixw(j, h) = 0xffffffffu;
                if (canonOK) ixw(j, 0) = capture(j, 0, ev, true) | 0xffff0000u;
                stamp++;
                live |= 1u << j;
                stg |= 1u << j;
                dirty |= 1u << j;
                whole |= 1u << j;
                pl0 &= ~(1u << j);
                pl1 &= ~(1u << j);
                seedP = false;
                if (G.chnEvery) {   // addEveryState: a blank clone with the partial's timestamp, staged
                    seedN = true;
                    seedTs = ev.ts;
                    created++;
                }
            }
        }
        return true;
    }

    // ---- a captured event's StreamEvent record (Lane::newEv), at pool entry `to`, from the batch
    __device__ __forceinline__ void storeEvent(uint32_t to, uint32_t pos) const {
        W64(sew(to, SE_SEQ), (int64_t)(sbase + (uint64_t)pos));
        W64(sew(to, SE_TS), gp(A.b.ts)[pos]);
        W(sew(to, SE_NEXT)) = GEN_NIL;
        W(sew(to, SE_RC)) = 1u;
        const int na = G.nattr[0];
        uint32_t nb = 0;
        for (int a = 0; a < na; a++) {
            const void* c = A.b.col[a];
            const uint32_t w = sew(to, SE_ATTR + 2 * (uint32_t)a);
            switch (G.attrType[0][a]) {
            case SG_T_LONG: case SG_T_DOUBLE: W64(w, (int64_t)gp((const uint64_t*)c)[pos]); break;
            case SG_T_BOOL: W(w) = gp((const uint8_t*)c)[pos] ? 1u : 0u; break;
            default: W(w) = gp((const uint32_t*)c)[pos];
            }
            if (A.b.nul[a] && gp(A.b.nul[a])[pos]) nb |= 1u << a;
        }
        W(sew(to, SE_NULL)) = nb;
    }

    // ---- store: the lists (rewritten), partial j = StateEvent j (rewritten when dirty), the seed = StateEvent R; the
    // events carried in stay where they are, the events captured in this batch take their canonical pool entries
    __device__ __forceinline__ void store() {
#pragma unroll
        for (int i = 0; i <= NE; ++i) W(ks(i) + KS_FLAGS) = fl[i];
        W(ks(0) + KS_PLEN) = seedP ? 1u : 0u;
        W(ks(0) + KS_NLEN) = seedN ? 1u : 0u;
        if (seedP || seedN) {
            W(ks(0) + KS_LISTS + (seedP ? 0u : G.L)) = (uint32_t)R;
            const uint32_t b = G.offST + (uint32_t)R * G.stWords;
            W64(b + ST_TS, seedTs);
            W(b + ST_TYPE) = 0u;
            W(b + ST_RC) = 1u;
            for (int q = 0; q < G.nslots; q++) W(b + ST_SLOTS + (uint32_t)q) = GEN_NIL;
        }
        // the pool entries below PA the events carried in hold; then the new events' entries
        const uint32_t PA = poolArea();
        unsigned long long occ = 0;
        for (uint32_t m = live; m; m &= m - 1u) {
            const int j = __ffs(m) - 1;
            const int s = (int)(((pl0 >> j) & 1u) | (((pl1 >> j) & 1u) << 1)) + 1;
            for (int i = 0; i < s; ++i) {
                const uint32_t e = canonOK ? canon(j, i) : getIx(j, i);
                if (e < PA) occ |= 1ull << e;
            }
        }
        if (canonOK) {   // the deferred events of the partials alive now, slot by slot (every lane at slot j writes
                         // the same rows of its key: adjacent words), and their StateEvents
            for (int j = 0; j < R; ++j) {
                if (!((dirty >> j) & 1u) || !((live >> j) & 1u)) continue;
                const int s = (int)(((pl0 >> j) & 1u) | (((pl1 >> j) & 1u) << 1)) + 1;
                const uint32_t sb = G.offST + (uint32_t)j * G.stWords;
                const bool all = (whole >> j) & 1u;
                if (all) {
                    for (int q = 0; q < G.nslots; q++) W(sb + ST_SLOTS + (uint32_t)q) = GEN_NIL;
                    W(sb + ST_TYPE) = 0u;
                    W(sb + ST_RC) = 1u;
                }
                for (int i = 0; i < s; ++i) {
                    const uint32_t h = getIx(j, i);
                    if (!(h & 0x8000u)) {   // (written when captured, or carried in)
                        if (all) W(sb + ST_SLOTS + sid(i)) = canon(j, i);
                        continue;
                    }
                    AbsEv<CHN_NW> ev;
                    abs_pay<CHN_NW>(A, runB + (h & 0x7fffu), tbase, ev);
                    putEvent(canon(j, i), ev);
                    W(sb + ST_SLOTS + sid(i)) = canon(j, i);
                    if (i == s - 1) W64(sb + ST_TS, ev.ts);
                }
            }
        }
        // the lists, row by row: each list's members in stamp order (lanes at the same position write adjacent words)
#pragma unroll
        for (int q = 1; q <= NE; ++q) {
            const uint32_t M = smask(q);
#pragma unroll
            for (uint32_t which = 0; which < 2u; ++which) {
                uint32_t r = 0;
                for (uint32_t m = M & (which ? stg : ~stg); m; r++) {
                    const int j = firstOf(m);
                    m &= ~(1u << j);
                    W(ks(q) + KS_LISTS + which * G.L + r) = (uint32_t)j;
                }
                W(ks(q) + KS_PLEN + which) = r;
            }
        }
        // the rewritten partials, slot by slot: partial j = StateEvent j, its new events at their canonical entries
        // (an entry an event carried in from a general layout holds: the lowest free one, and the block is stored
        // unmarked, to be read back through the checked path)
        bool canonical = true;
        for (int j = 0; j < R && !canonOK; ++j) {   // (canonOK: written as they were captured)
            if (!((dirty >> j) & 1u)) continue;
            const int s = (int)(((pl0 >> j) & 1u) | (((pl1 >> j) & 1u) << 1)) + 1;
            const uint32_t sb = G.offST + (uint32_t)j * G.stWords;
            const bool all = (whole >> j) & 1u;
            if (all)
                for (int q = 0; q < G.nslots; q++) W(sb + ST_SLOTS + (uint32_t)q) = GEN_NIL;
            for (int i = 0; i < s; ++i) {
                uint32_t e = getIx(j, i);
                const uint32_t pos = sqw(j, i);   // (captured in this batch: its batch position)
                if (e == 0xffffu) {
                    e = canon(j, i);
                    if ((occ >> e) & 1ull) e = (uint32_t)(__ffsll((long long)~occ) - 1);   // (< PA, chn_shape)
                    occ |= 1ull << e;
                    storeEvent(e, pos);
                    if (i == s - 1) W64(sb + ST_TS, gp(A.b.ts)[pos]);
                    W(sb + ST_SLOTS + sid(i)) = e;
                } else if (all) {
                    if (i == s - 1) W64(sb + ST_TS, R64(sew(e, SE_TS)));
                    W(sb + ST_SLOTS + sid(i)) = e;
                }
                canonical &= e == canon(j, i);
            }
            if (all) {
                W(sb + ST_TYPE) = 0u;
                W(sb + ST_RC) = 1u;
            }
        }
        // (a partial not rewritten was loaded from a marked, canonical block: a block loaded through the checked path
        // has every partial rewritten)
        W(0) = canonical ? (1u | GEN_W0_CHN) : 1u;
        // free bitmaps: StateEvents = the live slots and the seed; StreamEvents = the entries referenced
        const uint32_t seedBit = (seedP || seedN) ? 1u : 0u;   // (the seed is StateEvent R: word R / 32)
        W(G.offSTfree) = live | (R < 32 ? seedBit << (R & 31) : 0u);
        if (R >= 32) W(G.offSTfree + 1) = seedBit;
        if (stHigh)
            for (uint32_t q = R >= 32 ? 2u : 1u; q < (G.STCAP + 31) / 32; q++) W(G.offSTfree + q) = 0u;
        const uint32_t nw = (G.SECAP + 31) / 32;
        W(G.offSEfree) = (uint32_t)occ;
        if (nw > 1) W(G.offSEfree + 1) = (uint32_t)(occ >> 32);
        if (outside) {   // (events past PA carried in from a general-kernel layout: their words rebuilt)
            for (uint32_t q = 2; q < nw; q++) {
                uint32_t m = 0;
                for (uint32_t mm = live; mm; mm &= mm - 1u) {
                    const int j = __ffs(mm) - 1;
                    const int s = (int)(((pl0 >> j) & 1u) | (((pl1 >> j) & 1u) << 1)) + 1;
                    for (int i = 0; i < s; ++i) {
                        const uint32_t e = getIx(j, i);
                        if (e != 0xffffu && e / 32u == q) m |= 1u << (e % 32u);
                    }
                }
                W(G.offSEfree + q) = m;
            }
        }
    }
};

// an event's words from the batch columns (reg_common.h abs_gather, inlined: a call would take the event's address)
__device__ __forceinline__ void chn_gather(const GenArgs& a, const cGenProgram& G, uint32_t pos, AbsEv<CHN_NW>& ev) {
    ev.nb = 0;
#pragma unroll
    for (int q = 0; q < CHN_NW; ++q) ev.w[q] = 0;
    for (int at = 0; at < G.nattr[0]; at++) {
        const int ty = G.attrType[0][at];
        const void* c = a.b.col[at];
        uint32_t lo = 0, hi = 0;
        if (ty == SG_T_LONG || ty == SG_T_DOUBLE) {
            const uint64_t v = gp((const uint64_t*)c)[pos];
            lo = (uint32_t)v;
            hi = (uint32_t)(v >> 32);
        } else if (ty == SG_T_BOOL) {
            lo = gp((const uint8_t*)c)[pos] ? 1u : 0u;
        } else {
            lo = gp((const uint32_t*)c)[pos];
        }
        const uint32_t o = G.absOff[at];
        const bool wide = ty == SG_T_LONG || ty == SG_T_DOUBLE;
#pragma unroll
        for (int q = 0; q < CHN_NW; ++q) {
            ev.w[q] = (uint32_t)q == o ? lo : ev.w[q];
            ev.w[q] = (wide && (uint32_t)q == o + 1) ? hi : ev.w[q];
        }
        if (a.b.nul[at] && gp(a.b.nul[at])[pos]) ev.nb |= 1u << at;
    }
}

// ---- batch: one lane per key walks its events of the key-sorted batch ----
// ---- one key's run [b, e) of the key-sorted batch by one lane: false = handed over at `stop` (the general kernel,
// or the wide window, continues from the event where it stopped; stop = b: the block is not this kernel's)
template <int NE, int KW, int RR> struct ChnRun {
    unsigned long long scanned = 0, created = 0, matches = 0, keys = 0;
    uint32_t err = 0;
    bool fb = false;
    uint32_t stop = 0;
    __device__ __forceinline__ void run(const GenArgs& a, uint32_t key, uint32_t b, uint32_t e, uint32_t* cold) {
        ChnKey<NE, KW, RR> L(a, key);
        L.cold = cold;
        L.runB = b;
        bool walk = b < e;
        fb = false;
        stop = b;
        if (walk && !(CHN_ABL == 3 ? (L.seedN = true, true) : L.load())) {  // not this kernel's state: handed over whole
            fb = true;
            walk = false;
        }
        if (walk) {
            const cGenProgram& G = *(cGenProgram*)a.G;
            PayAhead<CHN_NW> ahead;
            ahead.first(a, b, e);
            uint32_t i = b;
            for (; i < e; i++) {
                AbsEv<CHN_NW> ev;
                uint32_t pos;
                if (a.b.pay) {
                    ahead.next(a, i, e, L.tbase, ev);
                    pos = (uint32_t)(ev.seq - a.b.seq_base);
                } else {
                    pos = a.b.sidx ? gp(a.b.sidx)[i] : i;
                    ev.ts = gp(a.b.ts)[pos];
                    ev.seq = a.b.seq_base + pos;
                    chn_gather(a, G, pos, ev);
                }
                if (CHN_ABL == 2) continue;
                L.cur = i;
                if (!L.event(ev, pos)) break;
            }
            if (CHN_ABL != 1) L.store();   // (a hand-over: the next kernel continues from the block)
            if (i < e) {
                fb = true;
                stop = i;
            } else {
                keys++;
            }
        }
        scanned += L.scanned;
        created += L.created;
        matches += L.matches;
        err |= L.err;
    }
};

// ---- batch: one lane per key walks its events of the key-sorted batch ----
template <int NE, int KW> __device__ __forceinline__ void chn_batch(const GenArgs& a) {
    constexpr int R = CHN_R(NE + 1);
    const uint32_t key = blockIdx.x * 64u + threadIdx.x;
    uint32_t b = 0, e = 0;
    if (key < a.K) {
        b = gp(a.b.seg_begin)[key];
        e = gp(a.b.seg_end)[key];
    }
    __shared__ uint32_t cold[R * (NE + (NE + 1) / 2) * 64];
    ChnRun<NE, KW, R> r;
    r.run(a, key < a.K ? key : 0u, b, e, cold);
    abs_fallback(a, r.fb, key, r.stop);
    abs_wave_stats(a, r.scanned, r.created, r.matches, r.keys, r.err, r.fb ? 1ull : 0ull);
}

// ---- the keys the chain kernel handed over (its window full, or a block it cannot take), in the wide window: a
// fixed grid of waves striding the list (its length is on the device), each key from the event where it stopped;
// what this window cannot hold goes on to the general kernel (fb2).  Its hand-overs are not counted again as
// window spills.
template <int NE, int KW> __device__ __forceinline__ void chn_wide(const GenArgs& a) {
    constexpr int R = CHN_RW(NE + 1);
    __shared__ uint32_t cold[R * (NE + (NE + 1) / 2) * 64];
    ChnRun<NE, KW, R> r;
    const unsigned long long n = *a.fb_n;
    for (unsigned long long base = (unsigned long long)blockIdx.x * 64u; base < n;
         base += (unsigned long long)gridDim.x * 64u) {   // (wave-uniform)
        const unsigned long long li = base + threadIdx.x;
        uint32_t key = 0, b = 0, e = 0;
        if (li < n) {
            key = gp(a.fb_list)[li];
            b = gp(a.fb_start)[key];
            e = gp(a.b.seg_end)[key];
        }
        r.run(a, key, b, e, cold);
        // (wave-aggregated append to the general kernel's list)
        const unsigned long long m = __ballot(r.fb);
        if (m) {
            const int lane = threadIdx.x & 63;
            unsigned long long b0 = 0;
            if (lane == __ffsll((long long)m) - 1) b0 = atomicAdd(a.fb2_n, (unsigned long long)__popcll(m));
            b0 = __shfl(b0, __ffsll((long long)m) - 1, 64);
            if (r.fb) {
                gp(a.fb2_list)[b0 + __popcll(m & ((1ull << lane) - 1ull))] = key;
                gp(a.fb2_start)[key] = r.stop;
            }
        }
    }
    abs_wave_stats(a, r.scanned, r.created, r.matches, r.keys, r.err, 0ull);
}

}  // namespace

// One kernel per (events a partial can hold, attribute words kept per captured event).  Occupancy floor 2 waves per
// SIMD (256 VGPRs): the window, the event in flight and the captured event's stores stay in registers — at 3 waves
// (168 VGPRs) the 3-state kernel spilled ~240 B per lane inside the walk and ran P3 at 8.7e8 events/s, at 2 at
// 1.09e9 (tools/exp_chain.py, one box, same build otherwise)
#ifndef SG_CHN_WAVES
#define SG_CHN_WAVES 2
#endif
#define CHN_KERNEL(NE, KW)                                                                                          \
    extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SG_CHN_WAVES, 8)))          \
    k_chn_batch_##NE##_##KW(const GenArgs ap) {                                                                     \
        (void)ap;   /* (read through the kernarg segment: a reference to the by-value parameter copies it to scratch) */ \
        chn_batch<NE, KW>(*(const GenArgs*)(const void*)__builtin_amdgcn_kernarg_segment_ptr());                    \
    }
CHN_KERNEL(1, 0)
CHN_KERNEL(1, 1)
CHN_KERNEL(1, 2)
CHN_KERNEL(2, 0)
CHN_KERNEL(2, 1)
CHN_KERNEL(2, 2)
CHN_KERNEL(3, 0)
CHN_KERNEL(3, 1)
CHN_KERNEL(3, 2)
// the wide window: one wave per SIMD (up to 512 VGPRs)
#define CHN_WIDE_KERNEL(NE, KW)                                                                                     \
    extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 8)))                     \
    k_chn_wide_##NE##_##KW(const GenArgs ap) {                                                                      \
        (void)ap;                                                                                                   \
        chn_wide<NE, KW>(*(const GenArgs*)(const void*)__builtin_amdgcn_kernarg_segment_ptr());                     \
    }
CHN_WIDE_KERNEL(1, 0)
CHN_WIDE_KERNEL(1, 1)
CHN_WIDE_KERNEL(1, 2)
CHN_WIDE_KERNEL(2, 0)
CHN_WIDE_KERNEL(2, 1)
CHN_WIDE_KERNEL(2, 2)
CHN_WIDE_KERNEL(3, 0)
CHN_WIDE_KERNEL(3, 1)
CHN_WIDE_KERNEL(3, 2)
