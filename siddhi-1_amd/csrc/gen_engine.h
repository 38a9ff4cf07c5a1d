// gen_engine.h — the general NFA engine: every query shape of the IR (stream / next / every / logical /
// count / absent states, PATTERN and SEQUENCE) on the device.  Shared by the host glue
// (gen_engine.hip, host part) and the advance kernels (gen_engine.hip, device part).
//
// The processor graph that StateInputStreamParser builds (util/parser/StateInputStreamParser.java:76-408)
// is lowered on the host into flat tables (GenProgram).  On the device one lane owns one partition key
// and runs that key's processors over its events in arrival order.  All per-key state lives in HBM,
// interleaved across keys (word w of key k at w * K + k) so that lanes reading the same field of
// their keys issue one coalesced access:
//   per processor  KeyState: flags, absent-state times, scheduler queue, pending and newAndEvery
//                  lists (StreamPreStateProcessor.StreamPreState, StreamPreStateProcessor.java:435-498)
//   StateEvent pool  partial matches (event/state/StateEvent.java:42-258), reference counted
//   StreamEvent pool slot events with their attributes captured at creation
//                  (event/stream/StreamEvent; count chains linked by `next`)
#pragma once

#include <stdint.h>

// Per-key state layout.  GEN_SPLIT = 0 (shipped): every word interleaved across keys, word w of key k at
// w * K + k, so a converged wave's access to one field is one coalesced transaction.  GEN_SPLIT = 1: the
// KeyState records (words [0, split), split = offST) interleaved, the StateEvent / StreamEvent pools and
// the deferred list contiguous per key (a record's words share cache lines).  Measured on C3_min1 / C4 /
// C4_deep: the split layout runs 0.69x / 0.73x / 0.78x — the kernel is bound by memory transactions, and
// per-key records turn each wave access into 64 of them.
#ifndef GEN_SPLIT
#define GEN_SPLIT 0
#endif
// GEN_GRAN_LOG2 = g (experiments): granules of 2^g consecutive words of one key interleaved across keys,
// word w of key k at ((w >> g) * K + k) << g | (w & (2^g - 1)); 0 (shipped) = one word per granule
#ifndef GEN_GRAN_LOG2
#define GEN_GRAN_LOG2 0
#endif
__host__ __device__ inline size_t gen_il(uint32_t K, uint32_t k, uint32_t w) {
    return ((((size_t)(w >> GEN_GRAN_LOG2)) * K + k) << GEN_GRAN_LOG2) | (w & ((1u << GEN_GRAN_LOG2) - 1u));
}
__host__ __device__ inline size_t gen_at(uint32_t K, uint32_t blockWords, uint32_t split, uint32_t k, uint32_t w) {
    if (!GEN_SPLIT || w < split) return gen_il(K, k, w);
    return (size_t)split * K + (size_t)k * (blockWords - split) + (w - split);
}

#define GEN_MAXP 16      // processors per query
#define GEN_MAXS 8       // input streams
#define GEN_MAXSLOT 16   // state slots
#define GEN_MAXA 16      // attributes per stream
#define GEN_MAXCODE 1024 // filter (+ projection) bytecode words
#define GEN_MAXPROJ 32   // selector items projected on the device (aggregator arguments + select + having)
#define GEN_MAXAGG 16    // aggregators of the selector on the device
#define GEN_NONE (-1)
#define GEN_NIL 0xffffu  // null pool index
#define GEN_RAWSEG 256   // raw-match reservation counters of a batch
#define GEN_RESCHUNK 4   // raw matches a lane reserves at a time
// a key block's word 0: bit 0 = initialised; GEN_W0_POOLC = abs_kernels.hip's layout with the constant words
// (type, refcounts, slot links) of pool entries [0, bits 2..7) in place, so its stores skip them (cleared by
// every other kernel that writes the block)
#define GEN_W0_POOLC 2u
// GEN_W0_DEEP: absd_kernels.hip keeps this key's absent-state lists and timer queue in its deep-store record
// (GenArgs.deep, one contiguous SoA record per key: coalesced for the key's one wave); the block then holds
// only the header words (flags, seed, list lengths, lastScheduledTime, queue length) and every component that
// reads the lists from the block flushes the record back first (gen_host.hip gen_flush_deep)
#define GEN_W0_DEEP 0x100u
// GEN_W0_REG: the register-window kernels (cnt_kernels.hip, abs_kernels.hip) keep this key's state in its
// register-native record (GenArgs.rec, interleaved like the blocks: row w of key k at w * K + k; gen_rec_words
// rows): a header (GEN_REC_EV rows: list lengths and memberships, flags, timestamps), the window's partials in
// list order (GEN_REC_R entries of seq i64, ts i64, null bits, attribute words) and, for the absent shape, its
// timer queue with the head at entry 0 (64-bit rows from gen_rec_q).  The block then holds only word 0; the
// kernels write back only what changed, and every component that reads the lists from the block flushes the
// records back first (gen_host.hip gen_flush_deep; k_gen_live / k_gen_min_seq read them in place)
#define GEN_W0_REG 0x200u
// GEN_W0_CHN: chn_kernels.hip stored this key's lists (in the general layout: partial j = StateEvent j, the seed =
// StateEvent CHN_R, events below min(64, SECAP)), so its next load skips the shape checks; the general kernel clears
// the mark when it takes the key over
#define GEN_W0_CHN 0x400u
// a deep-store record in 32-bit words: ts[L] i64, seq[L] u64, null bits[L], attribute words[NW][L], queue[Q] i64
struct GenDeepLayout {
    uint32_t oTs, oSeq, oNb, oW, oQ, words;
};
__host__ __device__ inline GenDeepLayout gen_deep_layout(uint32_t L, uint32_t Q, uint32_t NW) {
    GenDeepLayout d;
    d.oTs = 0;
    d.oSeq = 2 * L;
    d.oNb = 4 * L;
    d.oW = 5 * L;
    d.oQ = (5 + NW) * L;
    d.oQ += d.oQ & 1u;   // (8-B aligned: records start on even words)
    d.words = d.oQ + 2 * Q;
    return d;
}
#define ABS_R 8          // abs_kernels.hip: partials a key's register window holds
#define ABS_MAXNW 8      // abs_kernels.hip: attribute words of an event it captures
#define CNT_R 8          // cnt_kernels.hip: events a count chain in registers holds (the shape's max count)
#define GEN_REC_EV 8u     // a record's first partial row; each partial: seq lo, hi, ts lo, hi, null bits, NW words
#define GEN_REC_R 8u      // partials a record holds (= ABS_R = CNT_R)
static_assert(ABS_R == GEN_REC_R && CNT_R == GEN_REC_R, "the record holds the register windows");
// the first row of the timer queue (even: its 64-bit rows are 8-B aligned), the rows of a record
__host__ __device__ inline uint32_t gen_rec_q(uint32_t NW) {
    const uint32_t r = GEN_REC_EV + GEN_REC_R * (5u + NW);
    return r + (r & 1u);
}
__host__ __device__ inline uint32_t gen_rec_words(uint32_t NW, uint32_t Q) { return gen_rec_q(NW) + 2u * Q; }

enum { GK_STREAM = 0, GK_COUNT = 1, GK_LOGICAL = 2 };

// KeyState flag bits
enum {
    GF_CHANGED = 1u, GF_INIT = 2u, GF_SUCCESS = 4u, GF_SSRESET = 8u, GF_INACTIVE = 16u, GF_STARTED = 32u,
    GF_RUNNING = 64u
};

// A filter program of the form `operand CMP operand` (an attribute or a constant on each side, each widened
// to the compare domain), decoded once on the host (gen_host.hip jo_fast_decode) and evaluated by
// java_ops.h jo_fast without the interpreter: the common shapes `price > 20`, `price > e1.price`.
struct JoFast {
    uint32_t on, op, dom, pad;
    uint32_t isConst[2], from[2], slot[2], attr[2];
    int32_t chain[2];
    uint64_t cbits[2];  // constants, already in the compare domain
    uint32_t cnull[2], pad2[2];
};

struct GenPre {
    int32_t kind, absent, stateId, isStart;
    int64_t waiting;
    int32_t withinEvery, thisPost, thisLast, countPost;
    uint32_t fpc, flen;
    int32_t minCount, maxCount, logicalType, partner;
    JoFast ff;   // the filter as one decoded compare (java_ops.h), when it has that form (ff.on)
};

struct GenPost {
    int32_t kind, absent, stateId, thisPre;
    int32_t nextStatePre, nextEveryStatePre, callbackPre, hasNext;
    int32_t minCount, maxCount, logicalType, partnerPre, partnerPost, pad;
};

struct GenRecv {
    int32_t multi, n, nStateProcs, pad;
    int32_t procs[GEN_MAXP];        // nextProcessors (setup order); events visit them in reverse
    int32_t stateProcs[GEN_MAXP];   // stateProcessorsForStream
};

struct GenProgram {
    int32_t nprocs, nslots, qtype, playback, partitioned, nstreams;
    int64_t within;
    int32_t nStartIds, nInit, nReset, nUpdate, nAll, nStartup;
    int32_t startIds[GEN_MAXSLOT];
    int32_t initOrder[GEN_MAXP * 2], resetOrder[GEN_MAXP * 2], updateOrder[GEN_MAXP * 2];
    int32_t allProcs[GEN_MAXP], startup[GEN_MAXP];
    int32_t rootFirst, rootLast;
    GenPre pre[GEN_MAXP];
    GenPost post[GEN_MAXP];
    GenRecv recv[GEN_MAXS];
    int32_t slotStream[GEN_MAXSLOT];
    int32_t nattr[GEN_MAXS];
    int32_t attrType[GEN_MAXS][GEN_MAXA];
    uint32_t ncode;
    uint32_t code[GEN_MAXCODE];
    // capacities and the per-key block layout (words)
    uint32_t L, Q, STCAP, SECAP, NA, MC;  // list, timer queue, pools, attrs per event, max chain out
    uint32_t ksWords;                       // words of one processor's KeyState
    uint32_t offKS, offST, offSTfree, offSE, offSEfree, offDef, blockWords;
    uint32_t stWords, seWords, DEF;
    // on-device projection of the select list (sg_set_projection): item i = code[projPc[i], +projLen[i]);
    // items [0, projAgg) are aggregator arguments (siddhi_gpu_ir.h), the rest the select list and the optional
    // `having`, whose values go to the raw match record (3 words each from projOff)
    uint32_t projN, projOff;
    uint32_t projAgg;                     // aggregators; their per-key state: 5 words each from offAgg
    uint32_t offAgg;                      //   (count lo/hi, value lo/hi, has-value)
    uint32_t projPc[GEN_MAXPROJ], projLen[GEN_MAXPROJ], projType[GEN_MAXPROJ];
    // the absent-tail shape `[every] e1=S[f0] -> not S[f1] for T [within W]` (PATTERN, partitioned, playback,
    // one stream), which runs on the register-window kernels of abs_kernels.hip (gen_host.hip abs_shape):
    // absP0 / absP1 the start and absent processors, absEvery: `every` re-arms the start seed, absNW the
    // words an event's attributes take (2 for long / double), absOff[a] attribute a's first word
    int32_t absOk, absP0, absP1, absEvery, absListener;
    uint32_t absNW;
    uint32_t absOff[GEN_MAXA];
    // the counting sequence shape `every e1=S[f0]<m:n>, e2=S[fA] or e3=S[fB] [within W]` (SEQUENCE,
    // partitioned, one stream), which runs on the register-window kernel of cnt_kernels.hip (gen_host.hip
    // cnt_shape): cntP0 the count processor, cntPA / cntPB the logical OR pair in the order an event visits
    // them (the receiver's reverse order), cntWE: p0's withinEvery is p0 itself (an expired partial of p0's
    // lists is cloned into it, StreamPreStateProcessor.java:354-357); absNW / absOff give the word layout
    int32_t cntOk, cntP0, cntPA, cntPB, cntWE;
    int32_t cntAnd, cntPad;   // the pair is a logical AND (`e2=S[fA] and e3=S[fB]`) instead of an OR
    uint32_t absWordAt[ABS_MAXNW];  // the StreamEvent record word (SE_ATTR + ...) of each captured word
    // the chained stream states `[every] e1=S[f0] -> e2=S[f1] -> ... -> en=S[f(n-1)] [within W]` (PATTERN,
    // partitioned, one stream, 2 <= n <= CHN_MAXN), which run on the register-window kernel of chn_kernels.hip
    // (gen_host.hip chn_shape): chnP[i] the processor of state i, chnEvery: `every` re-arms p0's seed; the attribute
    // words later filters read of a captured event are kept in the window (chnKW of them: event word chnKeepW[c] of
    // attribute chnKeepA[c]; chnAttrK[a] = the kept index of attribute a's first word, or -1) and chnSlotEv[s] is
    // the event index (state) whose event slot s holds
    int32_t chnOk, chnN, chnEvery, chnKW;
    int32_t chnWide;   // the wide-window kernel takes the keys the chain kernel hands over (its window fits the block)
    int32_t chnP[4];
    uint32_t chnKeepW[2], chnKeepA[2];
    int32_t chnAttrK[GEN_MAXA];
    int32_t chnSlotEv[GEN_MAXSLOT];
};
#define CHN_MAXN 4       // chn_kernels.hip: states of a chain
#define CHN_MAXNW 4      // chn_kernels.hip CHN_NW: attribute words of a chained-state stream's event
// chn_kernels.hip: partials a key's register window holds, for a chain of n states (k_chn_batch, 2 waves per SIMD),
// and the wide window of the kernel the keys that outgrow it go to (k_chn_wide, 1 wave per SIMD: up to 512 VGPRs;
// its canonical pool entries, n - 1 per partial, stay below 64)
#ifndef CHN_R3
#define CHN_R3 24        // (the 3-state window: P3 per push 16 slots 3.63 ms, 20: 3.68-3.72, 24: 3.46-3.59 — 247 VGPRs,
                         // no spill at two waves per SIMD, 18 KB of LDS per wave; experiment builds override it)
#endif
#define CHN_R(n) ((n) == 2 ? 24 : (n) == 3 ? CHN_R3 : 12)
#define CHN_RW(n) ((n) == 2 ? 32 : (n) == 3 ? 32 : 21)

// KeyState field offsets inside a processor's record
#define KS_FLAGS 0
#define KS_LST 1    // lastScheduledTime (2 words)
#define KS_LAT 3    // lastArrivalTime (2)
#define KS_FIRE 5   // fireAt (2)
#define KS_ORDER 7  // scheduler order (1)
#define KS_QHEAD 8  // queue head index
#define KS_QLEN 9
#define KS_PLEN 10  // pending length
#define KS_NLEN 11  // newAndEvery length
#define KS_LISTS 12 // pending[L], newAndEvery[L], queue[Q] (2 words each)

// StateEvent record: ts(2) type(1) rc(1) slots[nslots]
#define ST_TS 0
#define ST_TYPE 2
#define ST_RC 3
#define ST_SLOTS 4
// StreamEvent record: seq(2) ts(2) next(1) rc(1) null(1) attrs[NA](2 each)
#define SE_SEQ 0
#define SE_TS 2
#define SE_NEXT 4
#define SE_RC 5
#define SE_NULL 6
#define SE_ATTR 7

// GST_LIVE0: SG_CFG_TIMING only; GST_SPILLS: keys the register-window kernels (abs_kernels.hip) handed to the
// general kernels (sg_stats.window_spills)
enum { GST_SCANNED = 0, GST_CREATED, GST_MATCHES, GST_KEYS, GST_LIVE0, GST_SPILLS, GST_N };
enum { GERR_CAP = 1, GERR_MATCHCAP = 2, GERR_KEY = 4, GERR_COLLAPSE = 8, GERR_CHAIN = 16, GERR_REF = 32 };

struct GenBatch {
    uint32_t n, stream;
    uint64_t seq_base;
    const int64_t* ts;
    const void* col[GEN_MAXA];
    const uint8_t* nul[GEN_MAXA];
    const uint32_t* sidx;      // key-sorted batch positions: sorted element i's at sidx[i * sidxStride]
    const uint32_t* seg_begin; // [K]
    const uint32_t* seg_end;
    // the key-sorted payload (pack.h Pay<W>: batch position, the attribute words in attribute order, the
    // null bits when payNull, the ts offset from ts[0] or SGD_TS_FAR), or NULL: then the kernels read the
    // columns at sidx positions
    const uint32_t* pay;
    uint32_t payStride;        // words per element (W + 2)
    uint32_t payNull;
    uint32_t sidxStride;       // 0 = 1
    // the fused grouping of the count kernel (gen_host.hip): the batch grouped by 64-key tile (Pay<W> elements, key &
    // 255 in the position's bits 24..31), tile t at [tile_lo[t], tile_lo[t + 1]) of tpay; k_cnt_split splits each
    // tile by key into `pay` and writes every key's bounds (its largest tile to tileMax)
    uint32_t pad2;
    const uint32_t* tile_lo;
    const uint32_t* tpay;
    uint32_t* tileMax;
};

struct GenOut {
    // raw matches: per match [trigger seq u64][ts i64][key u32][len[nslots] u32][seqs nslots*MC u64], as words
    uint32_t* raw;
    // matches reserved, per segment: a batch spreads its lanes' reservations over GEN_RAWSEG counters
    // (segment = wave % nseg, slots [s * seg_cap, (s + 1) * seg_cap)); one device-wide counter hit by
    // every lane serialises at the memory side.  Timer sweeps use one segment (their order sort reads
    // a dense prefix).
    unsigned long long* raw_count;
    uint64_t raw_cap;                // in matches
    uint64_t seg_cap;
    uint32_t nseg;
    uint32_t recWords;
    // per batch event: matches it triggered and the first raw index (contiguous)
    uint32_t* t_cnt;
    uint32_t* t_first;
    uint32_t* t_multi;   // GEN_M_TFIRST: set when a trigger emitted more than one match (the ordering scatters)
    // timer matches: sort keys per raw match (k1 sched or 0, k2 due/fireAt, k3 key, raw index)
    int64_t* tk2;
    uint32_t* tk1;
    uint32_t* tk3;
    unsigned long long* nvalid;      // timer matches emitted by a sweep
    unsigned long long* stats;
    // per-wave counter rows [wave][GST_N] of the register-window kernels (summed by k_gen_stats_reduce:
    // one device-wide atomic per wave and counter serialised ~16K atomics per counter at 2^20 keys)
    unsigned long long* wstats;
    uint32_t* err;
    unsigned long long* prof;        // GENX_PROF builds: shader-clock cycles per walk phase (summed over waves)
};

// Timers (sg_advance_time).  Each key's next deadline (the earliest queue head of its absent
// processors under the playback listener, the earliest caller fire time under the wall clock) is kept in
// nd[K] by every kernel that changes the key's timers; an advance to T compacts the keys with
// nd <= T into `due` and runs k_gen_timers over those only.  Under playback each due (key, listener)
// also records its queue head in dpair_key / dpair_i (slot due index * nStartup + listener), so that
// the host can detect two keys sharing a due time at one advance.
#define GEN_NO_DEADLINE INT64_MAX
#define GEN_PAIR_NONE 0xffffffffu
struct GenTimers {
    int64_t* nd;                     // [K] next deadline, GEN_NO_DEADLINE = none
    uint32_t* due;                   // [K] keys due at this advance
    unsigned long long* ndue;
    unsigned long long* dpair_key;   // [K * nStartup] order-preserving u64 of the head, or UINT64_MAX
    uint32_t* dpair_i;               // [K * nStartup] listener index, or GEN_PAIR_NONE
    // one listener (nStartup == 1, partitioned, playback): the timer matches are ordered through the due
    // keys sorted by head (gen_host.hip timer_order_keys) instead of a sort of the matches: the key of each
    // due slot and each due key's match count of the sweep (records carry their rank within the key)
    uint32_t* dpair_kid;             // [K] key of due slot di, or NULL
    uint32_t* kcnt;                  // [K] matches of the key at this sweep, or NULL; | GEN_KCNT_STAGED when
                                     //     k_abs_timers left them in tstage (not in the raw records)
    // k_abs_timers: a key's (e1 seq, fire time) per match of the sweep, rank-major ([rank][K] seqs, then
    // [rank][K] times): at most ABS_R per key (a sweep only emits partials that were live at its start)
    unsigned long long* tstage;
};
#define GEN_KCNT_STAGED 0x80000000u

struct GenArgs {
    const GenProgram* G;
    uint32_t* state;     // [blockWords][K] interleaved
    uint32_t K;
    GenBatch b;
    GenOut o;
    GenTimers t;
    int64_t now;         // engine clock during a push; the advance target for a timer sweep
    int64_t now0;        // the engine clock before a wall-clock timer sweep
    uint32_t kpl;        // k_gen_batch: keys per lane (lane l of block b walks keys (b*kpl + j)*64 + l)
    uint32_t mode;       // GEN_M_* below
    // keys the register-window kernels (abs_kernels.hip) hand to the general kernels: the list, its
    // length and, for a batch, the index of the key's first event still to walk (absolute, into sidx)
    uint32_t* fb_list;
    unsigned long long* fb_n;
    uint32_t* fb_start;
    // the wave-per-key kernels (absd_kernels.hip) take fb_list and hand what they cannot hold on in this one
    uint32_t* fb2_list;
    unsigned long long* fb2_n;
    uint32_t* fb2_start;
    // the deep store (GEN_W0_DEEP), deepWords words per key, or nullptr
    uint32_t* deep;
    uint32_t deepWords;
    uint32_t pad3;
    // the register-native records (GEN_W0_REG), gen_rec_words rows, or nullptr
    uint32_t* rec;
};
// GenArgs.mode
#define GEN_M_KEYLIST 1u   // k_gen_batch: lane i walks key fb_list[i] from fb_start[key]
#define GEN_M_NOPAIRS 2u   // k_gen_timers over fb_list: the collapse pairs were recorded by k_abs_timers
// a raw match record's word 1 (its rank within the trigger) with this bit: the slot chains are PACKED after the
// chain lengths, slot by slot in slot order (slot s's entries at the sum of the lengths of the slots before
// it), instead of at s * MC (cnt_kernels.hip: a match then writes its used words contiguously)
#define GEN_REC_PACKED 0x80000000u
#define GEN_M_NOCHUNK 8u   // k_absd_batch*: the per-event walk only (SG_NO_ABSD_CHUNK; A/B and parity tests)
#define GEN_M_TFIRST 4u    // batch kernels: each trigger emits at most one match; record its raw slot in t_first
                           // (the ordering then gathers output-major, gen_host.hip k_gen_gather1)
