// sg_engine.h — internal definitions shared by the host side of the C-ABI (sg_engine.hip, sg_jit.cpp),
// the ahead-of-time kernels (p2_kernels.hip) and the query-specialised advance kernel (p2_jit.hip,
// compiled at engine creation by hipRTC).  Not part of the public ABI (that is include/siddhi_gpu.h).
// Keep this header free of host-only includes: hipRTC compiles it as part of the JIT source.
#pragma once

#include <stdint.h>

// Ablation knobs that deliberately produce wrong results (timing experiments) exist only in builds made
// with EXTRA=-DSG_EXPERIMENTS; in the shipped library SG_EXP(x) is the constant 0 and their code is gone.
#ifndef SG_EXP
#ifdef SG_EXPERIMENTS
#define SG_EXP(x) (x)
#else
#define SG_EXP(x) 0u
#endif
#endif

#define SGD_MAX_PROG 64    // filter program length (instructions)
#define SGD_MAX_STACK 16   // filter evaluation stack depth
#define SGD_MAX_EVCOLS 8   // event columns a query's filters read (per stream)
#define SGD_MAX_CAPS 8     // slot-0 attributes captured into a partial match
#define SGD_MAX_CONST 32   // filter constants (kernel arguments, so equal-shaped queries share code)
#define SGD_MAX_REG 16     // register window (partials per lane) upper bound
#define SGD_MAX_REG_HBM 31 // the HBM pass's register window upper bound (a 32-bit slot mask, shifts by n < 32)
#define SGD_WAVE 64
#ifndef SGD_BLOCK
#define SGD_BLOCK 256      // lanes (= keys) per workgroup of the advance kernel
#endif
#define SGD_STAGE_MAX_BYTES 147456  // LDS per workgroup staging its keys' payload runs (upper bound; the
                                    // static LDS of the lane dealing sits beside it in the 160 KB)
// key-sorted payload timestamps are 32-bit offsets from the batch's first (arrival-order) timestamp;
// an event whose offset does not fit [-2^30, 2^30] (or whose ts is -1) carries SGD_TS_FAR and the
// advance kernel reads its full timestamp from the batch's ts column
#define SGD_TS_FAR ((int32_t)0x80000000)
#define SGD_TS_LIM (1ll << 30)
#define SGD_RAW_CHUNK 256  // raw match slots a wave reserves at a time (the raw buffer has 2 chunks of slack per wave)
#define SGD_TD_INLINE (1ull << 63)  // t_desc: the trigger's one match carried inline (no raw slot)
// t_desc word: [0, 32) first raw slot (or the inline e1 seq offset), [32, 47) match count (<= SGD_MAX_CAP), [47, 63)
// the batch's tag (an entry written under another batch's tag reads as "no match": the ordering never clears
// t_desc), bit 63 inline
#define SGD_TD_CNT(d) ((uint32_t)((d) >> 32) & 0x7fffu)
#define SGD_TD_TAGOF(d) ((uint32_t)((d) >> 47) & 0xffffu)
#define SGD_TD_TAG(epoch) ((uint64_t)(epoch) << 47)
// the fused grouping's LDS split keeps up to this many 64-event rounds per wave in registers (p2_jit.hip
// tile_split_lds): a tile of more than SGD_SPLIT_CHUNKS(stride) * SGD_BLOCK events goes to the HBM pass
#define SGD_SPLIT_CHUNKS(stride) (80u / ((stride) + 1u))
#define SGD_SPLIT_CNT_BYTES ((SGD_BLOCK / SGD_WAVE) * SGD_BLOCK * 2u)   // its per-(wave, key) u16 counters
#define SGD_HBM_STAGE_BYTES 32768u  // the HBM pass: LDS staging of one wave's runs (dynamic LDS of its 1-wave groups)

// ---- filters ------------------------------------------------------------------------------------
// A filter's IR bytecode (siddhi_gpu_ir.h) is lowered to DProg (variables resolved to event
// columns / captured slot-0 attributes), from which sg_jit.cpp generates typed HIP code.
enum { SGD_SRC_EV = 0, SGD_SRC_CAP = 1, SGD_SRC_CONST = 2, SGD_SRC_NULL = 3 };

struct DInst {
    uint8_t op;   // SG_OP_*
    uint8_t t;    // type / domain / from
    uint8_t t2;   // to (CVT), null flag (CONST)
    uint8_t src;  // SGD_SRC_* for VAR
    int32_t arg;  // event column / capture index
    uint64_t imm; // constant bits
};

struct DProg {
    uint32_t len;
    uint32_t pad;
    DInst ins[SGD_MAX_PROG];
};

// two-state pattern shapes handled by the P2 kernel family
enum {
    SGD_P2_EVERY_FIRST = 1,  // every e1 -> e2            (post0.nextEvery = pre0)
    SGD_P2_EVERY_BOTH = 2,   // every (e1 -> e2)          (post1.nextEvery = pre0, pre*.withinEvery = pre0)
};

// per-key header word
#define SGD_H_NPEND(h) ((h) & 0xfffu)
#define SGD_H_NSTG(h) (((h) >> 12) & 0xfffu)
#define SGD_H_SPEND(h) (((h) >> 24) & 0x3u)
#define SGD_H_SSTG(h) (((h) >> 26) & 0x3u)
#define SGD_H_INIT(h) (((h) >> 28) & 0x1u)
#define SGD_H_MAKE(np, ns, sp, ss, in) \
    ((uint32_t)(np) | ((uint32_t)(ns) << 12) | ((uint32_t)(sp) << 24) | ((uint32_t)(ss) << 26) | ((uint32_t)(in) << 28))
#define SGD_MAX_CAP 4095u
#define SGD_NO_RESUME 0xffffffffu
#define SGD_HOT_DONE 0xfffffffeu   // resume word: the hot-key pipeline advanced the key (the HBM pass skips it)
#define SGD_HOT_MARK 0xfffffffdu   // resume word: a hot key of a wave the staged pass left whole (counted there)
#define SGD_HOT_IDLE 8             // drained batches in a row without hot keys before the pipeline's buffers go back
#define SGD_HOT_CTL 8
#define SGD_HOT_CTL_BIG 6          // hot_ctl word: workgroups whose range exceeded SGD_BIG_TILE events
#define SGD_BIG_TILE 65536u
#define SGD_HOT_INFO 16

enum { SGD_ST_SCANNED = 0, SGD_ST_CREATED, SGD_ST_MATCHES, SGD_ST_KEYS, SGD_ST_LIVE0, SGD_ST_SPILLS, SGD_ST_HOTK,
       SGD_ST_HOTE, SGD_ST_N };

enum { SGD_ERR_PARTIAL_CAP = 1, SGD_ERR_MATCH_CAP = 2, SGD_ERR_KEY_RANGE = 4, SGD_ERR_PROJ = 8 };

// Advance-kernel arguments.  Everything that shapes the code (pattern mode, stream roles, column
// types, filter expressions, capture layout, register window) is compiled into the kernel; this
// struct carries only pointers, sizes and the filter constants.
struct P2Params {
    uint32_t n_keys;
    uint32_t cap;                      // partial capacity per key (HBM slab depth)
    uint64_t seq_base;
    int64_t within;                    // -1 = none
    // key-sorted batch: element i = [batch position][filter column words..][null bits?][ts lo, hi]
    const uint32_t* payload;
    const int64_t* ts_col;             // the batch's timestamps in arrival order (ts_col[0]: the offsets' base)
    uint32_t* seg_begin;               // [n_keys] (fused grouping: written by the staged pass for the keys it
    uint32_t* seg_end;                 //  leaves to the HBM pass, whose runs it writes to `payload`)
    // fused grouping (part.h sgd_group_tiles_fused; null: `payload` is key-sorted with seg_begin / seg_end): the
    // batch grouped by key tile (one tile = the SGD_BLOCK keys of one workgroup, arrival order within a tile,
    // position bits 24..31 = key & 255) in `tpay`, tile t at [tile_lo[t], tile_lo[t + 1]); the staged pass splits
    // its tile by key in LDS
    const uint32_t* tile_lo;
    const uint32_t* tpay;
    uint32_t write_sorted;             // fused: also write every key's run to `payload` + seg bounds (aggregators)
    uint32_t hbm_stage_chunks;         // the HBM pass's LDS staging per wave (16-B chunks; its dynamic LDS)
    // per-key state (SoA, partial j of key k at j * n_keys + k)
    uint32_t* hdr;
    int64_t* p_ts;
    uint64_t* p_seq;
    uint32_t* p_capw;                  // [n_capw][cap][n_keys] captured attribute words
    uint32_t* p_capnull;               // [cap][n_keys] null bits of the captures
    // matches: slot-0 event seq of every emitted match, appended in wave-reserved chunks; per batch
    // event t the number of matches it triggered and the position of the first (a trigger's matches
    // are contiguous, in emission order)
    uint64_t* raw_e1;
    unsigned long long* raw_count;
    uint64_t raw_capacity;
    uint64_t* t_desc;                  // [max_batch] count << 32 | first raw slot, or (SGD_TD_INLINE) one match
                                       // whose e1 seq - seq_base is the low word; zero outside the
                                       // advance -> scatter window
    unsigned long long* stats;         // [SGD_ST_N] cumulative (HBM pass adds here directly)
    unsigned long long* wstats;        // [n_keys / 64][SGD_ST_N] staged pass, this batch (k_stats_reduce)
    uint64_t raw_static;               // raw_e1 slots [0, raw_static) belong to the staged pass's waves
    uint32_t* err;
    uint32_t* deferred;                // [n_keys / 64] waves the staged pass left to the HBM pass:
                                       // 1 = the whole wave, 2 = the keys with a resume point
    uint32_t* dlist;                   // [n_keys / 64] the waves the HBM pass takes (appended by the staged pass)
    uint32_t* dlist_n;                 // [2] their number, then klist's (reset after the batch by k_stats_reduce)
    uint32_t* klist;                   // [n_keys] the keys the staged pass stopped (the HBM pass resumes them, a
                                       // lane each: a wave of them, not the waves they sit in)
    uint32_t* resume;                  // [n_keys] event index (in the key's run) where the HBM pass
                                       // resumes a key the staged pass stopped; SGD_NO_RESUME otherwise
    unsigned long long* prof;          // SGX_PROF experiments only (NULL otherwise)
    uint32_t* raw_capw;                // SGQ_PROJ: [n_capw][raw_capacity] the matched partial's captures
    uint32_t* raw_capnull;             // SGQ_PROJ: [raw_capacity] their null bits
    uint32_t stage_chunks;             // LDS staging per wave, 16-B chunks (dynamic LDS = waves x this)
    // hot keys (`every e1 -> e2` on one stream; p2_jit.hip k_hot_*): the staged pass leaves a key with at least
    // hot_min events in the batch, or more live partials than its register window, to the hot-key pipeline,
    // which advances all of its partials at once (a partial's fate is the first later event that expires or
    // matches it); 0 = off
    uint32_t hot_min;
    uint32_t hot_cap;                  // hot_list entries (further hot keys are walked by their lanes)
    uint32_t max_batch;                // (sizes the flat index space: <= max_batch events + hot_cap * cap carried in)
    uint32_t* hot_ctl;                 // [SGD_HOT_CTL] counters (hot_ctl[0]: hot keys listed; reset by the HBM pass)
    uint32_t* hot_list;                // [hot_cap] keys
    uint32_t* hot_info;                // [hot_cap][SGD_HOT_INFO] per hot key: run, offsets, checks, survivors
    uint32_t* hot_death;               // [flat] per partial: 2 * (ending event) + matched; or live / no partial
    uint32_t* hot_cur;                 // [flat] the next event its search scans
    uint32_t* hot_wl;                  // [2][flat][3] partials still open (flat index, key, cursor), by round
    uint32_t* hot_tcnt;                // [max_batch] matches per trigger (by flat event index)
    uint32_t* hot_tbase;               // [max_batch] their first raw slot
    uint32_t* hot_fbi;                 // [max_batch] the batch position of each flat event
    uint32_t* hot_alive;               // [flat] the survivors' flat indices, a region of min(cap, n0 + m) per key
    uint32_t* hot_fh;                  // [flat] the hot key of each flat index (round 0)
    uint32_t hot_round;                // the search round a k_hot_rn / k_hot_rc launch runs
    uint32_t hot_exmax;                // flat indices for carried-in partials (keys past it are given back)
    uint32_t hot_n0;                   // a key carrying in at least this many live partials is hot too
    uint64_t td_tag;                   // SGD_TD_TAG of this batch, or-ed into every t_desc entry written
    uint64_t cst[SGD_MAX_CONST];       // filter constants, already in their comparison domain
};

// payload packing (JIT kernel k_pack): batch arrival order or key-sorted order via sidx
struct PackParams {
    uint32_t n;
    uint32_t pad;
    const uint32_t* sidx;              // NULL: identity
    const int64_t* ts;
    const void* col[SGD_MAX_EVCOLS];   // the stream's filter columns (device)
    const uint8_t* nul[SGD_MAX_EVCOLS];
    uint32_t* payload;
};

// ahead-of-time launch wrappers (p2_kernels.hip)
struct ihipStream_t;
// ordered output of one batch: o_*[(out_count + t_off[t] + r) % capacity] for the r-th match of batch event t
struct ScatterParams {
    uint32_t n;
    uint64_t seq_base;
    const uint32_t* key;       // batch key ids (NULL: unpartitioned -> key 0)
    const int64_t* ts;
    const uint64_t* t_desc;    // per batch event: SGD_TD_CNT matches from the first raw slot (entries of this batch's tag)
    uint32_t epoch;            // this batch's t_desc tag
    uint32_t* tile_sum;        // [ceil(n / SGD_ORDER_TILE)] matches per tile of triggers
    const uint64_t* raw_e1;
    unsigned long long* out_count;     // matches ordered so far (monotonic; record r at r % capacity)
    unsigned long long* batch_total;
    uint64_t capacity;                 // ring of output records
    uint64_t win_start;                // matches handed out by polls so far (their records are free)
    uint64_t* o_trig;
    uint64_t* o_slot;          // [n][2]
    uint32_t* o_key;
    int64_t* o_ts;
    uint32_t* err;             // (o_len is constant 1/1 for two-state matches: filled at allocation)
    // on-device projection: the matched partials' captures follow their matches into output order
    const uint32_t* raw_capw;  // [n_capw][raw_capacity]
    const uint32_t* raw_capnull;
    uint64_t raw_capacity;
    uint32_t* o_capw;          // [n_capw][capacity] (NULL: no projection)
    uint32_t* o_capnull;
    uint32_t n_capw;
    uint64_t* out_first;       // aggregators: per batch event, count << 32 | ring position of its first
                               // record (0: no match); NULL otherwise
    uint32_t exp;              // ordering ablations (EXTRA=-DSG_EXPERIMENTS builds only: wrong results), 0 otherwise
};
#ifndef SGD_ORDER_TILE
#define SGD_ORDER_TILE 4096  // triggers per workgroup of the ordering kernels (256 threads x 16 rows)
#endif
// On-device projection of the select list (sg_set_projection) for the two-state kernel: after the ordering
// of a batch, item i of every match of the batch is evaluated (java_ops.h) over the match's e1 captures
// (VAR b = 0, w1 = capture index) and its trigger event's batch columns (VAR b = 1, w1 = attribute).
#define SGD_MAX_ATTR 16
#define SGD_MAX_PROJ 32
#define SGD_MAX_AGG 16
// Items (siddhi_gpu_ir.h): [0, n_agg) aggregator arguments, then n_sel select items, then the optional
// `having`.  Phase 0 evaluates the aggregator arguments into aggv; k_agg turns them into the aggregators'
// values per key in output order; phase 1 evaluates the select items and `having` into pval (VAR src 2 =
// select item x of the row, src 3 = aggregator x).
struct ProjParams {
    const uint32_t* code;       // rewritten item bytecode
    const uint32_t* item_pc;    // [n_items]
    const uint32_t* item_len;
    const uint32_t* capw_off;   // capture index -> first word
    const uint32_t* cap_type;
    uint32_t n_items;
    uint32_t pad;
    uint64_t seq_base;
    const void* col[SGD_MAX_ATTR];       // trigger stream's columns by attribute (NULL: not read)
    const uint8_t* col_null[SGD_MAX_ATTR];
    uint32_t col_type[SGD_MAX_ATTR];
    const uint64_t* o_trig;
    const uint32_t* o_capw;
    const uint32_t* o_capnull;
    uint64_t capacity;
    const unsigned long long* out_count;     // after the batch (k_bump ran)
    const unsigned long long* batch_total;
    uint64_t* pval;             // [n_items - n_agg][capacity]
    uint8_t* pnull;
    uint32_t* err;
    uint32_t phase;             // 0: aggregator arguments -> aggv; 1: select + having -> pval
    uint32_t n_agg;
    uint64_t* aggv;             // [n_agg][capacity]: argument, then (k_agg) the aggregator's value
    uint8_t* aggnull;
};
// per-key aggregator state in output order (QuerySelector + the aggregators' PartitionStateHolder): one
// thread per key walks its batch events in arrival order and their matches in emission order
struct AggParams {
    uint32_t K, n_agg;
    const uint32_t* seg_begin;
    const uint32_t* seg_end;
    const uint32_t* payload;    // element j's word 0 = its batch position
    uint32_t stride;            // payload words per element
    uint32_t pad;
    const uint64_t* out_first;
    uint64_t capacity;
    const uint32_t* agg_type;   // item type of each aggregator (arg type | fn << 8)
    uint64_t* aggv;
    uint8_t* aggnull;
    int64_t* st_n;              // [n_agg][K]
    uint64_t* st_v;
    uint8_t* st_has;
};
int sgd_launch_agg(const AggParams& a, ihipStream_t* stream);
// partition purge of the aggregator states of the listed (range-checked) keys
int sgd_launch_reset_agg(const uint32_t* keys, uint32_t n, uint32_t K, uint32_t n_agg, int64_t* st_n, uint64_t* st_v,
                         uint8_t* st_has, ihipStream_t* stream);
int sgd_launch_project(const ProjParams& p, ihipStream_t* stream);
// ordering of one batch's matches: per-tile totals, then per tile its prefix, the tile-local scan and the scatter;
// also bumps out_count
int sgd_launch_scatter(const ScatterParams& s, ihipStream_t* stream);
// partition purge: hdr[keys[i]] = 0 (key range errors -> err)
int sgd_launch_reset_keys(const uint32_t* keys, uint32_t n, uint32_t n_keys, uint32_t* hdr, uint32_t* err,
                          ihipStream_t* stream);
// *bad = 1 iff some keys[i] >= n_keys (device ids of sg_reset_keys, checked before any reset)
int sgd_launch_check_keys(const uint32_t* keys, uint32_t n, uint32_t n_keys, uint32_t* bad, ihipStream_t* stream);
int sgd_launch_min_seq(const uint32_t* hdr, const uint64_t* p_seq, uint32_t n_keys, unsigned long long* out,
                       ihipStream_t* stream);
// sums the staged pass's per-wave counters of one batch into stats[SGD_ST_N]
int sgd_launch_stats_reduce(const unsigned long long* wstats, uint32_t n_waves, unsigned long long* stats,
                            unsigned long long* raw_count, uint32_t* dlist_n, ihipStream_t* stream);
