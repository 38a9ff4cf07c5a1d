// sg_engine.h — internal definitions shared by the host side of the C-ABI (sg_engine.hip) and the
// gfx950 kernels (p2_kernels.hip).  Not part of the public ABI (that is include/siddhi_gpu.h).
#pragma once

#include <stdint.h>

#define SGD_MAX_PROG 48    // device filter program length (instructions)
#define SGD_MAX_STACK 8    // filter evaluation stack depth
#define SGD_MAX_EVCOLS 8   // event columns a query's filters read
#define SGD_MAX_CAPS 8     // slot-0 attributes captured into a partial match
#define SGD_MAX_ATOMS 4    // comparisons in a conjunctive predicate
#define SGD_WAVE 64
#define SGD_BLOCK 256      // lanes (= keys) per workgroup of the advance kernel
#define SGD_RAW_CHUNK 2048 // raw match slots a wave reserves at a time
#define SGD_STAGE_UNROLL 8 // 8-byte loads in flight per lane while staging a chunk

// ---- filters ------------------------------------------------------------------------------------
// Every filter is lowered twice from the IR bytecode (siddhi_gpu_ir.h):
//  * DPred: a conjunction of <= 4 typed comparisons whose operands are an event column, a captured
//    slot-0 attribute or a constant already converted to the comparison domain.  Nearly every
//    pattern filter has this form (`price > 20`, `price > e1.price and symbol == e1.symbol`); it is
//    evaluated with wave-uniform scalar branches only.
//  * DProg: the full stack program (every other filter), evaluated by a device interpreter.
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

struct DOperand {
    uint8_t kind;   // SGD_SRC_*
    uint8_t from;   // type of the value before conversion to the domain
    uint8_t idx;    // event column / capture index
    uint8_t pad;
    uint32_t pad2;
    uint64_t bits;  // constant (already in the domain)
};

struct DAtom {
    uint8_t op;     // SG_OP_EQ .. SG_OP_LE
    uint8_t dom;    // comparison domain (sg_type)
    uint8_t pad[6];
    DOperand l, r;
};

// DAtom packed into one word: op-EQ | dom<<4 | lkind<<8 | lfrom<<12 | lidx<<16 | rkind<<20 | rfrom<<24 |
// ridx<<28, plus the bits of the (at most one) constant operand
struct DPredPacked {
    uint32_t n;
    uint32_t prog;      // 1: not conjunctive, evaluate the stack program
    uint32_t code[SGD_MAX_ATOMS];
    uint64_t cbits[SGD_MAX_ATOMS];
};

struct DPred {
    uint32_t use_prog;  // 1: not conjunctive, evaluate the DProg
    uint32_t n_atoms;   // 0 = no filter (always true)
    DAtom atoms[SGD_MAX_ATOMS];
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

enum { SGD_ST_SCANNED = 0, SGD_ST_CREATED, SGD_ST_MATCHES, SGD_ST_KEYS, SGD_ST_LIVE0, SGD_ST_N };

enum { SGD_ERR_PARTIAL_CAP = 1, SGD_ERR_MATCH_CAP = 2, SGD_ERR_KEY_RANGE = 4 };

struct P2Params {
    // query shape
    uint32_t n_keys;
    uint32_t cap;          // partial capacity per key
    uint32_t mode;         // SGD_P2_*
    uint32_t multi;        // both states read the same stream (PatternMultiProcessStreamReceiver)
    uint32_t is_s0;        // this batch's stream feeds state 0
    uint32_t is_s1;        // ... state 1
    int64_t within;        // -1 = none
    // batch (device pointers)
    uint32_t n;
    uint32_t n_evcols;
    uint64_t seq_base;
    const int64_t* ts;
    const void* evcol[SGD_MAX_EVCOLS];
    const uint8_t* evnull[SGD_MAX_EVCOLS];
    uint8_t evtype[SGD_MAX_EVCOLS];
    uint8_t ev_word[SGD_MAX_EVCOLS];   // first LDS word of column c
    uint32_t n_evwords;                // 32-bit LDS words per staged event (64-bit columns take two)
    uint32_t chunk;                    // events staged in LDS per pass
    uint32_t any_null;                 // the batch carries null flags
    uint32_t lds_slots;                // partial-match window per lane in LDS
    uint32_t dbg;                      // profiling ablation switches (SGD_DBG), 0 in production
    unsigned long long* dbg_out;       // per-wave section stamps (dbg & 64)
    const uint32_t* sorted_idx;        // batch positions grouped by key, arrival order inside a key
    const uint32_t* payload;           // or: key-sorted events with payload [idx][cols..][ts] (NULL: gather)
    uint32_t pay_stride;               // words per payload element ([idx][cols..][ts]; even)
    uint32_t lds_stride;               // words per staged event in LDS (pay_stride (+2 with null bits))
    const uint32_t* seg_begin;         // [n_keys]
    const uint32_t* seg_end;           // [n_keys]
    // per-key state (SoA, partial j of key k at j * n_keys + k)
    uint32_t* hdr;
    int64_t* p_ts;
    uint64_t* p_seq;
    uint32_t* p_capw;                  // [n_capw][cap][n_keys] captured attribute words
    uint32_t* p_capnull;               // [cap][n_keys] null bits of the captures
    uint32_t n_caps;
    uint32_t n_capw;
    uint32_t nullable;                 // capture null bits are live
    uint8_t cap_col[SGD_MAX_CAPS];     // event column captured into capture c
    uint8_t cap_word[SGD_MAX_CAPS];    // first word of capture c
    uint8_t cap_type[SGD_MAX_CAPS];
    // matches: slot-0 event seq of every emitted match, appended in wave-reserved chunks; per batch
    // event t the number of matches it triggered and the position of the first (a trigger's matches
    // are contiguous, in emission order)
    uint64_t* raw_e1;
    unsigned long long* raw_count;
    uint64_t raw_capacity;
    uint32_t* t_cnt;                   // [max_batch], zero outside the advance -> scatter window
    uint32_t* t_first;                 // [max_batch]
    unsigned long long* stats;         // [SGD_ST_N]
    uint32_t* err;
    DPredPacked q0, q1;
    const DProg* f0g;                  // general filter programs (device memory)
    const DProg* f1g;
};

// launch wrappers (p2_kernels.hip)
struct ihipStream_t;
int sgd_launch_bounds(const uint32_t* sorted_keys, uint32_t n, uint32_t n_keys, uint32_t* seg_begin,
                      uint32_t* seg_end, uint32_t* err, ihipStream_t* stream);
int sgd_launch_p2(const P2Params& p, ihipStream_t* stream);
size_t sgd_p2_lds_bytes(const P2Params& p);
// ordered output of one batch: o_*[out_count + t_off[t] + r] for the r-th match of batch event t
struct ScatterParams {
    uint32_t n;
    uint64_t seq_base;
    const uint32_t* key;       // batch key ids (NULL: unpartitioned -> key 0)
    const int64_t* ts;
    uint32_t* t_cnt;
    const uint32_t* t_first;
    const uint32_t* t_off;     // exclusive scan of t_cnt
    const uint64_t* raw_e1;
    unsigned long long* out_count;
    unsigned long long* batch_total;
    uint64_t capacity;
    uint64_t* o_trig;
    uint64_t* o_slot;          // [n][2]
    uint32_t* o_key;
    int64_t* o_ts;
    uint32_t* o_len;           // [n][2]
    uint32_t* err;
};
int sgd_launch_scatter(const ScatterParams& s, ihipStream_t* stream);
