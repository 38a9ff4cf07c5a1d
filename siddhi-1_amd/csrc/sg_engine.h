// sg_engine.h — internal definitions shared by the host side of the C-ABI (sg_engine.hip) and the
// gfx950 kernels (p2_kernels.hip).  Not part of the public ABI (that is include/siddhi_gpu.h).
#pragma once

#include <stdint.h>

#define SGD_MAX_PROG 48    // device filter program length (instructions)
#define SGD_MAX_STACK 8    // filter evaluation stack depth
#define SGD_MAX_EVCOLS 8   // event columns a query's filters read
#define SGD_MAX_CAPS 8     // slot-0 attributes captured into a partial match
#define SGD_WAVE 64

// device filter program: the IR bytecode (siddhi_gpu_ir.h) with every variable resolved to where the
// kernel finds it — a column of the current event, a captured attribute of the partial's slot-0 event,
// or null (chain index outside a single-event slot)
enum { SGD_SRC_EV = 0, SGD_SRC_CAP = 1, SGD_SRC_NULL = 2 };

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
    const uint32_t* sorted_idx;   // batch positions grouped by key, arrival order inside a key
    const uint32_t* seg_begin;    // [n_keys]
    const uint32_t* seg_end;      // [n_keys]
    // per-key state (SoA, partial j of key k at j * n_keys + k)
    uint32_t* hdr;
    int64_t* p_ts;
    uint64_t* p_seq;
    uint64_t* p_cap;              // [n_caps][cap][n_keys]
    uint32_t* p_capnull;          // [cap][n_keys] null bits of the captures
    uint32_t n_caps;
    uint32_t nullable;            // capture null bits are live
    uint8_t cap_col[SGD_MAX_CAPS];// event column captured into capture c
    // matches (appended)
    uint64_t* m_trig;
    uint64_t* m_e1;
    uint32_t* m_key;
    int64_t* m_ts;
    unsigned long long* m_count;
    uint64_t m_capacity;
    unsigned long long* stats;    // [SGD_ST_N]
    uint32_t* err;
    DProg f0;
    DProg f1;
};

// launch wrappers (p2_kernels.hip)
struct ihipStream_t;
int sgd_launch_bounds(const uint32_t* sorted_keys, uint32_t n, uint32_t n_keys, uint32_t* seg_begin,
                      uint32_t* seg_end, uint32_t* err, ihipStream_t* stream);
int sgd_launch_p2(const P2Params& p, ihipStream_t* stream);
int sgd_launch_order(const uint64_t* trig, const uint64_t* e1, const uint32_t* key, const int64_t* ts,
                     const uint32_t* perm, uint64_t n, uint64_t* o_trig, uint64_t* o_slot, uint32_t* o_key,
                     int64_t* o_ts, uint32_t* o_len, ihipStream_t* stream);
int sgd_launch_rel_keys(const uint64_t* trig, uint64_t base, uint64_t n, uint32_t* out, ihipStream_t* stream);
