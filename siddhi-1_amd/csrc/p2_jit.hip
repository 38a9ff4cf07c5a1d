// p2_jit.hip — the NFA advance kernel for two-state partitioned patterns
//   every? e1=S0[f0] -> e2=S1[f1(e1,e2)] (within T)   and   every (e1=S0[f0] -> e2=S1[f1])
//
// This file is compiled by hipRTC when an engine is created (sg_jit.cpp), together with a generated
// header "sgq_query.h" that turns the query into code: the event layout of each stream, the filters
// f0 / f1 as typed straight-line HIP (Java value semantics below), the capture layout of a partial
// match and the register-window size SGQ_R.  Nothing in the hot loop interprets anything.
//
// Execution model: one lane owns one partition key (adjacent lanes = adjacent keys, so the SoA slabs
// "partial j of key k at j*K + k" are read and written coalesced).  The key-sorted micro-batch is a
// contiguous run of payload elements per key; a lane walks its own run in arrival order, the next
// element always in flight (software-pipelined loads), with the key's live partial matches held in
// registers: SGQ_R slots + a live mask + a staged mask (slot order = list order).  A key that
// outgrows the window spills to its HBM slab and continues there (exact, slower).
//
// Semantics restated from (paths under
// /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/query/input/):
//   stabilize: expire all states, then promote staged partials
//       stream/state/receiver/PatternMultiProcessStreamReceiver.java:42-51 (Single: :34-41)
//   expiry: StreamPreStateProcessor.java:118-129 (isExpired), :325-361 (prefix of pending, all of
//       staged, re-arm of the withinEvery start state)
//   promotion: StreamPreStateProcessor.java:308-323 (stable sort by ts, -1 last, :66-80)
//   state order per event: later state first (PatternMultiProcessStreamReceiver.java:31-40)
//   advance: StreamPreStateProcessor.java:364-403 + StreamPostStateProcessor.java:64-83
//   filters: FilterProcessor.java:48-60 and the typed executors under core/executor/
#include "siddhi_gpu_ir.h"
#include "sg_engine.h"

// ---- Java value semantics (executor/condition/compare/*, executor/math/*) -------------------------
template <class T> struct JV {
    T v;
    bool n;  // null
};
__device__ __forceinline__ bool jtrue(const JV<bool>& x) { return !x.n && x.v; }

// JLS 5.1.2 widening (int/long -> float/double round to nearest)
template <class TO, class FROM> __device__ __forceinline__ JV<TO> jcvt(const JV<FROM>& x) {
    return JV<TO>{(TO)x.v, x.n};
}

// CompareConditionExpressionExecutor.java:38-42: a null operand -> false; NotEqual: null -> true
template <int OP, class T> __device__ __forceinline__ JV<bool> jcmp(const JV<T>& a, const JV<T>& b) {
    bool r;
    if (OP == SG_OP_EQ) r = a.v == b.v;
    else if (OP == SG_OP_NE) r = a.v != b.v;
    else if (OP == SG_OP_GT) r = a.v > b.v;
    else if (OP == SG_OP_GE) r = a.v >= b.v;
    else if (OP == SG_OP_LT) r = a.v < b.v;
    else r = a.v <= b.v;
    return JV<bool>{(a.n || b.n) ? (OP == SG_OP_NE) : r, false};
}

// arithmetic: null in -> null; x/0, x%0 -> null; int/long wrap; MIN/-1 = MIN; MIN%-1 = 0
__device__ __forceinline__ JV<int32_t> jarith(int op, const JV<int32_t>& a, const JV<int32_t>& b) {
    const uint32_t x = (uint32_t)a.v, y = (uint32_t)b.v;
    const int32_t d = (b.v == 0 || b.v == -1) ? 1 : b.v;  // no undefined division on any lane
    JV<int32_t> o{0, a.n || b.n};
    switch (op) {
    case SG_OP_ADD: o.v = (int32_t)(x + y); break;
    case SG_OP_SUB: o.v = (int32_t)(x - y); break;
    case SG_OP_MUL: o.v = (int32_t)(x * y); break;
    case SG_OP_DIV: o.v = (b.v == -1) ? (int32_t)(0u - x) : a.v / d; o.n |= b.v == 0; break;
    default: o.v = (b.v == -1) ? 0 : a.v % d; o.n |= b.v == 0;
    }
    return o;
}
__device__ __forceinline__ JV<int64_t> jarith(int op, const JV<int64_t>& a, const JV<int64_t>& b) {
    const uint64_t x = (uint64_t)a.v, y = (uint64_t)b.v;
    const int64_t d = (b.v == 0 || b.v == -1) ? 1 : b.v;
    JV<int64_t> o{0, a.n || b.n};
    switch (op) {
    case SG_OP_ADD: o.v = (int64_t)(x + y); break;
    case SG_OP_SUB: o.v = (int64_t)(x - y); break;
    case SG_OP_MUL: o.v = (int64_t)(x * y); break;
    case SG_OP_DIV: o.v = (b.v == -1) ? (int64_t)(0ull - x) : a.v / d; o.n |= b.v == 0; break;
    default: o.v = (b.v == -1) ? 0 : a.v % d; o.n |= b.v == 0;
    }
    return o;
}
__device__ __forceinline__ JV<float> jarith(int op, const JV<float>& a, const JV<float>& b) {
    JV<float> o{0.f, a.n || b.n};
    switch (op) {
    case SG_OP_ADD: o.v = __fadd_rn(a.v, b.v); break;
    case SG_OP_SUB: o.v = __fsub_rn(a.v, b.v); break;
    case SG_OP_MUL: o.v = __fmul_rn(a.v, b.v); break;
    case SG_OP_DIV: o.v = __fdiv_rn(a.v, b.v); o.n |= b.v == 0.0f; break;
    default: o.v = fmodf(a.v, b.v); o.n |= b.v == 0.0f;
    }
    return o;
}
__device__ __forceinline__ JV<double> jarith(int op, const JV<double>& a, const JV<double>& b) {
    JV<double> o{0.0, a.n || b.n};
    switch (op) {
    case SG_OP_ADD: o.v = __dadd_rn(a.v, b.v); break;
    case SG_OP_SUB: o.v = __dsub_rn(a.v, b.v); break;
    case SG_OP_MUL: o.v = __dmul_rn(a.v, b.v); break;
    case SG_OP_DIV: o.v = __ddiv_rn(a.v, b.v); o.n |= b.v == 0.0; break;
    default: o.v = fmod(a.v, b.v); o.n |= b.v == 0.0;
    }
    return o;
}

__device__ __forceinline__ float sg_f32(uint32_t w) { return __uint_as_float(w); }
__device__ __forceinline__ double sg_f64(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)((uint64_t)lo | ((uint64_t)hi << 32)));
}
__device__ __forceinline__ int64_t sg_i64(uint32_t lo, uint32_t hi) {
    return (int64_t)((uint64_t)lo | ((uint64_t)hi << 32));
}

template <bool C, class A, class B> struct SgSel { typedef A type; };
template <bool B> struct SgBool { static constexpr bool value = B; };
template <class A, class B> struct SgSel<false, A, B> { typedef B type; };

// the query: SGQ_* constants, SgEv0/SgEv1 + sgq_ev0/1 (payload decode), sgq_f0, sgq_f1,
// sgq_capture, sgq_pack0/1
#include "sgq_query.h"

#define R SGQ_R
#ifndef SGQ_RH
#define SGQ_RH SGQ_R  // the HBM pass's register window (keys the staged pass stopped: often more partials)
#endif
// the hot-key pipeline (k_hot_*, end of file) exists for `every e1 -> e2` with both states on one stream
#if SGQ_MULTI && SGQ_MODE == 1  // (SGD_P2_EVERY_FIRST: an enum, invisible to #if)
#define SG_HOT 1
#else
#define SG_HOT 0
#endif

// ablation knobs for tools/exp_c2.py (JIT-time defines, experiment builds only); 0 in every shipped configuration
#ifndef SGX_NO_RAW
#define SGX_NO_RAW 0
#endif
#ifndef SGX_NO_TDESC
#define SGX_NO_TDESC 0
#endif
#ifndef SGX_NO_LOOP
#define SGX_NO_LOOP 0
#endif
#ifndef SGX_MAX_IT
#define SGX_MAX_IT 0x7fffffff
#endif
// SGX_GLB_WALK=1: the staged pass walks the payload in HBM (one element ahead) instead of LDS
// SGX_BRANCHLESS (1, shipped): the window scan evaluates the filter on every slot and masks with the pending
// set (no exec-mask branch per slot), and the matches are stored by a wave loop over the set bits of the
// hit mask (slot words picked by selects) instead of one predicated region per slot; 0: the per-slot branches
#ifndef SGX_BRANCHLESS
#define SGX_BRANCHLESS 1
#endif
#ifndef SGX_GLB_WALK
#define SGX_GLB_WALK 0
#endif
// SGX_PROF=1: s_memtime per walk phase, summed per wave into p.prof (tools/exp_c2.py prints it)
#ifndef SGX_PROF
#define SGX_PROF 0
#endif
#if SGX_PROF
#define SGX_T(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); prof_acc[i] += t_ - prof_t; prof_t = t_; } while (0)
#else
#define SGX_T(i) do { } while (0)
#endif

namespace {

// a wave-uniform value moved to an SGPR: branches on it are scalar (s_cbranch_scc), so the two
// sides of an if/else are disjoint paths for the compiler (no exec-masked sequencing of both)
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ int wave_max(int x) {
    for (int off = 32; off > 0; off >>= 1) x = max(x, __shfl_xor(x, off, SGD_WAVE));
    return x;
}
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, SGD_WAVE);
    return x;
}
// inclusive prefix sum over the wave (all 64 lanes must be active), in DPP lane moves (VALU only,
// no LDS round trip): shifts within each 16-lane row, then row_bcast:15 / row_bcast:31
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
    const int r = lane & 15;
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    if (r >= 1) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    if (r >= 2) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    if (r >= 4) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    if (r >= 8) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    if (lane & 16) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    if (lane >= 32) x += t;
    return x;
}

template <int S> struct PayEl { uint32_t w[S]; };
typedef uint32_t sg_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t sg_u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) void* sg_glb_ptr;
typedef __attribute__((address_space(3))) void* sg_lds_ptr;

// per-workgroup staging of the payload runs: SGD_BLOCK / 64 wave regions of p.stage_chunks 16-B
// chunks each (dynamic LDS, sized by the host from the batch density)
extern __shared__ sg_u32x4 sg_stage[];

template <int S> __device__ __forceinline__ PayEl<S> load_pay(const uint32_t* __restrict__ base, uint32_t i) {
    PayEl<S> x;
    if constexpr (S % 2 != 0) {  // 4-B aligned elements
#pragma unroll
        for (int q = 0; q < S; ++q) x.w[q] = __builtin_nontemporal_load(base + (size_t)i * S + q);
    } else if constexpr (S % 4 == 0) {
        const sg_u32x4* s = (const sg_u32x4*)(base + (size_t)i * S);
#pragma unroll
        for (int q = 0; q < S / 4; ++q) {
            const sg_u32x4 v = __builtin_nontemporal_load(s + q);
            x.w[4 * q] = v.x; x.w[4 * q + 1] = v.y; x.w[4 * q + 2] = v.z; x.w[4 * q + 3] = v.w;
        }
    } else {
        const sg_u32x2* s = (const sg_u32x2*)(base + (size_t)i * S);
#pragma unroll
        for (int q = 0; q < S / 2; ++q) {
            const sg_u32x2 v = __builtin_nontemporal_load(s + q);
            x.w[2 * q] = v.x; x.w[2 * q + 1] = v.y;
        }
    }
    return x;
}

// element i of a wave's payload run staged in LDS (base = element 0; 16-B aligned when the element
// size is a multiple of 16 B, 8-B aligned when it is a multiple of 8 B, 4-B aligned otherwise)
template <int S> __device__ __forceinline__ PayEl<S> lds_pay(const uint32_t* base, uint32_t i) {
    PayEl<S> x;
    if constexpr (S % 2 != 0) {  // 4-B aligned elements
#pragma unroll
        for (int q = 0; q < S; ++q) x.w[q] = base[(size_t)i * S + q];
    } else if constexpr (S % 4 == 0) {
        const sg_u32x4* s = (const sg_u32x4*)(base + (size_t)i * S);
#pragma unroll
        for (int q = 0; q < S / 4; ++q) {
            const sg_u32x4 v = s[q];
            x.w[4 * q] = v.x; x.w[4 * q + 1] = v.y; x.w[4 * q + 2] = v.z; x.w[4 * q + 3] = v.w;
        }
    } else {
        const sg_u32x2* s = (const sg_u32x2*)(base + (size_t)i * S);
#pragma unroll
        for (int q = 0; q < S / 2; ++q) {
            const sg_u32x2 v = s[q];
            x.w[2 * q] = v.x; x.w[2 * q + 1] = v.y;
        }
    }
    return x;
}

#define SG_OFF_LIM SGD_TS_LIM
// the payload's timestamp word (pack.h sgd_ts_off): ts - base, or SGD_TS_FAR when that does not fit
__device__ __forceinline__ int32_t ts_off32(int64_t t, int64_t base) {
    if (t == -1) return SGD_TS_FAR;
    const int64_t x = (int64_t)((uint64_t)t - (uint64_t)base);
    const bool wrapped = ((t ^ base) < 0) && ((x ^ t) < 0);
    return (wrapped || x < -SGD_TS_LIM || x > SGD_TS_LIM) ? SGD_TS_FAR : (int32_t)x;
}
__device__ __forceinline__ bool off_ok(int64_t d) { return d >= -SG_OFF_LIM && d <= SG_OFF_LIM; }
// t - base fits the staged pass's 32-bit offsets (no 64-bit wrap of the difference either)
__device__ __forceinline__ bool ts_off_ok(int64_t t, int64_t base) {
    int64_t d;
    return !__builtin_sub_overflow(t, base, &d) && off_ok(d);
}

__device__ __forceinline__ bool expired(int64_t pts, int64_t now, int64_t within) {
    const int64_t d = pts - now;  // StreamPreStateProcessor.isExpired: |slot0.ts - now| > within
    return (d < 0 ? -d : d) > within;
}
// eventTimeComparator (StreamPreStateProcessor.java:66-80): a sorts strictly before b; -1 sorts last
__device__ __forceinline__ bool ts_before(int64_t a, int64_t b) { return (a != -1) && (b == -1 || a < b); }

// one key's HBM slab (partial j at j * K)
struct Slab {
    int64_t* ts;
    uint64_t* seq;
    uint32_t* cap;
    uint32_t* nul;
    uint32_t K;
    size_t plane;  // cap * K
    __device__ __forceinline__ int64_t& TS(uint32_t j) const { return ts[(size_t)j * K]; }
    __device__ __forceinline__ uint64_t& SEQ(uint32_t j) const { return seq[(size_t)j * K]; }
    __device__ __forceinline__ uint32_t& CAP(uint32_t w, uint32_t j) const { return cap[w * plane + (size_t)j * K]; }
    __device__ __forceinline__ uint32_t& NUL(uint32_t j) const { return nul[(size_t)j * K]; }
    __device__ __forceinline__ void move(uint32_t dst, uint32_t src) const {
        TS(dst) = TS(src);
        SEQ(dst) = SEQ(src);
#pragma unroll
        for (int w = 0; w < SGQ_NCAPW; ++w) CAP(w, dst) = CAP(w, src);
        if (SGQ_CAPNULL) NUL(dst) = NUL(src);
    }
};

// the register window of one key: slot order = list order (pending slots before staged slots).
// OFF (the staged pass): timestamps and seqs are held as 32-bit offsets from a per-launch base (half
// the registers and VALU of 64-bit values); ts -1 (eventTimeComparator's "unset") never occurs there
// (such keys stop and go to the HBM pass), so the ts order is a plain compare.
template <bool OFF, int RR> struct Win {
    typedef typename SgSel<OFF, int32_t, int64_t>::type TS;
    typedef typename SgSel<OFF, int32_t, uint64_t>::type SQ;
    __device__ __forceinline__ static bool lt(TS a, TS b) { return OFF ? a < b : ts_before((int64_t)a, (int64_t)b); }
    TS ts[RR];
    SQ seq[RR];
    uint32_t cw[RR][SGQ_NCAPW > 0 ? SGQ_NCAPW : 1];
    uint32_t cn[RR];
    uint32_t live;  // slot holds a partial
    uint32_t stg;   // subset of live: staged (pre1's newAndEvery list), all above the pending slots
    uint32_t tail;  // appends go here (one past the highest live slot)
    TS slast;       // ts of the last staged append
    bool sbad;      // the staged slots may be out of ts order (promotion sorts them)

    __device__ __forceinline__ void copy_slot(int d, int s) {
        ts[d] = ts[s];
        seq[d] = seq[s];
#pragma unroll
        for (int w = 0; w < SGQ_NCAPW; ++w) cw[d][w] = cw[s][w];
        if (SGQ_CAPNULL) cn[d] = cn[s];
    }
    __device__ __forceinline__ void fix_tail() { tail = live ? 32u - __clz(live) : 0u; }

    // close the holes, keeping slot order: every live slot moves down by the number of free
    // slots below it, in log2(RR) collision-free steps of 1, 2, 4, ... (static register indices)
    __device__ __forceinline__ void compact() {
        if ((live & (live + 1u)) == 0u) { tail = __popc(live); return; }  // already a prefix
        uint32_t d[RR];
#pragma unroll
        for (int j = 0; j < RR; ++j) d[j] = __popc(~live & ((1u << j) - 1u));
        uint32_t cur = live;
#pragma unroll
        for (int s = 0; (1 << s) < RR; ++s) {
            const int sh = 1 << s;
#pragma unroll
            for (int j = sh; j < RR; ++j) {
                const bool mv = ((cur >> j) & 1u) && ((d[j] >> s) & 1u);
                if (mv) {
                    copy_slot(j - sh, j);
                    d[j - sh] = d[j];
                    cur = (cur & ~(1u << j)) | (1u << (j - sh));
                }
            }
        }
        const uint32_t n = __popc(live), ns = __popc(stg);
        live = (n >= 32u) ? 0xffffffffu : ((1u << n) - 1u);
        stg = live & ~((1u << (n - ns)) - 1u);
        tail = n;
    }

    // stable sort of the staged slots by ts (eventTimeComparator); the window is compacted
    __device__ __forceinline__ void sort_staged() {
        compact();
        const uint32_t n = tail, lo = n - __popc(stg);
#pragma unroll
        for (int pass = 0; pass < RR - 1; ++pass) {
#pragma unroll
            for (int j = 0; j + 1 < RR; ++j) {
                if ((uint32_t)j >= lo && (uint32_t)(j + 1) < n && lt(ts[j + 1], ts[j])) {
                    TS t = ts[j]; ts[j] = ts[j + 1]; ts[j + 1] = t;
                    SQ q = seq[j]; seq[j] = seq[j + 1]; seq[j + 1] = q;
#pragma unroll
                    for (int w = 0; w < SGQ_NCAPW; ++w) { uint32_t c = cw[j][w]; cw[j][w] = cw[j + 1][w]; cw[j + 1][w] = c; }
                    if (SGQ_CAPNULL) { uint32_t c = cn[j]; cn[j] = cn[j + 1]; cn[j + 1] = c; }
                }
            }
        }
    }
};

// per-lane NFA counters of one key during a batch
struct KeySt {
    uint32_t spend, sstg;              // start-state seeds: pending, staged
    uint32_t gnp, gns;                 // HBM mode: pending, staged list lengths
    unsigned long long scanned, created, matches;
};

// ---- HBM-mode list operations (a key with more than SGQ_R live partials) ------------------------
template <bool UPD0, bool UPD1>
__device__ __forceinline__ void glb_stabilize(const Slab& g, KeySt& s, int64_t ts, int64_t within) {
    if (SGQ_WITHIN && (s.gnp + s.gns) > 0) {
        uint32_t pre = 0;
        while (pre < s.gnp && expired(g.TS(pre), ts, within)) pre++;
        bool stg_exp = false;
        for (uint32_t r = s.gnp; r < s.gnp + s.gns; ++r) stg_exp |= expired(g.TS(r), ts, within);
        if (pre > 0 || stg_exp) {
            uint32_t w = 0, stg_drop = 0;
            const uint32_t end = s.gnp + s.gns;
            for (uint32_t r = pre; r < end; ++r) {
                if (r >= s.gnp && expired(g.TS(r), ts, within)) { stg_drop++; continue; }
                if (w != r) g.move(w, r);
                w++;
            }
            s.gnp -= pre;
            s.gns -= stg_drop;
            if (SGQ_MODE & SGD_P2_EVERY_BOTH) {  // withinEveryPreStateProcessor.addEveryState + updateState
                s.spend += s.sstg + 1;
                s.sstg = 0;
                s.created++;
            }
        }
    }
    if (UPD0) { s.spend += s.sstg; s.sstg = 0; }
    if (UPD1 && s.gns > 0) {
        // stable insertion sort of the staged region by ts
        for (uint32_t r = s.gnp + 1; r < s.gnp + s.gns; ++r) {
            const int64_t kt = g.TS(r);
            if (!ts_before(kt, g.TS(r - 1))) continue;
            const uint64_t ks = g.SEQ(r);
            const uint32_t kn = SGQ_CAPNULL ? g.NUL(r) : 0u;
            uint32_t kw[SGQ_NCAPW > 0 ? SGQ_NCAPW : 1];
#pragma unroll
            for (int w = 0; w < SGQ_NCAPW; ++w) kw[w] = g.CAP(w, r);
            uint32_t q = r;
            while (q > s.gnp && ts_before(kt, g.TS(q - 1))) { g.move(q, q - 1); q--; }
            g.TS(q) = kt;
            g.SEQ(q) = ks;
#pragma unroll
            for (int w = 0; w < SGQ_NCAPW; ++w) g.CAP(w, q) = kw[w];
            if (SGQ_CAPNULL) g.NUL(q) = kn;
        }
        s.gnp += s.gns;
        s.gns = 0;
    }
}

template <class Ev>
__device__ __forceinline__ bool glb_hit(const Slab& g, uint32_t j, const Ev& ev, const P2Params& p) {
    uint32_t cw[SGQ_NCAPW > 0 ? SGQ_NCAPW : 1];
#pragma unroll
    for (int w = 0; w < SGQ_NCAPW; ++w) cw[w] = g.CAP(w, j);
    return sgq_f1(ev, cw, SGQ_CAPNULL ? g.NUL(j) : 0u, p);
}

// e2's filter over the pending partials: count and the hit bits of the first 64
template <class Ev>
__device__ __forceinline__ uint32_t glb_scan(const Slab& g, const KeySt& s, const Ev& ev, const P2Params& p,
                                          uint64_t& mask) {
    uint32_t c = 0;
    mask = 0;
    for (uint32_t j = 0; j < s.gnp; ++j) {
        if (glb_hit(g, j, ev, p)) {
            if (j < 64) mask |= 1ull << j;
            c++;
        }
    }
    return c;
}

// emit the matches of one event (raw[pos ..]) and compact the survivors, pending-list order
template <class Ev>
__device__ __forceinline__ void glb_emit(const Slab& g, KeySt& s, const Ev& ev, const P2Params& p, uint64_t mask,
                                      unsigned long long pos) {
    uint32_t w1 = 0;
    for (uint32_t j = 0; j < s.gnp; ++j) {
        const bool hit = (j < 64) ? ((mask >> j) & 1ull) != 0 : glb_hit(g, j, ev, p);
        if (hit) {
            if (pos < p.raw_capacity) {
                p.raw_e1[pos] = g.SEQ(j);
#if SGQ_PROJ
#pragma unroll
                for (int w = 0; w < SGQ_NCAPW; ++w) p.raw_capw[(size_t)w * p.raw_capacity + pos] = g.CAP(w, j);
                if (SGQ_CAPNULL) p.raw_capnull[pos] = g.NUL(j);
#endif
            }
            pos++;
        } else {
            if (w1 != j) g.move(w1, j);
            w1++;
        }
    }
    s.gnp = w1;
}

// ---- the fused grouping: a workgroup's tile split by key (part.h sgd_group_tiles_fused) ------------------------
// The tile holds the events of the workgroup's SGD_BLOCK keys in arrival order, key & 255 in the position's top
// byte.  Each wave takes a contiguous share of it, in rounds of 64, and ranks every event among its own earlier
// events of the same key (wave ballots: "match any" over the 8 key bits, a u16 running count per (wave, key)
// updated by the group's first lane: no atomics); lane x then turns the waves' counts of key x into the key's run
// [kb, kb + kc) in the tile and each wave's place in it; the events move to their places (positions cleared of
// the tag).  The result is what a key sort of the batch gives for these keys: the runs in key order, arrival
// order within a run (PartitionStreamReceiver.java:175-260).
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t match_key8(uint32_t v, uint64_t act) {
    uint64_t m = act;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const bool x = (v >> b) & 1u;
        const uint64_t bb = __ballot(x);
        m &= x ? bb : ~bb;
    }
    return m;
}

// lane = key: from the waves' counts cnt[w][lane], the key's run (kb, kc) and each wave's place (into cnt)
template <class C>
__device__ __forceinline__ void split_places(C* cnt, uint32_t& kb, uint32_t& kc) {
    constexpr uint32_t NW = SGD_BLOCK / SGD_WAVE;
    __shared__ uint32_t ws[NW];
    const uint32_t tid = threadIdx.x, lane = tid & (SGD_WAVE - 1), w = tid / SGD_WAVE;
    uint32_t cw[NW], t = 0;
#pragma unroll
    for (uint32_t q = 0; q < NW; ++q) { cw[q] = cnt[q * SGD_BLOCK + tid]; t += cw[q]; }
    const uint32_t incl = wave_incl_scan(t, (int)lane);
    if (lane == SGD_WAVE - 1) ws[w] = incl;
    __syncthreads();
    uint32_t run = incl - t;
    for (uint32_t q = 0; q < w; ++q) run += ws[q];
    kb = run;
    kc = t;
#pragma unroll
    for (uint32_t q = 0; q < NW; ++q) { cnt[q * SGD_BLOCK + tid] = (C)run; run += cw[q]; }
    __syncthreads();
}

// the tile staged in LDS (`run`: element 0), nt <= SGD_SPLIT_CHUNKS(S) * SGD_BLOCK events: every element read into
// registers before the places are known, written to its place after; cnt: NW * SGD_BLOCK u16 of LDS (after the
// staging region: dynamic, so the launches without the split do not hold it)
template <int S>
__device__ __forceinline__ void tile_split_lds(uint32_t* run, uint32_t nt, uint16_t* cnt, uint32_t& kb, uint32_t& kc) {
    constexpr uint32_t NW = SGD_BLOCK / SGD_WAVE;
    constexpr uint32_t MC = SGD_SPLIT_CHUNKS(S);
    const uint32_t tid = threadIdx.x, lane = tid & (SGD_WAVE - 1), w = tid / SGD_WAVE;
    for (uint32_t x = tid; x < NW * SGD_BLOCK / 2; x += SGD_BLOCK) ((uint32_t*)cnt)[x] = 0u;
    __syncthreads();
    const uint32_t q = ((nt + NW - 1) / NW + SGD_WAVE - 1) & ~(uint32_t)(SGD_WAVE - 1);
    const uint32_t lo = min(nt, w * q), hi = min(nt, lo + q);
    uint16_t* mine = cnt + w * SGD_BLOCK;
    uint32_t rk[MC];
    uint32_t el[MC][S];
#pragma unroll
    for (uint32_t c = 0; c < MC; ++c) {
        rk[c] = 0;
        if (lo + c * SGD_WAVE < hi) {  // (wave-uniform)
            const uint32_t j = lo + c * SGD_WAVE + lane;
            const bool v = j < hi;
            uint32_t kl = 0;
            if (v) {
#pragma unroll
                for (int u = 0; u < S; ++u) el[c][u] = run[j * S + u];
                kl = el[c][0] >> 24;
            }
            const uint64_t m = match_key8(kl, __ballot(v));
            if (v) {
                const uint32_t before = lane_rank(m);
                const uint32_t base = mine[kl];
                if (before == 0) mine[kl] = (uint16_t)(base + (uint32_t)__popcll(m));
                rk[c] = kl | ((base + before) << 8) | 0x80000000u;
            }
        }
    }
    __syncthreads();
    split_places(cnt, kb, kc);
#pragma unroll
    for (uint32_t c = 0; c < MC; ++c) {
        if (rk[c] >> 31) {
            const uint32_t d = mine[rk[c] & 255u] + ((rk[c] >> 8) & 0x7fffu);
            el[c][0] &= 0xffffffu;
#pragma unroll
            for (int u = 0; u < S; ++u) run[d * S + u] = el[c][u];
        }
    }
    __syncthreads();
}

// a tile too large for the LDS split: split from `src` (HBM) into `dst` (the key-sorted payload at the tile's
// place), counted in one pass and placed in a second; cnt: NW * SGD_BLOCK words of LDS
template <int S>
__device__ __forceinline__ void tile_split_glb(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t nt,
                                               uint32_t* cnt, uint32_t& kb, uint32_t& kc) {
    constexpr uint32_t NW = SGD_BLOCK / SGD_WAVE;
    const uint32_t tid = threadIdx.x, lane = tid & (SGD_WAVE - 1), w = tid / SGD_WAVE;
    for (uint32_t x = tid; x < NW * SGD_BLOCK; x += SGD_BLOCK) cnt[x] = 0u;
    __syncthreads();
    const uint32_t q = ((nt + NW - 1) / NW + SGD_WAVE - 1) & ~(uint32_t)(SGD_WAVE - 1);
    const uint32_t lo = min(nt, w * q), hi = min(nt, lo + q);
    uint32_t* mine = cnt + w * SGD_BLOCK;
    for (uint32_t r0 = lo; r0 < hi; r0 += SGD_WAVE) {  // (wave-uniform trips)
        const uint32_t j = r0 + lane;
        const bool v = j < hi;
        const uint32_t kl = v ? src[(size_t)j * S] >> 24 : 0u;
        const uint64_t m = match_key8(kl, __ballot(v));
        if (v && lane_rank(m) == 0) mine[kl] += (uint32_t)__popcll(m);
    }
    __syncthreads();
    split_places(cnt, kb, kc);
    for (uint32_t r0 = lo; r0 < hi; r0 += SGD_WAVE) {
        const uint32_t j = r0 + lane;
        const bool v = j < hi;
        uint32_t el[S];
        uint32_t kl = 0;
        if (v) {
#pragma unroll
            for (int u = 0; u < S; ++u) el[u] = src[(size_t)j * S + u];
            kl = el[0] >> 24;
        }
        const uint64_t m = match_key8(kl, __ballot(v));
        if (v) {
            const uint32_t before = lane_rank(m);
            const uint32_t base = mine[kl];
            if (before == 0) mine[kl] = base + (uint32_t)__popcll(m);
            el[0] &= 0xffffffu;
#pragma unroll
            for (int u = 0; u < S; ++u) dst[(size_t)(base + before) * S + u] = el[u];
        }
    }
    __syncthreads();
}

// ---- the kernel ---------------------------------------------------------------------------------
// a hot key (SG_HOT): at least p.hot_min events in the batch, or more live partials than the register window
// holds (the staged pass would leave it to the HBM pass's slab walk); listed for the hot-key pipeline (while its
// list has room), its lane then walks nothing
__device__ __forceinline__ bool list_hot(const P2Params& p, uint32_t k, uint32_t nev, uint32_t h) {
#if SG_HOT
    const uint32_t n0 = SGD_H_INIT(h) ? SGD_H_NPEND(h) + SGD_H_NSTG(h) : 0u;
    const bool want = p.hot_min != 0u && k < p.n_keys && nev > 0u && (nev >= p.hot_min || n0 >= p.hot_n0);
    const uint64_t bal = __ballot(want);  // (one atomic per wave that has any)
    if (bal == 0ull) return false;
    uint32_t base = 0;
    if ((threadIdx.x & (SGD_WAVE - 1)) == 0) base = atomicAdd(p.hot_ctl, (uint32_t)__popcll(bal));
    base = (uint32_t)__shfl((int)base, 0, SGD_WAVE);
    const uint32_t slot = base + lane_rank(bal);
    if (want && slot < p.hot_cap) {
        p.hot_list[slot] = k;
        return true;
    }
#endif
    return false;
}

__device__ __forceinline__ uint32_t wave_min_u(uint32_t x) {
    for (int off = 32; off > 0; off >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, off, SGD_WAVE));
    return x;
}
__device__ __forceinline__ uint32_t wave_max_u(uint32_t x) {
    for (int off = 32; off > 0; off >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, off, SGD_WAVE));
    return x;
}

// STG: the staged pass.  Every wave whose payload range fits its LDS region walks it there with the
// keys' partials in the register window only; a key whose window could overflow at its next event
// stops before that event and is resumed from there by the HBM pass (p.resume), and a wave whose
// range does not fit is left whole to the HBM pass (p.deferred).  !STG: the HBM pass over those
// waves and keys (payload read from HBM, register window spilling to the slab when full).  Two
// kernels, so the staged walk carries no global load and no vmcnt wait behind the match stores.
// gid: the lane's global index (key): blockIdx.x * SGD_BLOCK + threadIdx.x in the staged pass; the HBM pass
// runs one wave per work-group over the list of deferred waves (gid = wave * 64 + lane)
template <bool S0, bool S1, bool STG, int RR, bool KL = false>
__device__ __forceinline__ void advance(const P2Params& p, const uint32_t gid) {
    typedef typename SgSel<S0, SgEv0, SgEv1>::type Ev;
    constexpr int STRIDE = S0 ? SGQ_STRIDE0 : SGQ_STRIDE1;
    constexpr uint32_t SB = STRIDE * 4;  // bytes per payload element
    constexpr uint32_t NW = SGD_BLOCK / SGD_WAVE;
    const int lane = threadIdx.x & (SGD_WAVE - 1);
    const uint32_t wv = threadIdx.x / SGD_WAVE;
    // KL (the HBM pass over the stopped keys): lane gid takes the gid-th listed key (none past the list's end)
    const uint32_t k = KL ? (gid < p.dlist_n[1] ? p.klist[gid] : 0xffffffffu) : gid;
    const uint32_t K = p.n_keys;
    // round trip 1: the key's segment of the sorted batch and its header (independent loads)
    const uint32_t wave_id = gid / SGD_WAVE;
    const bool fused = STG && p.tile_lo != nullptr;  // (uniform) the batch is grouped by tile, split here
    uint32_t b = 0, e = 0, h = 0, dfr = 0, rsm = SGD_NO_RESUME;
    if (k < K) {
        if (!fused) {
            b = p.seg_begin[k];
            e = p.seg_end[k];
        }
        h = p.hdr[k];
    }
    // The staged pass stages the workgroup's runs whole (its keys are consecutive, so their runs are one
    // byte range of the sorted payload): the wave ranges meet in LDS, one barrier.  (Dealing keys to lanes
    // by run length was measured: 22% fewer VALU instructions, no faster — the workgroup's LDS is held
    // until its longest lane ends, so occupancy, not lane idling, bounds the walk.)
    uint32_t blo = 0, bhi = 0, rlo = 0;  // the workgroup's payload range; the wave's first event
    uint32_t gb = 0, ge = 0;              // the longest hot run inside it (not staged: the pipeline's)
    bool hot = false;
    bool fits = true;
    bool tile_glb = false;  // fused: the tile was too large for LDS, split into the key-sorted payload in HBM
    if constexpr (STG) {
        if (fused) {
            // the workgroup's tile: staged in LDS and split by key there, or (too large: ~1 in 4096 at the C2
            // density) split into the key-sorted payload in HBM by this workgroup and walked from there (L2)
            blo = uni(p.tile_lo[blockIdx.x]);
            bhi = uni(p.tile_lo[blockIdx.x + 1]);
            const uint32_t nt = bhi - blo;
            const uint64_t f_lo = (uint64_t)blo * SB / 16u, f_hi = ((uint64_t)bhi * SB + 15u) / 16u;
            fits = nt <= SGD_SPLIT_CHUNKS(STRIDE) * SGD_BLOCK && f_hi - f_lo <= (uint64_t)p.stage_chunks * NW;
            if (nt > SGD_BIG_TILE && threadIdx.x == 0 && p.hot_ctl) atomicAdd(&p.hot_ctl[SGD_HOT_CTL_BIG], 1u);
            uint32_t kb = 0, kc = 0;
            if (nt > 0 && fits) {
                const uint32_t nch = (uint32_t)(f_hi - f_lo);
                const sg_u32x4* src = (const sg_u32x4*)p.tpay + f_lo;
                for (uint32_t c = wv * SGD_WAVE; c < nch; c += SGD_BLOCK)
                    if (c + (uint32_t)lane < nch)
                        __builtin_amdgcn_global_load_lds((sg_glb_ptr)(src + c + lane), (sg_lds_ptr)(sg_stage + c), 16, 0, 0);
                __builtin_amdgcn_s_waitcnt(0);
                __syncthreads();
                uint32_t* tile = (uint32_t*)sg_stage + ((uint64_t)blo * SB - f_lo * 16u) / 4u;
                tile_split_lds<STRIDE>(tile, nt, (uint16_t*)(sg_stage + (size_t)p.stage_chunks * NW), kb, kc);
                if (p.write_sorted) {  // every key's run to the key-sorted payload (the aggregators read it)
                    for (uint32_t x = threadIdx.x; x < nt * STRIDE; x += SGD_BLOCK)
                        ((uint32_t*)p.payload)[(size_t)blo * STRIDE + x] = tile[x];
                }
            } else if (nt > 0) {
                tile_split_glb<STRIDE>(p.tpay + (size_t)blo * STRIDE, (uint32_t*)p.payload + (size_t)blo * STRIDE, nt,
                                       (uint32_t*)sg_stage, kb, kc);
                tile_glb = true;
                fits = true;
            }
            b = blo + kb;
            e = b + kc;
            hot = list_hot(p, k, e - b, h);
            if ((tile_glb || p.write_sorted) && k < K) {
                p.seg_begin[k] = b;
                p.seg_end[k] = e;
            }
            rlo = uni(wave_min_u(e > b ? b : 0xffffffffu));
        } else {
            __shared__ uint32_t s_lo[NW], s_hi[NW], s_gl[NW], s_gb[NW];
            const uint32_t nv = e - b;
            hot = list_hot(p, k, nv, h);
            rlo = uni(wave_min_u(nv > 0 ? b : 0xffffffffu));
            const uint32_t hi = uni(wave_max_u(nv > 0 ? e : 0u));
            // the wave's longest hot run: left out of the LDS staging (the range of a workgroup holding a head key
            // of a skewed stream then still fits)
            const uint32_t gl = uni(wave_max_u(hot ? nv : 0u));
            const uint64_t gm = __ballot(hot && nv == gl);
            const uint32_t gw = gm ? (uint32_t)__shfl((int)b, __builtin_ctzll(gm), SGD_WAVE) : 0u;
            if (lane == 0) { s_lo[wv] = rlo; s_hi[wv] = hi; s_gl[wv] = gl; s_gb[wv] = gw; }
            __syncthreads();
            blo = 0xffffffffu;
            uint32_t glen = 0;
#pragma unroll
            for (uint32_t w = 0; w < NW; ++w) {
                blo = min(blo, s_lo[w]);
                bhi = max(bhi, s_hi[w]);
                if (s_gl[w] > glen) { glen = s_gl[w]; gb = s_gb[w]; }
            }
            blo = uni(blo);
            bhi = uni(bhi);
            gb = uni(gb);
            ge = gb + uni(glen);
        }
    }
    bool count_key = true;  // this pass owns the key's keys_touched / live_at_batch_start counts
    if constexpr (!STG) {
        dfr = KL ? 2u : uni(p.deferred[wave_id]);  // 1: the whole wave; 2: the keys with a resume point
        if (dfr == 0u) return;
        if (k < K) rsm = p.resume[k];
        if (rsm == SGD_HOT_DONE) {  // advanced by the hot-key pipeline
            p.resume[k] = SGD_NO_RESUME;
            count_key = false;
            e = b;
        } else if (dfr == 1u) {
            if (rsm == SGD_HOT_MARK) {  // a hot key the pipeline gave back (counted by the staged pass)
                p.resume[k] = SGD_NO_RESUME;
                count_key = false;
            }
        } else {
            count_key = false;
            if (rsm != SGD_NO_RESUME) {
                b += rsm;
                p.resume[k] = SGD_NO_RESUME;
            } else {
                e = b;
            }
        }
    }
    const int nev = (int)(e - b);
    if (nev <= 0) h = 0;
    int iters = (int)uni((uint32_t)wave_max(hot ? 0 : nev));
    // the HBM pass stages its wave's runs in LDS too when they fit (its keys are consecutive: one range of the
    // key-sorted payload), so its walk waits on LDS, not on a dependent HBM load per event
    bool from_lds = STG && !SGX_GLB_WALK && !tile_glb;
    if constexpr (!STG) {
        const uint32_t wl = uni(wave_min_u(nev > 0 ? b : 0xffffffffu));
        const uint32_t wh = uni(wave_max_u(nev > 0 ? e : 0u));
        if (wh > wl) {
            const uint64_t h_lo = (uint64_t)wl * SB / 16u, h_hi = ((uint64_t)wh * SB + 15u) / 16u;
            if (h_hi - h_lo <= (uint64_t)p.hbm_stage_chunks) {
                blo = wl;
                bhi = wh;
                from_lds = true;
                const uint32_t nch = (uint32_t)(h_hi - h_lo);
                const sg_u32x4* src = (const sg_u32x4*)p.payload + h_lo;
                for (uint32_t c = 0; c < nch; c += SGD_WAVE)
                    if (c + (uint32_t)lane < nch)
                        __builtin_amdgcn_global_load_lds((sg_glb_ptr)(src + c + lane), (sg_lds_ptr)(sg_stage + c), 16, 0, 0);
            }
        }
    }
    // The workgroup's keys are consecutive, so their runs of the key-sorted payload form ONE
    // contiguous byte range: the waves copy it into LDS with 16-B global_load_lds (all copies in
    // flight at once, no VGPRs) and the lanes then walk their own runs out of LDS (a lane-private walk
    // through HBM touches every line ~8x, once per iteration, and thrashes L2).
    const uint64_t c_lo = (uint64_t)blo * SB / 16u, c_hi = ((uint64_t)bhi * SB + 15u) / 16u;
    // the gap: the 16-B chunks wholly inside the longest hot run [gb, ge) (the staging skips them)
    const uint64_t c_g0 = ((uint64_t)gb * SB + 15u) / 16u, c_g1 = (uint64_t)ge * SB / 16u;
    const uint32_t gap_ch = (ge > gb && c_g1 > c_g0) ? (uint32_t)(c_g1 - c_g0) : 0u;
    if constexpr (STG) {
        if (!fused) fits = SGX_GLB_WALK || bhi <= blo || c_hi - c_lo - gap_ch <= (uint64_t)p.stage_chunks * NW;
        // (a giant workgroup range: the host keeps the sorted grouping while batches have them)
        if (!fused && bhi > blo && bhi - blo > SGD_BIG_TILE && threadIdx.x == 0 && p.hot_ctl)
            atomicAdd(&p.hot_ctl[SGD_HOT_CTL_BIG], 1u);
        // this wave's p.deferred entry: 1 = the HBM pass takes the whole workgroup (its range does not
        // fit); keys stopped early raise it to 2 after the walk (written after the barrier below)
        if (lane == 0) p.deferred[wave_id] = (!fits && bhi > blo) ? 1u : 0u;
        if (!fits && bhi > blo && lane == 0) p.dlist[atomicAdd(p.dlist_n, 1u)] = wave_id;  // the HBM pass's list
        if (!fits) iters = 0;
    }
    const uint32_t* lds_run = (const uint32_t*)sg_stage + ((uint64_t)blo * SB - c_lo * 16u) / 4u;  // element blo
    const uint32_t* lrun = lds_run - ((gap_ch != 0u && b >= ge) ? gap_ch * 4u : 0u);  // (this lane's side of the gap)

    // round trip 2: the partials of the register window, the raw-slot reservation and the LDS copy,
    // all in flight together (nothing below reads a result before the barrier)
    KeySt s{SGD_H_SPEND(h), SGD_H_SSTG(h), SGD_H_NPEND(h), SGD_H_NSTG(h), 0, 0, 0};
    if (nev > 0 && !SGD_H_INIT(h)) s.sstg = 1;  // PartitionRuntimeImpl.initPartition -> init(): one seed
    const uint32_t n0 = s.gnp + s.gns;
    const unsigned long long st_live0 = (nev > 0 && count_key) ? (unsigned long long)n0 : 0ull;
    const Slab G{p.p_ts + k, p.p_seq + k, p.p_capw + k, p.p_capnull + k, K, (size_t)p.cap * K};
    bool hbm = n0 > (uint32_t)RR;
    // events of the run this pass walks (the staged pass may stop a key early: resume point `rs`)
    int run = hot ? 0 : nev;
    uint32_t rs = (hot && fits) ? 0u : SGD_NO_RESUME;  // (a hot key resumes from 0 if the pipeline gives it back)
    if (STG && hbm && nev > 0) {  // more live partials than the window holds: all of it to the HBM pass
        rs = 0;
        run = 0;
        hbm = false;
    }
    bool overflow = false;
    unsigned long long spills = 0;
    const int64_t within = p.within;
    constexpr bool GLB = !STG;  // only the HBM pass has the slab (spill) mode

    // the payload's timestamps are 32-bit offsets from obase, the batch's first timestamp (pack.h); the
    // staged pass keeps the window's timestamps as offsets from the same base (tbase) and seqs from the
    // batch's seq_base; a key with a value out of range goes to the HBM pass (`far` below)
    const int64_t obase = p.ts_col[0];
    const int64_t tbase = STG ? obase : 0;
    const uint64_t sbase = STG ? p.seq_base : 0;
    Win<STG, RR> W;
    typedef typename Win<STG, RR>::TS WTS;
    typedef typename Win<STG, RR>::SQ WSQ;
    bool far = false;
    W.live = 0; W.stg = 0; W.tail = 0;
#pragma unroll
    for (int j = 0; j < RR; ++j) {
        const bool ld = run > 0 && !hbm && (uint32_t)j < n0;
        const int64_t t = ld ? G.TS(j) : 0;
        const uint64_t q = ld ? G.SEQ(j) : 0;
        if (STG && ld) far |= !ts_off_ok(t, tbase) || !off_ok((int64_t)(q - sbase)) || t == -1;
        W.ts[j] = (WTS)(t - tbase);
        W.seq[j] = (WSQ)(q - sbase);
#pragma unroll
        for (int w = 0; w < SGQ_NCAPW; ++w) W.cw[j][w] = ld ? G.CAP(w, j) : 0u;
        W.cn[j] = (SGQ_CAPNULL && ld) ? G.NUL(j) : 0u;
    }
    if (run > 0 && !hbm) {
        W.live = (1u << n0) - 1u;
        W.stg = W.live & ~((1u << s.gnp) - 1u);
        W.tail = n0;
    }
    // staged partials carried over from the previous batch may be out of ts order (sorted at promotion)
    W.sbad = s.gns > 1;
    W.slast = 0;

    // Raw match slots.  Without `every` around the whole pattern a key holds at most one start seed,
    // so each event creates at most one partial and each partial is matched at most once: a lane
    // emits at most n0 + nev matches in this batch.  In the staged pass n0 <= R (larger keys go to the
    // HBM pass), so the wave's matches fit [rlo + w*64R, rhi + (w+1)*64R) of raw_e1 — disjoint from
    // every other wave's range, found without any atomic (one device-wide counter hit by every wave
    // serialises at the memory side and cost 0.8 ms per 2^24-event batch).  The HBM pass (few waves)
    // and `every (e1 -> e2)` (seeds multiply: chunks reserved as the wave goes, the next one
    // prefetched, lane 0 keeping its base until the switch) take slots above p.raw_static by atomics.
    constexpr bool BOUNDED = !(SGQ_MODE & SGD_P2_EVERY_BOTH);
    unsigned long long chunk_base = 0, next_l0 = 0;
    uint32_t chunk_left = 0;
    bool have_next = false;
    if constexpr (S1) {
        if constexpr (BOUNDED && STG) {
            // the wave's events + 64 R window partials bound its matches: [rlo + w*64R, ...) is disjoint
            // from every other wave's range
            chunk_base = (unsigned long long)rlo + (unsigned long long)wave_id * (unsigned long long)(SGD_WAVE * RR);
        } else if constexpr (BOUNDED) {
            const uint32_t bound = nev > 0 ? n0 + (S0 ? (uint32_t)nev : 0u) : 0u;
            const uint32_t wb = (uint32_t)wave_sum((unsigned long long)bound);
            if (lane == 0 && wb) next_l0 = p.raw_static + atomicAdd(p.raw_count, (unsigned long long)wb);
            chunk_left = wb;
        } else {
            have_next = iters > 0;
            if (have_next && lane == 0)
                next_l0 = p.raw_static + atomicAdd(p.raw_count, (unsigned long long)SGD_RAW_CHUNK);
        }
    }
    if (!SGX_GLB_WALK && STG && !fused && fits && bhi > blo) {  // (fused: staged and split above)
        const uint32_t nch = (uint32_t)(c_hi - c_lo) - gap_ch;
        const uint32_t ga = gap_ch ? (uint32_t)(c_g0 - c_lo) : nch;  // chunks before the gap
        const sg_u32x4* src = (const sg_u32x4*)p.payload + c_lo;
        for (uint32_t c = wv * SGD_WAVE; c < nch; c += SGD_BLOCK) {
            const uint32_t cc = c + (uint32_t)lane;
            if (cc < nch)
                __builtin_amdgcn_global_load_lds((sg_glb_ptr)(src + cc + (cc >= ga ? gap_ch : 0u)), (sg_lds_ptr)(sg_stage + c),
                                                 16, 0, 0);
        }
    }
    if constexpr (STG) {
        // every wave's LDS copies have landed (a wave reads runs other waves copied: each waits for its
        // own global_load_lds before the barrier)
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }
    // (a wave with hot keys in a staged workgroup goes on: their runs and resume points are written below)
    if (iters == 0 && !(STG && fits && __ballot(hot) != 0ull)) {
        // no key of this wave has an event here (wave-uniform), or the HBM pass has it; hot keys of a wave left
        // to the HBM pass are counted here (the pipeline or, given back, the HBM pass advances them)
        const unsigned long long hk = wave_sum(hot ? 1ull : 0ull), hl = wave_sum(hot ? (unsigned long long)n0 : 0ull);
        if (STG && hot) p.resume[k] = SGD_HOT_MARK;
        if (STG && lane == 0) {
#pragma unroll
            for (int i = 0; i < SGD_ST_N; ++i) p.wstats[(size_t)wave_id * SGD_ST_N + i] = 0;
            p.wstats[(size_t)wave_id * SGD_ST_N + SGD_ST_KEYS] = hk;
            p.wstats[(size_t)wave_id * SGD_ST_N + SGD_ST_LIVE0] = hl;
        }
        return;
    }
    // every prologue load has landed: an explicit full wait here clears the compiler's scoreboard, so
    // the walk below carries no vmcnt waits for the window registers (which would also drain the
    // match stores of every earlier iteration)
    __builtin_amdgcn_s_waitcnt(0);
    if (S1 && BOUNDED && !STG) chunk_base = __shfl(next_l0, 0, SGD_WAVE);
    if constexpr (STG) {
        // the staged walk holds 32-bit offsets (|offset| <= 2^30) and tests expiry as
        // `off < now - within || off > now + within`, exact in 32-bit arithmetic while 0 <= `within` < 2^30
        // (StreamPreStateProcessor.isExpired's long arithmetic never wraps in that range, and off ± within
        // stays inside int32); a key outside it goes to the HBM pass whole
        if (SGQ_WITHIN && (within >= SG_OFF_LIM || within < 0)) far = true;
        if (run > 0 && far) {
            rs = 0;
            run = 0;
            W.live = 0;
            W.stg = 0;
            W.tail = 0;
        }
    }

    PayEl<STRIDE> cur, nxt;
    if (run > 0) cur = from_lds ? lds_pay<STRIDE>(lrun, b - blo) : load_pay<STRIDE>(p.payload, b);

#if SGX_PROF
    uint64_t prof_acc[5] = {0, 0, 0, 0, 0};
    uint64_t prof_t = __builtin_amdgcn_s_memtime();
#endif
    for (int it = 0; it < (SGX_NO_LOOP ? 0 : min(iters, SGX_MAX_IT)); ++it) {
        bool act = it < run;
        if constexpr (STG) {
            // the partials this event can add: every start seed fires at most once (+1: the
            // withinEvery re-arm of `every (e1 -> e2)`); stop here if the window could overflow, or
            // if the event's timestamp is outside the range of the band expiry test
            if (act && (__popc(W.live) + s.spend + s.sstg + ((SGQ_MODE & SGD_P2_EVERY_BOTH) ? 1u : 0u) > (uint32_t)RR ||
                        (int32_t)cur.w[STRIDE - 1] == SGD_TS_FAR || cur.w[0] > 0x7fffffffu)) {
                rs = (uint32_t)it;
                run = it;
                act = false;
                spills++;
            }
        }
        if (it + 1 < run)  // next event in flight
            nxt = from_lds ? lds_pay<STRIDE>(lrun, b - blo + (uint32_t)it + 1)
                           : load_pay<STRIDE>(p.payload, b + (uint32_t)it + 1);
        Ev ev;
        int64_t ts = 0;
        uint32_t bi = 0;
        if (act) {
            bi = cur.w[0];
            const int32_t toff = (int32_t)cur.w[STRIDE - 1];
            ts = (STG || toff != SGD_TS_FAR) ? obase + (int64_t)toff : p.ts_col[bi];
            if constexpr (S0) ev = sgq_ev0(cur.w); else ev = sgq_ev1(cur.w);
            SGX_T(0);
            // ---- stabilize (receiver.stabilizeStates) ----
            if (!GLB || !hbm) {
                if (SGQ_WITHIN && W.live) {
                    uint32_t X = 0;
                    if constexpr (STG) {  // band form on the offsets (see the prologue): two compares per slot
                        const int32_t tn = toff, w32 = (int32_t)within;
                        const int32_t lo = tn - w32, hi = tn + w32;
#pragma unroll
                        for (int j = 0; j < RR; ++j) X |= (((W.ts[j] < lo) | (W.ts[j] > hi)) ? 1u : 0u) << j;
                    } else {
#pragma unroll
                        for (int j = 0; j < RR; ++j) X |= (expired((int64_t)W.ts[j], ts, within) ? 1u : 0u) << j;
                    }
                    X &= W.live;
                    if (X) {
                        const uint32_t P = W.live & ~W.stg;
                        const uint32_t f = P & ~X;  // first live pending partial that survives
                        const uint32_t pre = f ? (P & X & ((f & (0u - f)) - 1u)) : (P & X);
                        const uint32_t sx = W.stg & X;
                        if (pre | sx) {
                            W.live &= ~(pre | sx);
                            W.stg &= ~sx;
                            W.fix_tail();
                            if (SGQ_MODE & SGD_P2_EVERY_BOTH) {
                                s.spend += s.sstg + 1;
                                s.sstg = 0;
                                s.created++;
                            }
                        }
                    }
                }
                if (S0) { s.spend += s.sstg; s.sstg = 0; }
                if (S1 && W.stg) {
                    // promotion: staged partials join the pending list sorted by ts (stable); the
                    // appends tracked whether they arrived out of ts order
                    if (W.sbad) W.sort_staged();
                    W.stg = 0;
                    W.sbad = false;
                }
            } else {
                glb_stabilize<S0, S1>(G, s, ts, within);
            }
        }
        SGX_T(1);
        // ---- state 1 first (reverse state order, PatternMultiProcessStreamReceiver.java:31-40) ----
        uint32_t c1 = 0, H = 0;
        uint64_t gmask = 0;
        if constexpr (S1) {
            if (act) {
                if (!GLB || !hbm) {
                    const uint32_t P = W.live & ~W.stg;
                    if (SGX_BRANCHLESS) {
#pragma unroll
                        for (int j = 0; j < RR; ++j) H |= (sgq_f1(ev, W.cw[j], W.cn[j], p) ? 1u : 0u) << j;
                        H &= P;
                    } else {
#pragma unroll
                        for (int j = 0; j < RR; ++j) {
                            if (((P >> j) & 1u) && sgq_f1(ev, W.cw[j], W.cn[j], p)) H |= 1u << j;
                        }
                    }
                    c1 = __popc(H);
                    s.scanned += __popc(P);
                } else {
                    c1 = glb_scan(G, s, ev, p, gmask);
                    s.scanned += s.gnp;
                }
            }
        }
        SGX_T(2);
        // wave-wide reservation of the emitted matches (one atomic per wave chunk of slots)
        if constexpr (S1) {
        const uint32_t incl = wave_incl_scan(c1, lane);
        const uint32_t total = __builtin_amdgcn_readlane(incl, SGD_WAVE - 1);
        if (total) {
            if (!BOUNDED && total > chunk_left) {
                if (have_next && total <= (uint32_t)SGD_RAW_CHUNK) {  // switch to the prefetched chunk
                    chunk_base = __shfl(next_l0, 0, SGD_WAVE);
                    chunk_left = SGD_RAW_CHUNK;
                    have_next = false;
                } else {
                    const uint32_t want = max(total, (uint32_t)SGD_RAW_CHUNK);
                    unsigned long long nb = 0;
                    if (lane == 0) nb = p.raw_static + atomicAdd(p.raw_count, (unsigned long long)want);
                    chunk_base = __shfl(nb, 0, SGD_WAVE);
                    chunk_left = want;
                }
            }
            if (c1) {
                unsigned long long pos = chunk_base + incl - c1;
                // the staged pass's single match without captures to carry: its e1 seq (a 32-bit offset from the
                // batch's seq base) rides in the trigger's descriptor, so the ordering reads no raw slot for it
                const bool inl = STG && SGX_BRANCHLESS && !SGQ_PROJ && c1 == 1u;
                if (pos + c1 <= p.raw_capacity) {
                    if (!SGX_NO_TDESC && !inl) p.t_desc[bi] = p.td_tag | ((uint64_t)c1 << 32) | (uint64_t)(uint32_t)pos;  // count | first slot
                } else {
                    atomicOr(p.err, (uint32_t)SGD_ERR_MATCH_CAP);
                }
                if ((!GLB || !hbm) && SGX_BRANCHLESS) {
                    // the hit slots in slot order: one trip per set bit of the wave's widest mask
                    for (uint32_t m = H; __builtin_amdgcn_read_exec() & __ballot(m != 0u);) {
                        if (m) {
                            const int jj = __ffs(m) - 1;
                            m &= m - 1u;
                            WSQ sq = 0;
#if SGQ_PROJ
                            uint32_t cw[SGQ_NCAPW > 0 ? SGQ_NCAPW : 1], cn = 0;
#pragma unroll
                            for (int w = 0; w < SGQ_NCAPW; ++w) cw[w] = 0;
#endif
#pragma unroll
                            for (int j = 0; j < RR; ++j) {
                                const bool here = j == jj;
                                sq = here ? W.seq[j] : sq;
#if SGQ_PROJ
#pragma unroll
                                for (int w = 0; w < SGQ_NCAPW; ++w) cw[w] = here ? W.cw[j][w] : cw[w];
                                if (SGQ_CAPNULL) cn = here ? W.cn[j] : cn;
#endif
                            }
                            if (inl) {
                                if (!SGX_NO_TDESC && pos < p.raw_capacity)
                                    p.t_desc[bi] = SGD_TD_INLINE | p.td_tag | (1ull << 32) | (uint64_t)(uint32_t)(int32_t)sq;
                            } else if (!SGX_NO_RAW && pos < p.raw_capacity) {
                                p.raw_e1[pos] = sbase + (uint64_t)(int64_t)sq;
#if SGQ_PROJ
#pragma unroll
                                for (int w = 0; w < SGQ_NCAPW; ++w) p.raw_capw[(size_t)w * p.raw_capacity + pos] = cw[w];
                                if (SGQ_CAPNULL) p.raw_capnull[pos] = cn;
#endif
                            }
                            pos++;
                        }
                    }
                    W.live &= ~H;
                    W.fix_tail();
                } else if (!GLB || !hbm) {
#pragma unroll
                    for (int j = 0; j < RR; ++j) {
                        if ((H >> j) & 1u) {
                            if (!SGX_NO_RAW && pos < p.raw_capacity) {
                                p.raw_e1[pos] = sbase + (uint64_t)(int64_t)W.seq[j];
#if SGQ_PROJ
#pragma unroll
                                for (int w = 0; w < SGQ_NCAPW; ++w)
                                    p.raw_capw[(size_t)w * p.raw_capacity + pos] = W.cw[j][w];
                                if (SGQ_CAPNULL) p.raw_capnull[pos] = W.cn[j];
#endif
                            }
                            pos++;
                        }
                    }
                    W.live &= ~H;
                    W.fix_tail();
                } else {
                    glb_emit(G, s, ev, p, gmask, pos);
                }
                if (SGQ_MODE & SGD_P2_EVERY_BOTH) s.sstg += c1;  // post1 -> pre0.addEveryState
                s.matches += c1;
            }
            chunk_base += total;
            chunk_left -= total;
            if (!BOUNDED && !have_next && chunk_left < (uint32_t)SGD_RAW_CHUNK / 2) {  // prefetch the next chunk
                if (lane == 0) next_l0 = p.raw_static + atomicAdd(p.raw_count, (unsigned long long)SGD_RAW_CHUNK);
                have_next = true;
            }
        }
        }
        SGX_T(3);
        // ---- state 0: the start-state seeds ----
        if constexpr (S0) {
            if (act && s.spend > 0) {
                s.scanned += s.spend;
                if (sgq_f0(ev, p)) {
                    // post0: partial (slot0 = this event, ts = its ts) -> pre1.addState (staged);
                    // every e1: pre0.addEveryState (a new seed, staged)
                    uint32_t cw[SGQ_NCAPW > 0 ? SGQ_NCAPW : 1];
                    uint32_t cn = 0;
                    sgq_capture(ev, cw, cn);
                    const uint64_t seq = p.seq_base + bi;
                    for (uint32_t q = 0; q < s.spend; ++q) {
                        if ((!GLB || !hbm) && W.tail >= (uint32_t)RR) W.compact();
                        if (!GLB && W.tail >= (uint32_t)RR) { overflow = true; break; }  // excluded by the stop rule
                        if (GLB && !hbm && W.tail >= (uint32_t)RR) {
                            // the window is full of live partials: move the list to the HBM slab
#pragma unroll
                            for (int j = 0; j < RR; ++j) {
                                G.TS(j) = tbase + (int64_t)W.ts[j];
                                G.SEQ(j) = sbase + (uint64_t)(int64_t)W.seq[j];
#pragma unroll
                                for (int w = 0; w < SGQ_NCAPW; ++w) G.CAP(w, j) = W.cw[j][w];
                                if (SGQ_CAPNULL) G.NUL(j) = W.cn[j];
                            }
                            s.gns = __popc(W.stg);
                            s.gnp = RR - s.gns;
                            hbm = true;
                            spills++;
                        }
                        if (!GLB || !hbm) {
                            const uint32_t t = W.tail;
#pragma unroll
                            for (int j = 0; j < RR; ++j) {
                                if ((uint32_t)j == t) {
                                    W.ts[j] = (WTS)(ts - tbase);
                                    W.seq[j] = (WSQ)(seq - sbase);
#pragma unroll
                                    for (int w = 0; w < SGQ_NCAPW; ++w) W.cw[j][w] = cw[w];
                                    if (SGQ_CAPNULL) W.cn[j] = cn;
                                }
                            }
                            const WTS to = (WTS)(ts - tbase);
                            if (W.stg && Win<STG, RR>::lt(to, W.slast)) W.sbad = true;
                            W.slast = to;
                            W.live |= 1u << t;
                            W.stg |= 1u << t;
                            W.tail = t + 1;
                        } else {
                            const uint32_t j = s.gnp + s.gns;
                            if (j >= p.cap) { overflow = true; break; }
                            G.TS(j) = ts;
                            G.SEQ(j) = seq;
#pragma unroll
                            for (int w = 0; w < SGQ_NCAPW; ++w) G.CAP(w, j) = cw[w];
                            if (SGQ_CAPNULL) G.NUL(j) = cn;
                            s.gns++;
                        }
                        s.created++;
                    }
                    if (SGQ_MODE & SGD_P2_EVERY_FIRST) s.sstg += s.spend;
                    s.spend = 0;
                }
            }
        }
        cur = nxt;
        SGX_T(4);
    }
#if SGX_PROF
    if (lane == 0 && p.prof)  // one row per wave (no device-wide atomics), summed by the host
        for (int i = 0; i < 5; ++i) p.prof[(size_t)wave_id * 8 + i] += prof_acc[i];
#endif
    if (STG && fused && !tile_glb && !p.write_sorted) {
        // fused: the runs of the keys the HBM pass resumes (or the hot-key pipeline takes) were only in LDS; the
        // wave copies them to the key-sorted payload one key at a time, coalesced
        for (uint64_t need = __ballot(rs != SGD_NO_RESUME); need; need &= need - 1ull) {
            const int l = __builtin_ctzll(need);
            const uint32_t lb = (uint32_t)__shfl((int)b, l, SGD_WAVE), ln = (uint32_t)__shfl(nev, l, SGD_WAVE);
            uint32_t* dst = (uint32_t*)p.payload + (size_t)lb * STRIDE;
            const uint32_t* src = lds_run + (size_t)(lb - blo) * STRIDE;
            for (uint32_t x = (uint32_t)lane; x < ln * STRIDE; x += SGD_WAVE) dst[x] = src[x];
        }
    }
    if (STG && rs != SGD_NO_RESUME) {  // the HBM pass resumes the key
        if (fused && !tile_glb && !p.write_sorted) {
            p.seg_begin[k] = b;
            p.seg_end[k] = e;
        }
        p.resume[k] = rs;
        p.deferred[wave_id] = 2u;
    }
    if constexpr (STG) {  // the resumed keys join the HBM pass's key list (one reservation per wave)
        const uint64_t rb = __ballot(rs != SGD_NO_RESUME);
        if (rb && !p.klist) {
            if (lane == 0) p.dlist[atomicAdd(p.dlist_n, 1u)] = wave_id;
        } else if (rb) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&p.dlist_n[1], (uint32_t)__popcll(rb));
            base = (uint32_t)__shfl((int)base, 0, SGD_WAVE);
            if (rs != SGD_NO_RESUME) p.klist[base + lane_rank(rb)] = k;
        }
    }
    if (run > 0) {
        uint32_t np, ns;
        if (!GLB || !hbm) {
            W.compact();
            const uint32_t n = W.tail;
#pragma unroll
            for (int j = 0; j < RR; ++j) {
                if ((uint32_t)j < n) {
                    G.TS(j) = tbase + (int64_t)W.ts[j];
                    G.SEQ(j) = sbase + (uint64_t)(int64_t)W.seq[j];
#pragma unroll
                    for (int w = 0; w < SGQ_NCAPW; ++w) G.CAP(w, j) = W.cw[j][w];
                    if (SGQ_CAPNULL) G.NUL(j) = W.cn[j];
                }
            }
            ns = __popc(W.stg);
            np = n - ns;
        } else {
            np = s.gnp;
            ns = s.gns;
        }
        if (s.sstg > 3 || s.spend > 3) overflow = true;
        p.hdr[k] = SGD_H_MAKE(np, ns, min(s.spend, 3u), min(s.sstg, 3u), 1);
    }
    if (overflow) atomicOr(p.err, (uint32_t)SGD_ERR_PARTIAL_CAP);
    // exact work counters, wave-reduced: the staged pass writes its wave's row of p.wstats (summed by
    // k_stats_reduce: no device-wide atomics from every wave), the HBM pass adds to p.stats directly
    const unsigned long long v0 = wave_sum(s.scanned), v1 = wave_sum(s.created), v2 = wave_sum(s.matches);
    const unsigned long long v3 = wave_sum((nev > 0 && count_key) ? 1ull : 0ull), v4 = wave_sum(st_live0),
                             v5 = wave_sum(spills);
    if (STG && lane == 0) {
        unsigned long long* w = p.wstats + (size_t)wave_id * SGD_ST_N;
        w[SGD_ST_SCANNED] = v0;
        w[SGD_ST_CREATED] = v1;
        w[SGD_ST_MATCHES] = v2;
        w[SGD_ST_KEYS] = v3;
        w[SGD_ST_LIVE0] = v4;
        w[SGD_ST_SPILLS] = v5;
        w[SGD_ST_HOTK] = 0;  // (the hot-key pipeline counts its keys into p.stats)
        w[SGD_ST_HOTE] = 0;
    }
    if (!STG && lane == 0) {
        if (v0) atomicAdd(&p.stats[SGD_ST_SCANNED], v0);
        if (v1) atomicAdd(&p.stats[SGD_ST_CREATED], v1);
        if (v2) atomicAdd(&p.stats[SGD_ST_MATCHES], v2);
        if (v3) atomicAdd(&p.stats[SGD_ST_KEYS], v3);
        if (v4) atomicAdd(&p.stats[SGD_ST_LIVE0], v4);
        if (v5) atomicAdd(&p.stats[SGD_ST_SPILLS], v5);
    }
}

template <int STRIDE, int WHICH>
__device__ __forceinline__ void pack(const PackParams& q) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= q.n) return;
    const uint32_t j = q.sidx ? q.sidx[i] : i;
    PayEl<STRIDE> x;
#pragma unroll
    for (int w = 0; w < STRIDE; ++w) x.w[w] = 0;
    x.w[0] = j;
    if constexpr (WHICH == 0) sgq_pack0(q, j, x.w); else sgq_pack1(q, j, x.w);
    x.w[STRIDE - 1] = (uint32_t)ts_off32(q.ts[j], q.ts[0]);
    uint32_t* d = q.payload + (size_t)i * STRIDE;
#pragma unroll
    for (int w = 0; w < STRIDE; ++w) d[w] = x.w[w];
}

}  // namespace

// occupancy target of the advance kernel (waves per SIMD); the register allocator keeps within it
#ifndef SGQ_WAVES
#define SGQ_WAVES 2
#endif
#define SGQ_OCC __attribute__((amdgpu_waves_per_eu(SGQ_WAVES, 8)))
// the HBM pass over the stopped keys (k_adv_*_k), with a window wider than the staged pass's: one wave per SIMD may
// hold it all in registers (its few waves walk the keys the staged pass stopped, where the slab walk's dependent HBM
// loads per partial were the cost)
#if SGQ_RH > SGQ_R
#define SGQ_OCC_H __attribute__((amdgpu_waves_per_eu(1, 8)))
#else
#define SGQ_OCC_H SGQ_OCC
#endif
// k_adv_*: the staged pass; k_adv_*_h: the HBM pass over the waves the staged pass deferred
// the HBM pass: one wave per work-group, striding over the waves the staged pass listed (p.dlist: the
// workgroups whose range did not fit LDS, the waves with resumed keys), so a batch with few of them
// costs few work-groups
template <bool S0, bool S1> __device__ __forceinline__ void hbm_pass(const P2Params& p) {
    const uint32_t n = __builtin_amdgcn_readfirstlane(*p.dlist_n);
    if (p.hot_ctl && blockIdx.x == 0 && threadIdx.x == 0) {
        // the batch's hot keys (after the pipeline) and giant workgroup ranges: into the status block's spare word
        // (the host runs the pipeline / the sorted grouping while batches have them); reset for the next batch
        p.err[1] = min(p.hot_ctl[0], 0xffffu) | (min(p.hot_ctl[SGD_HOT_CTL_BIG], 0xffffu) << 16);
        p.hot_ctl[0] = 0u;
        p.hot_ctl[SGD_HOT_CTL_BIG] = 0u;
    }
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t w = __builtin_amdgcn_readfirstlane(p.dlist[i]);
        advance<S0, S1, false, SGQ_R>(p, w * SGD_WAVE + threadIdx.x);
    }
}
// the keys the staged pass stopped (p.klist), 64 to a wave, with the HBM pass's wider window
template <bool S0, bool S1> __device__ __forceinline__ void hbm_keys(const P2Params& p) {
    const uint32_t nk = p.klist ? __builtin_amdgcn_readfirstlane(p.dlist_n[1]) : 0u;
    for (uint32_t i = blockIdx.x; i * SGD_WAVE < nk; i += gridDim.x)
        advance<S0, S1, false, SGQ_RH, true>(p, i * SGD_WAVE + threadIdx.x);
}
#define SG_GID (blockIdx.x * SGD_BLOCK + threadIdx.x)
#if SGQ_MULTI
extern "C" __global__ void __launch_bounds__(SGD_BLOCK) SGQ_OCC k_adv_m(const P2Params p) { advance<true, true, true, SGQ_R>(p, SG_GID); }
extern "C" __global__ void __launch_bounds__(SGD_WAVE) SGQ_OCC k_adv_m_h(const P2Params p) { hbm_pass<true, true>(p); }
extern "C" __global__ void __launch_bounds__(SGD_WAVE) SGQ_OCC_H k_adv_m_k(const P2Params p) { hbm_keys<true, true>(p); }
#else
extern "C" __global__ void __launch_bounds__(SGD_BLOCK) SGQ_OCC k_adv_s0(const P2Params p) { advance<true, false, true, SGQ_R>(p, SG_GID); }
extern "C" __global__ void __launch_bounds__(SGD_BLOCK) SGQ_OCC k_adv_s1(const P2Params p) { advance<false, true, true, SGQ_R>(p, SG_GID); }
extern "C" __global__ void __launch_bounds__(SGD_WAVE) SGQ_OCC k_adv_s0_h(const P2Params p) { hbm_pass<true, false>(p); }
extern "C" __global__ void __launch_bounds__(SGD_WAVE) SGQ_OCC k_adv_s1_h(const P2Params p) { hbm_pass<false, true>(p); }
extern "C" __global__ void __launch_bounds__(SGD_WAVE) SGQ_OCC_H k_adv_s0_k(const P2Params p) { hbm_keys<true, false>(p); }
extern "C" __global__ void __launch_bounds__(SGD_WAVE) SGQ_OCC_H k_adv_s1_k(const P2Params p) { hbm_keys<false, true>(p); }
#endif
extern "C" __global__ void __launch_bounds__(256) k_pack0(const PackParams q) { pack<SGQ_STRIDE0, 0>(q); }
extern "C" __global__ void __launch_bounds__(256) k_pack1(const PackParams q) { pack<SGQ_STRIDE1, 1>(q); }

// ---- hot keys -----------------------------------------------------------------------------------------------
// `every e1=S[f0] -> e2=S[f1(e1, e2)] within T` on one stream.  A key with thousands of events in one batch (the
// head of a Zipf key stream; the single key of an unpartitioned query) would serialise one lane of the staged walk.
// Its run is advanced here instead, all partials at once.  When the run's timestamps are nondecreasing (and the
// carried-in list is ts- and seq-ordered, with one start seed armed) the walk decomposes exactly:
//   - every event e_j with f0 creates one partial (the start state's one seed fires and re-arms at each event:
//     PatternMultiProcessStreamReceiver.java:31-40 with StreamPreStateProcessor.java:364-403), staged until the
//     next event, whose stabilize promotes it (:308-323, identity order: its ts is the newest);
//   - a pending partial dies at the first later event e_i that either expires it (|ts_j - ts_i| > T, tested at
//     stabilize, before the state-1 scan: :118-129 / :325-361 — with ordered timestamps the expired partials
//     are a prefix of the list, as the reference's prefix rule assumes) or satisfies f1(e_j, e_i) (a match,
//     emitted by e_i; StreamPostStateProcessor.java:64-83);
//   - the matches of one trigger are its matched partials in list order (creation order = seq order).
// So a partial's fate is a first-hit search over the run, done in rounds: a thread per partial over the
// SGD_HOT_L0 events after it (staged in LDS), a wave per partial still open over SGD_HOT_L1 more, then blocks of
// SGD_HOT_L1 events in parallel over spans 8x longer each round (atomicMin of the hit; the partials still open
// are about inversely proportional to the distance scanned, so every round costs about the same).  The
// triggers' match counts, their raw slots, the slot fill and the in-trigger seq order follow; the survivors
// (ordered) become the key's slab list.  A key whose run breaks the conditions is left to the HBM pass (its
// resume word untouched), which walks it as before.
#if SG_HOT
#define SGD_HOT_C 256u     // round 0: events per workgroup
#define SGD_HOT_L0 128u    // round 0: events each partial scans (staged in LDS after the workgroup's)
#define SGD_HOT_R0A 16u    // round 0: of them, the events a lane scans for its own partial (then a wave per partial)
#define SGD_HOT_L1 512u    // round 1: events each open partial scans; rounds >= 2: x8 per round
#define SGD_HOT_G 16u      // elements per thread of the list / reservation kernels (one atomic per 4096)
#define SGD_HOT_FILL 4096u // k_hot_fill: run events per workgroup pass
namespace {
constexpr uint32_t HOT_NOTP = 0xfffffffeu;  // death word of a run event that made no partial
constexpr uint32_t HOT_LIVE = 0xffffffffu;  // no event of the run ends the partial (or not found yet)
enum { HI_B = 0, HI_M, HI_EXOFF, HI_EVOFF, HI_N0, HI_BAD, HI_ALIVE, HI_KEY, HI_BLKOFF, HI_ALOFF };
enum { HC_N = 0, HC_EX, HC_EV, HC_L0, HC_L1, HC_MAXM, HC_BIG, HC_NBLK };
constexpr int HST = SGQ_STRIDE0;

// Flat index space of one batch's pipeline: [0, nex) the carried-in partials of the hot keys (key after key, list
// order), then [nex, nex + nev) the events of their runs (key after key, run order).  Flat order within a key is
// list order, so the survivors sorted by flat index are the key's new list.
struct HotPart {
    int64_t ts;
    uint64_t seq;
    uint32_t cw[SGQ_NCAPW > 0 ? SGQ_NCAPW : 1];
    uint32_t cn;
};

// the last hot key h whose `field` offset is <= x (keys with nothing there share the next key's offset)
__device__ __forceinline__ uint32_t hot_find(const uint32_t* info, uint32_t n, uint32_t x, int field) {
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) / 2u;
        if (info[mid * SGD_HOT_INFO + field] <= x) lo = mid; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int64_t hot_ts(const P2Params& p, const PayEl<HST>& x, int64_t obase) {
    const int32_t toff = (int32_t)x.w[HST - 1];
    return toff != SGD_TS_FAR ? obase + (int64_t)toff : p.ts_col[x.w[0]];
}
__device__ __forceinline__ HotPart hot_created(const P2Params& p, uint32_t pos, int64_t obase) {
    const PayEl<HST> x = load_pay<HST>(p.payload, pos);
    HotPart P;
    P.ts = hot_ts(p, x, obase);
    P.seq = p.seq_base + x.w[0];
    P.cn = 0;
#pragma unroll
    for (int w = 0; w < (SGQ_NCAPW > 0 ? SGQ_NCAPW : 1); ++w) P.cw[w] = 0;
    sgq_capture(sgq_ev0(x.w), P.cw, P.cn);
    return P;
}
__device__ __forceinline__ Slab hot_slab(const P2Params& p, uint32_t k) {
    return Slab{p.p_ts + k, p.p_seq + k, p.p_capw + k, p.p_capnull + k, p.n_keys, (size_t)p.cap * p.n_keys};
}
__device__ __forceinline__ HotPart hot_existing(const P2Params& p, uint32_t k, uint32_t j) {
    const Slab G = hot_slab(p, k);
    HotPart P;
    P.ts = G.TS(j);
    P.seq = G.SEQ(j);
#pragma unroll
    for (int w = 0; w < (SGQ_NCAPW > 0 ? SGQ_NCAPW : 1); ++w) P.cw[w] = w < SGQ_NCAPW ? G.CAP(w, j) : 0u;
    P.cn = SGQ_CAPNULL ? G.NUL(j) : 0u;
    return P;
}
// the partial at flat index x (key info hi): carried in (run index -1) or created by run event x - nex - evoff
__device__ __forceinline__ HotPart hot_part(const P2Params& p, uint32_t x, uint32_t nex, const uint32_t* hi,
                                            int64_t obase, int& start) {
    if (x < nex) {
        start = -1;
        return hot_existing(p, hi[HI_KEY], x - hi[HI_EXOFF]);
    }
    const uint32_t i = x - nex - hi[HI_EVOFF];
    start = (int)i;
    return hot_created(p, hi[HI_B] + i, obase);
}
// event i of the run (payload position pos) ends partial P: 2i (expired) or 2i + 1 (matched); HOT_LIVE otherwise
__device__ __forceinline__ uint32_t hot_test(const P2Params& p, const HotPart& P, uint32_t pos, uint32_t i,
                                             int64_t obase) {
    const PayEl<HST> x = load_pay<HST>(p.payload, pos);
    if (SGQ_WITHIN && expired(P.ts, hot_ts(p, x, obase), p.within)) return i * 2u;
    return sgq_f1(sgq_ev1(x.w), P.cw, P.cn, p) ? i * 2u + 1u : HOT_LIVE;
}
// a wave scans events [lo, end) of a run for partial P, 64 at a time: the first that ends it, or HOT_LIVE.  The
// payload of SGD_HOT_SB consecutive 64-event chunks is loaded at once (one round trip per 256 events instead of
// one per 64: the partials scanned here are the long-lived ones)
#define SGD_HOT_SB 4
__device__ __forceinline__ uint32_t hot_wave_scan(const P2Params& p, const HotPart& P, uint32_t b, uint32_t lo,
                                                  uint32_t end, int64_t obase) {
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1);
    for (uint32_t i0 = lo; i0 < end; i0 += SGD_WAVE * SGD_HOT_SB) {
        PayEl<HST> x[SGD_HOT_SB];
#pragma unroll
        for (int u = 0; u < SGD_HOT_SB; ++u) {
            const uint32_t i = i0 + (uint32_t)u * SGD_WAVE + lane;
            if (i < end) x[u] = load_pay<HST>(p.payload, b + i);
        }
#pragma unroll
        for (int u = 0; u < SGD_HOT_SB; ++u) {
            const uint32_t i = i0 + (uint32_t)u * SGD_WAVE + lane;
            uint32_t c = HOT_LIVE;
            if (i < end) {
                if (SGQ_WITHIN && expired(P.ts, hot_ts(p, x[u], obase), p.within)) c = i * 2u;
                else if (sgq_f1(sgq_ev1(x[u].w), P.cw, P.cn, p)) c = i * 2u + 1u;
            }
            const uint64_t hit = __ballot(c != HOT_LIVE);
            if (hit) return (uint32_t)__shfl((int)c, __builtin_ctzll(hit), SGD_WAVE);
        }
    }
    return HOT_LIVE;
}
__device__ __forceinline__ uint32_t hot_wl_cap(const P2Params& p) { return p.max_batch + p.hot_exmax; }
__device__ __forceinline__ uint32_t* hot_list_buf(const P2Params& p, uint32_t which) {
    return p.hot_wl + 3u * (size_t)hot_wl_cap(p) * which;
}
// workgroup-wide exclusive scan of one value per thread (blockDim.x = 256); *total = the sum
__device__ __forceinline__ uint32_t hot_block_scan(uint32_t v, uint32_t* s_w, uint32_t& total) {
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1), w = threadIdx.x / SGD_WAVE;
    const uint32_t incl = wave_incl_scan(v, (int)lane);
    if (lane == SGD_WAVE - 1) s_w[w] = incl;
    __syncthreads();
    uint32_t off = incl - v, tot = 0;
    for (uint32_t u = 0; u < blockDim.x / SGD_WAVE; ++u) {
        if (u < w) off += s_w[u];
        tot += s_w[u];
    }
    __syncthreads();
    total = tot;
    return off;
}
}  // namespace

// per hot key (a thread each): its run, its state and the conditions
extern "C" __global__ void __launch_bounds__(256) k_hot_prep(const P2Params p) {
    const uint32_t n = min(p.hot_ctl[HC_N], p.hot_cap);
    for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < n; h += gridDim.x * blockDim.x) {
        const uint32_t k = p.hot_list[h];
        uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        const uint32_t b = p.seg_begin[k], m = p.seg_end[k] - b;
        const uint32_t hd = p.hdr[k];
        const uint32_t sp = SGD_H_SPEND(hd), ss = SGD_H_SSTG(hd) + (SGD_H_INIT(hd) ? 0u : 1u);
        const uint32_t n0 = SGD_H_INIT(hd) ? SGD_H_NPEND(hd) + SGD_H_NSTG(hd) : 0u;
        // (the carried-in list's order is checked by round 0, a thread per partial)
        const bool bad = sp + ss != 1u || n0 > p.cap || m == 0u;
        hi[HI_B] = b;
        hi[HI_M] = bad ? 0u : m;
        hi[HI_N0] = bad ? 0u : n0;
        hi[HI_BAD] = bad ? 1u : 0u;
        hi[HI_ALIVE] = 0u;
        hi[HI_KEY] = k;
    }
}

// the offsets of the hot keys' carried-in partials, run events, fill blocks and survivor regions in their index
// spaces (exclusive scans, one workgroup: each thread a contiguous span of keys).  Keys whose carried-in partials
// would pass the space's end (p.hot_exmax) are given back and the scans run again.
__device__ __forceinline__ void hot_scan_pass(const P2Params& p, uint32_t n, bool last) {
    __shared__ uint32_t s_x[16], s_e[16], s_m[16], s_b[16], s_a[16];
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1), w = threadIdx.x / SGD_WAVE;
    const uint32_t per = (n + blockDim.x - 1u) / blockDim.x;
    const uint32_t lo = min(n, threadIdx.x * per), hi_ = min(n, lo + per);
    uint32_t sx = 0, se = 0, mm = 0, sb = 0, sa = 0;
    for (uint32_t h = lo; h < hi_; ++h) {
        const uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        const uint32_t n0 = hi[HI_N0], m = hi[HI_M];
        sx += n0;
        se += m;
        sb += (m + SGD_HOT_FILL - 1u) / SGD_HOT_FILL;
        sa += min(p.cap, n0 + m);
        mm = max(mm, m);
    }
    const uint32_t ix = wave_incl_scan(sx, (int)lane), ie = wave_incl_scan(se, (int)lane);
    const uint32_t ib = wave_incl_scan(sb, (int)lane), ia = wave_incl_scan(sa, (int)lane);
    mm = wave_max_u(mm);
    if (lane == SGD_WAVE - 1) { s_x[w] = ix; s_e[w] = ie; s_m[w] = mm; s_b[w] = ib; s_a[w] = ia; }
    __syncthreads();
    uint32_t ox = ix - sx, oe = ie - se, ob = ib - sb, oa = ia - sa;
    for (uint32_t u = 0; u < w; ++u) { ox += s_x[u]; oe += s_e[u]; ob += s_b[u]; oa += s_a[u]; }
    for (uint32_t h = lo; h < hi_; ++h) {
        uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        const uint32_t n0 = hi[HI_N0], m = hi[HI_M];
        if (!last && n0 && ox + n0 > p.hot_exmax) {  // (given back: the HBM pass walks it)
            hi[HI_BAD] = 1u;
            hi[HI_N0] = 0u;
            hi[HI_M] = 0u;
            continue;
        }
        hi[HI_EXOFF] = ox;
        hi[HI_EVOFF] = oe;
        hi[HI_BLKOFF] = ob;
        hi[HI_ALOFF] = oa;
        ox += n0;
        oe += m;
        ob += (m + SGD_HOT_FILL - 1u) / SGD_HOT_FILL;
        oa += min(p.cap, n0 + m);
    }
    if (threadIdx.x == 0) {
        uint32_t tx = 0, te = 0, tm = 0, tb = 0;
        for (uint32_t u = 0; u < blockDim.x / SGD_WAVE; ++u) { tx += s_x[u]; te += s_e[u]; tm = max(tm, s_m[u]); tb += s_b[u]; }
        uint32_t* ctl = p.hot_ctl;
        ctl[HC_EX] = tx;
        ctl[HC_EV] = te;
        ctl[HC_NBLK] = tb;
        ctl[HC_MAXM] = tm;
        ctl[HC_L0] = 0u;
        ctl[HC_L1] = 0u;
    }
    __syncthreads();
}
extern "C" __global__ void __launch_bounds__(1024) k_hot_scan(const P2Params p) {
    const uint32_t n = min(p.hot_ctl[HC_N], p.hot_cap);
    hot_scan_pass(p, n, false);
    if (p.hot_ctl[HC_EX] > p.hot_exmax) hot_scan_pass(p, n, true);  // (uniform: after the pass's barrier)
}

// the hot key of every run event (hot_fh): a workgroup per SGD_HOT_FILL events of one run (every thread finds
// the run by the same binary search: broadcast loads, no barrier)
extern "C" __global__ void __launch_bounds__(256) k_hot_fill(const P2Params p) {
    const uint32_t* ctl = p.hot_ctl;
    const uint32_t n = min(ctl[HC_N], p.hot_cap), nex = ctl[HC_EX], nblk = ctl[HC_NBLK];
    for (uint32_t q = blockIdx.x; q < nblk; q += gridDim.x) {
        const uint32_t h = hot_find(p.hot_info, n, q, HI_BLKOFF);
        const uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        const uint32_t j0 = (q - hi[HI_BLKOFF]) * SGD_HOT_FILL, j1 = min(hi[HI_M], j0 + SGD_HOT_FILL);
        uint32_t* dst = p.hot_fh + nex + hi[HI_EVOFF];
        for (uint32_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) dst[j] = h;
    }
}

// round 0.  The carried-in partials: a thread each over the first SGD_HOT_L0 events of the run (from HBM).  The
// runs' events: a workgroup per SGD_HOT_C consecutive flat events, staged in LDS with the SGD_HOT_L0 events after
// them; a thread per event checks it (timestamps nondecreasing, none -1), evaluates f0 (a partial or not) and scans
// the staged events after it.  Per flat index: its key (hot_fh), the partial's end so far (hot_death) and where the
// scan goes on (hot_cur).  No list is built here: round 1 finds the open partials by their death word.
extern "C" __global__ void __launch_bounds__(SGD_HOT_C) k_hot_r0(const P2Params p) {
    const uint32_t* ctl = p.hot_ctl;
    const uint32_t n = min(ctl[HC_N], p.hot_cap), nex = ctl[HC_EX], total = nex + ctl[HC_EV];
    const int64_t obase = p.ts_col[0];
    const uint32_t tid = threadIdx.x;
    for (uint32_t x = blockIdx.x * SGD_HOT_C + tid; x < nex; x += gridDim.x * SGD_HOT_C) {
        const uint32_t h = hot_find(p.hot_info, n, x, HI_EXOFF);
        p.hot_fh[x] = h;
        const uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        const uint32_t b = hi[HI_B], m = hi[HI_M], j = x - hi[HI_EXOFF];
        const HotPart P = hot_existing(p, hi[HI_KEY], j);
        {  // the carried-in list: ts and seq ordered, no ts -1, none newer than the run's first event
            const Slab G = hot_slab(p, hi[HI_KEY]);
            const int64_t t0 = hot_ts(p, load_pay<HST>(p.payload, b), obase);
            bool bad = P.ts == -1 || t0 == -1 || P.ts > t0;
            if (j > 0u) bad |= P.ts < G.TS(j - 1u) || P.seq <= G.SEQ(j - 1u);
            if (bad) p.hot_info[(size_t)h * SGD_HOT_INFO + HI_BAD] = 1u;
        }
        uint32_t d = HOT_LIVE;
        const uint32_t i1 = min(m, SGD_HOT_L0);
        for (uint32_t i = 0; i < i1 && d == HOT_LIVE; ++i) d = hot_test(p, P, b + i, i, obase);
        p.hot_death[x] = d;
        p.hot_cur[x] = i1;
    }
    constexpr uint32_t ST = SGD_HOT_C + SGD_HOT_L0;
    __shared__ uint32_t s_w[ST * HST];
    __shared__ int64_t s_ts[ST];
    __shared__ uint32_t s_open[SGD_HOT_C], s_oi[SGD_HOT_C], s_onj[SGD_HOT_C], s_nopen;
    const uint32_t lane = tid & (SGD_WAVE - 1), wv = tid / SGD_WAVE;
    for (uint32_t x0 = nex + blockIdx.x * SGD_HOT_C; x0 < total; x0 += gridDim.x * SGD_HOT_C) {
        uint32_t h = 0, pos = 0, i = 0, m = 0;
        for (uint32_t t = tid; t < ST; t += SGD_HOT_C) {
            const uint32_t x = x0 + t;
            if (x >= total) break;
            const uint32_t hx = p.hot_fh[x];
            const uint32_t* hi = p.hot_info + (size_t)hx * SGD_HOT_INFO;
            const uint32_t ix = x - nex - hi[HI_EVOFF], px = hi[HI_B] + ix;
            const PayEl<HST> ev = load_pay<HST>(p.payload, px);
#pragma unroll
            for (int u = 0; u < HST; ++u) s_w[t * HST + u] = ev.w[u];
            s_ts[t] = hot_ts(p, ev, obase);
            if (t < SGD_HOT_C) {
                h = hx;
                pos = px;
                i = ix;
                m = hi[HI_M];
                p.hot_fbi[x - nex] = ev.w[0];
            }
        }
        if (tid == 0) s_nopen = 0u;
        __syncthreads();
        const uint32_t x = x0 + tid;
        if (x < total) {
            const int64_t ts = s_ts[tid];
            const int64_t tp = i == 0u ? ts : tid > 0u ? s_ts[tid - 1] : hot_ts(p, load_pay<HST>(p.payload, pos - 1u), obase);
            if (ts == -1 || tp > ts) p.hot_info[(size_t)h * SGD_HOT_INFO + HI_BAD] = 1u;
            p.hot_tcnt[x - nex] = 0u;
            const SgEv0 e0 = sgq_ev0(&s_w[tid * HST]);
            uint32_t d = HOT_NOTP, cur = 0;
            if (sgq_f0(e0, p)) {
                HotPart P;
                P.ts = ts;
                P.cn = 0;
#pragma unroll
                for (int w = 0; w < (SGQ_NCAPW > 0 ? SGQ_NCAPW : 1); ++w) P.cw[w] = 0;
                sgq_capture(e0, P.cw, P.cn);
                d = HOT_LIVE;
                const uint32_t nj = min(m - 1u - i, SGD_HOT_L0);
                // the first SGD_HOT_R0A events a lane each (most partials end there); the rest of the window below,
                // a wave per partial still open (a lane-per-partial scan ran every wave to its longest scan)
                const uint32_t na = min(nj, SGD_HOT_R0A);
                for (uint32_t j = 1; j <= na && d == HOT_LIVE; ++j) {
                    const uint32_t t = tid + j;
                    if (SGQ_WITHIN && expired(P.ts, s_ts[t], p.within)) d = (i + j) * 2u;
                    else if (sgq_f1(sgq_ev1(&s_w[t * HST]), P.cw, P.cn, p)) d = (i + j) * 2u + 1u;
                }
                cur = i + 1u + nj;
                if (d == HOT_LIVE && nj > na) {  // (its death word is written by the wave that finishes it)
                    const uint32_t o = atomicAdd(&s_nopen, 1u);
                    s_open[o] = tid;
                    s_oi[o] = i;
                    s_onj[o] = nj;
                    d = HOT_NOTP - 1u;  // (marker: not written here)
                }
            }
            if (d != HOT_NOTP - 1u) p.hot_death[x] = d;
            p.hot_cur[x] = cur;
        }
        __syncthreads();
        const uint32_t no = s_nopen;
        for (uint32_t q = wv; q < no; q += SGD_HOT_C / SGD_WAVE) {
            const uint32_t tq = s_open[q], iq = s_oi[q], njq = s_onj[q];
            HotPart P;
            P.ts = s_ts[tq];
            P.cn = 0;
#pragma unroll
            for (int w = 0; w < (SGQ_NCAPW > 0 ? SGQ_NCAPW : 1); ++w) P.cw[w] = 0;
            sgq_capture(sgq_ev0(&s_w[tq * HST]), P.cw, P.cn);
            uint32_t d = HOT_LIVE;
            for (uint32_t j0 = SGD_HOT_R0A + 1u; j0 <= njq; j0 += SGD_WAVE) {
                const uint32_t j = j0 + lane;
                uint32_t c = HOT_LIVE;
                if (j <= njq) {
                    const uint32_t t = tq + j;
                    if (SGQ_WITHIN && expired(P.ts, s_ts[t], p.within)) c = (iq + j) * 2u;
                    else if (sgq_f1(sgq_ev1(&s_w[t * HST]), P.cw, P.cn, p)) c = (iq + j) * 2u + 1u;
                }
                const uint64_t hit = __ballot(c != HOT_LIVE);
                if (hit) {
                    d = (uint32_t)__shfl((int)c, __builtin_ctzll(hit), SGD_WAVE);
                    break;
                }
            }
            if (lane == 0) p.hot_death[x0 + tq] = d;
        }
        __syncthreads();
    }
}

// round 1: a wave per 64 flat indices; each partial still open there scans its next SGD_HOT_L1 events (the wave
// together, 64 at a time)
extern "C" __global__ void __launch_bounds__(256) k_hot_r1(const P2Params p) {
    const uint32_t* ctl = p.hot_ctl;
    const uint32_t nex = ctl[HC_EX], total = nex + ctl[HC_EV];
    const int64_t obase = p.ts_col[0];
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1);
    const uint32_t nw = gridDim.x * (blockDim.x / SGD_WAVE);
    for (uint32_t x0 = (blockIdx.x * (blockDim.x / SGD_WAVE) + threadIdx.x / SGD_WAVE) * SGD_WAVE; x0 < total;
         x0 += nw * SGD_WAVE) {
        const uint32_t x = x0 + lane;
        uint32_t h = 0, cur = 0;
        bool open = false;
        if (x < total && p.hot_death[x] == HOT_LIVE) {
            h = p.hot_fh[x];
            cur = p.hot_cur[x];
            open = cur < p.hot_info[(size_t)h * SGD_HOT_INFO + HI_M];
        }
        for (uint64_t bits = __ballot(open); bits; bits &= bits - 1ull) {
            const int l = __builtin_ctzll(bits);
            const uint32_t xl = (uint32_t)__shfl((int)x, l, SGD_WAVE), hl = (uint32_t)__shfl((int)h, l, SGD_WAVE);
            const uint32_t cl = (uint32_t)__shfl((int)cur, l, SGD_WAVE);
            const uint32_t* hi = p.hot_info + (size_t)hl * SGD_HOT_INFO;
            const uint32_t b = uni(hi[HI_B]), m = uni(hi[HI_M]);
            int start;
            const HotPart P = hot_part(p, xl, nex, hi, obase, start);
            const uint32_t end = min(m, cl + SGD_HOT_L1);
            const uint32_t d = hot_wave_scan(p, P, b, cl, end, obase);
            if (lane == 0) {
                p.hot_death[xl] = d;
                p.hot_cur[xl] = end;
            }
        }
    }
}

// the partials still open after round 1, listed for round 2: SGD_HOT_G flat indices per thread, one atomic per
// workgroup pass
extern "C" __global__ void __launch_bounds__(256) k_hot_r1c(const P2Params p) {
    const uint32_t* ctl = p.hot_ctl;
    const uint32_t total = ctl[HC_EX] + ctl[HC_EV];
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_base;
    uint32_t* out = hot_list_buf(p, 0);
    const uint32_t step = blockDim.x * SGD_HOT_G;
    for (uint32_t x0 = blockIdx.x * step; x0 < total; x0 += gridDim.x * step) {
        uint32_t mine = 0;
        for (uint32_t g = 0; g < SGD_HOT_G; ++g) {
            const uint32_t x = x0 + g * blockDim.x + threadIdx.x;
            if (x < total && p.hot_death[x] == HOT_LIVE &&
                p.hot_cur[x] < p.hot_info[(size_t)p.hot_fh[x] * SGD_HOT_INFO + HI_M])
                mine++;
        }
        uint32_t tot;
        uint32_t off = hot_block_scan(mine, s_w, tot);
        if (tot == 0u) continue;
        if (threadIdx.x == 0) s_base = atomicAdd(&p.hot_ctl[HC_L0], tot);
        __syncthreads();
        off += s_base;
        for (uint32_t g = 0; g < SGD_HOT_G && mine; ++g) {
            const uint32_t x = x0 + g * blockDim.x + threadIdx.x;
            if (x < total && p.hot_death[x] == HOT_LIVE) {
                const uint32_t h = p.hot_fh[x], c = p.hot_cur[x];
                if (c < p.hot_info[(size_t)h * SGD_HOT_INFO + HI_M]) {
                    out[3u * off] = x;
                    out[3u * off + 1u] = h;
                    out[3u * off + 2u] = c;
                    off++;
                    mine--;
                }
            }
        }
        __syncthreads();
    }
}

// rounds 2, 3, ... (p.hot_round): the partials still open scan their next SGD_HOT_L1 << 3 (round - 1) events, a
// wave per (partial, SGD_HOT_L1-event block), nearest blocks first, a block behind a hit already found skipped;
// the hit is the least (atomicMin).  The round reads list (round & 1) and zeroes the other one, which k_hot_rc
// fills with the partials still open after it.
__device__ __forceinline__ uint32_t hot_span(uint32_t round) { return SGD_HOT_L1 << (3u * (round - 1u)); }
extern "C" __global__ void __launch_bounds__(256) k_hot_rn(const P2Params p) {
    const uint32_t in = p.hot_round & 1u;
    const uint32_t nq = p.hot_ctl[HC_L0 + in], nex = p.hot_ctl[HC_EX];
    if (blockIdx.x == 0 && threadIdx.x == 0) p.hot_ctl[HC_L0 + (in ^ 1u)] = 0u;
    if (nq == 0u) return;
    const uint32_t span = hot_span(p.hot_round), nblk = span / SGD_HOT_L1;
    const uint64_t total = (uint64_t)nq * nblk;
    const int64_t obase = p.ts_col[0];
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1);
    const uint32_t nw = gridDim.x * (blockDim.x / SGD_WAVE);
    const uint32_t* wl = hot_list_buf(p, in);
    for (uint64_t t = blockIdx.x * (blockDim.x / SGD_WAVE) + threadIdx.x / SGD_WAVE; t < total; t += nw) {
        const uint32_t q = (uint32_t)(t % nq), blk = (uint32_t)(t / nq);
        const uint32_t x = uni(wl[3u * q]), h = uni(wl[3u * q + 1u]), cur = uni(wl[3u * q + 2u]);
        const uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        const uint32_t b = uni(hi[HI_B]), m = uni(hi[HI_M]);
        const uint64_t lo64 = (uint64_t)cur + (uint64_t)blk * SGD_HOT_L1;
        if (lo64 >= m) continue;
        const uint32_t lo = (uint32_t)lo64, end = min(m, lo + SGD_HOT_L1);
        if (uni(__hip_atomic_load(&p.hot_death[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < 2u * lo) continue;
        int start;
        const HotPart P = hot_part(p, x, nex, hi, obase, start);
        const uint32_t d = hot_wave_scan(p, P, b, lo, end, obase);
        if (lane == 0 && d != HOT_LIVE) atomicMin(&p.hot_death[x], d);
    }
}
// after round p.hot_round: the partials it left open with events still ahead, to the next round's list
extern "C" __global__ void __launch_bounds__(256) k_hot_rc(const P2Params p) {
    const uint32_t in = p.hot_round & 1u;
    const uint32_t nq = p.hot_ctl[HC_L0 + in];
    const uint32_t span = hot_span(p.hot_round);
    const uint32_t* wl = hot_list_buf(p, in);
    uint32_t* out = hot_list_buf(p, in ^ 1u);
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1);
    for (uint32_t x0 = blockIdx.x * blockDim.x + (threadIdx.x & ~(SGD_WAVE - 1)); x0 < nq; x0 += gridDim.x * blockDim.x) {
        const uint32_t q = x0 + lane;
        bool open = false;
        uint32_t x = 0, h = 0, nxt = 0;
        if (q < nq) {
            x = wl[3u * q];
            h = wl[3u * q + 1u];
            const uint64_t e64 = (uint64_t)wl[3u * q + 2u] + span;
            open = p.hot_death[x] == HOT_LIVE && e64 < p.hot_info[(size_t)h * SGD_HOT_INFO + HI_M];
            nxt = (uint32_t)min(e64, (uint64_t)0xffffffffu);
        }
        const uint64_t bal = __ballot(open);  // (few: one atomic per wave that has any)
        if (bal == 0ull) continue;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&p.hot_ctl[HC_L0 + (in ^ 1u)], (uint32_t)__popcll(bal));
        base = (uint32_t)__shfl((int)base, 0, SGD_WAVE);
        if (open) {
            const uint32_t o = base + lane_rank(bal);
            out[3u * o] = x;
            out[3u * o + 1u] = h;
            out[3u * o + 2u] = nxt;
        }
    }
}

// per flat index: the counters (exact, as the walk counts them), the trigger's match count, the survivors
extern "C" __global__ void __launch_bounds__(256) k_hot_emit(const P2Params p) {
    const uint32_t* ctl = p.hot_ctl;
    const uint32_t nex = ctl[HC_EX], total = nex + ctl[HC_EV];
    unsigned long long sc = 0, cr = 0, mt = 0;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < total; x += gridDim.x * blockDim.x) {
        const uint32_t h = p.hot_fh[x];
        uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        if (hi[HI_BAD]) continue;
        const uint32_t m = hi[HI_M];
        const bool ex = x < nex;
        const int start = ex ? -1 : (int)(x - nex - hi[HI_EVOFF]);
        if (!ex) sc += 1;  // the start state's seed tests every event (one seed armed)
        const uint32_t d = p.hot_death[x];
        if (d == HOT_NOTP) continue;
        if (!ex) cr += 1;
        if (d == HOT_LIVE) {  // scanned by every later event of the run; a survivor
            sc += (unsigned long long)((int64_t)m - 1 - start);
            const uint32_t a = atomicAdd(&hi[HI_ALIVE], 1u);
            if (a < min(p.cap, hi[HI_N0] + m)) p.hot_alive[hi[HI_ALOFF] + a] = x;
        } else {  // scanned up to its end; the expiring event removes it before its scan
            const uint32_t i = d >> 1;
            sc += (unsigned long long)((int64_t)i - start - 1 + (int64_t)(d & 1u));
            if (d & 1u) {
                mt += 1;
                atomicAdd(&p.hot_tcnt[hi[HI_EVOFF] + i], 1u);
            }
        }
    }
    __shared__ unsigned long long s_r[3][4];
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1), w = threadIdx.x / SGD_WAVE;
    sc = wave_sum(sc);
    cr = wave_sum(cr);
    mt = wave_sum(mt);
    if (lane == 0) { s_r[0][w] = sc; s_r[1][w] = cr; s_r[2][w] = mt; }
    __syncthreads();
    if (threadIdx.x < 3) {
        unsigned long long v = 0;
        for (uint32_t u = 0; u < blockDim.x / SGD_WAVE; ++u) v += s_r[threadIdx.x][u];
        const int which = threadIdx.x == 0 ? SGD_ST_SCANNED : threadIdx.x == 1 ? SGD_ST_CREATED : SGD_ST_MATCHES;
        if (v) atomicAdd(&p.stats[which], v);
    }
}

// per run event: its matches' raw slots (SGD_HOT_G events per thread, one reservation per workgroup pass) and its
// trigger descriptor (the events of keys given back have no count)
extern "C" __global__ void __launch_bounds__(256) k_hot_trig(const P2Params p) {
    const uint32_t nev = p.hot_ctl[HC_EV];
    __shared__ uint32_t s_w[4];
    __shared__ unsigned long long s_base;
    const uint32_t step = blockDim.x * SGD_HOT_G;
    for (uint32_t x0 = blockIdx.x * step; x0 < nev; x0 += gridDim.x * step) {
        uint32_t c[SGD_HOT_G], mine = 0;
#pragma unroll
        for (uint32_t g = 0; g < SGD_HOT_G; ++g) {
            const uint32_t x = x0 + g * blockDim.x + threadIdx.x;
            c[g] = x < nev ? p.hot_tcnt[x] : 0u;
            mine += c[g];
        }
        uint32_t tot;
        const uint32_t off = hot_block_scan(mine, s_w, tot);
        if (tot == 0u) continue;
        if (threadIdx.x == 0) s_base = atomicAdd(p.raw_count, (unsigned long long)tot);
        __syncthreads();
        unsigned long long first = p.raw_static + s_base + off;
#pragma unroll
        for (uint32_t g = 0; g < SGD_HOT_G; ++g) {
            if (c[g]) {
                const uint32_t x = x0 + g * blockDim.x + threadIdx.x;
                if (first + c[g] <= p.raw_capacity)
                    p.t_desc[p.hot_fbi[x]] = p.td_tag | ((uint64_t)c[g] << 32) | (uint64_t)(uint32_t)first;
                else
                    atomicOr(p.err, (uint32_t)SGD_ERR_MATCH_CAP);
                p.hot_tbase[x] = (uint32_t)first;
                p.hot_tcnt[x] = 0u;  // (the fill's rank counter)
                first += c[g];
            }
        }
        __syncthreads();
    }
}

// per matched partial: its e1 seq (and captures) into a slot of its trigger's range
extern "C" __global__ void __launch_bounds__(256) k_hot_place(const P2Params p) {
    const uint32_t* ctl = p.hot_ctl;
    const uint32_t nex = ctl[HC_EX], total = nex + ctl[HC_EV];
    const int64_t obase = p.ts_col[0];
    (void)obase;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < total; x += gridDim.x * blockDim.x) {
        const uint32_t d = p.hot_death[x];
        if (d == HOT_NOTP || d == HOT_LIVE || !(d & 1u)) continue;
        const uint32_t* hi = p.hot_info + (size_t)p.hot_fh[x] * SGD_HOT_INFO;
        if (hi[HI_BAD]) continue;
        const uint32_t tp = hi[HI_EVOFF] + (d >> 1);
        const uint64_t dst = (uint64_t)p.hot_tbase[tp] + atomicAdd(&p.hot_tcnt[tp], 1u);
        if (dst >= p.raw_capacity) continue;
#if SGQ_PROJ
        int start;
        const HotPart P = hot_part(p, x, nex, hi, obase, start);
        p.raw_e1[dst] = P.seq;
#pragma unroll
        for (int w = 0; w < SGQ_NCAPW; ++w) p.raw_capw[(size_t)w * p.raw_capacity + dst] = P.cw[w];
        if (SGQ_CAPNULL) p.raw_capnull[dst] = P.cn;
#else
        p.raw_e1[dst] = x >= nex ? p.seq_base + p.hot_fbi[x - nex] : hot_slab(p, hi[HI_KEY]).SEQ(x - hi[HI_EXOFF]);
#endif
    }
}

// per trigger with several matches: its range into list order (= e1 seq order).  A range of 2..8 by its thread
// (values in registers, ranked by counting); longer ones by the wave of its 64 run events (one match per lane,
// ranks by shuffles), beyond 64 by lane 0 (insertion sort)
extern "C" __global__ void __launch_bounds__(256) k_hot_sort(const P2Params p) {
    const uint32_t nev = p.hot_ctl[HC_EV];
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1);
    const uint32_t nw = gridDim.x * (blockDim.x / SGD_WAVE);
    const uint64_t RC = p.raw_capacity;
    for (uint32_t x0 = (blockIdx.x * (blockDim.x / SGD_WAVE) + threadIdx.x / SGD_WAVE) * SGD_WAVE; x0 < nev;
         x0 += nw * SGD_WAVE) {
        const uint32_t x = x0 + lane;
        const uint32_t c = x < nev ? p.hot_tcnt[x] : 0u;
        const uint32_t fb = c >= 2u ? p.hot_tbase[x] : 0u;
        constexpr uint32_t SMALL = 8;
        if (c >= 2u && c <= SMALL && (uint64_t)fb + c <= RC) {
            uint64_t v[SMALL];
#if SGQ_PROJ
            uint32_t cw[SMALL][SGQ_NCAPW > 0 ? SGQ_NCAPW : 1], cn[SMALL];
#endif
#pragma unroll
            for (uint32_t a = 0; a < SMALL; ++a) {
                v[a] = a < c ? p.raw_e1[fb + a] : ~0ull;
#if SGQ_PROJ
#pragma unroll
                for (int w = 0; w < SGQ_NCAPW; ++w) cw[a][w] = a < c ? p.raw_capw[(size_t)w * RC + fb + a] : 0u;
                cn[a] = (SGQ_CAPNULL && a < c) ? p.raw_capnull[fb + a] : 0u;
#endif
            }
#pragma unroll
            for (uint32_t a = 0; a < SMALL; ++a) {
                if (a < c) {
                    uint32_t r = 0;
#pragma unroll
                    for (uint32_t u = 0; u < SMALL; ++u) r += v[u] < v[a] ? 1u : 0u;  // (distinct; ~0 pads rank last)
                    p.raw_e1[fb + r] = v[a];
#if SGQ_PROJ
#pragma unroll
                    for (int w = 0; w < SGQ_NCAPW; ++w) p.raw_capw[(size_t)w * RC + fb + r] = cw[a][w];
                    if (SGQ_CAPNULL) p.raw_capnull[fb + r] = cn[a];
#endif
                }
            }
        }
        for (uint64_t bits = __ballot(c > SMALL && (uint64_t)fb + c <= RC); bits; bits &= bits - 1ull) {
            const int l = __builtin_ctzll(bits);
            const uint32_t cl = uni((uint32_t)__shfl((int)c, l, SGD_WAVE));
            const uint64_t f = uni((uint32_t)__shfl((int)fb, l, SGD_WAVE));
            if (cl <= SGD_WAVE) {
                const bool in = lane < cl;
                const uint64_t v = in ? p.raw_e1[f + lane] : ~0ull;
#if SGQ_PROJ
                uint32_t cw[SGQ_NCAPW > 0 ? SGQ_NCAPW : 1], cn = 0;
#pragma unroll
                for (int w = 0; w < SGQ_NCAPW; ++w) cw[w] = in ? p.raw_capw[(size_t)w * RC + f + lane] : 0u;
                if (SGQ_CAPNULL) cn = in ? p.raw_capnull[f + lane] : 0u;
#endif
                const uint32_t vlo = (uint32_t)v, vhi = (uint32_t)(v >> 32);
                uint32_t r = 0;
                for (uint32_t j = 0; j < cl; ++j) {  // (seqs are distinct)
                    const uint64_t vj = (uint64_t)(uint32_t)__shfl((int)vlo, (int)j, SGD_WAVE) |
                                        ((uint64_t)(uint32_t)__shfl((int)vhi, (int)j, SGD_WAVE) << 32);
                    r += vj < v ? 1u : 0u;
                }
                if (in) {
                    p.raw_e1[f + r] = v;
#if SGQ_PROJ
#pragma unroll
                    for (int w = 0; w < SGQ_NCAPW; ++w) p.raw_capw[(size_t)w * RC + f + r] = cw[w];
                    if (SGQ_CAPNULL) p.raw_capnull[f + r] = cn;
#endif
                }
            } else if (lane == 0) {
                for (uint32_t a = 1; a < cl; ++a) {
                    const uint64_t v = p.raw_e1[f + a];
#if SGQ_PROJ
                    uint32_t cw[SGQ_NCAPW > 0 ? SGQ_NCAPW : 1], cn = 0;
#pragma unroll
                    for (int w = 0; w < SGQ_NCAPW; ++w) cw[w] = p.raw_capw[(size_t)w * RC + f + a];
                    if (SGQ_CAPNULL) cn = p.raw_capnull[f + a];
#endif
                    uint32_t z = a;
                    while (z > 0u && p.raw_e1[f + z - 1u] > v) {
                        p.raw_e1[f + z] = p.raw_e1[f + z - 1u];
#if SGQ_PROJ
#pragma unroll
                        for (int w = 0; w < SGQ_NCAPW; ++w) p.raw_capw[(size_t)w * RC + f + z] = p.raw_capw[(size_t)w * RC + f + z - 1u];
                        if (SGQ_CAPNULL) p.raw_capnull[f + z] = p.raw_capnull[f + z - 1u];
#endif
                        --z;
                    }
                    p.raw_e1[f + z] = v;
#if SGQ_PROJ
#pragma unroll
                    for (int w = 0; w < SGQ_NCAPW; ++w) p.raw_capw[(size_t)w * RC + f + z] = cw[w];
                    if (SGQ_CAPNULL) p.raw_capnull[f + z] = cn;
#endif
                }
            }
        }
    }
}

// the key's header and the resume word that tells the HBM pass the key is done: the last event's partial (if f0
// held) is still staged, and the seed it used re-arms at the next event
__device__ __forceinline__ void hot_close(const P2Params& p, const uint32_t* hi, uint32_t nex, uint32_t na) {
    const uint32_t k = hi[HI_KEY];
    const bool lastf0 = p.hot_death[nex + hi[HI_EVOFF] + hi[HI_M] - 1u] != HOT_NOTP;
    const uint32_t gns = lastf0 ? 1u : 0u;
    p.hdr[k] = SGD_H_MAKE(na - gns, gns, lastf0 ? 0u : 1u, lastf0 ? 1u : 0u, 1u);
    p.resume[k] = SGD_HOT_DONE;
    atomicAdd(&p.stats[SGD_ST_HOTK], 1ull);
    atomicAdd(&p.stats[SGD_ST_HOTE], (unsigned long long)hi[HI_M]);
}
__device__ __forceinline__ void hot_store(const P2Params& p, const Slab& G, uint32_t o, const HotPart& P) {
    G.TS(o) = P.ts;
    G.SEQ(o) = P.seq;
#pragma unroll
    for (int w = 0; w < SGQ_NCAPW; ++w) G.CAP(w, o) = P.cw[w];
    if (SGQ_CAPNULL) G.NUL(o) = P.cn;
}

// a wave per hot key with at most SGD_HOT_FW survivors: ranked by flat index (= list order) in the wave's LDS, then
// moved to the key's slab 64 at a time in rank order (survivor o comes from list index >= o, so a round's writes
// land below every later round's reads), the header, the resume word
#define SGD_HOT_FW 256u
extern "C" __global__ void __launch_bounds__(256) k_hot_final(const P2Params p) {
    const uint32_t n = min(p.hot_ctl[HC_N], p.hot_cap), nex = p.hot_ctl[HC_EX];
    const int64_t obase = p.ts_col[0];
    const uint32_t lane = threadIdx.x & (SGD_WAVE - 1), wv = threadIdx.x / SGD_WAVE;
    const uint32_t nw = gridDim.x * (blockDim.x / SGD_WAVE);
    __shared__ uint32_t s_ord[4][SGD_HOT_FW];
    for (uint32_t h = blockIdx.x * (blockDim.x / SGD_WAVE) + wv; h < n; h += nw) {
        const uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        if (uni(hi[HI_BAD])) continue;  // left to the HBM pass
        const uint32_t na = uni(hi[HI_ALIVE]);
        if (na > p.cap) {  // more partials than the slab holds
            if (lane == 0) {
                atomicOr(p.err, (uint32_t)SGD_ERR_PARTIAL_CAP);
                p.resume[hi[HI_KEY]] = SGD_HOT_DONE;
            }
            continue;
        }
        if (na > SGD_HOT_FW) continue;  // (k_hot_final_big)
        const uint32_t* pool = p.hot_alive + hi[HI_ALOFF];
        // the survivors (listed in emit's atomic order) sorted by flat index — list order — with a bitonic network
        // over the next power of two (padding sorts last): log^2 stages of 64-lane compare-exchanges instead of a
        // rank count over all pairs
        uint32_t np2 = 1;
        while (np2 < na) np2 <<= 1;
        uint32_t* so = s_ord[wv];
        for (uint32_t a = lane; a < np2; a += SGD_WAVE) so[a] = a < na ? pool[a] : 0xffffffffu;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (uint32_t kk = 2; kk <= np2; kk <<= 1) {
            for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
                for (uint32_t i = lane; i < np2; i += SGD_WAVE) {
                    const uint32_t ij = i ^ j;
                    if (ij > i) {
                        const uint32_t va = so[i], vb = so[ij];
                        if ((va > vb) == ((i & kk) == 0u)) {
                            so[i] = vb;
                            so[ij] = va;
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
        }
        const Slab G = hot_slab(p, hi[HI_KEY]);
        for (uint32_t c0 = 0; c0 < na; c0 += SGD_WAVE) {
            const uint32_t o = c0 + lane;
            HotPart P;
            int start;
            if (o < na) P = hot_part(p, s_ord[wv][o], nex, hi, obase, start);
            __builtin_amdgcn_s_waitcnt(0);  // (every lane's read of the round before any write)
            __builtin_amdgcn_wave_barrier();
            if (o < na) hot_store(p, G, o, P);
        }
        if (lane == 0) hot_close(p, hi, nex, na);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// a workgroup per hot key with more than SGD_HOT_FW survivors (rare): ranked in LDS, moved 256 at a time in order
extern "C" __global__ void __launch_bounds__(256) k_hot_final_big(const P2Params p) {
    const uint32_t n = min(p.hot_ctl[HC_N], p.hot_cap), nex = p.hot_ctl[HC_EX];
    const int64_t obase = p.ts_col[0];
    __shared__ uint32_t s_x[SGD_MAX_CAP + 1], s_ord[SGD_MAX_CAP + 1];
    for (uint32_t h = blockIdx.x; h < n; h += gridDim.x) {
        const uint32_t* hi = p.hot_info + (size_t)h * SGD_HOT_INFO;
        const uint32_t na = hi[HI_ALIVE];
        if (hi[HI_BAD] || na <= SGD_HOT_FW || na > p.cap) continue;  // (uniform)
        for (uint32_t a = threadIdx.x; a < na; a += blockDim.x) s_x[a] = p.hot_alive[hi[HI_ALOFF] + a];
        __syncthreads();
        for (uint32_t a = threadIdx.x; a < na; a += blockDim.x) {  // rank by flat index (distinct)
            uint32_t r = 0;
            const uint32_t xa = s_x[a];
            for (uint32_t u = 0; u < na; ++u) r += s_x[u] < xa ? 1u : 0u;
            s_ord[r] = xa;
        }
        __syncthreads();
        // in place, 256 at a time: survivor o comes from list index >= o, so a chunk's writes land below every
        // later chunk's reads
        const Slab G = hot_slab(p, hi[HI_KEY]);
        for (uint32_t c0 = 0; c0 < na; c0 += blockDim.x) {
            const uint32_t o = c0 + threadIdx.x;
            HotPart P;
            int start;
            if (o < na) P = hot_part(p, s_ord[o], nex, hi, obase, start);
            __syncthreads();
            if (o < na) hot_store(p, G, o, P);
            __syncthreads();
        }
        if (threadIdx.x == 0) hot_close(p, hi, nex, na);
        __syncthreads();
    }
}
#endif  // SG_HOT
