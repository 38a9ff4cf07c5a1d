// p2_kernels.hip — gfx950 kernels for two-state partitioned patterns
//   every? e1=S0[f0] -> e2=S1[f1(e1,e2)] (within T)   and   every (e1=S0[f0] -> e2=S1[f1])
//
// One lane owns one partition key (adjacent lanes = adjacent keys, so the SoA partial-match slabs
// partial j of key k at j*K+k are read and written coalesced), a wavefront walks 64 keys' events of
// the micro-batch in arrival order, and emitted matches are compacted wave-wide (shuffle prefix sum,
// one global atomic per wave step).  Semantics restated from (paths under
// /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/query/input/):
//   stabilize: expire all states, then promote staged partials
//       stream/state/receiver/PatternMultiProcessStreamReceiver.java:42-51 (Single: :34-41)
//   expiry: StreamPreStateProcessor.java:118-129 (isExpired), :325-361 (prefix of pending, all of
//       staged, re-arm of the withinEvery start state)
//   promotion: StreamPreStateProcessor.java:308-323 (stable sort by ts, -1 last, :66-80)
//   state order per event: later state first (PatternMultiProcessStreamReceiver.java:31-40)
//   advance: StreamPreStateProcessor.java:364-403 + StreamPostStateProcessor.java:64-83
//   filters: FilterProcessor.java:48-60 and the typed executors (see eval_prog)
#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu_ir.h"
#include "sg_engine.h"

namespace {

struct DVal {
    uint64_t b;
    uint32_t null;
};

__device__ __forceinline__ float f32_of(uint64_t b) { return __uint_as_float((uint32_t)b); }
__device__ __forceinline__ double f64_of(uint64_t b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ uint64_t bits_f32(float f) { return (uint64_t)__float_as_uint(f); }
__device__ __forceinline__ uint64_t bits_f64(double d) { return (uint64_t)__double_as_longlong(d); }

// Java widening conversions (JLS 5.1.2: int/long -> float/double round to nearest)
__device__ __forceinline__ uint64_t cvt_bits(uint64_t b, uint32_t from, uint32_t to) {
    if (from == SG_T_INT) {
        int32_t x = (int32_t)(uint32_t)b;
        if (to == SG_T_LONG) return (uint64_t)(int64_t)x;
        if (to == SG_T_FLOAT) return bits_f32((float)x);
        return bits_f64((double)x);
    }
    if (from == SG_T_LONG) {
        int64_t x = (int64_t)b;
        if (to == SG_T_FLOAT) return bits_f32((float)x);
        return bits_f64((double)x);
    }
    return bits_f64((double)f32_of(b));  // FLOAT -> DOUBLE
}

template <class T> __device__ __forceinline__ bool cmp_t(uint32_t op, T a, T b) {
    switch (op) {
    case SG_OP_EQ: return a == b;
    case SG_OP_NE: return a != b;
    case SG_OP_GT: return a > b;
    case SG_OP_GE: return a >= b;
    case SG_OP_LT: return a < b;
    default: return a <= b;
    }
}

__device__ __forceinline__ bool compare(uint32_t op, uint32_t dom, DVal l, DVal r) {
    // CompareConditionExpressionExecutor.java:38-42 (null -> false); NotEqual...: null -> true
    if (l.null | r.null) return op == SG_OP_NE;
    switch (dom) {
    case SG_T_INT: return cmp_t(op, (int32_t)(uint32_t)l.b, (int32_t)(uint32_t)r.b);
    case SG_T_LONG: return cmp_t(op, (int64_t)l.b, (int64_t)r.b);
    case SG_T_FLOAT: return cmp_t(op, f32_of(l.b), f32_of(r.b));
    case SG_T_DOUBLE: return cmp_t(op, f64_of(l.b), f64_of(r.b));
    case SG_T_STRING: return cmp_t(op, (uint32_t)l.b, (uint32_t)r.b);
    default: return cmp_t(op, (uint32_t)(l.b & 1), (uint32_t)(r.b & 1));
    }
}

// executor/math/*: null in -> null, x/0 and x%0 -> null, int/long wrap, MIN/-1 = MIN, MIN%-1 = 0
__device__ __forceinline__ DVal arith(uint32_t op, uint32_t t, DVal l, DVal r) {
    DVal o{0, 0};
    if (l.null | r.null) { o.null = 1; return o; }
    if (t == SG_T_INT) {
        uint32_t a = (uint32_t)l.b, b = (uint32_t)r.b;
        int32_t sa = (int32_t)a, sb = (int32_t)b;
        switch (op) {
        case SG_OP_ADD: o.b = (uint32_t)(a + b); break;
        case SG_OP_SUB: o.b = (uint32_t)(a - b); break;
        case SG_OP_MUL: o.b = (uint32_t)(a * b); break;
        case SG_OP_DIV:
            if (sb == 0) o.null = 1;
            else o.b = (sb == -1) ? (uint32_t)(0u - a) : (uint32_t)(sa / sb);
            break;
        default:
            if (sb == 0) o.null = 1;
            else o.b = (sb == -1) ? 0u : (uint32_t)(sa % sb);
        }
        return o;
    }
    if (t == SG_T_LONG) {
        uint64_t a = l.b, b = r.b;
        int64_t sa = (int64_t)a, sb = (int64_t)b;
        switch (op) {
        case SG_OP_ADD: o.b = a + b; break;
        case SG_OP_SUB: o.b = a - b; break;
        case SG_OP_MUL: o.b = a * b; break;
        case SG_OP_DIV:
            if (sb == 0) o.null = 1;
            else o.b = (sb == -1) ? (0ull - a) : (uint64_t)(sa / sb);
            break;
        default:
            if (sb == 0) o.null = 1;
            else o.b = (sb == -1) ? 0ull : (uint64_t)(sa % sb);
        }
        return o;
    }
    if (t == SG_T_FLOAT) {
        float a = f32_of(l.b), b = f32_of(r.b);
        switch (op) {
        case SG_OP_ADD: o.b = bits_f32(__fadd_rn(a, b)); break;
        case SG_OP_SUB: o.b = bits_f32(__fsub_rn(a, b)); break;
        case SG_OP_MUL: o.b = bits_f32(__fmul_rn(a, b)); break;
        case SG_OP_DIV: if (b == 0.0f) o.null = 1; else o.b = bits_f32(__fdiv_rn(a, b)); break;
        default: if (b == 0.0f) o.null = 1; else o.b = bits_f32(fmodf(a, b));
        }
        return o;
    }
    double a = f64_of(l.b), b = f64_of(r.b);
    switch (op) {
    case SG_OP_ADD: o.b = bits_f64(__dadd_rn(a, b)); break;
    case SG_OP_SUB: o.b = bits_f64(__dsub_rn(a, b)); break;
    case SG_OP_MUL: o.b = bits_f64(__dmul_rn(a, b)); break;
    case SG_OP_DIV: if (b == 0.0) o.null = 1; else o.b = bits_f64(__ddiv_rn(a, b)); break;
    default: if (b == 0.0) o.null = 1; else o.b = bits_f64(fmod(a, b));
    }
    return o;
}

// register file of the evaluation stack; all indices are wave-uniform (the program is), so the
// switch lowers to scalar branches, not scratch memory
struct Stack {
    DVal r0, r1, r2, r3, r4, r5, r6, r7;
    __device__ __forceinline__ DVal get(int i) const {
        switch (i) {
        case 0: return r0; case 1: return r1; case 2: return r2; case 3: return r3;
        case 4: return r4; case 5: return r5; case 6: return r6; default: return r7;
        }
    }
    __device__ __forceinline__ void set(int i, DVal v) {
        switch (i) {
        case 0: r0 = v; break; case 1: r1 = v; break; case 2: r2 = v; break; case 3: r3 = v; break;
        case 4: r4 = v; break; case 5: r5 = v; break; case 6: r6 = v; break; default: r7 = v;
        }
    }
};

struct EvRegs {  // the current event's columns used by the filters (static indices only)
    DVal c0, c1, c2, c3, c4, c5, c6, c7;
    __device__ __forceinline__ DVal get(int i) const {
        switch (i) {
        case 0: return c0; case 1: return c1; case 2: return c2; case 3: return c3;
        case 4: return c4; case 5: return c5; case 6: return c6; default: return c7;
        }
    }
    __device__ __forceinline__ void set(int i, DVal v) {
        switch (i) {
        case 0: c0 = v; break; case 1: c1 = v; break; case 2: c2 = v; break; case 3: c3 = v; break;
        case 4: c4 = v; break; case 5: c5 = v; break; case 6: c6 = v; break; default: c7 = v;
        }
    }
};

// full stack-program interpreter (filters that are not a conjunction of comparisons)
template <class CapFn>
__device__ __forceinline__ bool eval_prog(const DProg& P, const EvRegs& ev, CapFn caps) {
    Stack s;
    int sp = 0;
    for (uint32_t pc = 0; pc < P.len; ++pc) {
        const DInst I = P.ins[pc];
        switch (I.op) {
        case SG_OP_VAR: {
            DVal v;
            if (I.src == SGD_SRC_EV) v = ev.get(I.arg);
            else if (I.src == SGD_SRC_CAP) v = caps(I.arg);
            else v = DVal{0, 1};
            s.set(sp++, v);
            break;
        }
        case SG_OP_CONST: s.set(sp++, DVal{I.imm, (uint32_t)I.t2}); break;
        case SG_OP_CVT: {
            DVal v = s.get(sp - 1);
            if (!v.null) v.b = cvt_bits(v.b, I.t, I.t2);
            s.set(sp - 1, v);
            break;
        }
        case SG_OP_ADD: case SG_OP_SUB: case SG_OP_MUL: case SG_OP_DIV: case SG_OP_MOD:
            s.set(sp - 2, arith(I.op, I.t, s.get(sp - 2), s.get(sp - 1)));
            sp--;
            break;
        case SG_OP_EQ: case SG_OP_NE: case SG_OP_GT: case SG_OP_GE: case SG_OP_LT: case SG_OP_LE:
            s.set(sp - 2, DVal{(uint64_t)compare(I.op, I.t, s.get(sp - 2), s.get(sp - 1)), 0});
            sp--;
            break;
        case SG_OP_AND: case SG_OP_OR: {  // And/OrConditionExpressionExecutor: null counts as false
            DVal l = s.get(sp - 2), r = s.get(sp - 1);
            bool lb = !l.null && (l.b & 1), rb = !r.null && (r.b & 1);
            s.set(sp - 2, DVal{(uint64_t)(I.op == SG_OP_AND ? (lb && rb) : (lb || rb)), 0});
            sp--;
            break;
        }
        case SG_OP_NOT: {  // NotConditionExpressionExecutor: not(null) = true
            DVal v = s.get(sp - 1);
            s.set(sp - 1, DVal{(uint64_t)!(!v.null && (v.b & 1)), 0});
            break;
        }
        default: {  // SG_OP_ISNULL
            DVal v = s.get(sp - 1);
            s.set(sp - 1, DVal{(uint64_t)v.null, 0});
        }
        }
    }
    if (P.len == 0) return true;
    DVal r = s.get(sp - 1);
    return !r.null && (r.b & 1);
}

// conjunctive predicate in registers: atom a = code[a] (packed DAtom, see sg_engine.h) + const bits
struct PredRegs {
    uint32_t n;
    uint32_t prog;
    uint32_t code[SGD_MAX_ATOMS];
    uint64_t cbits[SGD_MAX_ATOMS];
};

template <class CapFn>
__device__ __forceinline__ DVal operand(uint32_t kind, uint32_t from, uint32_t idx, uint64_t cb, uint32_t dom,
                                        const EvRegs& ev, CapFn caps) {
    DVal v;
    switch (kind) {
    case SGD_SRC_EV: v = ev.get((int)idx); break;
    case SGD_SRC_CAP: v = caps((int)idx); break;
    case SGD_SRC_CONST: return DVal{cb, 0};
    default: return DVal{0, 1};
    }
    if (from != dom && !v.null) v.b = cvt_bits(v.b, from, dom);
    return v;
}

// out-of-line general interpreter: program in global memory, captures preloaded into registers
__device__ __noinline__ bool eval_prog_ool(const DProg* __restrict__ P, EvRegs ev, EvRegs cp) {
    auto caps = [&](int c) -> DVal { return cp.get(c); };
    return eval_prog(*P, ev, caps);
}

// every descriptor field is wave-uniform and already in registers: scalar branches only
template <bool PROG, class CapFn>
__device__ __forceinline__ bool eval_pred(const PredRegs& P, const DProg* F, uint32_t n_caps, const EvRegs& ev,
                                          CapFn caps) {
    if constexpr (PROG) {
        if (P.prog) {
            EvRegs cp;
#pragma unroll
            for (int c = 0; c < SGD_MAX_CAPS; ++c)
                if (c < (int)n_caps) cp.set(c, caps(c));
            return eval_prog_ool(F, ev, cp);
        }
    }
    bool ok = true;
#pragma unroll
    for (int a = 0; a < SGD_MAX_ATOMS; ++a) {
        if (a < (int)P.n) {
            const uint32_t c = P.code[a];
            const uint32_t dom = (c >> 4) & 15u;
            const DVal l = operand((c >> 8) & 15u, (c >> 12) & 15u, (c >> 16) & 15u, P.cbits[a], dom, ev, caps);
            const DVal r = operand((c >> 20) & 15u, (c >> 24) & 15u, c >> 28, P.cbits[a], dom, ev, caps);
            ok = ok && compare(SG_OP_EQ + (c & 15u), dom, l, r);
        }
    }
    return ok;
}

__device__ __forceinline__ PredRegs load_pred(const DPredPacked& d) {
    PredRegs r;
    r.n = d.n;
    r.prog = d.prog;
#pragma unroll
    for (int a = 0; a < SGD_MAX_ATOMS; ++a) {
        r.code[a] = d.code[a];
        r.cbits[a] = d.cbits[a];
    }
    return r;
}

__device__ __forceinline__ uint64_t load_col(const void* base, uint32_t type, uint32_t i) {
    switch (type) {
    case SG_T_LONG: case SG_T_DOUBLE: return ((const uint64_t*)base)[i];
    case SG_T_BOOL: return ((const uint8_t*)base)[i] ? 1u : 0u;
    default: return ((const uint32_t*)base)[i];
    }
}

__device__ __forceinline__ int wave_max(int x) {
    for (int off = 32; off > 0; off >>= 1) x = max(x, __shfl_xor(x, off, SGD_WAVE));
    return x;
}
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, SGD_WAVE);
    return x;
}
// inclusive prefix sum over the wave (all 64 lanes must be active)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
    for (int off = 1; off < SGD_WAVE; off <<= 1) {
        uint32_t y = __shfl_up(x, off, SGD_WAVE);
        if (lane >= off) x += y;
    }
    return x;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// segment bounds of the key-sorted batch: seg_begin[k], seg_end[k]
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_seg_bounds(const uint32_t* __restrict__ skeys, uint32_t n,
                                                    uint32_t n_keys, uint32_t* __restrict__ seg_begin,
                                                    uint32_t* __restrict__ seg_end, uint32_t* __restrict__ err) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k = skeys[i];
    if (k >= n_keys) {  // key id outside [0, n_keys): reject the batch loudly, never write out of bounds
        atomicOr(err, (uint32_t)SGD_ERR_KEY_RANGE);
        return;
    }
    if (i == 0 || skeys[i - 1] != k) seg_begin[k] = i;
    if (i == n - 1 || skeys[i + 1] != k) seg_end[k] = i + 1;
}

// ------------------------------------------------------------------------------------------------
// the NFA advance: one lane per key, events of the key in arrival order
//
// A workgroup owns SGD_BLOCK consecutive keys; in the key-sorted batch their events form one
// contiguous range, which the workgroup stages into LDS in chunks (one coalesced index read plus a
// wide gather of the timestamp and the filter columns, all issued before any lane starts walking its
// key), so the per-event serial work of a lane reads LDS, not HBM.  Partial matches stay in the HBM
// slabs (partial j of key k at j*K+k: every wave access to partial j is one coalesced line).
// ------------------------------------------------------------------------------------------------
// One lane's partial-match list.  During a batch it lives in an LDS window of R slots (the common
// case: a key rarely holds more than a handful of live partials) or, when it outgrows the window, in
// the HBM slab; both are addressed through flat pointers and strides so one code path serves both.
// One lane's partial-match list.  During a batch it lives in an LDS window of R slots per lane
// (the common case: a key rarely holds more than a handful of live partials) or, once it outgrows
// the window, in the HBM slab.  The two are separate types so that every access compiles to ds_* or
// global_* instructions (never flat, whose waits would serialise LDS and memory traffic).
struct LdsList {
    int64_t* ts;
    uint64_t* seq;
    uint32_t* cap;
    uint32_t* nul;
    uint32_t ws;  // words between capture planes
    __device__ __forceinline__ int64_t& TS(uint32_t j) const { return ts[j * SGD_BLOCK]; }
    __device__ __forceinline__ uint64_t& SEQ(uint32_t j) const { return seq[j * SGD_BLOCK]; }
    __device__ __forceinline__ uint32_t& CAP(uint32_t w, uint32_t j) const { return cap[w * ws + j * SGD_BLOCK]; }
    __device__ __forceinline__ uint32_t& NUL(uint32_t j) const { return nul[j * SGD_BLOCK]; }
};
struct GlbList {
    int64_t* ts;
    uint64_t* seq;
    uint32_t* cap;
    uint32_t* nul;
    uint32_t s;   // n_keys
    size_t ws;    // cap * n_keys
    __device__ __forceinline__ int64_t& TS(uint32_t j) const { return ts[(size_t)j * s]; }
    __device__ __forceinline__ uint64_t& SEQ(uint32_t j) const { return seq[(size_t)j * s]; }
    __device__ __forceinline__ uint32_t& CAP(uint32_t w, uint32_t j) const { return cap[w * ws + (size_t)j * s]; }
    __device__ __forceinline__ uint32_t& NUL(uint32_t j) const { return nul[(size_t)j * s]; }
};

template <class D, class S>
__device__ __forceinline__ void pl_copy(const D& d, const S& src, uint32_t n, uint32_t n_capw, bool nullable) {
    for (uint32_t j = 0; j < n; ++j) {
        d.TS(j) = src.TS(j);
        d.SEQ(j) = src.SEQ(j);
        for (uint32_t w = 0; w < n_capw; ++w) d.CAP(w, j) = src.CAP(w, j);
        if (nullable) d.NUL(j) = src.NUL(j);
    }
}
template <class L>
__device__ __forceinline__ void pl_move(const L& l, uint32_t n_capw, bool nullable, uint32_t dst, uint32_t src) {
    l.TS(dst) = l.TS(src);
    l.SEQ(dst) = l.SEQ(src);
    for (uint32_t w = 0; w < n_capw; ++w) l.CAP(w, dst) = l.CAP(w, src);
    if (nullable) l.NUL(dst) = l.NUL(src);
}

template <class L>
struct PartRef {  // capture accessor of partial j
    const L& l;
    uint32_t j;
    uint32_t cn;
    uint64_t wide;   // bit c: capture c is 64-bit
    uint64_t words;  // byte c: first word of capture c
    __device__ __forceinline__ DVal operator()(int c) const {
        const uint32_t w = (uint32_t)(words >> (8 * c)) & 0xffu;
        uint64_t b = l.CAP(w, j);
        if ((wide >> c) & 1u) b |= (uint64_t)l.CAP(w + 1, j) << 32;
        return DVal{b, (cn >> c) & 1u};
    }
};

__device__ __forceinline__ bool expired(int64_t pts, int64_t now, int64_t within) {
    const int64_t d = pts - now;  // StreamPreStateProcessor.isExpired: |slot0.ts - now| > within
    return (d < 0 ? -d : d) > within;
}

// per-lane NFA state of one key during a batch
struct KeySt {
    uint32_t npend, nstg, spend, sstg;
    unsigned long long scanned, created, matches;
};

// stabilize (expire + promote) for one event: StreamPreStateProcessor.expireEvents :325-361 and
// updateState :308-323, in receiver order (PatternMulti/SingleProcessStreamReceiver.stabilizeStates)
template <class L>
__device__ __forceinline__ void stabilize(const P2Params& p, const L& l, KeySt& s, int64_t ts, bool upd0, bool upd1,
                                          uint32_t ncw, bool nullable) {
    if (p.within >= 0 && (s.npend + s.nstg) > 0) {
        uint32_t pre = 0;
        while (pre < s.npend && expired(l.TS(pre), ts, p.within)) pre++;
        bool stg_exp = false;
        for (uint32_t r = s.npend; r < s.npend + s.nstg; ++r) stg_exp |= expired(l.TS(r), ts, p.within);
        if (pre > 0 || stg_exp) {
            uint32_t w = 0, stg_drop = 0;
            const uint32_t end = s.npend + s.nstg;
            for (uint32_t r = pre; r < end; ++r) {
                if (r >= s.npend && expired(l.TS(r), ts, p.within)) { stg_drop++; continue; }
                if (w != r) pl_move(l, ncw, nullable, w, r);
                w++;
            }
            s.npend -= pre;
            s.nstg -= stg_drop;
            if (p.mode & SGD_P2_EVERY_BOTH) {
                // withinEveryPreStateProcessor.addEveryState(expired) + updateState()
                s.spend += s.sstg + 1;
                s.sstg = 0;
                s.created++;
            }
        }
    }
    if (upd0) { s.spend += s.sstg; s.sstg = 0; }
    if (upd1 && s.nstg > 0) {
        // stable insertion sort of the staged region by ts (eventTimeComparator: -1 sorts last)
        for (uint32_t r = s.npend + 1; r < s.npend + s.nstg; ++r) {
            const int64_t kt = l.TS(r);
            const int64_t pt = l.TS(r - 1);
            if (!((kt != -1) && (pt == -1 || kt < pt))) continue;
            const uint64_t ks = l.SEQ(r);
            const uint32_t kn = nullable ? l.NUL(r) : 0u;
            uint32_t kw[2 * SGD_MAX_CAPS];
#pragma unroll
            for (int w = 0; w < 2 * SGD_MAX_CAPS; ++w) kw[w] = (w < (int)ncw) ? l.CAP(w, r) : 0u;
            uint32_t q = r;
            while (q > s.npend) {
                const int64_t qt = l.TS(q - 1);
                if (!((kt != -1) && (qt == -1 || kt < qt))) break;
                pl_move(l, ncw, nullable, q, q - 1);
                q--;
            }
            l.TS(q) = kt;
            l.SEQ(q) = ks;
#pragma unroll
            for (int w = 0; w < 2 * SGD_MAX_CAPS; ++w)
                if (w < (int)ncw) l.CAP(w, q) = kw[w];
            if (nullable) l.NUL(q) = kn;
        }
        s.npend += s.nstg;
        s.nstg = 0;
    }
}

// e2's filter over the pending partials: count and the hit bits of the first 64
template <bool PROG, class L>
__device__ __forceinline__ uint32_t scan1(const P2Params& p, const PredRegs& P1, const L& l, const KeySt& s,
                                          const EvRegs& ev, bool nullable, uint64_t wide, uint64_t words,
                                          uint64_t& mask) {
    uint32_t c = 0;
    mask = 0;
    for (uint32_t j = 0; j < s.npend; ++j) {
        PartRef<L> caps{l, j, nullable ? l.NUL(j) : 0u, wide, words};
        if (eval_pred<PROG>(P1, p.f1g, p.n_caps, ev, caps)) {
            if (j < 64) mask |= 1ull << j;
            c++;
        }
    }
    return c;
}

// emit the matches of one event (raw[pos ..]) and compact the survivors, pending-list order
template <bool PROG, class L>
__device__ __forceinline__ void emit1(const P2Params& p, const PredRegs& P1, const L& l, KeySt& s, const EvRegs& ev,
                                      uint64_t mask,
                                      unsigned long long pos, uint32_t ncw, bool nullable, uint64_t wide,
                                      uint64_t words) {
    uint32_t w1 = 0;
    for (uint32_t j = 0; j < s.npend; ++j) {
        bool hit;
        if (j < 64) {
            hit = (mask >> j) & 1ull;
        } else {  // rare: more than 64 pending partials, re-evaluate
            PartRef<L> caps{l, j, nullable ? l.NUL(j) : 0u, wide, words};
            hit = eval_pred<PROG>(P1, p.f1g, p.n_caps, ev, caps);
        }
        if (hit) {
            if (pos < p.raw_capacity && !(p.dbg & 256)) p.raw_e1[pos] = l.SEQ(j);
            pos++;
            if (p.mode & SGD_P2_EVERY_BOTH) s.sstg++;  // post1 -> pre0.addEveryState
        } else {
            if (w1 != j) pl_move(l, ncw, nullable, w1, j);
            w1++;
        }
    }
    s.npend = w1;
}

// post0 for `cnt` seeds: append a partial (slot0 = this event) to e2's staged list
template <class L>
__device__ __forceinline__ void append0(const P2Params& p, const L& l, uint32_t j, int64_t ts, uint64_t seq,
                                        const EvRegs& ev, uint64_t wide, bool nullable) {
    l.TS(j) = ts;
    l.SEQ(j) = seq;
    uint32_t cn = 0;
    for (uint32_t c = 0; c < p.n_caps; ++c) {
        const DVal v = ev.get(p.cap_col[c]);
        const uint32_t w = p.cap_word[c];
        l.CAP(w, j) = (uint32_t)v.b;
        if ((wide >> c) & 1u) l.CAP(w + 1, j) = (uint32_t)(v.b >> 32);
        cn |= v.null << c;
    }
    if (nullable) l.NUL(j) = cn;
}

template <bool PROG>
__global__ void __launch_bounds__(SGD_BLOCK) k_p2_advance(const P2Params p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint32_t s_rb, s_re;
    const int lane = threadIdx.x & (SGD_WAVE - 1);
    const uint32_t k = blockIdx.x * SGD_BLOCK + threadIdx.x;
    const bool valid = k < p.n_keys;
    const uint32_t K = p.n_keys;
    const uint32_t CH = p.chunk;
    const uint32_t R = p.lds_slots;
    // LDS: the partial windows (SoA, lane-minor: conflict-free), then the staged events (AoS in the
    // payload layout [idx][cols..][ts(2)] (+ [null bits] in gather mode), SS words each)
    const uint32_t SS = p.lds_stride;
    int64_t* w_ts = (int64_t*)smem;                                   // [R][BLOCK]
    uint64_t* w_seq = (uint64_t*)(w_ts + (size_t)R * SGD_BLOCK);      // [R][BLOCK]
    uint32_t* w_cap = (uint32_t*)(w_seq + (size_t)R * SGD_BLOCK);     // [n_capw][R][BLOCK]
    uint32_t* w_nul = w_cap + (size_t)p.n_capw * R * SGD_BLOCK;       // [R][BLOCK]
    uint32_t* l_ev = w_nul + (size_t)R * SGD_BLOCK;                   // [CH][SS], 8-byte aligned

    uint32_t b = 0, e = 0, h = 0;
    if (valid) {
        b = p.seg_begin[k];
        e = p.seg_end[k];
        if (e > b) h = p.hdr[k];
    }
    if (threadIdx.x == 0) { s_rb = 0xffffffffu; s_re = 0; }
    __syncthreads();
    if (e > b) { atomicMin(&s_rb, b); atomicMax(&s_re, e); }
    __syncthreads();
    const uint32_t rb = s_rb, re = s_re;
    if (rb >= re) return;  // no key of this workgroup has an event in the batch (block-uniform)
    const uint32_t dbg = p.dbg;  // ablation switches for profiling (0 in production)
    if (dbg & 16) return;
    uint64_t tsec[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tmark = __builtin_amdgcn_s_memtime();
#define SGD_STAMP(i)                                                      \
    do {                                                                  \
        if (dbg & 64) {                                                   \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();           \
            tsec[i] += now_ - tmark;                                      \
            tmark = now_;                                                 \
        }                                                                 \
    } while (0)

    const int nev = (int)(e - b);
    KeySt s{SGD_H_NPEND(h), SGD_H_NSTG(h), SGD_H_SPEND(h), SGD_H_SSTG(h), 0, 0, 0};
    if (nev > 0 && !SGD_H_INIT(h)) s.sstg = 1;  // PartitionRuntimeImpl.initPartition -> init(): one seed
    const unsigned long long st_live0 = (nev > 0) ? (unsigned long long)(s.npend + s.nstg) : 0ull;
    bool overflow = false;
    const bool upd0 = p.multi || p.is_s0;
    const bool upd1 = p.multi || p.is_s1;
    const bool nullable = p.nullable != 0;
    const uint32_t ncw = p.n_capw;
    uint64_t wide = 0, words = 0;
#pragma unroll
    for (int c = 0; c < SGD_MAX_CAPS; ++c) {
        words |= (uint64_t)p.cap_word[c] << (8 * c);
        if (p.cap_type[c] == SG_T_LONG || p.cap_type[c] == SG_T_DOUBLE) wide |= 1ull << c;
    }
    const PredRegs P0 = load_pred(p.q0), P1 = load_pred(p.q1);  // filters, once, into registers
    unsigned long long chunk_base = 0;  // this wave's reserved slots of the raw match buffer
    uint32_t chunk_left = 0;

    const GlbList G{p.p_ts + k, p.p_seq + k, p.p_capw + k, p.p_capnull + k, K, (size_t)p.cap * K};
    const LdsList W{w_ts + threadIdx.x, w_seq + threadIdx.x, w_cap + threadIdx.x, w_nul + threadIdx.x,
                    R * SGD_BLOCK};
    bool in_lds = (s.npend + s.nstg) <= R;
    if (nev > 0 && in_lds && !(dbg & 32)) pl_copy(W, G, s.npend + s.nstg, ncw, nullable);  // load the window
    uint32_t limit = in_lds ? R : p.cap;
    SGD_STAMP(0);

    for (uint32_t cb = rb; cb < re; cb += CH) {
        const uint32_t ce = min(re, cb + CH);
        // ---- stage the chunk's events in LDS ----
        if (p.payload) {
            // the batch is key-sorted WITH its payload: the chunk is one contiguous byte range, copied
            // 8 bytes per lane with SGD_STAGE_UNROLL loads in flight per lane before any LDS write
            const uint2* src = (const uint2*)(p.payload + (size_t)cb * SS);
            uint2* dst = (uint2*)l_ev;
            const uint32_t n8 = (ce - cb) * (SS / 2);
            for (uint32_t base = 0; base < n8; base += SGD_BLOCK * SGD_STAGE_UNROLL) {
                uint2 v[SGD_STAGE_UNROLL];
#pragma unroll
                for (int u = 0; u < SGD_STAGE_UNROLL; ++u) {
                    const uint32_t q = base + u * SGD_BLOCK + threadIdx.x;
                    if (q < n8) v[u] = src[q];
                }
#pragma unroll
                for (int u = 0; u < SGD_STAGE_UNROLL; ++u) {
                    const uint32_t q = base + u * SGD_BLOCK + threadIdx.x;
                    if (q < n8) dst[q] = v[u];
                }
            }
        } else {
            for (uint32_t t = threadIdx.x; t < ce - cb && !(dbg & 8); t += SGD_BLOCK) {
                uint32_t* d = l_ev + (size_t)t * SS;
                const uint32_t i = p.sorted_idx[cb + t];
                d[0] = i;
                *(int64_t*)(d + p.pay_stride - 2) = p.ts[i];
                uint32_t nb = 0;
#pragma unroll
                for (int c = 0; c < SGD_MAX_EVCOLS; ++c) {
                    if (c < (int)p.n_evcols) {
                        const uint32_t w = 1 + p.ev_word[c];
                        const uint32_t ty = p.evtype[c];
                        if (ty == SG_T_LONG || ty == SG_T_DOUBLE) {
                            const uint64_t v = ((const uint64_t*)p.evcol[c])[i];
                            d[w] = (uint32_t)v;
                            d[w + 1] = (uint32_t)(v >> 32);
                        } else if (ty == SG_T_BOOL) {
                            d[w] = ((const uint8_t*)p.evcol[c])[i] ? 1u : 0u;
                        } else {
                            d[w] = ((const uint32_t*)p.evcol[c])[i];
                        }
                        if (p.any_null && p.evnull[c]) nb |= (uint32_t)(p.evnull[c][i] != 0) << c;
                    }
                }
                if (SS > p.pay_stride) d[p.pay_stride] = nb;
            }
        }
        SGD_STAMP(1);
        __syncthreads();
        SGD_STAMP(2);

        const uint32_t lo = max(b, cb), hi = min(e, ce);
        const int cnt = (hi > lo) ? (int)(hi - lo) : 0;
        const int iters = wave_max(cnt);
        for (int it = 0; it < iters; ++it) {
            const bool act = it < cnt;
            const uint32_t t = lo - cb + (uint32_t)it;
            int64_t ts = 0;
            uint64_t seq = 0;
            EvRegs ev;
            if (act) {
                const uint32_t* d = l_ev + (size_t)t * SS;
                ts = *(const int64_t*)(d + p.pay_stride - 2);
                seq = p.seq_base + d[0];
                const uint32_t nb = (SS > p.pay_stride) ? d[p.pay_stride] : 0u;
#pragma unroll
                for (int c = 0; c < SGD_MAX_EVCOLS; ++c) {
                    if (c < (int)p.n_evcols) {
                        const uint32_t w = 1 + p.ev_word[c];
                        uint64_t v = d[w];
                        const uint32_t ty = p.evtype[c];
                        if (ty == SG_T_LONG || ty == SG_T_DOUBLE) v |= (uint64_t)d[w + 1] << 32;
                        ev.set(c, DVal{v, (nb >> c) & 1u});
                    }
                }
                SGD_STAMP(3);
                if (!(dbg & 1)) {
                    if (in_lds) stabilize(p, W, s, ts, upd0, upd1, ncw, nullable);
                    else stabilize(p, G, s, ts, upd0, upd1, ncw, nullable);
                }
            }
            SGD_STAMP(4);
            // ---- state 1 first (reverse state order, PatternMultiProcessStreamReceiver.java:31-40) ----
            uint64_t mask = 0;
            uint32_t c1 = 0;
            if (act && p.is_s1 && !(dbg & 2)) {
                c1 = in_lds ? scan1<PROG>(p, P1, W, s, ev, nullable, wide, words, mask)
                            : scan1<PROG>(p, P1, G, s, ev, nullable, wide, words, mask);
                s.scanned += s.npend;
            }
            SGD_STAMP(5);
            // wave-wide reservation of the emitted matches (one atomic per wave chunk of slots)
            const uint32_t incl = wave_incl_scan(c1, lane);
            const uint32_t total = __shfl(incl, SGD_WAVE - 1, SGD_WAVE);
            if (total) {
                if (total > chunk_left) {
                    const uint32_t want = max(total, (uint32_t)SGD_RAW_CHUNK);
                    unsigned long long nb = 0;
                    if (lane == 0) nb = atomicAdd(p.raw_count, (unsigned long long)want);
                    chunk_base = __shfl(nb, 0, SGD_WAVE);
                    chunk_left = want;
                }
                if (c1) {
                    const unsigned long long pos = chunk_base + incl - c1;
                    if (dbg & 128) {
                    } else if (pos + c1 <= p.raw_capacity) {
                        const uint32_t bi = l_ev[(size_t)t * SS];  // batch position of the trigger
                        p.t_cnt[bi] = c1;
                        p.t_first[bi] = (uint32_t)pos;
                    } else {
                        atomicOr(p.err, (uint32_t)SGD_ERR_MATCH_CAP);
                    }
                    if (in_lds) emit1<PROG>(p, P1, W, s, ev, mask, pos, ncw, nullable, wide, words);
                    else emit1<PROG>(p, P1, G, s, ev, mask, pos, ncw, nullable, wide, words);
                    s.matches += c1;
                }
                chunk_base += total;
                chunk_left -= total;
            }
            SGD_STAMP(6);
            // ---- state 0: the start-state seeds ----
            if (act && p.is_s0 && s.spend > 0 && !(dbg & 4)) {
                s.scanned += s.spend;
                auto nocap = [](int) -> DVal { return DVal{0, 1}; };
                if (eval_pred<PROG>(P0, p.f0g, 0, ev, nocap)) {
                    // post0: partial (slot0 = this event, ts = its ts) -> pre1.addState (staged);
                    // every e1: pre0.addEveryState (a new seed, staged)
                    for (uint32_t q = 0; q < s.spend; ++q) {
                        const uint32_t j = s.npend + s.nstg;
                        if (j >= limit && in_lds) {  // the window is full: move the list to HBM
                            pl_copy(G, W, j, ncw, nullable);
                            in_lds = false;
                            limit = p.cap;
                        }
                        if (j >= limit) { overflow = true; break; }
                        if (in_lds) append0(p, W, j, ts, seq, ev, wide, nullable);
                        else append0(p, G, j, ts, seq, ev, wide, nullable);
                        s.nstg++;
                        s.created++;
                    }
                    if (p.mode & SGD_P2_EVERY_FIRST) s.sstg += s.spend;
                    s.spend = 0;
                }
            }
            SGD_STAMP(7);
        }
        __syncthreads();  // the next chunk overwrites the LDS staging area
    }
    if (nev > 0) {
        if (in_lds && !(dbg & 32)) pl_copy(G, W, s.npend + s.nstg, ncw, nullable);  // write the window back
        if (s.sstg > 3 || s.spend > 3) overflow = true;
        p.hdr[k] = SGD_H_MAKE(s.npend, s.nstg, min(s.spend, 3u), min(s.sstg, 3u), 1);
    }
    if (overflow) atomicOr(p.err, (uint32_t)SGD_ERR_PARTIAL_CAP);
    if ((dbg & 64) && lane == 0 && p.dbg_out) {
        const uint32_t wv = (blockIdx.x * SGD_BLOCK + threadIdx.x) / SGD_WAVE;
#pragma unroll
        for (int i = 0; i < 8; ++i) p.dbg_out[(size_t)wv * 8 + i] = tsec[i];
    }
    // exact work counters (wave-reduced, one atomic per wave and counter)
    const unsigned long long v0 = wave_sum(s.scanned), v1 = wave_sum(s.created), v2 = wave_sum(s.matches);
    const unsigned long long v3 = wave_sum(nev > 0 ? 1ull : 0ull), v4 = wave_sum(st_live0);
    if (lane == 0) {
        if (v0) atomicAdd(&p.stats[SGD_ST_SCANNED], v0);
        if (v1) atomicAdd(&p.stats[SGD_ST_CREATED], v1);
        if (v2) atomicAdd(&p.stats[SGD_ST_MATCHES], v2);
        if (v3) atomicAdd(&p.stats[SGD_ST_KEYS], v3);
        if (v4) atomicAdd(&p.stats[SGD_ST_LIVE0], v4);
    }
}

// ------------------------------------------------------------------------------------------------
// match ordering: batch event t's matches go to out_count + t_off[t] (t_off = exclusive scan of
// t_cnt), i.e. ascending trigger seq, then emission order — the reference's callback order
// (MultiProcessStreamReceiver.java:119-121).  Resets t_cnt for the next batch.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_scatter(const ScatterParams s) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= s.n) return;
    const uint32_t c = s.t_cnt[t];
    const uint64_t base = *s.out_count;
    if (t == s.n - 1) *s.batch_total = (unsigned long long)s.t_off[t] + c;
    if (c == 0) return;
    s.t_cnt[t] = 0;
    const uint64_t o = base + s.t_off[t];
    const uint32_t f = s.t_first[t];
    const uint64_t trig = s.seq_base + t;
    const uint32_t key = s.key ? s.key[t] : 0u;
    const int64_t ts = s.ts[t];
    if (o + c > s.capacity) {
        atomicOr(s.err, (uint32_t)SGD_ERR_MATCH_CAP);
        return;
    }
    for (uint32_t r = 0; r < c; ++r) {
        const uint64_t d = o + r;
        s.o_trig[d] = trig;
        s.o_slot[2 * d] = s.raw_e1[f + r];
        s.o_slot[2 * d + 1] = trig;
        s.o_key[d] = key;
        s.o_ts[d] = ts;  // StreamPostStateProcessor.java:68: StateEvent ts = ts of the e2 event
        s.o_len[2 * d] = 1;
        s.o_len[2 * d + 1] = 1;
    }
}

__global__ void k_bump(unsigned long long* out_count, const unsigned long long* batch_total) {
    *out_count += *batch_total;
}

// ------------------------------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------------------------------
int sgd_launch_bounds(const uint32_t* skeys, uint32_t n, uint32_t n_keys, uint32_t* seg_begin, uint32_t* seg_end,
                      uint32_t* err, ihipStream_t* stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_seg_bounds, dim3((n + 255) / 256), dim3(256), 0, stream, skeys, n, n_keys, seg_begin,
                       seg_end, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t sgd_p2_lds_bytes(const P2Params& p) {
    return (size_t)p.chunk * 4 * p.lds_stride + (size_t)p.lds_slots * SGD_BLOCK * (16 + 4 * p.n_capw + 4);
}

int sgd_launch_p2(const P2Params& p, ihipStream_t* stream) {
    const uint32_t blocks = (p.n_keys + SGD_BLOCK - 1) / SGD_BLOCK;
    const size_t lds = sgd_p2_lds_bytes(p);
    if (p.q0.prog || p.q1.prog)
        hipLaunchKernelGGL(k_p2_advance<true>, dim3(blocks), dim3(SGD_BLOCK), lds, stream, p);
    else
        hipLaunchKernelGGL(k_p2_advance<false>, dim3(blocks), dim3(SGD_BLOCK), lds, stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_scatter(const ScatterParams& s, ihipStream_t* stream) {
    if (s.n == 0) return 0;
    hipLaunchKernelGGL(k_scatter, dim3((s.n + 255) / 256), dim3(256), 0, stream, s);
    hipLaunchKernelGGL(k_bump, dim3(1), dim3(1), 0, stream, s.out_count, s.batch_total);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
