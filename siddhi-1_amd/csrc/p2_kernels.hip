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

struct EvRegs {  // the current event's columns used by the filters
    DVal c[SGD_MAX_EVCOLS];
    __device__ __forceinline__ DVal get(int i) const {
        switch (i) {
        case 0: return c[0]; case 1: return c[1]; case 2: return c[2]; case 3: return c[3];
        case 4: return c[4]; case 5: return c[5]; case 6: return c[6]; default: return c[7];
        }
    }
};

// evaluate a filter program; caps(i) fetches capture i of the partial (slot-0 event)
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
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_p2_advance(P2Params p) {
    const int lane = threadIdx.x & (SGD_WAVE - 1);
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = k < p.n_keys;
    const uint32_t K = p.n_keys;

    uint32_t b = 0, e = 0, h = 0;
    if (valid) {
        b = p.seg_begin[k];
        e = p.seg_end[k];
        if (e > b) h = p.hdr[k];
    }
    const int nev = (int)(e - b);
    uint32_t npend = SGD_H_NPEND(h), nstg = SGD_H_NSTG(h), spend = SGD_H_SPEND(h), sstg = SGD_H_SSTG(h);
    if (nev > 0 && !SGD_H_INIT(h)) {
        // PartitionRuntimeImpl.initPartition -> StreamPreStateProcessor.init: one start-state seed
        sstg = 1;
    }
    unsigned long long st_scanned = 0, st_created = 0, st_matches = 0;
    unsigned long long st_live0 = (nev > 0) ? (unsigned long long)(npend + nstg) : 0ull;
    bool overflow = false;

    const int iters = wave_max(nev);
    for (int it = 0; it < iters; ++it) {
        const bool act = it < nev;
        int64_t ts = 0;
        uint64_t seq = 0;
        EvRegs ev;
        if (act) {
            const uint32_t i = p.sorted_idx[b + it];
            ts = p.ts[i];
            seq = p.seq_base + i;
            for (uint32_t c = 0; c < p.n_evcols; ++c) {
                ev.c[c].b = load_col(p.evcol[c], p.evtype[c], i);
                ev.c[c].null = p.evnull[c] ? p.evnull[c][i] : 0u;
            }
            // ---- stabilize: expire (StreamPreStateProcessor.expireEvents) ----
            if (p.within >= 0 && (npend + nstg) > 0) {
                uint32_t pre = 0;
                while (pre < npend) {
                    int64_t d = p.p_ts[(size_t)pre * K + k] - ts;
                    if ((d < 0 ? -d : d) > p.within) pre++;
                    else break;
                }
                uint32_t w = 0, nexp = pre, stg_drop = 0;
                const uint32_t end = npend + nstg;
                for (uint32_t r = pre; r < end; ++r) {
                    const size_t src = (size_t)r * K + k;
                    if (r >= npend) {
                        int64_t d = p.p_ts[src] - ts;
                        if ((d < 0 ? -d : d) > p.within) {
                            nexp++;
                            stg_drop++;
                            continue;
                        }
                    }
                    if (w != r) {
                        const size_t dst = (size_t)w * K + k;
                        p.p_ts[dst] = p.p_ts[src];
                        p.p_seq[dst] = p.p_seq[src];
                        for (uint32_t c = 0; c < p.n_caps; ++c)
                            p.p_cap[(size_t)c * p.cap * K + dst] = p.p_cap[(size_t)c * p.cap * K + src];
                        if (p.nullable) p.p_capnull[dst] = p.p_capnull[src];
                    }
                    w++;
                }
                nstg -= stg_drop;
                npend -= pre;
                if (nexp > 0 && (p.mode & SGD_P2_EVERY_BOTH)) {
                    // withinEveryPreStateProcessor.addEveryState(expired) + updateState()
                    spend += sstg + 1;
                    sstg = 0;
                    st_created++;
                }
            }
            // ---- stabilize: promote staged (updateState) ----
            const bool upd0 = p.multi || p.is_s0;
            const bool upd1 = p.multi || p.is_s1;
            if (upd0) { spend += sstg; sstg = 0; }
            if (upd1 && nstg > 0) {
                // stable insertion sort of the staged region by ts (eventTimeComparator, -1 last)
                for (uint32_t r = npend + 1; r < npend + nstg; ++r) {
                    const size_t ir = (size_t)r * K + k;
                    int64_t kt = p.p_ts[ir];
                    int64_t pt = p.p_ts[ir - K];
                    bool before = (kt != -1) && (pt == -1 || kt < pt);
                    if (!before) continue;
                    uint64_t ks = p.p_seq[ir];
                    uint64_t kc[SGD_MAX_CAPS];
                    for (uint32_t c = 0; c < p.n_caps; ++c) kc[c] = p.p_cap[(size_t)c * p.cap * K + ir];
                    uint32_t kn = p.nullable ? p.p_capnull[ir] : 0u;
                    uint32_t q = r;
                    while (q > npend) {
                        const size_t iq = (size_t)(q - 1) * K + k;
                        int64_t qt = p.p_ts[iq];
                        if (!((kt != -1) && (qt == -1 || kt < qt))) break;
                        const size_t dq = (size_t)q * K + k;
                        p.p_ts[dq] = qt;
                        p.p_seq[dq] = p.p_seq[iq];
                        for (uint32_t c = 0; c < p.n_caps; ++c)
                            p.p_cap[(size_t)c * p.cap * K + dq] = p.p_cap[(size_t)c * p.cap * K + iq];
                        if (p.nullable) p.p_capnull[dq] = p.p_capnull[iq];
                        q--;
                    }
                    const size_t dq = (size_t)q * K + k;
                    p.p_ts[dq] = kt;
                    p.p_seq[dq] = ks;
                    for (uint32_t c = 0; c < p.n_caps; ++c) p.p_cap[(size_t)c * p.cap * K + dq] = kc[c];
                    if (p.nullable) p.p_capnull[dq] = kn;
                }
                npend += nstg;
                nstg = 0;
            }
        }

        // ---- state 1 (evaluated first: reverse state order) in chunks of 64 partials ----
        const int nch = (act && p.is_s1) ? (int)((npend + 63) >> 6) : 0;
        const int wch = wave_max(nch);
        uint32_t w1 = 0;  // survivors written so far
        for (int ch = 0; ch < wch; ++ch) {
            uint64_t mask = 0;
            const uint32_t j0 = (uint32_t)ch << 6;
            uint32_t cnt = 0;
            if (ch < nch) {
                const uint32_t j1 = min(npend, j0 + 64);
                for (uint32_t j = j0; j < j1; ++j) {
                    const size_t ij = (size_t)j * K + k;
                    const uint32_t cn = p.nullable ? p.p_capnull[ij] : 0u;
                    auto caps = [&](int c) -> DVal {
                        return DVal{p.p_cap[(size_t)c * p.cap * K + ij], (cn >> c) & 1u};
                    };
                    if (eval_prog(p.f1, ev, caps)) mask |= 1ull << (j - j0);
                }
                st_scanned += j1 - j0;
                cnt = (uint32_t)__popcll(mask);
            }
            // wave-wide compaction of the emitted matches: one atomic per wave step
            const uint32_t incl = wave_incl_scan(cnt, lane);
            const uint32_t total = __shfl(incl, SGD_WAVE - 1, SGD_WAVE);
            unsigned long long base = 0;
            if (lane == SGD_WAVE - 1 && total) base = atomicAdd(p.m_count, (unsigned long long)total);
            base = __shfl(base, SGD_WAVE - 1, SGD_WAVE);
            if (ch < nch) {
                unsigned long long pos = base + incl - cnt;
                const uint32_t j1 = min(npend, j0 + 64);
                for (uint32_t j = j0; j < j1; ++j) {
                    const size_t ij = (size_t)j * K + k;
                    if ((mask >> (j - j0)) & 1ull) {
                        if (pos < p.m_capacity) {
                            p.m_trig[pos] = seq;
                            p.m_e1[pos] = p.p_seq[ij];
                            p.m_key[pos] = k;
                            p.m_ts[pos] = ts;  // StreamPostStateProcessor: StateEvent ts = e2 ts
                        } else {
                            atomicOr(p.err, (uint32_t)SGD_ERR_MATCH_CAP);
                        }
                        pos++;
                        st_matches++;
                        if (p.mode & SGD_P2_EVERY_BOTH) sstg++;  // post1 -> pre0.addEveryState
                    } else {
                        if (w1 != j) {
                            const size_t dst = (size_t)w1 * K + k;
                            p.p_ts[dst] = p.p_ts[ij];
                            p.p_seq[dst] = p.p_seq[ij];
                            for (uint32_t c = 0; c < p.n_caps; ++c)
                                p.p_cap[(size_t)c * p.cap * K + dst] = p.p_cap[(size_t)c * p.cap * K + ij];
                            if (p.nullable) p.p_capnull[dst] = p.p_capnull[ij];
                        }
                        w1++;
                    }
                }
            }
        }
        if (act && p.is_s1) npend = w1;

        // ---- state 0: the start-state seeds ----
        if (act && p.is_s0 && spend > 0) {
            st_scanned += spend;
            auto nocap = [&](int) -> DVal { return DVal{0, 1}; };
            if (eval_prog(p.f0, ev, nocap)) {
                // post0: partial (slot0 = this event, ts = event ts) -> pre1.addState (staged);
                // every e1: pre0.addEveryState (a new seed, staged)
                for (uint32_t s = 0; s < spend; ++s) {
                    const uint32_t j = npend + nstg;
                    if (j >= p.cap) { overflow = true; break; }
                    const size_t ij = (size_t)j * K + k;
                    p.p_ts[ij] = ts;
                    p.p_seq[ij] = seq;
                    uint32_t cn = 0;
                    for (uint32_t c = 0; c < p.n_caps; ++c) {
                        DVal v = ev.get(p.cap_col[c]);
                        p.p_cap[(size_t)c * p.cap * K + ij] = v.b;
                        cn |= v.null << c;
                    }
                    if (p.nullable) p.p_capnull[ij] = cn;
                    nstg++;
                    st_created++;
                }
                if (p.mode & SGD_P2_EVERY_FIRST) sstg += spend;
                spend = 0;
            }
        }
    }
    if (nev > 0) {
        if (sstg > 3 || spend > 3) overflow = true;
        p.hdr[k] = SGD_H_MAKE(npend, nstg, min(spend, 3u), min(sstg, 3u), 1);
    }
    if (overflow) atomicOr(p.err, (uint32_t)SGD_ERR_PARTIAL_CAP);
    // exact work counters (wave-reduced, one atomic per wave and counter)
    unsigned long long v0 = wave_sum(st_scanned), v1 = wave_sum(st_created), v2 = wave_sum(st_matches);
    unsigned long long v3 = wave_sum(nev > 0 ? 1ull : 0ull), v4 = wave_sum(st_live0);
    if (lane == 0) {
        if (v0) atomicAdd(&p.stats[SGD_ST_SCANNED], v0);
        if (v1) atomicAdd(&p.stats[SGD_ST_CREATED], v1);
        if (v2) atomicAdd(&p.stats[SGD_ST_MATCHES], v2);
        if (v3) atomicAdd(&p.stats[SGD_ST_KEYS], v3);
        if (v4) atomicAdd(&p.stats[SGD_ST_LIVE0], v4);
    }
}

// ------------------------------------------------------------------------------------------------
// match ordering: gather the (trigger, emission)-ordered permutation into the output layout
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_rel_keys(const uint64_t* __restrict__ trig, uint64_t base, uint64_t n,
                                                  uint32_t* __restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)(trig[i] - base);
}

__global__ void __launch_bounds__(256) k_order(const uint64_t* __restrict__ trig, const uint64_t* __restrict__ e1,
                                               const uint32_t* __restrict__ key, const int64_t* __restrict__ ts,
                                               const uint32_t* __restrict__ perm, uint64_t n,
                                               uint64_t* __restrict__ o_trig, uint64_t* __restrict__ o_slot,
                                               uint32_t* __restrict__ o_key, int64_t* __restrict__ o_ts,
                                               uint32_t* __restrict__ o_len) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t s = perm ? perm[i] : (uint32_t)i;
    uint64_t t = trig[s];
    o_trig[i] = t;
    o_slot[2 * i] = e1[s];
    o_slot[2 * i + 1] = t;
    o_key[i] = key[s];
    o_ts[i] = ts[s];
    o_len[2 * i] = 1;
    o_len[2 * i + 1] = 1;
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

int sgd_launch_p2(const P2Params& p, ihipStream_t* stream) {
    uint32_t blocks = (p.n_keys + 255) / 256;
    hipLaunchKernelGGL(k_p2_advance, dim3(blocks), dim3(256), 0, stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_rel_keys(const uint64_t* trig, uint64_t base, uint64_t n, uint32_t* out, ihipStream_t* stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_rel_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, trig, base, n, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_order(const uint64_t* trig, const uint64_t* e1, const uint32_t* key, const int64_t* ts,
                     const uint32_t* perm, uint64_t n, uint64_t* o_trig, uint64_t* o_slot, uint32_t* o_key,
                     int64_t* o_ts, uint32_t* o_len, ihipStream_t* stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_order, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, trig, e1, key, ts, perm, n,
                       o_trig, o_slot, o_key, o_ts, o_len);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
