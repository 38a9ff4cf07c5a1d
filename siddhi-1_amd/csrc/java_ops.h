// java_ops.h — Java value semantics of the expression bytecode (include/siddhi_gpu_ir.h) on the device,
// shared by the general engine's filters and selector (gen_kernels.hip) and the two-state engine's
// on-device projection (p2_kernels.hip).  Restated from (paths under
// /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/):
//   executor/condition/compare/**       null operand -> false (!= -> true), promotion per compare domain
//   executor/math/**                    null in -> null, x/0 and x%0 -> null, int/long wrap, no FMA
//   executor/condition/{And,Or,Not,IsNull}ConditionExpressionExecutor.java
//   executor/function/IfThenElseFunctionExecutor.java
//   util/parser/ExpressionParser.java   widening conversions (JLS 5.1.2)
#pragma once

#include <stdint.h>

struct GVal {
    uint64_t b;  // value bits (int / float / string id / bool in the low 32 bits)
    bool null;
};

// instruction length in words (siddhi_gpu_ir.h)
__device__ __forceinline__ uint32_t op_len(uint32_t op) {
    op &= 0xffu;
    return (op == SG_OP_VAR || op == SG_OP_CONST) ? 3u : (op == SG_OP_ISNULL_EV ? 2u : 1u);
}

__device__ __forceinline__ float gf32(uint64_t b) { return __uint_as_float((uint32_t)b); }
__device__ __forceinline__ double gf64(uint64_t b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ uint64_t gbf32(float f) { return (uint64_t)__float_as_uint(f); }
__device__ __forceinline__ uint64_t gbf64(double d) { return (uint64_t)__double_as_longlong(d); }

__device__ __forceinline__ GVal jo_cvt(GVal v, int from, int to) {
    if (v.null) return v;
    if (from == SG_T_INT) {
        const int32_t x = (int32_t)(uint32_t)v.b;
        if (to == SG_T_LONG) return {(uint64_t)(int64_t)x, false};
        if (to == SG_T_FLOAT) return {gbf32((float)x), false};
        if (to == SG_T_DOUBLE) return {gbf64((double)x), false};
    } else if (from == SG_T_LONG) {
        const int64_t x = (int64_t)v.b;
        if (to == SG_T_FLOAT) return {gbf32((float)x), false};
        if (to == SG_T_DOUBLE) return {gbf64((double)x), false};
    } else if (from == SG_T_FLOAT && to == SG_T_DOUBLE) {
        return {gbf64((double)gf32(v.b)), false};
    }
    return v;
}

__device__ __forceinline__ GVal jo_arith(int op, int t, GVal l, GVal r) {
    if (l.null || r.null) return {0, true};
    switch (t) {
    case SG_T_INT: {
        const int32_t a = (int32_t)(uint32_t)l.b, b = (int32_t)(uint32_t)r.b;
        const uint32_t ua = (uint32_t)a, ub = (uint32_t)b;
        switch (op) {
        case SG_OP_ADD: return {(uint64_t)(uint32_t)(ua + ub), false};
        case SG_OP_SUB: return {(uint64_t)(uint32_t)(ua - ub), false};
        case SG_OP_MUL: return {(uint64_t)(uint32_t)(ua * ub), false};
        case SG_OP_DIV:
            if (b == 0) return {0, true};
            if (b == -1) return {(uint64_t)(uint32_t)(0u - ua), false};
            return {(uint64_t)(uint32_t)(a / b), false};
        default:
            if (b == 0) return {0, true};
            if (b == -1) return {0, false};
            return {(uint64_t)(uint32_t)(a % b), false};
        }
    }
    case SG_T_LONG: {
        const int64_t a = (int64_t)l.b, b = (int64_t)r.b;
        const uint64_t ua = (uint64_t)a, ub = (uint64_t)b;
        switch (op) {
        case SG_OP_ADD: return {ua + ub, false};
        case SG_OP_SUB: return {ua - ub, false};
        case SG_OP_MUL: return {ua * ub, false};
        case SG_OP_DIV:
            if (b == 0) return {0, true};
            if (b == -1) return {0ull - ua, false};
            return {(uint64_t)(a / b), false};
        default:
            if (b == 0) return {0, true};
            if (b == -1) return {0, false};
            return {(uint64_t)(a % b), false};
        }
    }
    case SG_T_FLOAT: {
        const float a = gf32(l.b), b = gf32(r.b);
        switch (op) {
        case SG_OP_ADD: return {gbf32(__fadd_rn(a, b)), false};
        case SG_OP_SUB: return {gbf32(__fsub_rn(a, b)), false};
        case SG_OP_MUL: return {gbf32(__fmul_rn(a, b)), false};
        case SG_OP_DIV: if (b == 0.0f) return {0, true}; return {gbf32(__fdiv_rn(a, b)), false};
        default: if (b == 0.0f) return {0, true}; return {gbf32(fmodf(a, b)), false};
        }
    }
    default: {
        const double a = gf64(l.b), b = gf64(r.b);
        switch (op) {
        case SG_OP_ADD: return {gbf64(__dadd_rn(a, b)), false};
        case SG_OP_SUB: return {gbf64(__dsub_rn(a, b)), false};
        case SG_OP_MUL: return {gbf64(__dmul_rn(a, b)), false};
        case SG_OP_DIV: if (b == 0.0) return {0, true}; return {gbf64(__ddiv_rn(a, b)), false};
        default: if (b == 0.0) return {0, true}; return {gbf64(fmod(a, b)), false};
        }
    }
    }
}

template <class T> __device__ __forceinline__ bool jo_cmp_op(int op, T a, T b) {
    switch (op) {
    case SG_OP_EQ: return a == b;
    case SG_OP_NE: return a != b;
    case SG_OP_GT: return a > b;
    case SG_OP_GE: return a >= b;
    case SG_OP_LT: return a < b;
    default: return a <= b;
    }
}

__device__ __forceinline__ bool jo_compare(int op, int dom, GVal l, GVal r) {
    if (l.null || r.null) return op == SG_OP_NE;  // CompareConditionExpressionExecutor.java:38-42
    switch (dom) {
    case SG_T_INT: return jo_cmp_op(op, (int32_t)(uint32_t)l.b, (int32_t)(uint32_t)r.b);
    case SG_T_LONG: return jo_cmp_op(op, (int64_t)l.b, (int64_t)r.b);
    case SG_T_FLOAT: return jo_cmp_op(op, gf32(l.b), gf32(r.b));
    case SG_T_DOUBLE: return jo_cmp_op(op, gf64(l.b), gf64(r.b));
    case SG_T_BOOL: return jo_cmp_op(op, (uint32_t)(l.b & 1), (uint32_t)(r.b & 1));
    default: return jo_cmp_op(op, (uint32_t)l.b, (uint32_t)r.b);
    }
}

// A filter program of the form `operand CMP operand` (operands: an attribute, or a constant, each widened
// to the compare domain), decoded once on the host (gen_host.hip jo_fast_decode) and evaluated without the
// interpreter's loop and dispatch: the common shapes `price > 20`, `price > e1.price`.
// (F: gen_engine.h JoFast)
template <class F, class VarFn> __device__ __forceinline__ bool jo_fast(const F& f, VarFn var) {
    GVal o[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
        o[i] = f.isConst[i] ? GVal{f.cbits[i], f.cnull[i] != 0u}
                            : jo_cvt(var(f.slot[i], f.attr[i], f.chain[i]), (int)f.from[i], (int)f.dom);
    return jo_compare((int)f.op, (int)f.dom, o[0], o[1]);
}

// The value of one expression program code[pc, pc + n).  Leaves: var(slot, attr, chain) -> GVal and
// evnull(slot, chain) -> bool (`e1 is null`).  The two top entries live in registers (t0 = top, t1 =
// below it); deeper ones in stk[] (stk[i] = entry i from the bottom), touched only by programs deeper
// than two.  Malformed code sets err bit 32 (GERR_REF) / 1 (stack too deep) and yields null.
// DEEP = false: programs at most two entries deep (checked on the host, jo_depth): no stack array at all,
// so a kernel that only evaluates such programs keeps every value in registers (no scratch)
template <bool DEEP = true, class CodePtr, class VarFn, class EvNullFn>
__device__ __forceinline__ GVal jo_eval(CodePtr code, uint32_t pc, uint32_t n, uint32_t& err, VarFn var,
                                        EvNullFn evnull) {
    GVal stk[DEEP ? 24 : 1];
    GVal t0{0, true}, t1{0, true};
    int sp = 0;
    const uint32_t end = pc + n;
    while (pc < end) {
        const uint32_t w = code[pc];
        const uint32_t op = w & 0xff, a = (w >> 8) & 0xff, b = (w >> 16) & 0xff;
        if (sp > (DEEP ? 22 : 2)) { err |= 1u; return GVal{0, true}; }
        GVal v;
        bool push = false, binary = false;
        switch (op) {
        case SG_OP_VAR:
            v = var(b, code[pc + 1], (int32_t)code[pc + 2]);
            push = true;
            break;
        case SG_OP_CONST:
            v = {(uint64_t)code[pc + 1] | ((uint64_t)code[pc + 2] << 32), b != 0};
            push = true;
            break;
        case SG_OP_ISNULL_EV:
            v = {(uint64_t)evnull(b, (int32_t)code[pc + 1]), false};
            push = true;
            break;
        case SG_OP_CVT: t0 = jo_cvt(t0, (int)a, (int)b); break;
        case SG_OP_ADD: case SG_OP_SUB: case SG_OP_MUL: case SG_OP_DIV: case SG_OP_MOD:
            t0 = jo_arith((int)op, (int)a, t1, t0);
            binary = true;
            break;
        case SG_OP_EQ: case SG_OP_NE: case SG_OP_GT: case SG_OP_GE: case SG_OP_LT: case SG_OP_LE:
            t0 = {(uint64_t)jo_compare((int)op, (int)a, t1, t0), false};
            binary = true;
            break;
        case SG_OP_AND: {  // AndConditionExpressionExecutor.java:65-74 (never null)
            const bool l = !t1.null && (t1.b & 1), r = !t0.null && (t0.b & 1);
            t0 = {(uint64_t)(l && r), false};
            binary = true;
            break;
        }
        case SG_OP_OR: {  // OrConditionExpressionExecutor.java:65-75
            const bool l = !t1.null && (t1.b & 1), r = !t0.null && (t0.b & 1);
            t0 = {(uint64_t)(l || r), false};
            binary = true;
            break;
        }
        case SG_OP_NOT: {  // NotConditionExpressionExecutor.java:43-49: not(null) = true
            const bool t = !t0.null && (t0.b & 1);
            t0 = {(uint64_t)(!t), false};
            break;
        }
        case SG_OP_ISNULL: t0 = {(uint64_t)t0.null, false}; break;
        case SG_OP_IFELSE: {  // ifThenElse(cond, then, else): three popped, one pushed
            if constexpr (!DEEP) { err |= 1u; return GVal{0, true}; }
            const GVal c = sp >= 3 ? stk[sp - 3] : GVal{0, true};
            t0 = (!c.null && (c.b & 1)) ? t1 : t0;
            t1 = sp >= 4 ? stk[sp - 4] : GVal{0, true};
            sp -= 2;
            pc += op_len(op);
            continue;
        }
        default: err |= 32u; return GVal{0, true};
        }
        if (push) {
            if constexpr (DEEP) {
                if (sp >= 2) stk[sp - 2] = t1;
            } else if (sp >= 2) {
                err |= 1u;
                return GVal{0, true};
            }
            t1 = t0;
            t0 = v;
            sp++;
        } else if (binary) {  // two popped, one pushed: the entry below the operands moves up
            if constexpr (DEEP) {
                if (sp >= 3) t1 = stk[sp - 3];
            }
            sp--;
        }
        pc += op_len(op);
    }
    return sp > 0 ? t0 : GVal{0, true};
}

// One aggregator's processAdd for a CURRENT event of one partition key (AttributeAggregatorExecutor.java:
// 60-100 over Count / Sum / Avg / Min / Max*AttributeAggregatorExecutor.java): `arg` of type `at`, the
// per-key state (n events added, v value bits, has = a value exists); returns the aggregator's value after
// the event.  A null argument leaves the state and returns the current value (null before any value).
// Sums add in arrival order from 0 / 0.0, like the reference's running sums.
__device__ __forceinline__ GVal jo_agg(uint32_t fn, int at, GVal arg, int64_t& n, uint64_t& v, bool& has) {
    if (fn == SG_AGG_COUNT) {
        n += 1;
        return {(uint64_t)n, false};
    }
    const bool wide_int = at == SG_T_INT || at == SG_T_LONG;
    if (fn == SG_AGG_SUM || fn == SG_AGG_AVG) {
        if (!arg.null) {
            if (fn == SG_AGG_SUM && wide_int) {
                const int64_t x = at == SG_T_INT ? (int64_t)(int32_t)(uint32_t)arg.b : (int64_t)arg.b;
                v = (uint64_t)((has ? (int64_t)v : 0) + x);   // two's-complement wrap, as long addition
            } else {
                double x = 0.0;
                switch (at) {
                case SG_T_INT: x = (double)(int32_t)(uint32_t)arg.b; break;
                case SG_T_LONG: x = (double)(int64_t)arg.b; break;
                case SG_T_FLOAT: x = (double)gf32(arg.b); break;
                default: x = gf64(arg.b);
                }
                v = gbf64(__dadd_rn(has ? gf64(v) : 0.0, x));
            }
            has = true;
            n += 1;
        }
        if (!has) return {0, true};
        if (fn == SG_AGG_SUM) return {v, false};
        return {gbf64(__ddiv_rn(gf64(v), (double)n)), false};
    }
    // min / max in the argument's domain
    if (!arg.null) {
        bool take = !has;
        if (!take) {
            switch (at) {
            case SG_T_INT: {
                const int32_t c = (int32_t)(uint32_t)v, x = (int32_t)(uint32_t)arg.b;
                take = fn == SG_AGG_MIN ? c > x : c < x;
                break;
            }
            case SG_T_LONG: {
                const int64_t c = (int64_t)v, x = (int64_t)arg.b;
                take = fn == SG_AGG_MIN ? c > x : c < x;
                break;
            }
            case SG_T_FLOAT: {
                const float c = gf32(v), x = gf32(arg.b);
                take = fn == SG_AGG_MIN ? c > x : c < x;
                break;
            }
            default: {
                const double c = gf64(v), x = gf64(arg.b);
                take = fn == SG_AGG_MIN ? c > x : c < x;
            }
            }
        }
        if (take) {
            v = arg.b;
            has = true;
        }
        n += 1;
    }
    return has ? GVal{v, false} : GVal{0, true};
}
