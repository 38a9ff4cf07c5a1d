// reg_common.h — pieces shared by the register-window kernels (abs_kernels.hip: the absent-tail shape,
// cnt_kernels.hip: the counting sequence shape): an event of the key-sorted payload in registers, the
// per-wave counter rows, the hand-over of keys to the general kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu.h"
#include "../../include/siddhi_gpu_ir.h"
#include "gen_engine.h"
#include "sg_engine.h"

namespace {

typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(4))) const GenProgram cGenProgram;
template <class T> __device__ __forceinline__ __attribute__((address_space(1))) T* gp(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

__device__ __forceinline__ bool ts_before(int64_t a, int64_t b) { return (a != -1) && (b == -1 || a < b); }

template <int NW> struct AbsEv {
    int64_t ts;
    uint64_t seq;
    uint32_t w[NW];
    uint32_t nb;
};

// the lanes' work counters, reduced over the wave (all 64 lanes call this): one atomic per wave
// (the wave's row of a.o.wstats: every wave writes its row, k_gen_stats_reduce sums them afterwards)
__device__ void abs_wave_stats(const GenArgs& a, unsigned long long sc, unsigned long long cr, unsigned long long ma,
                               unsigned long long ky, uint32_t er, unsigned long long fb) {
    for (int off = 32; off > 0; off >>= 1) {
        fb += __shfl_xor(fb, off, 64);
        sc += __shfl_xor(sc, off, 64);
        cr += __shfl_xor(cr, off, 64);
        ma += __shfl_xor(ma, off, 64);
        ky += __shfl_xor(ky, off, 64);
        er |= (uint32_t)__shfl_xor((int)er, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (er) atomicOr(a.o.err, er);
        auto w = gp(a.o.wstats) + (size_t)blockIdx.x * GST_N;
        w[GST_SCANNED] = sc;
        w[GST_CREATED] = cr;
        w[GST_MATCHES] = ma;
        w[GST_KEYS] = ky;
        w[GST_LIVE0] = 0;
        w[GST_SPILLS] = fb;
    }
}

// hand a key to the general kernels (wave-aggregated append to the fallback list)
__device__ __forceinline__ void abs_fallback(const GenArgs& a, bool mine, uint32_t key, uint32_t start) {
    const unsigned long long m = __ballot(mine);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    unsigned long long b0 = 0;
    if (lane == __ffsll((long long)m) - 1) b0 = atomicAdd(a.fb_n, (unsigned long long)__popcll(m));
    b0 = __shfl(b0, __ffsll((long long)m) - 1, 64);
    if (mine) {
        gp(a.fb_list)[b0 + __popcll(m & ((1ull << lane) - 1ull))] = key;
        if (a.fb_start) gp(a.fb_start)[key] = start;
    }
}

template <int NW> __device__ void abs_gather(const GenArgs& a, const cGenProgram& G, uint32_t pos, AbsEv<NW>& ev) {
    const int s = (int)a.b.stream;
    const int na = G.nattr[s];
    ev.nb = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) ev.w[q] = 0;
    for (int at = 0; at < na; at++) {
        const int ty = G.attrType[s][at];
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
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            if ((uint32_t)q == o) ev.w[q] = lo;
            if ((ty == SG_T_LONG || ty == SG_T_DOUBLE) && (uint32_t)q == o + 1) ev.w[q] = hi;
        }
        if (a.b.nul[at] && gp(a.b.nul[at])[pos]) ev.nb |= 1u << at;
    }
}

// event i of the key-sorted payload (pack.h Pay<W>): the batch position, the attribute words in attribute
// order (= the window's word layout), the null bits when present, the timestamp offset from ts[0]
// (split in two so that a walk can load event i + 1's words while it processes event i)
template <int NW> __device__ __forceinline__ void abs_pay_raw(const GenArgs& a, uint32_t i, uint32_t (&x)[NW + 3]) {
    const uint32_t st = a.b.payStride;
    const gu32* p = gp(a.b.pay) + (size_t)i * st;
#pragma unroll
    for (int q = 0; q < NW + 3; ++q) x[q] = (uint32_t)q < st ? p[q] : 0u;
}
template <int NW> __device__ __forceinline__ void abs_pay_decode(const GenArgs& a, const uint32_t (&x)[NW + 3],
                                                                 int64_t tbase, AbsEv<NW>& ev) {
    constexpr int MW = NW + 3;
    const uint32_t st = a.b.payStride;
    const uint32_t pos = x[0];
#pragma unroll
    for (int q = 0; q < NW; ++q) ev.w[q] = x[1 + q];
    uint32_t toff = 0, nb = 0;
#pragma unroll
    for (int q = 1; q < MW; ++q) {
        if ((uint32_t)q == st - 1) toff = x[q];
        if (a.b.payNull && (uint32_t)q == st - 2) nb = x[q];
    }
    ev.nb = nb;
    ev.ts = (int32_t)toff == SGD_TS_FAR ? gp(a.b.ts)[pos] : tbase + (int64_t)(int32_t)toff;
    ev.seq = a.b.seq_base + pos;
}
template <int NW> __device__ __forceinline__ void abs_pay(const GenArgs& a, uint32_t i, int64_t tbase, AbsEv<NW>& ev) {
    uint32_t x[NW + 3];
    abs_pay_raw<NW>(a, i, x);
    abs_pay_decode<NW>(a, x, tbase, ev);
}
// the walk's payload words, one event ahead
template <int NW> struct PayAhead {
    uint32_t x[NW + 3];
    __device__ __forceinline__ void first(const GenArgs& a, uint32_t b, uint32_t e) {
#pragma unroll
        for (int q = 0; q < NW + 3; ++q) x[q] = 0;
        if (a.b.pay && b < e) abs_pay_raw<NW>(a, b, x);
    }
    // event i decoded, event i + 1's words requested
    __device__ __forceinline__ void next(const GenArgs& a, uint32_t i, uint32_t e, int64_t tbase, AbsEv<NW>& ev) {
        uint32_t c[NW + 3];
#pragma unroll
        for (int q = 0; q < NW + 3; ++q) c[q] = x[q];
        if (i + 1 < e) abs_pay_raw<NW>(a, i + 1, x);
        abs_pay_decode<NW>(a, c, tbase, ev);
    }
};

}  // namespace
