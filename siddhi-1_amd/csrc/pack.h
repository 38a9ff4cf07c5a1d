// pack.h — the key-sorted payload element of the engines and its gather from the SoA batch columns (the first
// pass of the grouping, part_kernels.hip)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sg_engine.h"

// key-sorted event payload: batch position, the filter columns (32-bit words), timestamp as a 32-bit
// offset from the batch's first timestamp (SGD_TS_FAR when it does not fit)
template <int W> struct Pay {
    uint32_t idx;
    uint32_t w[W];
    int32_t ts;
};
static_assert(sizeof(Pay<1>) == 12 && sizeof(Pay<2>) == 16 && sizeof(Pay<3>) == 20 && sizeof(Pay<4>) == 24,
              "payload layout: 4-B words, the ts offset last");

__host__ __device__ __forceinline__ int32_t sgd_ts_off(int64_t t, int64_t base) {
    if (t == -1) return SGD_TS_FAR;
    const uint64_t d = (uint64_t)t - (uint64_t)base;  // two's-complement difference
    const int64_t x = (int64_t)d;
    // exact only when t - base does not wrap: same signs or the difference keeps the sign of t - base
    const bool wrapped = ((t ^ base) < 0) && ((x ^ t) < 0);
    return (wrapped || x < -SGD_TS_LIM || x > SGD_TS_LIM) ? SGD_TS_FAR : (int32_t)x;
}

struct PackSrc {
    const void* p[4];
    uint8_t kind[4];  // 0: 32-bit column, 1: low / 2: high word of a 64-bit column, 3: bool byte,
                      // 4: null bits of the columns, 5: zero
    const uint8_t* nul[SGD_MAX_EVCOLS];
    const int64_t* ts;
};

template <int W> struct PackFn {
    PackSrc s;
    __host__ __device__ Pay<W> operator()(uint32_t i) const {
        Pay<W> o;
        o.idx = i;
        o.ts = sgd_ts_off(s.ts[i], s.ts[0]);
        for (int w = 0; w < W; ++w) {
            switch (s.kind[w]) {
            case 0: o.w[w] = ((const uint32_t*)s.p[w])[i]; break;
            case 1: o.w[w] = (uint32_t)((const uint64_t*)s.p[w])[i]; break;
            case 2: o.w[w] = (uint32_t)(((const uint64_t*)s.p[w])[i] >> 32); break;
            case 3: o.w[w] = ((const uint8_t*)s.p[w])[i] ? 1u : 0u; break;
            case 4: {
                uint32_t nb = 0;
                for (int c = 0; c < SGD_MAX_EVCOLS; ++c)
                    if (s.nul[c]) nb |= (s.nul[c][i] != 0 ? 1u : 0u) << c;
                o.w[w] = nb;
                break;
            }
            default: o.w[w] = 0u;
            }
        }
        return o;
    }
};
