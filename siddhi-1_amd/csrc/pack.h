// pack.h — the key-sorted payload element of the two-state engine and its gather from the SoA batch
// columns (shared by the rocPRIM grouping in sg_engine.hip and the tile grouping in grp_kernels.hip)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sg_engine.h"

// key-sorted event payload: batch position, the filter columns (32-bit words), timestamp
template <int W> struct alignas(8) Pay {
    uint32_t idx;
    uint32_t w[W];
    int64_t ts;
};
static_assert(sizeof(Pay<1>) == 16 && sizeof(Pay<2>) == 24 && sizeof(Pay<3>) == 24 && sizeof(Pay<4>) == 32,
              "payload layout: ts in the last 8 bytes");

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
        o.ts = s.ts[i];
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
