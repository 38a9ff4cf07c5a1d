// grp_kernels.hip — key grouping of a two-state micro-batch by key tile (see grp.h).
//
// Replaces the key-run grouping of PartitionStreamReceiver.receive(Event[])
// (partition/PartitionStreamReceiver.java:175-260: the events of a batch handed to each partition key's
// state in arrival order).  The product is the same as the stable rocPRIM payload sort's: the batch as
// key-sorted payload elements (arrival order within a key) + seg_begin / seg_end per key.
//
// Why not a radix sort: the advance kernel only needs each workgroup's 256 keys as one contiguous range,
// split by key.  So the device-wide pass buckets by key TILE (key >> 8, up to 4096 tiles), and the split
// inside a tile (~4K events at C2) happens in LDS.  Both steps are stable rankings built from wave ballots
// ("match any": the lanes of a wave holding the same tile id), no radix passes over digits:
//   k_grp_hist     one read of the keys, per-block tile counts in LDS -> mat (tile-major)
//   scan           rocPRIM exclusive scan of mat -> each (tile, block) range
//   k_grp_scatter  each wave ranks its 4096 events among its tile peers (two passes over the keys: the
//                  counts, then the ranks from the offsets), the payload is gathered from the SoA
//                  columns and written to its tile range (a block's events of one tile are ~16
//                  consecutive elements, so the writes fill whole lines)
//   k_grp_tile     one workgroup per tile: the tile's range staged in LDS (global_load_lds), the same
//                  two-pass ranking by key & 255, the elements written out key-sorted and the 256 keys'
//                  bounds (a tile larger than the LDS region is ranked from HBM, same code)
#include "grp.h"

#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>

namespace {

typedef uint32_t grp_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) void* grp_glb_ptr;
typedef __attribute__((address_space(3))) void* grp_lds_ptr;

// number of set bits of m below this lane
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// the lanes (among `act`) whose BITS-bit value equals this lane's; every lane of the wave runs it
template <int BITS> __device__ __forceinline__ uint64_t match_any(uint32_t v, uint64_t act) {
    uint64_t m = act;
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const bool x = (v >> b) & 1u;
        const uint64_t bb = __ballot(x);
        m &= x ? bb : ~bb;
    }
    return m;
}

__device__ __forceinline__ bool key_ok(uint32_t k, uint32_t K) { return k < K; }

#define GRP_CPL (SGD_GRP_WAVE_EVENTS / 64)          // chunks (of 64 consecutive events) per wave
#define GRP_KPT (SGD_GRP_BLOCK_EVENTS / 1024)        // keys per thread of the histogram

// ---- per-block tile counts ----------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_grp_hist(const GrpArgs a) {
    extern __shared__ uint32_t cnt[];  // [n_tiles]
    for (uint32_t t = threadIdx.x; t < a.n_tiles; t += 1024) cnt[t] = 0;
    const uint32_t i0 = blockIdx.x * SGD_GRP_BLOCK_EVENTS + threadIdx.x;
    uint32_t k[GRP_KPT];
#pragma unroll
    for (uint32_t c = 0; c < GRP_KPT; ++c) {  // every load in flight at once
        const uint32_t i = i0 + c * 1024;
        k[c] = i < a.n ? a.keys[i] : 0u;
    }
    __syncthreads();
    bool bad = false;
#pragma unroll
    for (uint32_t c = 0; c < GRP_KPT; ++c) {
        if (i0 + c * 1024 >= a.n) continue;
        if (key_ok(k[c], a.K)) atomicAdd(&cnt[k[c] >> 8], 1u);
        else if (!(a.drop_null && k[c] == 0xffffffffu)) bad = true;
    }
    // an out-of-range id is reported (the batch's other events go on), never written anywhere
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(a.err, (uint32_t)SGD_ERR_KEY_RANGE);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < a.n_tiles; t += 1024) a.mat[(size_t)t * a.nblk + blockIdx.x] = cnt[t];
    if (blockIdx.x == 0 && threadIdx.x == 0) a.mat[(size_t)a.n_tiles * a.nblk] = 0;  // scans to the total
}

// ---- tile bucketing ----------------------------------------------------------------------------
// wave w of block b owns events [b*BE + w*2048, +2048): 32 chunks of 64 consecutive events, loaded at
// once.  Pass 1 ranks each event among the wave's earlier events of its tile (u16 counters in LDS,
// updated by the lowest lane of each group of tile peers: no atomics) and keeps key | rank << 20 in a
// register; the counters become the wave's offsets within the block's range of each tile; pass 2
// gathers the payload (2-8 chunks' loads in flight at a time) and writes element i to
// mscan[tile][block] + wave offset + rank.
template <int W> __global__ void __launch_bounds__(1024) k_grp_scatter(const GrpArgs a, const PackSrc src) {
    extern __shared__ uint32_t lds[];
    const uint32_t NT = a.n_tiles;
    const uint32_t NTP = (NT + 1u) & ~1u;     // u16 counters per wave, a whole number of words
    uint16_t* wc = (uint16_t*)lds;            // [SGD_GRP_WAVES][NTP]
    uint32_t* boff = lds + (SGD_GRP_WAVES / 2) * NTP;  // [NT] the block's start in each tile's range
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t x = threadIdx.x; x < (SGD_GRP_WAVES / 2) * NTP; x += 1024) lds[x] = 0;
    const uint32_t i0 = blockIdx.x * SGD_GRP_BLOCK_EVENTS + w * SGD_GRP_WAVE_EVENTS + lane;
    uint32_t pk[GRP_CPL];
#pragma unroll
    for (uint32_t c = 0; c < GRP_CPL; ++c) {
        const uint32_t i = i0 + c * 64;
        pk[c] = i < a.n ? a.keys[i] : 0xffffffffu;
    }
    __syncthreads();
    uint16_t* mine = wc + w * NTP;
    uint32_t vm = 0;  // bit c: chunk c's event is kept
#pragma unroll
    for (uint32_t c = 0; c < GRP_CPL; ++c) {
        const uint32_t k = pk[c];
        const bool v = key_ok(k, a.K);
        const uint64_t act = __ballot(v);
        uint32_t r = 0;
        if (act && !(SG_EXP(a.exp) & 2)) {  // wave-uniform
            const uint64_t m = match_any<12>(k >> 8, act);
            if (v) {
                const uint32_t t = k >> 8;
                const uint32_t before = lane_rank(m);
                const uint32_t base = mine[t];
                if (before == 0) mine[t] = (uint16_t)(base + (uint32_t)__popcll(m));
                r = base + before;
            }
        }
        vm |= (v ? 1u : 0u) << c;
        pk[c] = (k & 0xfffffu) | (r << 20);  // key < 2^20, rank < 2048
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < NT; t += 1024) {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t q = 0; q < SGD_GRP_WAVES; ++q) {
            const uint32_t c = wc[q * NTP + t];
            wc[q * NTP + t] = (uint16_t)run;  // < 32768: the block's events before this wave's
            run += c;
        }
        boff[t] = a.mscan[(size_t)t * a.nblk + blockIdx.x];
    }
    __syncthreads();
    const PackFn<W> pf{src};
    Pay<W>* out = (Pay<W>*)a.tpay;
    constexpr uint32_t G = W == 1 ? 8 : (W == 4 ? 2 : 4);  // chunks whose loads are in flight together
#pragma unroll
    for (uint32_t g = 0; g < GRP_CPL; g += G) {
        Pay<W> el[G];
#pragma unroll
        for (uint32_t q = 0; q < G; ++q)
            if ((vm >> (g + q)) & 1u) el[q] = pf(i0 + (g + q) * 64);
#pragma unroll
        for (uint32_t q = 0; q < G; ++q) {
            const uint32_t c = g + q;
            if ((vm >> c) & 1u) {
                const uint32_t k = pk[c] & 0xfffffu, t = k >> 8;
                // the tile sort's split key rides in the position's top byte
                el[q].idx = (i0 + c * 64) | ((k & 255u) << 24);
                out[(SG_EXP(a.exp) & 1) ? i0 + c * 64 : boff[t] + mine[t] + (pk[c] >> 20)] = el[q];
            }
        }
    }
}

// inclusive prefix sum over a wave
__device__ __forceinline__ uint32_t wave_scan(uint32_t x, uint32_t lane) {
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

// ---- the split of one tile by key -----------------------------------------------------------------
// 8 waves; wave w takes the w-th eighth of the tile (arrival order).  Pass 1 counts each key's events per
// wave (LDS atomics: order does not matter for counts); lanes 0..255 turn the counts into each key's
// range and the waves' offsets in it; pass 2 ranks each event among its wave's earlier events of its key
// (ballots + a running counter per key) and writes it out.
#define GT_W SGD_GRP_TILE_WAVES
template <int W> __global__ void __launch_bounds__(GT_W * 64) k_grp_tile(const GrpArgs a) {
    extern __shared__ grp_u32x4 stage[];
    __shared__ uint32_t cnt[GT_W][256];
    __shared__ uint32_t wsum[4];
    constexpr uint32_t SB = sizeof(Pay<W>);
    const uint32_t t = blockIdx.x;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63, x = threadIdx.x;
    const uint32_t blo = a.mscan[(size_t)t * a.nblk], bhi = a.mscan[(size_t)(t + 1) * a.nblk];
    const uint32_t n = bhi - blo;
    const uint64_t c_lo = (uint64_t)blo * SB / 16u, c_hi = ((uint64_t)bhi * SB + 15u) / 16u;
    const bool in_lds = (c_hi - c_lo) * 16u <= a.tile_lds;
    const Pay<W>* gsrc = (const Pay<W>*)a.tpay + blo;
    if (in_lds && n) {
        const uint32_t nch = (uint32_t)(c_hi - c_lo);
        const grp_u32x4* s16 = (const grp_u32x4*)a.tpay + c_lo;
        for (uint32_t c = w * 64; c < nch; c += GT_W * 64)
            if (c + lane < nch)
                __builtin_amdgcn_global_load_lds((grp_glb_ptr)(s16 + c + lane), (grp_lds_ptr)(stage + c), 16, 0, 0);
    }
    for (uint32_t q = x; q < GT_W * 256; q += GT_W * 64) (&cnt[0][0])[q] = 0;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const Pay<W>* e = in_lds ? (const Pay<W>*)((const char*)stage + ((uint64_t)blo * SB - c_lo * 16u)) : gsrc;
    const uint32_t qn = (n + GT_W - 1) / GT_W;
    const uint32_t lo = min(n, w * qn), hi = min(n, lo + qn);
    for (uint32_t j = lo + lane; j < hi; j += 64) atomicAdd(&cnt[w][e[j].idx >> 24], 1u);
    __syncthreads();
    uint32_t c[GT_W], tot = 0, incl = 0;
    if (x < 256) {  // lane x of waves 0..3 = key t*256 + x: its events' range, the waves' offsets in it
#pragma unroll
        for (uint32_t q = 0; q < GT_W; ++q) { c[q] = cnt[q][x]; tot += c[q]; }
        incl = wave_scan(tot, lane);
        if (lane == 63) wsum[w] = incl;
    }
    __syncthreads();
    if (x < 256) {
        uint32_t run = incl - tot;
        for (uint32_t q = 0; q < w; ++q) run += wsum[q];
        const uint32_t key = t * 256u + x;
        if (key < a.K) {
            a.seg_begin[key] = blo + run;
            a.seg_end[key] = blo + run + tot;
        }
#pragma unroll
        for (uint32_t q = 0; q < GT_W; ++q) { cnt[q][x] = run; run += c[q]; }
    }
    __syncthreads();
    Pay<W>* out = (Pay<W>*)a.pay + blo;
    for (uint32_t j0 = lo; j0 < hi; j0 += 64) {  // wave-uniform
        const uint32_t j = j0 + lane;
        const bool v = j < hi;
        constexpr uint32_t Q = SB / 4;  // the element as 4-B words
        uint32_t el[Q];
        if (v) {
            const uint32_t* ep = (const uint32_t*)(e + j);
#pragma unroll
            for (uint32_t q = 0; q < Q; ++q) el[q] = ep[q];
        }
        const uint32_t s = v ? (el[0] >> 24) : 0u;
        const uint64_t m = match_any<8>(s, __ballot(v));
        if (v) {
            const uint32_t before = lane_rank(m);
            const uint32_t base = cnt[w][s];
            if (before == 0) cnt[w][s] = base + (uint32_t)__popcll(m);
            el[0] &= 0xffffffu;
            uint32_t* op = (uint32_t*)(out + base + before);
#pragma unroll
            for (uint32_t q = 0; q < Q; ++q) op[q] = el[q];
        }
    }
}

template <int W> hipError_t group_w(const GrpArgs& a, const PackSrc& src, hipStream_t stream) {
    static bool attrs = [] {  // dynamic LDS above 64 KB (gfx950: 160 KB per workgroup)
        (void)hipFuncSetAttribute((const void*)k_grp_scatter<W>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        (void)hipFuncSetAttribute((const void*)k_grp_tile<W>, hipFuncAttributeMaxDynamicSharedMemorySize, 148 * 1024);
        (void)hipGetLastError();  // (an attribute the runtime does not need is not an error of this batch)
        return true;
    }();
    (void)attrs;
    const uint32_t NTP = (a.n_tiles + 1u) & ~1u;
    const size_t sc_lds = (size_t)(SGD_GRP_WAVES / 2) * NTP * 4 + (size_t)a.n_tiles * 4;
    hipLaunchKernelGGL(k_grp_scatter<W>, dim3(a.nblk), dim3(1024), sc_lds, stream, a, src);
    if (hipError_t e = hipGetLastError()) return e;
    hipLaunchKernelGGL(k_grp_tile<W>, dim3(a.n_tiles), dim3(GT_W * 64), a.tile_lds, stream, a);
    return hipGetLastError();
}

// ---- the bucket split: the second half of the grouping after one radix pass on the high key bits --------
// The radix pass (rocPRIM onesweep on bits [SGD_BK_BITS, bits)) leaves the batch stably grouped by bucket =
// key >> SGD_BK_BITS (1024 keys).  One workgroup per bucket then splits it by key in three phases, with the
// 16 waves each owning a contiguous eighth... sixteenth of the bucket (arrival order):
//   count   each wave's events per key (LDS atomics: counts are order-free)
//   scan    per key its range in the bucket (seg_begin / seg_end written here: no k_seg_bounds) and each
//           wave's first position in it
//   place   in passes over key windows whose output fits the LDS stage: every wave re-walks its events in
//           order, ranks each of the window's events among its wave peers of the same key (ballots, a
//           running offset per (wave, key): stable), stores it into the stage; the stage goes out as one
//           contiguous, coalesced range.  A window too large for the stage (hot keys) is placed directly.
#define BK_WAVES 16
#define BK_STAGE_BYTES (88u * 1024u)   // beside 68 KB of counters and key starts (160 KB per CU)
__global__ void __launch_bounds__(256) k_bucket_bounds(const uint32_t* __restrict__ skeys, uint32_t n, uint32_t bits,
                                                       uint32_t nb, uint32_t K, uint32_t drop_null,
                                                       uint32_t* __restrict__ blo, uint32_t* __restrict__ err) {
    // blo[b] = first element of bucket b (b in [0, nb]); skeys sorted by (key & (2^bits - 1)) >> SGD_BK_BITS.
    // Elements past the last bucket are dropped null keys or out-of-range ids (reported here: no split sees them)
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const uint32_t m = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
    const uint32_t ki = i < n ? skeys[i] : 0u;
    const uint32_t cur = i < n ? min((ki & m) >> SGD_BK_BITS, nb) : nb;
    if (i < n && cur == nb && ki >= K && !(drop_null && ki == 0xffffffffu)) atomicOr(err, (uint32_t)SGD_ERR_KEY_RANGE);
    const uint32_t prv = i > 0 ? min((skeys[i - 1] & m) >> SGD_BK_BITS, nb) : 0u;
    if (i == 0) {
        for (uint32_t b = 0; b <= cur; ++b) blo[b] = 0;
    } else if (cur != prv) {
        for (uint32_t b = prv + 1; b <= cur; ++b) blo[b] = i;
    }
    if (i == n && n > 0)
        for (uint32_t b = cur + 1; b <= nb; ++b) blo[b] = n;  // (cur == nb here)
}

template <int W> __global__ void __launch_bounds__(BK_WAVES * 64) k_bucket_split(const BucketArgs a) {
    __shared__ uint32_t cnt[BK_WAVES][1u << SGD_BK_BITS];  // counts, then each wave's running offset per key
    __shared__ uint32_t wsum[BK_WAVES];
    __shared__ uint32_t kstart[(1u << SGD_BK_BITS) + 1];
    extern __shared__ uint32_t bk_stage[];
    constexpr uint32_t KB = 1u << SGD_BK_BITS;
    constexpr uint32_t SW = sizeof(Pay<W>) / 4;  // words per element
    const uint32_t b = blockIdx.x;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63, x = threadIdx.x;
    const uint32_t lo = a.blo[b], hi = a.blo[b + 1];
    const uint32_t n = hi - lo;
    const uint32_t m = a.bits >= 32 ? 0xffffffffu : ((1u << a.bits) - 1u);
    const uint32_t k0 = b * KB;  // first key of the bucket
    for (uint32_t q = x; q < BK_WAVES * KB; q += BK_WAVES * 64) (&cnt[0][0])[q] = 0;
    __syncthreads();
    // wave w: events [lo + w*qn, lo + (w+1)*qn) of the bucket (qn a multiple of 64)
    const uint32_t qn = ((n + BK_WAVES - 1) / BK_WAVES + 63u) & ~63u;
    const uint32_t wlo = min(n, w * qn), whi = min(n, wlo + qn);
    bool bad = false;
    for (uint32_t j = wlo + lane; j < whi; j += 64) {
        const uint32_t key = a.skeys[lo + j];
        if (key < a.K && (key & m) >= k0 && (key & m) < k0 + KB) atomicAdd(&cnt[w][key - k0], 1u);
        else if (!(a.drop_null && key == 0xffffffffu)) bad = true;
    }
    if (__ballot(bad) && lane == 0) atomicOr(a.err, (uint32_t)SGD_ERR_KEY_RANGE);
    __syncthreads();
    // scan: thread x = key k0 + x
    uint32_t c[BK_WAVES], tot = 0;
#pragma unroll
    for (uint32_t q = 0; q < BK_WAVES; ++q) { c[q] = cnt[q][x]; tot += c[q]; }
    const uint32_t incl = wave_scan(tot, lane);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t run = incl - tot;
    for (uint32_t q = 0; q < w; ++q) run += wsum[q];
    kstart[x] = run;
    if (x == KB - 1) kstart[KB] = run + tot;
    if (k0 + x < a.K) {
        a.seg_begin[k0 + x] = lo + run;
        a.seg_end[k0 + x] = lo + run + tot;
    }
#pragma unroll
    for (uint32_t q = 0; q < BK_WAVES; ++q) { cnt[q][x] = run; run += c[q]; }
    __syncthreads();
    // place, window by window of keys
    const uint32_t cap = a.stage_bytes / (SW * 4);   // elements the stage holds
    const Pay<W>* in = (const Pay<W>*)a.tpay + lo;
    uint32_t* out = (uint32_t*)((Pay<W>*)a.pay + lo);
    for (uint32_t p0 = 0; p0 < KB;) {
        // the window: as many keys from p0 as fit the stage (at least one); wave-uniform (LDS reads)
        uint32_t p1 = p0 + 1;
        for (uint32_t step = KB / 2; step >= 1; step >>= 1)
            if (p1 + step <= KB && kstart[p1 + step] - kstart[p0] <= cap) p1 += step;
        const uint32_t s0 = kstart[p0], s1 = kstart[p1];
        const bool staged = s1 - s0 <= cap;
        for (uint32_t j0 = wlo; j0 < whi; j0 += 64) {   // wave-uniform trips
            const uint32_t j = j0 + lane;
            const bool v = j < whi;
            const uint32_t key = v ? a.skeys[lo + j] : 0xffffffffu;
            const uint32_t sub = key - k0;
            const bool sel = v && key < a.K && sub >= p0 && sub < p1;
            const uint64_t act = __ballot(sel);
            if (!act) continue;
            const uint64_t mm = match_any<SGD_BK_BITS>(sub, act);
            if (sel) {
                const uint32_t before = lane_rank(mm);
                const uint32_t base = cnt[w][sub];
                if (before == 0) cnt[w][sub] = base + (uint32_t)__popcll(mm);
                const uint32_t d = base + before;   // position in the bucket
                const uint32_t* src = (const uint32_t*)(in + j);
                uint32_t el[SW];
#pragma unroll
                for (uint32_t q = 0; q < SW; ++q) el[q] = src[q];
                if (staged) {
#pragma unroll
                    for (uint32_t q = 0; q < SW; ++q) bk_stage[(d - s0) * SW + q] = el[q];
                } else {
#pragma unroll
                    for (uint32_t q = 0; q < SW; ++q) out[(size_t)d * SW + q] = el[q];
                }
            }
        }
        __syncthreads();
        if (staged) {   // the window's output range, coalesced
            const uint32_t nw = (s1 - s0) * SW;
            uint32_t* o = out + (size_t)s0 * SW;
            for (uint32_t q = x; q < nw; q += BK_WAVES * 64) o[q] = bk_stage[q];
            __syncthreads();
        }
        p0 = p1;
    }
}

template <int W> hipError_t bucket_w(const BucketArgs& a, hipStream_t stream) {
    static bool attrs = [] {
        (void)hipFuncSetAttribute((const void*)k_bucket_split<W>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  BK_STAGE_BYTES);
        (void)hipGetLastError();
        return true;
    }();
    (void)attrs;
    hipLaunchKernelGGL(k_bucket_split<W>, dim3(a.nb), dim3(BK_WAVES * 64), a.stage_bytes, stream, a);
    return hipGetLastError();
}

}  // namespace

size_t sgd_group_scan_bytes(uint64_t max_entries) {
    size_t b = 0;
    if (rocprim::exclusive_scan(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)max_entries,
                                rocprim::plus<uint32_t>()) != hipSuccess)
        return 0;
    return b;
}

// LDS region of the tile sort: the tile's payload bytes at this density (n / K events per key, 256 keys)
// plus 4 standard deviations of the Poisson count (larger tiles are ranked from HBM, exactly)
uint32_t sgd_group_tile_lds(uint64_t n, uint64_t K, uint32_t words) {
    const uint32_t sb = 4u * (words + 2u);  // sizeof(Pay<words>)
    const double mean = (double)n * 256.0 / (double)(K ? K : 1);
    const double want = (mean + 4.0 * std::sqrt(mean) + 32.0) * sb + 32.0;
    const double lim = 148.0 * 1024.0;  // beside the 8 KB of counters
    return (uint32_t)(std::ceil(std::min(std::max(want, 16384.0), lim) / 16.0) * 16.0);
}

hipError_t sgd_group_tiles(const GrpArgs& a, const PackSrc& src, int W, hipStream_t stream) {
    const size_t entries = (size_t)a.n_tiles * a.nblk + 1;
    hipLaunchKernelGGL(k_grp_hist, dim3(a.nblk), dim3(1024), (size_t)a.n_tiles * 4, stream, a);
    if (hipError_t e = hipGetLastError()) return e;
    size_t tb = a.scan_tmp_bytes;
    if (hipError_t e = rocprim::exclusive_scan(a.scan_tmp, tb, (const uint32_t*)a.mat, a.mscan, 0u, entries,
                                               rocprim::plus<uint32_t>(), stream))
        return e;
    switch (W) {
    case 1: return group_w<1>(a, src, stream);
    case 2: return group_w<2>(a, src, stream);
    case 3: return group_w<3>(a, src, stream);
    default: return group_w<4>(a, src, stream);
    }
}

hipError_t sgd_bucket_split(const BucketArgs& a0, int W, hipStream_t stream) {
    BucketArgs a = a0;
    a.stage_bytes = BK_STAGE_BYTES;
    hipLaunchKernelGGL(k_bucket_bounds, dim3((a.n + 1 + 255) / 256), dim3(256), 0, stream, a.skeys, a.n, a.bits, a.nb,
                       a.K, a.drop_null, a.blo, a.err);
    if (hipError_t e = hipGetLastError()) return e;
    switch (W) {
    case 1: return bucket_w<1>(a, stream);
    case 2: return bucket_w<2>(a, stream);
    case 3: return bucket_w<3>(a, stream);
    default: return bucket_w<4>(a, stream);
    }
}
