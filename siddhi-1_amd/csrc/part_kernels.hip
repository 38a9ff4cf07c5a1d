// part_kernels.hip — hand-written stable partitioning by key digit (see part.h): the key-run grouping of
// every micro-batch (partition/PartitionStreamReceiver.java:175-260, util/snapshot/state/
// PartitionStateHolder.java:43-80) and the engine's key / value sorts, for gfx950.
//
// A pass partitions the batch by one digit of the key (<= 8 bits) and keeps arrival order within a digit:
//
//   k_part_hist     chunk c (4096 events; 2048 for elements wider than 16 B) counts its events per digit in
//                   LDS -> mat[d * nblk + c]
//   k_part_scan     one workgroup per digit: exclusive scan of mat's row d over the chunks, tot[d]
//   k_part_scatter  chunk c: each wave ranks its events among the wave's earlier events of the same digit
//                   ("match any" over the digit bits by wave ballots, a u16 running count per (wave, digit) in
//                   LDS updated by the group's first lane: no atomics); the counts give every event its place
//                   in the chunk's digit-sorted order; the elements are gathered and placed there in LDS; then
//                   the chunk goes out in that order, each digit's run to its start (the digit totals scanned
//                   + the row scan), consecutive lanes to consecutive addresses.
//
// Why staged runs: a lane-scattered store (each lane of a wave store to a different digit's range) is one
// memory request per lane; measured on a 4096-way single pass (tools/ubench/part_bench), the stores alone took
// 300 of 500 us per 2^24 events, and a dwordx3 store per element did not help.  With <= 256 digits a chunk's
// run of one digit is 16+ elements, so a wave's store instruction covers a few runs.
//
// Chunks are dealt XCD-aware: block b takes chunk (b % 8) * nb8 + b / 8, so (under the round-robin placement of
// blocks over the 8 XCDs, speed only, never correctness) each XCD works through one contiguous run of chunks,
// and the runs that neighbouring chunks write into one digit's range meet in that XCD's L2.
#include "part.h"

#include <algorithm>

namespace {

enum { PT_RANGE = 1, PT_DESC = 2 };
enum { PT_GATHER = 0, PT_IDX = 1, PT_MOVE = 2 };    // element source
enum { PD_U32 = 0, PD_U64 = 1, PD_U16 = 2 };        // digit source: keys u32 / u64, or u16 tile codes
enum { PS_NONE = 0, PS_KEY = 1, PS_CODE = 2 };      // side output: the key, or a u16 code of it

struct PassArgs {
    uint32_t n;               // elements (upper bound)
    const uint32_t* n_dev;    // valid elements (a previous pass's count on the device), or null: all n
    uint32_t nblk, nb8;       // chunks, chunks per XCD
    uint32_t shift, dbits, ndig;
    uint32_t mode;            // PT_RANGE: keys >= K are dropped (SG_KEY_NULL silently when drop_null, others
                              // reported in err); PT_DESC: descending digit order
    uint32_t K, drop_null;
    uint32_t cshift, cmask;   // PS_CODE: code = (key >> cshift) & cmask
    const void* keys;         // [n] digit source
    void* side_out;           // [n] keys or codes written beside the elements
    uint32_t* mat;
    uint32_t* tot;
    uint32_t* lo;             // [ndig + 1]: digit starts, then the valid count (written by chunk 0)
    uint32_t* err;
};

struct ElemArgs {
    PackSrc ps;               // PT_GATHER: the SoA batch columns
    const void* in;           // PT_MOVE: [n] elements of S words
    void* out;                // [n] elements of S words
    uint32_t tag;             // PT_GATHER: key & 255 in the position's bits 24..31 (the fused C2 grouping)
    uint32_t pad;
};

template <int DS> struct DKey { typedef uint32_t T; };
template <> struct DKey<PD_U64> { typedef uint64_t T; };
template <> struct DKey<PD_U16> { typedef uint16_t T; };

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// the lanes (among `act`) whose low nb bits of v equal this lane's (every lane of the wave runs it; nb uniform)
__device__ __forceinline__ uint64_t match_any(uint32_t v, uint64_t act, uint32_t nb) {
    uint64_t m = act;
#pragma unroll
    for (uint32_t b = 0; b < SGD_PT_MAX_BITS; ++b) {
        if (b < nb) {
            const bool x = (v >> b) & 1u;
            const uint64_t bb = __ballot(x);
            m &= x ? bb : ~bb;
        }
    }
    return m;
}

__device__ __forceinline__ uint32_t pt_chunk(uint32_t b, uint32_t nb8) { return (b & 7u) * nb8 + (b >> 3); }

// digit of key k; false: the element is left out (bad: to be reported)
template <class T>
__device__ __forceinline__ bool pt_digit(const PassArgs& a, T k, uint32_t& d, bool& bad) {
    if (a.mode & PT_RANGE) {
        if ((uint64_t)k >= (uint64_t)a.K) {
            if (!(a.drop_null && (uint64_t)k == 0xffffffffull)) bad = true;
            return false;
        }
    }
    const uint32_t m = (1u << a.dbits) - 1u;
    uint32_t x = (uint32_t)((uint64_t)k >> a.shift) & m;
    if (a.mode & PT_DESC) x = m - x;
    d = x;
    return true;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane) {
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

// ---- per-chunk digit counts ----------------------------------------------------------------------
// one block counts HC consecutive chunks (HC * CE keys in flight at once: the read is one round trip)
template <int DS, int EPT, int HC> __global__ void __launch_bounds__(SGD_PT_THREADS) k_part_hist(const PassArgs a) {
    typedef typename DKey<DS>::T T;
    constexpr uint32_t CE = SGD_PT_THREADS * EPT;
    __shared__ uint32_t cnt[HC][SGD_PT_MAX_DIG];
    const uint32_t c0 = blockIdx.x * HC;
    if (c0 >= a.nblk) return;  // (the whole block)
    const uint32_t tid = threadIdx.x;
    for (uint32_t x = tid; x < HC * SGD_PT_MAX_DIG; x += SGD_PT_THREADS) (&cnt[0][0])[x] = 0;
    const uint32_t nv = a.n_dev ? *a.n_dev : a.n;
    const uint64_t i0 = (uint64_t)c0 * CE + tid;
    T k[EPT * HC];
#pragma unroll
    for (uint32_t j = 0; j < EPT * HC; ++j) {  // every load in flight at once
        const uint64_t i = i0 + (uint64_t)j * SGD_PT_THREADS;
        k[j] = i < nv ? ((const T*)a.keys)[i] : (T)0;
    }
    __syncthreads();
    bool bad = false;
#pragma unroll
    for (uint32_t j = 0; j < EPT * HC; ++j) {
        uint32_t d;
        if (i0 + (uint64_t)j * SGD_PT_THREADS < nv && pt_digit(a, k[j], d, bad)) atomicAdd(&cnt[j / EPT][d], 1u);
    }
    // an out-of-range id is reported (the batch's other events go on), never written anywhere
    if ((a.mode & PT_RANGE) && __ballot(bad) && (tid & 63u) == 0) atomicOr(a.err, (uint32_t)SGD_ERR_KEY_RANGE);
    __syncthreads();
    for (uint32_t x = tid; x < HC * a.ndig; x += SGD_PT_THREADS) {
        const uint32_t d = x / HC, h = x % HC;
        if (c0 + h < a.nblk) a.mat[(size_t)d * a.nblk + c0 + h] = cnt[h][d];
    }
}

// ---- per digit: exclusive scan of its chunk counts, the digit's total ------------------------------
__global__ void __launch_bounds__(256) k_part_scan(uint32_t* __restrict__ mat, uint32_t nblk,
                                                   uint32_t* __restrict__ tot) {
    __shared__ uint32_t ws[4];
    uint32_t* row = mat + (size_t)blockIdx.x * nblk;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    uint32_t run = 0;
    for (uint32_t base = 0; base < nblk; base += 256u * 4u) {  // (uniform trips)
        const uint32_t j0 = base + tid * 4u;
        uint32_t v[4], s = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            v[q] = j0 + q < nblk ? row[j0 + q] : 0u;
            s += v[q];
        }
        const uint32_t incl = wave_incl_scan(s, lane);
        if (lane == 63) ws[w] = incl;
        __syncthreads();
        uint32_t pre = run, all = run;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            pre += q < w ? ws[q] : 0u;
            all += ws[q];
        }
        uint32_t x = pre + incl - s;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            if (j0 + q < nblk) row[j0 + q] = x;
            x += v[q];
        }
        run = all;
        __syncthreads();
    }
    if (tid == 0) tot[blockIdx.x] = run;
}

template <int SIDE, class T> struct SideT { typedef uint8_t U; static constexpr uint32_t B = 0; };
template <class T> struct SideT<PS_KEY, T> { typedef T U; static constexpr uint32_t B = sizeof(T); };
template <class T> struct SideT<PS_CODE, T> { typedef uint16_t U; static constexpr uint32_t B = 2; };

template <int S> __device__ __forceinline__ void st_elem(uint32_t* o, const uint32_t* v) {
    if constexpr (S == 3) {
        typedef uint32_t v3 __attribute__((ext_vector_type(3)));
        typedef v3 __attribute__((aligned(4))) v3a;
        *(v3a*)o = v3{v[0], v[1], v[2]};
    } else if constexpr (S == 4) {
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        *(v4*)o = v4{v[0], v[1], v[2], v[3]};
    } else if constexpr (S == 6) {
        typedef uint32_t v2 __attribute__((ext_vector_type(2)));
        ((v2*)o)[0] = v2{v[0], v[1]};
        ((v2*)o)[1] = v2{v[2], v[3]};
        ((v2*)o)[2] = v2{v[4], v[5]};
    } else {
#pragma unroll
        for (int u = 0; u < S; ++u) o[u] = v[u];
    }
}

// LDS bytes of a scatter block
__host__ __device__ constexpr uint32_t pt_scatter_lds(uint32_t ce, uint32_t S, uint32_t side_b, uint32_t nd) {
    return ce * S * 4u + ce * side_b + ce + (nd * SGD_PT_WAVES + 2u) * 2u + nd * 8u + 64u;
}

// ---- the stable scatter of one chunk --------------------------------------------------------------
// per event: digit (8 bits) | wave rank << 8 (9 bits) | key & 255 << 17 | valid << 31
template <int DS, int SRC, int S, int SIDE, int EPT>
__global__ void __launch_bounds__(SGD_PT_THREADS) k_part_scatter(const PassArgs a, const ElemArgs e) {
    typedef typename DKey<DS>::T T;
    typedef SideT<SIDE, T> SD;
    constexpr uint32_t CE = SGD_PT_THREADS * EPT, WE = 64u * EPT;
    static_assert(WE <= 512u, "wave ranks are 9 bits");
    extern __shared__ uint32_t lds[];
    const uint32_t c = pt_chunk(blockIdx.x, a.nb8);
    if (c >= a.nblk) return;
    const uint32_t ND = a.ndig;
    uint32_t* el_l = lds;                                               // [CE][S] digit-sorted elements
    typename SD::U* side_l = (typename SD::U*)(el_l + CE * S);          // [CE] their keys / codes
    uint8_t* dg = (uint8_t*)(el_l + CE * S) + CE * SD::B;               // [CE] their digits
    uint16_t* wc = (uint16_t*)(dg + CE);                                // [8][ND] per wave: counts, then places
    uint32_t* bst = (uint32_t*)(wc + SGD_PT_WAVES * ND + 2u);           // [ND] digit run starts in the chunk
    uint32_t* gof = bst + ND;                                           // [ND] their global starts
    uint32_t* ws = gof + ND;                                            // [16] scan scratch; ws[15]: valid events
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = tid & 63u;
    const uint32_t nv = a.n_dev ? *a.n_dev : a.n;

    // the wave's events: c * CE + w * WE + j * 64 + lane, every load in flight at once
    const uint64_t i0 = (uint64_t)c * CE + (uint64_t)w * WE + lane;
    T k[EPT];
#pragma unroll
    for (uint32_t j = 0; j < EPT; ++j) {
        const uint64_t i = i0 + (uint64_t)j * 64u;
        k[j] = i < nv ? ((const T*)a.keys)[i] : (T)0;
    }
    // the events' elements, loaded with the keys (their places are ranked below: the loads' latency overlaps
    // the ranking instead of following it)
    uint32_t el[EPT][S];
#pragma unroll
    for (uint32_t j = 0; j < EPT; ++j) {
        const uint64_t i64 = i0 + (uint64_t)j * 64u;
        const uint32_t i = (uint32_t)i64;
        if (i64 < nv) {
            if constexpr (SRC == PT_GATHER) {
                const Pay<S - 2> p = PackFn<S - 2>{e.ps}(i);
                el[j][0] = p.idx;
#pragma unroll
                for (int u = 0; u < S - 2; ++u) el[j][1 + u] = p.w[u];
                el[j][S - 1] = (uint32_t)p.ts;
            } else if constexpr (SRC == PT_IDX) {
                el[j][0] = i;
            } else {
#pragma unroll
                for (int u = 0; u < S; ++u) el[j][u] = ((const uint32_t*)e.in)[(size_t)i * S + u];
            }
        } else {
#pragma unroll
            for (int u = 0; u < S; ++u) el[j][u] = 0u;
        }
    }
    // the chunk's global start in each digit's range: digit starts (tot scanned, wave 0) + the row scan
    if (w == 0) {
        const uint32_t q = (ND + 63u) / 64u;  // <= 4
        uint32_t v[4], s = 0;
#pragma unroll
        for (uint32_t x = 0; x < 4; ++x) {
            const uint32_t d = lane * q + x;
            v[x] = (x < q && d < ND) ? a.tot[d] : 0u;
            s += v[x];
        }
        const uint32_t incl = wave_incl_scan(s, lane);
        uint32_t ex = incl - s;
#pragma unroll
        for (uint32_t x = 0; x < 4; ++x) {
            const uint32_t d = lane * q + x;
            if (x < q && d < ND) {
                gof[d] = ex + a.mat[(size_t)d * a.nblk + c];
                if (c == 0) a.lo[d] = ex;
            }
            ex += v[x];
        }
        if (c == 0 && lane == 63) a.lo[ND] = incl;
    }
    for (uint32_t x = tid; x < (SGD_PT_WAVES * ND + 1u) / 2u; x += SGD_PT_THREADS) ((uint32_t*)wc)[x] = 0u;
    __syncthreads();

    // ranks among the wave's earlier events of the same digit (arrival order: round j before j + 1, lanes in order)
    uint16_t* mine = wc + w * ND;
    uint32_t pk[EPT];
    bool bad = false;
#pragma unroll
    for (uint32_t j = 0; j < EPT; ++j) {
        uint32_t d = 0;
        const bool v = i0 + (uint64_t)j * 64u < nv && pt_digit(a, k[j], d, bad);
        const uint64_t act = __ballot(v);
        uint32_t r = 0;
        if (act) {  // (wave-uniform)
            const uint64_t m = match_any(d, act, a.dbits);
            if (v) {
                const uint32_t before = lane_rank(m);
                const uint32_t base = mine[d];
                if (before == 0) mine[d] = (uint16_t)(base + (uint32_t)__popcll(m));
                r = base + before;
            }
        }
        pk[j] = v ? (d | (r << 8) | (((uint32_t)k[j] & 255u) << 17) | 0x80000000u) : 0u;
    }
    (void)bad;  // (reported by k_part_hist)
    __syncthreads();
    // per digit: the chunk's run start (exclusive scan over the digits of the chunk's counts) and each wave's
    // place in the run (threads 0..ND-1, ND <= 256: waves 0..3)
    {
        uint32_t cw[SGD_PT_WAVES], t = 0;
        const uint32_t d = tid;
        if (d < ND) {
#pragma unroll
            for (uint32_t q = 0; q < SGD_PT_WAVES; ++q) { cw[q] = wc[q * ND + d]; t += cw[q]; }
        }
        const uint32_t incl = wave_incl_scan(d < ND ? t : 0u, lane);
        if (lane == 63 && w < 4) ws[w] = incl;
        __syncthreads();
        if (d < ND) {
            uint32_t run = incl - t;
            for (uint32_t q = 0; q < w; ++q) run += ws[q];
            bst[d] = run;
#pragma unroll
            for (uint32_t q = 0; q < SGD_PT_WAVES; ++q) { wc[q * ND + d] = (uint16_t)run; run += cw[q]; }
            if (d == ND - 1) ws[15] = run;
        }
    }
    __syncthreads();

    // gather each event's element and place it in LDS, digit-sorted
#pragma unroll
    for (uint32_t j = 0; j < EPT; ++j) {
        const uint32_t x = pk[j];
        if (x >> 31) {
            if constexpr (SRC == PT_GATHER) {
                if (e.tag) el[j][0] |= ((x >> 17) & 255u) << 24;
            }
            const uint32_t d = x & 255u;
            const uint32_t pos = mine[d] + ((x >> 8) & 511u);
#pragma unroll
            for (int u = 0; u < S; ++u) el_l[pos * S + u] = el[j][u];
            dg[pos] = (uint8_t)d;
            if constexpr (SIDE == PS_KEY) side_l[pos] = k[j];
            if constexpr (SIDE == PS_CODE) side_l[pos] = (uint16_t)(((uint64_t)k[j] >> a.cshift) & a.cmask);
        }
    }
    __syncthreads();

    // out in digit-sorted order: each digit's run to its global start, consecutive lanes to consecutive places
    const uint32_t nvc = ws[15];
    for (uint32_t p = tid; p < nvc; p += SGD_PT_THREADS) {
        const uint32_t d = dg[p];
        const uint32_t dst = gof[d] + (p - bst[d]);
        uint32_t v[S];
#pragma unroll
        for (int u = 0; u < S; ++u) v[u] = el_l[p * S + u];
        st_elem<S>((uint32_t*)e.out + (size_t)dst * S, v);
        if constexpr (SIDE != PS_NONE) ((typename SD::U*)a.side_out)[dst] = side_l[p];
    }
}

// ---- the fused grouping's tile starts, from the tile codes of the sorted elements -------------------------------
// tile_lo[t] = first element of tile t (tiles without events: the next tile's start), tile_lo[n_tiles] = nv
__global__ void __launch_bounds__(256) k_tile_bounds(const uint16_t* __restrict__ code, const uint32_t* __restrict__ n_dev,
                                                     uint32_t n_tiles, uint32_t* __restrict__ tile_lo) {
    const uint32_t nv = *n_dev;
    const uint32_t i0 = (blockIdx.x * blockDim.x + threadIdx.x) * 8u;  // 8 consecutive elements per thread
    if (i0 > nv) return;
    int32_t c[9];
    c[0] = i0 > 0 ? (int32_t)code[i0 - 1] : -1;
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) c[q + 1] = i0 + q < nv ? (int32_t)code[i0 + q] : (int32_t)n_tiles;
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
        if (i0 + q > nv) break;
        for (int32_t t = c[q] + 1; t <= c[q + 1]; ++t) tile_lo[t] = i0 + q;
    }
}

// ---- per-key bounds ----------------------------------------------------------------------------------
// from the digit starts of a single pass whose digit is the whole key (K <= 256)
__global__ void __launch_bounds__(256) k_part_lo_bounds(const uint32_t* __restrict__ lo, uint32_t K,
                                                        uint32_t* __restrict__ seg_begin, uint32_t* __restrict__ seg_end) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    seg_begin[k] = lo[k];
    seg_end[k] = lo[k + 1];
}

// from the sorted keys of the last pass (nv valid on the device); keys without events get an empty [i, i)
__global__ void __launch_bounds__(256) k_part_bounds(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ n_dev,
                                                     uint32_t K, uint32_t* __restrict__ seg_begin,
                                                     uint32_t* __restrict__ seg_end) {
    const uint32_t nv = *n_dev;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > nv) return;
    const uint32_t cur = i < nv ? sk[i] : K;            // (K: past the last run)
    const uint32_t prv = i > 0 ? sk[i - 1] : 0xffffffffu;
    if (cur == prv) return;
    if (i > 0) seg_end[prv] = i;
    for (uint32_t g = (i == 0) ? 0u : prv + 1u; g < cur; ++g) seg_begin[g] = seg_end[g] = i;
    if (cur < K) seg_begin[cur] = i;
}

// ---- host side ----------------------------------------------------------------------------------------
#ifndef SGD_PT_EPT_NARROW
#define SGD_PT_EPT_NARROW 4
#endif
constexpr uint32_t ept_of(uint32_t S) { return S <= 4 ? (uint32_t)SGD_PT_EPT_NARROW : 2u; }
constexpr uint32_t PT_HC = 8;  // chunks per histogram block

uint32_t nblk_of(uint64_t n, uint32_t S) {
    const uint64_t ce = (uint64_t)SGD_PT_THREADS * ept_of(S);
    return (uint32_t)std::max<uint64_t>(1, (n + ce - 1) / ce);
}

template <int DS, int SRC, int S, int SIDE> hipError_t run_pass(PassArgs a, const ElemArgs& e, hipStream_t st) {
    typedef typename DKey<DS>::T T;
    constexpr uint32_t EPT = ept_of(S);
    a.nblk = nblk_of(a.n, S);
    a.nb8 = (a.nblk + 7u) / 8u;
    const uint32_t grid = 8u * a.nb8;
    hipLaunchKernelGGL((k_part_hist<DS, EPT, PT_HC>), dim3((a.nblk + PT_HC - 1) / PT_HC), dim3(SGD_PT_THREADS), 0, st, a);
    if (hipError_t x = hipGetLastError()) return x;
    hipLaunchKernelGGL(k_part_scan, dim3(a.ndig), dim3(256), 0, st, a.mat, a.nblk, a.tot);
    if (hipError_t x = hipGetLastError()) return x;
    constexpr uint32_t SB = SideT<SIDE, T>::B;
    const size_t sl = pt_scatter_lds(SGD_PT_THREADS * EPT, S, SB, a.ndig);
    static bool attr = [] {
        (void)hipFuncSetAttribute((const void*)k_part_scatter<DS, SRC, S, SIDE, EPT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)pt_scatter_lds(SGD_PT_THREADS * EPT, S, SB, SGD_PT_MAX_DIG));
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
    hipLaunchKernelGGL((k_part_scatter<DS, SRC, S, SIDE, EPT>), dim3(grid), dim3(SGD_PT_THREADS), sl, st, a, e);
    return hipGetLastError();
}

// first pass of a grouping: elements gathered from the batch (W payload words; 0: positions)
template <int SIDE> hipError_t run_gather(const PassArgs& a, const ElemArgs& e, uint32_t W, hipStream_t st) {
    switch (W) {
    case 0: return run_pass<PD_U32, PT_IDX, 1, SIDE>(a, e, st);
    case 1: return run_pass<PD_U32, PT_GATHER, 3, SIDE>(a, e, st);
    case 2: return run_pass<PD_U32, PT_GATHER, 4, SIDE>(a, e, st);
    case 3: return run_pass<PD_U32, PT_GATHER, 5, SIDE>(a, e, st);
    default: return run_pass<PD_U32, PT_GATHER, 6, SIDE>(a, e, st);
    }
}

// a later pass: elements of S words moved
template <int DS, int SIDE> hipError_t run_move(const PassArgs& a, const ElemArgs& e, uint32_t S, hipStream_t st) {
    switch (S) {
    case 1: return run_pass<DS, PT_MOVE, 1, SIDE>(a, e, st);
    case 3: return run_pass<DS, PT_MOVE, 3, SIDE>(a, e, st);
    case 4: return run_pass<DS, PT_MOVE, 4, SIDE>(a, e, st);
    case 5: return run_pass<DS, PT_MOVE, 5, SIDE>(a, e, st);
    default: return run_pass<DS, PT_MOVE, 6, SIDE>(a, e, st);
    }
}

PassArgs base_args(uint32_t n, const PartScratch& s) {
    PassArgs a{};
    a.n = n;
    a.mat = s.mat;
    a.tot = s.tot;
    return a;
}

uint32_t bits_for(uint64_t K) {
    uint32_t b = 0;
    while (b < 64 && (1ull << b) < K) b++;
    return b;
}

}  // namespace

size_t sgd_part_scratch_bytes(uint64_t max_n) {
    const uint64_t nblk = nblk_of(max_n, 6);  // (the smallest chunks: the most of them)
    size_t b = 0;
    b += (size_t)SGD_PT_MAX_DIG * nblk * 4 + 256;
    b += (size_t)SGD_PT_MAX_DIG * 4 + 256;
    b += 2 * ((size_t)(SGD_PT_MAX_DIG + 1) * 4 + 256);
    b += 2 * ((size_t)max_n * 8 + 256);
    b += 2 * ((size_t)max_n * 24 + 256);
    return b;
}

PartScratch sgd_part_scratch(void* base, uint64_t max_n) {
    const uint64_t nblk = nblk_of(max_n, 6);
    char* p = (char*)base;
    auto take = [&](size_t bytes) {
        void* r = p;
        p += (bytes + 255) & ~(size_t)255;
        return r;
    };
    PartScratch s{};
    s.mat = (uint32_t*)take((size_t)SGD_PT_MAX_DIG * nblk * 4);
    s.tot = (uint32_t*)take((size_t)SGD_PT_MAX_DIG * 4);
    s.lo[0] = (uint32_t*)take((size_t)(SGD_PT_MAX_DIG + 1) * 4);
    s.lo[1] = (uint32_t*)take((size_t)(SGD_PT_MAX_DIG + 1) * 4);
    s.keys[0] = take((size_t)max_n * 8);
    s.keys[1] = take((size_t)max_n * 8);
    s.el[0] = take((size_t)max_n * 24);
    s.el[1] = take((size_t)max_n * 24);
    return s;
}

hipError_t sgd_group_tiles_fused(const GroupArgs& g, uint32_t* tile_lo, hipStream_t stream) {
    const uint32_t tbits = g.tile_bits ? g.tile_bits : SGD_PT_TILE_BITS;
    if (tbits > 8u || !sgd_fused_ok(g.K, g.n, g.W, tbits) || g.n == 0) return hipErrorInvalidValue;
    const uint32_t nt = (g.K + (1u << tbits) - 1) >> tbits;
    const uint32_t tb = bits_for(nt);
    ElemArgs e{};
    e.ps = g.src;
    e.tag = 1;
    PassArgs a = base_args(g.n, g.s);
    a.mode = PT_RANGE;
    a.K = g.K;
    a.drop_null = g.drop_null;
    a.keys = g.keys;
    a.err = g.err;
    a.shift = tbits;
    if (tb <= SGD_PT_MAX_BITS) {  // one pass on the whole tile id: its digit starts are the tile starts
        a.dbits = tb;
        a.ndig = nt;
        a.lo = tile_lo;
        e.out = g.out;
        return run_gather<PS_NONE>(a, e, g.W, stream);
    }
    // LSD: the low tile bits carrying the tile id as a u16 code, then the high bits (the codes follow the
    // elements), then the tile starts from the sorted codes
    const uint32_t b1 = tb / 2, b2 = tb - b1;
    a.dbits = b1;
    a.ndig = 1u << b1;
    a.cshift = tbits;
    a.cmask = 0xffffu;
    a.side_out = g.s.keys[0];
    a.lo = g.s.lo[0];
    e.out = g.s.el[0];
    if (hipError_t x = run_gather<PS_CODE>(a, e, g.W, stream)) return x;
    PassArgs b = base_args(g.n, g.s);
    b.n_dev = g.s.lo[0] + a.ndig;
    b.shift = b1;
    b.dbits = b2;
    b.ndig = ((nt - 1) >> b1) + 1;
    b.keys = g.s.keys[0];
    b.cmask = 0xffffu;
    b.side_out = g.s.keys[1];
    b.lo = g.s.lo[1];
    ElemArgs f{};
    f.in = g.s.el[0];
    f.out = g.out;
    if (hipError_t x = run_move<PD_U16, PS_CODE>(b, f, g.W + 2, stream)) return x;
    hipLaunchKernelGGL(k_tile_bounds, dim3((g.n + 1 + 2047) / 2048), dim3(256), 0, stream, (const uint16_t*)g.s.keys[1],
                       (const uint32_t*)(g.s.lo[1] + b.ndig), nt, tile_lo);
    return hipGetLastError();
}

hipError_t sgd_group_sorted(const GroupArgs& g, hipStream_t stream) {
    if (g.n == 0) return hipSuccess;
    const uint32_t bits = bits_for(g.K);
    const uint32_t np = std::max(1u, (bits + SGD_PT_MAX_BITS - 1) / SGD_PT_MAX_BITS);
    const uint32_t S = g.W == 0 ? 1u : g.W + 2u;
    const uint32_t* n_dev = nullptr;
    uint32_t shift = 0;
    for (uint32_t p = 0; p < np; ++p) {
        const bool last = p + 1 == np;
        PassArgs a = base_args(g.n, g.s);
        a.n_dev = n_dev;
        a.shift = shift;
        a.dbits = (bits - shift + (np - p) - 1) / (np - p);  // the remaining bits split evenly
        a.ndig = np == 1 ? std::max(1u, g.K) : (1u << a.dbits);
        a.mode = p == 0 ? PT_RANGE : 0u;
        a.K = g.K;
        a.drop_null = g.drop_null;
        a.keys = p == 0 ? (const void*)g.keys : (const void*)g.s.keys[(p - 1) & 1];
        a.side_out = g.s.keys[p & 1];
        a.lo = g.s.lo[p & 1];
        a.err = g.err;
        ElemArgs e{};
        e.ps = g.src;
        e.in = p == 0 ? nullptr : g.s.el[(p - 1) & 1];
        e.out = last ? g.out : g.s.el[p & 1];
        hipError_t x;
        if (np == 1) x = run_gather<PS_NONE>(a, e, g.W, stream);
        else if (p == 0) x = run_gather<PS_KEY>(a, e, g.W, stream);
        else x = run_move<PD_U32, PS_KEY>(a, e, S, stream);
        if (x) return x;
        n_dev = a.lo + a.ndig;
        shift += a.dbits;
    }
    if (np == 1) {
        hipLaunchKernelGGL(k_part_lo_bounds, dim3((g.K + 255) / 256), dim3(256), 0, stream, g.s.lo[0], g.K, g.seg_begin,
                           g.seg_end);
    } else {
        hipLaunchKernelGGL(k_part_bounds, dim3((g.n + 1 + 255) / 256), dim3(256), 0, stream,
                           (const uint32_t*)g.s.keys[(np - 1) & 1], n_dev, g.K, g.seg_begin, g.seg_end);
    }
    return hipGetLastError();
}

hipError_t sgd_sort_pairs(const void* keys_in, void* keys_out, const uint32_t* vals_in, uint32_t* vals_out, uint32_t n,
                          uint32_t bits, bool key64, bool desc, const PartScratch& s, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t np = std::max(1u, (bits + SGD_PT_MAX_BITS - 1) / SGD_PT_MAX_BITS);
    uint32_t shift = 0;
    for (uint32_t p = 0; p < np; ++p) {
        const bool last = p + 1 == np;
        PassArgs a = base_args(n, s);
        a.shift = shift;
        a.dbits = (bits - shift + (np - p) - 1) / (np - p);
        a.ndig = 1u << a.dbits;
        a.mode = desc ? PT_DESC : 0u;
        a.keys = p == 0 ? keys_in : (const void*)s.keys[(p - 1) & 1];
        a.side_out = last ? keys_out : s.keys[p & 1];
        a.lo = s.lo[p & 1];
        ElemArgs e{};
        e.in = p == 0 ? (const void*)vals_in : s.el[(p - 1) & 1];
        e.out = last ? (void*)vals_out : s.el[p & 1];
        hipError_t x = key64 ? run_pass<PD_U64, PT_MOVE, 1, PS_KEY>(a, e, stream)
                             : run_pass<PD_U32, PT_MOVE, 1, PS_KEY>(a, e, stream);
        if (x) return x;
        shift += a.dbits;
    }
    return hipSuccess;
}
