// p2_kernels.hip — ahead-of-time gfx950 kernels around the NFA advance: the ordered scatter of the emitted
// matches, projection, aggregators, purge and the small helpers.  The advance kernel itself is
// query-specialised and compiled at engine creation (p2_jit.hip, sg_jit.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/siddhi_gpu_ir.h"
#include "java_ops.h"
#include "sg_engine.h"

// ------------------------------------------------------------------------------------------------
// match ordering: batch event t's matches go to out_count + (exclusive prefix of the per-event counts
// over arrival order), i.e. ascending trigger seq, then emission order — the reference's callback
// order (MultiProcessStreamReceiver.java:119-121).  Tiles of SGD_ORDER_TILE triggers: k_order_sums (tile
// totals), then k_order_scatter, a workgroup per tile: the tile's prefix reduced from the earlier tiles'
// totals, its 16 rows of counts scanned (256 consecutive triggers per row, so the lanes' output records are
// consecutive), the records written.  t_desc entries count only under this batch's tag, so nothing is
// cleared behind the batch.  chain_len is the constant 1/1 of a two-state match and was written once at
// allocation.  (A one-pass decoupled look-back over the tiles was measured: 0.67 ms against 0.23 ms for the
// two kernels — each tile's wait on its predecessors' words crossed the XCDs' L2s.)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ord_wave_incl_scan(uint32_t x, int lane) {
    const int r = lane & 15;
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false); if (r >= 1) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false); if (r >= 2) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false); if (r >= 4) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false); if (r >= 8) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false); if (lane & 16) x += t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false); if (lane >= 32) x += t;
    return x;
}

__global__ void __launch_bounds__(256) k_order_sums(const uint64_t* __restrict__ t_desc, uint32_t n, uint32_t ep,
                                                    uint32_t* __restrict__ tile_sum) {
    __shared__ uint32_t part[4];
    const uint32_t base = blockIdx.x * SGD_ORDER_TILE;
    uint32_t c = 0;
    for (uint32_t j = 0; j < SGD_ORDER_TILE / 256; ++j) {
        const uint32_t t = base + j * 256 + threadIdx.x;
        if (t < n) {
            const uint64_t d = t_desc[t];
            c += SGD_TD_TAGOF(d) == ep ? SGD_TD_CNT(d) : 0u;
        }
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

#ifndef SGD_ORDER_U
#define SGD_ORDER_U 8   // (records per thread per round; 40-step A/B: 2 / 4 / 8 -> ordering 0.215 / 0.211 / 0.209 ms)
#endif
__global__ void __launch_bounds__(256) k_order_scatter(const ScatterParams s, uint32_t ntiles) {
    // Phase 1: all rows' descriptors are loaded up front, the 16 rows' wave scans combined through one
    // LDS round trip: every trigger of the tile gets its tile-local output offset.  Phase 2 is output-major: each thread owns consecutive output records (coalesced
    // stores); a window of WIN records at a time, each record's trigger found through an owner map in LDS.
    constexpr int ROWS = SGD_ORDER_TILE / 256;
    constexpr uint32_t WIN = SGD_ORDER_TILE / 2;
    __shared__ uint32_t wtot[ROWS][4];
    __shared__ uint32_t owner[WIN];          // window record -> tile-local trigger index
    __shared__ uint32_t loc[SGD_ORDER_TILE]; // tile-local trigger -> its first record (tile-local)
    __shared__ uint16_t cnt[SGD_ORDER_TILE]; // tile-local trigger -> its record count (<= SGD_MAX_CAP) | inline << 15
    __shared__ uint32_t fst[SGD_ORDER_TILE]; // tile-local trigger -> its first raw slot (inline: e1 seq - seq_base)
    __shared__ unsigned long long s_excl[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.x;
    const uint32_t base = tile * SGD_ORDER_TILE;
    // the tile's prefix: the sum of every earlier tile's count (k_order_sums), reduced here (at most 4096 tiles at
    // 2^24 triggers: a few L2-resident loads per thread instead of a scan kernel and its launch)
    {
        unsigned long long v = 0;
        for (uint32_t i = threadIdx.x; i < tile; i += 256) v += s.tile_sum[i];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) s_excl[wv] = v;
    }
    const uint32_t ep = s.epoch;
    uint64_t d[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
        const uint32_t t = base + j * 256 + threadIdx.x;
        const uint64_t x = t < s.n ? s.t_desc[t] : 0ull;
        d[j] = SGD_TD_TAGOF(x) == ep ? x : 0ull;
    }
    uint32_t incl[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
        incl[j] = ord_wave_incl_scan(SGD_TD_CNT(d[j]), lane);
        if (lane == 63) wtot[j][wv] = incl[j];
    }
    __syncthreads();
    uint32_t running = 0;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
        uint32_t before = 0, row = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t x = wtot[j][w];
            before += (w < wv) ? x : 0u;
            row += x;
        }
        const uint32_t c = SGD_TD_CNT(d[j]);
        const uint32_t tl = j * 256 + threadIdx.x;
        loc[tl] = running + before + incl[j] - c;
        cnt[tl] = (uint16_t)(c | ((d[j] & SGD_TD_INLINE) ? 0x8000u : 0u));
        if (c) fst[tl] = (uint32_t)d[j];
        running += row;
    }
    const uint32_t total = running;  // records of this tile
    const unsigned long long toff = s_excl[0] + s_excl[1] + s_excl[2] + s_excl[3];
    if (s.out_first) {  // aggregators: where each trigger's records start
#pragma unroll 1
        for (int j = 0; j < ROWS; ++j) {
            const uint32_t tl = j * 256 + threadIdx.x;
            if (base + tl < s.n) {
                const uint32_t c = cnt[tl] & 0x7fffu;
                const uint64_t r = (*s.out_count + toff + loc[tl]) % s.capacity;
                s.out_first[base + tl] = c ? (((uint64_t)c << 32) | r) : 0ull;
            }
        }
    }
    const uint64_t out0 = *s.out_count + toff;   // monotonic record number
    if (tile == ntiles - 1 && threadIdx.x == 0) *s.batch_total = toff + total;
    if (out0 + total - s.win_start > s.capacity) {  // the ring would overwrite unpolled records: fail loudly
        if (threadIdx.x == 0 && total) atomicOr(s.err, (uint32_t)SGD_ERR_MATCH_CAP);
        return;
    }
    for (uint32_t w0 = 0; w0 < total; w0 += WIN) {
        const uint32_t w1 = min(total, w0 + WIN);
#pragma unroll 1
        for (int j = 0; j < ROWS; ++j) {
            const uint32_t tl = j * 256 + threadIdx.x;
            const uint32_t l0 = loc[tl], c = cnt[tl] & 0x7fffu;
            const uint32_t a = max(l0, w0), b = min(l0 + c, w1);
            for (uint32_t r = a; r < b; ++r) owner[r - w0] = tl;
        }
        __syncthreads();
        const uint64_t ring0 = out0 % s.capacity;
        // SGD_ORDER_U records per thread per round: their owner lookups and their loads of the trigger's
        // key / timestamp / e1 seq issued together before any store, so the loads' latencies overlap
        for (uint32_t q0 = w0 + threadIdx.x; q0 < w1; q0 += 256 * SGD_ORDER_U) {
            uint32_t tlu[SGD_ORDER_U], kyu[SGD_ORDER_U];
            uint64_t e1u[SGD_ORDER_U], tsu[SGD_ORDER_U];
#pragma unroll
            for (int u = 0; u < SGD_ORDER_U; ++u) {
                const uint32_t q = q0 + u * 256;
                if (q < w1) {
                    const uint32_t tl = owner[q - w0];
                    const uint32_t t = base + tl;
                    tlu[u] = tl;
                    kyu[u] = s.key ? s.key[t] : 0u;
                    tsu[u] = s.ts[t];
                    e1u[u] = (SG_EXP(s.exp) & 1) ? 0ull
                             : (cnt[tl] & 0x8000u) ? s.seq_base + (uint64_t)(int64_t)(int32_t)fst[tl]
                                                   : s.raw_e1[fst[tl] + (q - loc[tl])];
                }
            }
#pragma unroll
            for (int u = 0; u < SGD_ORDER_U; ++u) {
                const uint32_t q = q0 + u * 256;
                if (q >= w1) break;
                const uint32_t tl = tlu[u];
                const uint64_t trig = s.seq_base + base + tl;
                uint64_t o = ring0 + q;
                if (o >= s.capacity) o -= s.capacity;
                s.o_trig[o] = trig;
                *reinterpret_cast<ulonglong2*>(s.o_slot + 2 * o) = make_ulonglong2(e1u[u], trig);  // {e1, e2} seqs
                s.o_key[o] = kyu[u];
                s.o_ts[o] = tsu[u];  // StreamPostStateProcessor.java:68: StateEvent ts = ts of the e2 event
                if (s.o_capw) {      // on-device projection: the partial's captures in output order
                    const uint64_t r = fst[tl] + (q - loc[tl]);
                    for (uint32_t w = 0; w < s.n_capw; ++w)
                        s.o_capw[(size_t)w * s.capacity + o] = s.raw_capw[(size_t)w * s.raw_capacity + r];
                    s.o_capnull[o] = s.raw_capnull[r];
                }
            }
        }
        __syncthreads();  // the owner map is rebuilt for the next window
    }
}

// QuerySelector.processNoGroupBy (QuerySelector.java:162-206) on the device for the batch's matches,
// output slots [out_count - batch_total, out_count): e1's attributes from the captures the partial
// carried, e2's (the trigger's) from the batch columns; Java numerics from java_ops.h
__global__ void __launch_bounds__(256) k_project(const ProjParams p) {
    const uint64_t total = *p.batch_total, o0 = (*p.out_count - total) % p.capacity;
    uint32_t err = 0;
    if (total > p.capacity) return;  // (the ordering reported the overflow)
    const uint32_t it0 = p.phase == 0 ? 0u : p.n_agg, it1 = p.phase == 0 ? p.n_agg : p.n_items;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t o = o0 + i;
        if (o >= p.capacity) o -= p.capacity;
        const uint64_t t = p.o_trig[o] - p.seq_base;
        const uint32_t cn = p.o_capnull[o];
        for (uint32_t it = it0; it < it1; ++it) {
            const GVal v = jo_eval(
                p.code, p.item_pc[it], p.item_len[it], err,
                [&](uint32_t src, uint32_t x, int32_t chain) -> GVal {
                    if (src == 2) {  // select item x of this row (evaluated before `having`)
                        const size_t r = (size_t)x * p.capacity + o;
                        return GVal{p.pval[r], p.pnull[r] != 0};
                    }
                    if (src == 3) {  // aggregator x after this row's event (k_agg)
                        const size_t r = (size_t)x * p.capacity + o;
                        return GVal{p.aggv[r], p.aggnull[r] != 0};
                    }
                    if (!(chain == 0 || chain == -1)) return GVal{0, true};  // a single-event slot
                    if (src == 0) {  // e1 capture x
                        const uint32_t w = p.capw_off[x];
                        uint64_t b = p.o_capw[(size_t)w * p.capacity + o];
                        const uint32_t ty = p.cap_type[x];
                        if (ty == SG_T_LONG || ty == SG_T_DOUBLE) b |= (uint64_t)p.o_capw[(size_t)(w + 1) * p.capacity + o] << 32;
                        return GVal{b, ((cn >> x) & 1u) != 0};
                    }
                    const void* c = p.col[x];  // the trigger event's attribute x
                    uint64_t b;
                    switch (p.col_type[x]) {
                    case SG_T_LONG: case SG_T_DOUBLE: b = ((const uint64_t*)c)[t]; break;
                    case SG_T_BOOL: b = ((const uint8_t*)c)[t] ? 1u : 0u; break;
                    default: b = ((const uint32_t*)c)[t];
                    }
                    return GVal{b, p.col_null[x] && p.col_null[x][t] != 0};
                },
                [&](uint32_t, int32_t chain) -> bool { return !(chain == 0 || chain == -1); });
            if (p.phase == 0) {
                p.aggv[(size_t)it * p.capacity + o] = v.b;
                p.aggnull[(size_t)it * p.capacity + o] = v.null ? 1 : 0;
            } else {
                p.pval[(size_t)(it - p.n_agg) * p.capacity + o] = v.b;
                p.pnull[(size_t)(it - p.n_agg) * p.capacity + o] = v.null ? 1 : 0;
            }
        }
    }
    if (err) atomicOr(p.err, (uint32_t)SGD_ERR_PROJ);
}

// The aggregators of QuerySelector.processNoGroupBy (QuerySelector.java:162-206) run per partition key
// over the key's matches in output order: one thread per key walks its batch events in arrival order
// (the key's run of the grouped payload) and each event's records in emission order, applying processAdd
// (java_ops.h jo_agg) to the argument phase 0 wrote and leaving the aggregator's value in its place.  The
// state (count, value, has-value) persists per key across batches.
__global__ void __launch_bounds__(256) k_agg(const AggParams a) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.K) return;
    const uint32_t b = a.seg_begin[k], e = a.seg_end[k];
    if (b >= e) return;
    for (uint32_t f = 0; f < a.n_agg; ++f) {
        const size_t si = (size_t)f * a.K + k;
        int64_t n = a.st_n[si];
        uint64_t v = a.st_v[si];
        bool has = a.st_has[si] != 0;
        const uint32_t ty = a.agg_type[f];
        const uint32_t fn = (ty >> 8) & 0xffu;
        const int at = (int)(ty & 0xffu);
        bool touched = false;
        for (uint32_t j = b; j < e; ++j) {
            const uint32_t t = a.payload[(size_t)j * a.stride];
            const uint64_t d = a.out_first[t];
            const uint32_t c = (uint32_t)(d >> 32);
            uint64_t r = (uint32_t)d;
            for (uint32_t q = 0; q < c; ++q) {
                const size_t x = (size_t)f * a.capacity + r;
                const GVal res = jo_agg(fn, at, GVal{a.aggv[x], a.aggnull[x] != 0}, n, v, has);
                a.aggv[x] = res.b;
                a.aggnull[x] = res.null ? 1 : 0;
                touched = true;
                if (++r == a.capacity) r = 0;
            }
        }
        if (touched) {
            a.st_n[si] = n;
            a.st_v[si] = v;
            a.st_has[si] = has ? 1 : 0;
        }
    }
}

__global__ void __launch_bounds__(256) k_reset_agg(const uint32_t* __restrict__ keys, uint32_t n, uint32_t K,
                                                   uint32_t n_agg, int64_t* st_n, uint64_t* st_v, uint8_t* st_has) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || keys[i] >= K) return;
    for (uint32_t f = 0; f < n_agg; ++f) {
        const size_t si = (size_t)f * K + keys[i];
        st_n[si] = 0;
        st_v[si] = 0;
        st_has[si] = 0;
    }
}

int sgd_launch_project(const ProjParams& p, ihipStream_t* stream) {
    hipLaunchKernelGGL(k_project, dim3(1024), dim3(256), 0, stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_agg(const AggParams& a, ihipStream_t* stream) {
    hipLaunchKernelGGL(k_agg, dim3((a.K + 255) / 256), dim3(256), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_reset_agg(const uint32_t* keys, uint32_t n, uint32_t K, uint32_t n_agg, int64_t* st_n, uint64_t* st_v,
                         uint8_t* st_has, ihipStream_t* stream) {
    if (n == 0 || n_agg == 0) return 0;
    hipLaunchKernelGGL(k_reset_agg, dim3((n + 255) / 256), dim3(256), 0, stream, keys, n, K, n_agg, st_n, st_v, st_has);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// partition purge: the listed keys' headers go back to "never seen" (INIT clear, no partials); the
// slab rows they held are dead once the counts are zero
__global__ void __launch_bounds__(256) k_reset_keys(const uint32_t* __restrict__ keys, uint32_t n, uint32_t n_keys,
                                                    uint32_t* __restrict__ hdr, uint32_t* __restrict__ err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = keys[i];
    if (k >= n_keys) {
        atomicOr(err, (uint32_t)SGD_ERR_KEY_RANGE);
        return;
    }
    hdr[k] = 0u;
}

// validation of a device array of key ids: *bad = 1 if any id is outside [0, n_keys) (*bad is cleared
// by the wrapper first)
__global__ void __launch_bounds__(256) k_check_keys(const uint32_t* __restrict__ keys, uint32_t n, uint32_t n_keys,
                                                    uint32_t* __restrict__ bad) {
    bool b = false;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b |= keys[i] >= n_keys;
    if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

__global__ void k_bump(unsigned long long* out_count, const unsigned long long* batch_total) {
    *out_count += *batch_total;
}

// per-batch counters of the staged advance pass: one row per wave -> the cumulative totals (blocks stride
// over the rows; one atomic per counter per block)
__global__ void __launch_bounds__(256) k_stats_reduce(const unsigned long long* __restrict__ wstats,
                                                      uint32_t n_waves, unsigned long long* __restrict__ stats,
                                                      unsigned long long* __restrict__ raw_count,
                                                      uint32_t* __restrict__ dlist_n) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the next advance's atomic slot counter and HBM-pass list
        *raw_count = 0;
        dlist_n[0] = 0;
        dlist_n[1] = 0;
    }
    __shared__ unsigned long long part[SGD_ST_N][4];
    unsigned long long acc[SGD_ST_N];
    for (int i = 0; i < SGD_ST_N; ++i) acc[i] = 0;
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < n_waves; w += gridDim.x * blockDim.x)
        for (int i = 0; i < SGD_ST_N; ++i) acc[i] += wstats[(size_t)w * SGD_ST_N + i];
    for (int i = 0; i < SGD_ST_N; ++i)
        for (int off = 32; off > 0; off >>= 1) acc[i] += __shfl_xor(acc[i], off, 64);
    const int wv = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0)
        for (int i = 0; i < SGD_ST_N; ++i) part[i][wv] = acc[i];
    __syncthreads();
    if (threadIdx.x < SGD_ST_N) {
        const unsigned long long t = part[threadIdx.x][0] + part[threadIdx.x][1] + part[threadIdx.x][2] + part[threadIdx.x][3];
        if (t) atomicAdd(&stats[threadIdx.x], t);
    }
}

// the smallest e1 seq a live partial holds (pending + staged rows of every key; the multi-device engine trims
// its seq maps below it)
__global__ void __launch_bounds__(256) k_min_seq(const uint32_t* __restrict__ hdr, const uint64_t* __restrict__ p_seq,
                                                 uint32_t n_keys, unsigned long long* out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long m = ~0ull;
    if (k < n_keys) {
        const uint32_t h = hdr[k];
        const uint32_t c = SGD_H_NPEND(h) + SGD_H_NSTG(h);
        for (uint32_t j = 0; j < c; j++) {
            const unsigned long long q = p_seq[(size_t)j * n_keys + k];
            m = q < m ? q : m;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, 64);
        m = o < m ? o : m;
    }
    if ((threadIdx.x & 63) == 0 && m != ~0ull) atomicMin(out, m);
}

// ------------------------------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------------------------------
int sgd_launch_reset_keys(const uint32_t* keys, uint32_t n, uint32_t n_keys, uint32_t* hdr, uint32_t* err,
                          ihipStream_t* stream) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_reset_keys, dim3((n + 255) / 256), dim3(256), 0, stream, keys, n, n_keys, hdr, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_check_keys(const uint32_t* keys, uint32_t n, uint32_t n_keys, uint32_t* bad, ihipStream_t* stream) {
    if (hipMemsetAsync(bad, 0, 4, stream) != hipSuccess) return -1;
    if (n == 0) return 0;
    const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 1024u);
    hipLaunchKernelGGL(k_check_keys, dim3(blocks), dim3(256), 0, stream, keys, n, n_keys, bad);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_stats_reduce(const unsigned long long* wstats, uint32_t n_waves, unsigned long long* stats,
                            unsigned long long* raw_count, uint32_t* dlist_n, ihipStream_t* stream) {
    const uint32_t blocks = std::max(1u, std::min(64u, (n_waves + 255u) / 256u));
    hipLaunchKernelGGL(k_stats_reduce, dim3(blocks), dim3(256), 0, stream, wstats, n_waves, stats, raw_count, dlist_n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_scatter(const ScatterParams& s, ihipStream_t* stream) {
    if (s.n == 0) return 0;
    const uint32_t nt = (s.n + SGD_ORDER_TILE - 1) / SGD_ORDER_TILE;
    hipLaunchKernelGGL(k_order_sums, dim3(nt), dim3(256), 0, stream, s.t_desc, s.n, s.epoch, s.tile_sum);
    hipLaunchKernelGGL(k_order_scatter, dim3(nt), dim3(256), 0, stream, s, nt);
    hipLaunchKernelGGL(k_bump, dim3(1), dim3(1), 0, stream, s.out_count, s.batch_total);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_min_seq(const uint32_t* hdr, const uint64_t* p_seq, uint32_t n_keys, unsigned long long* out,
                       ihipStream_t* stream) {
    hipLaunchKernelGGL(k_min_seq, dim3((n_keys + 255) / 256), dim3(256), 0, stream, hdr, p_seq, n_keys, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
