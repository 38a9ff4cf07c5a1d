// shard_kernels.hip — multi-GPU ingest: bucket one rank's slice of the arrival-ordered
// stream by the rank that owns each event's partition key, as packed rows ready for one RCCL
// all_to_all, and unpack the received rows into the SoA columns sg_push_batch takes.
//
// Partition keys shard with no cross-key state (PartitionStateHolder.java:43-49,
// PartitionStreamReceiver.send :262-272): owner = key % world, local key = key / world.  The pack is
// a STABLE partition (arrival order kept within each destination), so a rank that receives the chunks
// of all source ranks in rank order holds its keys' events in global arrival order — per key exactly
// the order the reference processes them in.
//
// Layout: rows of W = 3 + n_cols 32-bit words {local key, ts lo, ts hi, col 0, ..}; the rows for
// destination d are contiguous and in arrival order, destinations in rank order.
//
// Kernels (tiles of SH_TILE events, one workgroup each, SH_WAVES waves; wave w owns the contiguous
// sub-range [w * SH_TILE / SH_WAVES, ...) of its tile, walked in rounds of 64 events):
//   k_sh_count   per (destination, tile) counts, destination-major (so one exclusive scan gives every
//                tile's first row per destination: k_sh_scan, one workgroup — world x tiles counts, 8K for 8
//                ranks at 4M events)
//   k_sh_scatter stable rank per event by ballot per destination and round, rows written
//   k_sh_unpack  rows -> SoA columns
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/siddhi_gpu.h"
#include "sg_sharded.h"

namespace {

constexpr uint32_t SH_TILE = 4096;
constexpr uint32_t SH_WAVES = 4;
constexpr uint32_t SH_PER_WAVE = SH_TILE / SH_WAVES;  // 1024 = 16 rounds of 64
constexpr uint32_t SH_MAX_WORLD = 64;
constexpr uint32_t SH_MAX_COLS = 8;

struct ShardArgs {
    uint64_t n;
    const uint32_t* key;   // global key ids
    const int64_t* ts;
    const uint32_t* col[SH_MAX_COLS];
    uint32_t ncols;
    uint32_t world;
    uint32_t ntiles;
    uint32_t* counts;      // [world][ntiles] (count pass) -> exclusive offsets (after the scan)
    uint32_t* rows;        // [n][3 + ncols], or [world][cap][3 + ncols] in block mode
    uint32_t cap;          // block mode (> 0): destination d's rows at [d * cap, d * cap + count_d)
    uint32_t* overflow;    // block mode: set when a destination receives more than cap rows
};

__global__ void __launch_bounds__(SH_WAVES * 64) k_sh_count(const ShardArgs a) {
    __shared__ uint32_t c[SH_MAX_WORLD];
    if (threadIdx.x < SH_MAX_WORLD) c[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * SH_TILE;
    for (uint32_t i = threadIdx.x; i < SH_TILE; i += blockDim.x) {
        const uint64_t e = base + i;
        if (e < a.n) atomicAdd(&c[a.key[e] % a.world], 1u);  // LDS atomics (order-free counts)
    }
    __syncthreads();
    if (threadIdx.x < a.world) a.counts[(size_t)threadIdx.x * a.ntiles + blockIdx.x] = c[threadIdx.x];
}

__global__ void __launch_bounds__(SH_WAVES * 64) k_sh_scatter(const ShardArgs a) {
    __shared__ uint32_t wtot[SH_WAVES][SH_MAX_WORLD];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x / 64;
    const uint64_t wbase = (uint64_t)blockIdx.x * SH_TILE + (uint64_t)wv * SH_PER_WAVE;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));  // the lanes below this one
    // pass 1: this wave's count per destination (lane d keeps destination d's)
    uint32_t mine = 0;
    for (uint32_t r = 0; r < SH_PER_WAVE / 64; ++r) {
        const uint64_t e = wbase + r * 64 + lane;
        const uint32_t d = e < a.n ? a.key[e] % a.world : 0xffffffffu;
        for (uint32_t dd = 0; dd < a.world; ++dd) {
            const uint64_t m = __ballot(d == dd);
            if (lane == dd) mine += (uint32_t)__popcll(m);
        }
    }
    wtot[wv][lane] = mine;
    __syncthreads();
    // lane d: first row of destination d for this wave = the tile's offset + the tile's earlier waves
    uint32_t base = 0;
    if (lane < a.world) {
        base = a.counts[(size_t)lane * a.ntiles + blockIdx.x];
        for (uint32_t w2 = 0; w2 < wv; ++w2) base += wtot[w2][lane];
    }
    // pass 2: stable rank (arrival order = round, then lane) and the packed row
    const uint32_t W = 3 + a.ncols;
    for (uint32_t r = 0; r < SH_PER_WAVE / 64; ++r) {
        const uint64_t e = wbase + r * 64 + lane;
        const bool in = e < a.n;
        const uint32_t k = in ? a.key[e] : 0u;
        const uint32_t d = in ? k % a.world : 0xffffffffu;
        uint32_t pos = 0;
        for (uint32_t dd = 0; dd < a.world; ++dd) {
            const uint64_t m = __ballot(d == dd);
            const uint32_t bdd = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)dd);
            if (d == dd) pos = bdd + (uint32_t)__popcll(m & lt);
            if (lane == dd) base += (uint32_t)__popcll(m);
        }
        if (in && a.cap) {  // block mode: the rank of the row within its destination, in d's block
            const uint32_t r0 = pos - a.counts[(size_t)d * a.ntiles];
            if (r0 >= a.cap) {
                atomicOr(a.overflow, 1u);
                continue;
            }
            pos = d * a.cap + r0;
        }
        if (in) {
            uint32_t* row = a.rows + (size_t)pos * W;
            row[0] = k / a.world;
            const uint64_t t = (uint64_t)a.ts[e];
            row[1] = (uint32_t)t;
            row[2] = (uint32_t)(t >> 32);
            for (uint32_t c = 0; c < a.ncols; ++c) row[3 + c] = a.col[c][e];
        }
    }
}

// block mode: the rows past each destination's count are padding (local key SG_KEY_NULL, dropped by an
// engine created with SG_CFG_NULL_KEYS; ts and columns zero)
__global__ void __launch_bounds__(256) k_sh_pad(uint32_t* __restrict__ rows, const unsigned long long* __restrict__ totals,
                                                uint32_t world, uint32_t cap, uint32_t W) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)world * cap) return;
    const uint32_t d = (uint32_t)(i / cap), r = (uint32_t)(i % cap);
    if (r < totals[d]) return;
    uint32_t* row = rows + i * W;
    row[0] = SG_KEY_NULL;
    for (uint32_t c = 1; c < W; ++c) row[c] = 0u;
}

__global__ void __launch_bounds__(256) k_sh_unpack(uint64_t n, const uint32_t* __restrict__ rows, uint32_t ncols,
                                                   uint32_t* __restrict__ key, int64_t* __restrict__ ts,
                                                   uint32_t* const* __restrict__ cols) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t W = 3 + ncols;
    const uint32_t* row = rows + i * W;
    key[i] = row[0];
    ts[i] = (int64_t)((uint64_t)row[1] | ((uint64_t)row[2] << 32));
    for (uint32_t c = 0; c < ncols; ++c) cols[c][i] = row[3 + c];
}

// destination totals from the scanned offsets (dest-major): total[d] = off[d+1][0] - off[d][0]
__global__ void k_sh_totals(const uint32_t* off, const uint32_t* last_counts, uint32_t world, uint32_t ntiles,
                            uint64_t n, unsigned long long* totals) {
    const uint32_t d = threadIdx.x;
    if (d >= world) return;
    const uint64_t a = off[(size_t)d * ntiles];
    const uint64_t b = (d + 1 < world) ? off[(size_t)(d + 1) * ntiles] : n;
    totals[d] = b - a;
    (void)last_counts;
}

// ---- the multi-device engine's split of a device batch (sg_sharded.cpp): SoA in, SoA out ----
// The batch stays on the device it was handed over on: every event gets its owner shard (key % world; local
// key key / world) and its stable rank within the owner (arrival order kept, as k_sh_scatter), and each column
// is scattered into one destination-major copy of the batch, shard r's events contiguous at [off_r, off_r +
// count_r).  opos[j] = the batch position of output row j (the shard's local -> global seq map, 4 B per event:
// the only thing copied to the host besides the per-shard counts).  Keys outside [0, K) set *err (an
// SG_KEY_NULL with null_keys is dropped instead).
struct FanArgs {
    uint64_t n;
    const uint32_t* key;
    uint32_t K, world, ntiles, null_keys;
    uint32_t* counts;   // [world][ntiles] counts, then (scanned) first output row per (shard, tile)
    uint32_t* pos;      // [n] output row of event i (0xffffffff: dropped)
    uint32_t* opos;     // [n] batch position of output row j
    uint32_t* okey;     // [n] local key of output row j
    uint32_t* err;
};

__device__ __forceinline__ uint32_t fan_owner(const FanArgs& a, uint64_t e) {
    if (e >= a.n) return 0xffffffffu;
    const uint32_t k = a.key[e];
    if (k < a.K) return k % a.world;
    if (!(a.null_keys && k == SG_KEY_NULL)) atomicOr(a.err, 1u);
    return 0xffffffffu;
}

__global__ void __launch_bounds__(SH_WAVES * 64) k_fan_count(const FanArgs a) {
    __shared__ uint32_t c[SH_MAX_WORLD];
    if (threadIdx.x < SH_MAX_WORLD) c[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * SH_TILE;
    for (uint32_t i = threadIdx.x; i < SH_TILE; i += blockDim.x) {
        const uint32_t d = fan_owner(a, base + i);
        if (d != 0xffffffffu) atomicAdd(&c[d], 1u);
    }
    __syncthreads();
    if (threadIdx.x < a.world) a.counts[(size_t)threadIdx.x * a.ntiles + blockIdx.x] = c[threadIdx.x];
}

__global__ void __launch_bounds__(SH_WAVES * 64) k_fan_rank(const FanArgs a) {
    __shared__ uint32_t wtot[SH_WAVES][SH_MAX_WORLD];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x / 64;
    const uint64_t wbase = (uint64_t)blockIdx.x * SH_TILE + (uint64_t)wv * SH_PER_WAVE;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t mine = 0;
    for (uint32_t r = 0; r < SH_PER_WAVE / 64; ++r) {
        const uint64_t e = wbase + r * 64 + lane;
        const uint32_t d = e < a.n ? (a.key[e] < a.K ? a.key[e] % a.world : 0xffffffffu) : 0xffffffffu;
        for (uint32_t dd = 0; dd < a.world; ++dd) {
            const uint64_t m = __ballot(d == dd);
            if (lane == dd) mine += (uint32_t)__popcll(m);
        }
    }
    wtot[wv][lane] = mine;
    __syncthreads();
    uint32_t base = 0;
    if (lane < a.world) {
        base = a.counts[(size_t)lane * a.ntiles + blockIdx.x];
        for (uint32_t w2 = 0; w2 < wv; ++w2) base += wtot[w2][lane];
    }
    for (uint32_t r = 0; r < SH_PER_WAVE / 64; ++r) {
        const uint64_t e = wbase + r * 64 + lane;
        const bool in = e < a.n;
        const uint32_t k = in ? a.key[e] : 0u;
        const uint32_t d = (in && k < a.K) ? k % a.world : 0xffffffffu;
        uint32_t p = 0xffffffffu;
        for (uint32_t dd = 0; dd < a.world; ++dd) {
            const uint64_t m = __ballot(d == dd);
            const uint32_t bdd = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)dd);
            if (d == dd) p = bdd + (uint32_t)__popcll(m & lt);
            if (lane == dd) base += (uint32_t)__popcll(m);
        }
        if (in) {
            a.pos[e] = p;
            if (p != 0xffffffffu) {
                a.opos[p] = (uint32_t)e;
                a.okey[p] = k / a.world;
            }
        }
    }
}

// one column: out[pos[e]] = in[e] (W = 1, 4 or 8 bytes)
template <typename T>
__global__ void __launch_bounds__(256) k_fan_col(uint64_t n, const uint32_t* __restrict__ pos, const T* __restrict__ in,
                                                 T* __restrict__ out) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const uint32_t p = pos[e];
    if (p != 0xffffffffu) out[p] = in[e];
}

// exclusive scan of the (destination, tile) counts by one workgroup: each thread sums a contiguous slice, the
// slice sums are scanned across the block (wave DPP-free shuffles + one LDS round), then each thread writes its
// slice's prefixes (the counts are world x tiles: thousands, a few reads per thread)
__global__ void __launch_bounds__(1024) k_sh_scan(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t n) {
    __shared__ uint32_t wsum[16];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint64_t per = (n + 1023) / 1024, a = (uint64_t)t * per, b = a + per < n ? a + per : n;
    uint32_t s = 0;
    for (uint64_t i = a; i < b; ++i) s += in[i];
    uint32_t x = s;   // inclusive scan over the wave
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if ((int)lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t v = 0; v < w; ++v) before += wsum[v];
    uint32_t run = before + x - s;   // exclusive prefix of this thread's slice
    for (uint64_t i = a; i < b; ++i) {
        const uint32_t c = in[i];
        out[i] = run;
        run += c;
    }
}

// per-shard totals from the scanned offsets (shard-major): total[d] = off[d + 1][0] - off[d][0]
__global__ void k_fan_totals(const uint32_t* off, uint32_t world, uint32_t ntiles, const uint32_t* last_cnt,
                             uint32_t* totals) {
    const uint32_t d = threadIdx.x;
    if (d >= world) return;
    const uint32_t a = off[(size_t)d * ntiles];
    const uint32_t b = (d + 1 < world) ? off[(size_t)(d + 1) * ntiles]
                                       : off[(size_t)d * ntiles + ntiles - 1] + last_cnt[(size_t)d * ntiles + ntiles - 1];
    totals[d] = b - a;
}

}  // namespace

extern "C" {

static int shard_pack(uint64_t n, const uint32_t* key, const int64_t* ts, const uint32_t* const* cols, uint32_t n_cols,
                      uint32_t world, uint32_t cap, uint32_t* rows, unsigned long long* dest_counts, uint32_t* overflow,
                      void* scratch, size_t scratch_len, void* stream) {
    if (world == 0 || world > SH_MAX_WORLD || n_cols > SH_MAX_COLS || n >= (1ull << 32)) return SG_ERR_INVALID;
    const hipStream_t s = (hipStream_t)stream;
    ShardArgs a{};
    a.n = n;
    a.key = key;
    a.ts = ts;
    for (uint32_t c = 0; c < n_cols; ++c) a.col[c] = cols[c];
    a.ncols = n_cols;
    a.world = world;
    a.cap = cap;
    a.overflow = overflow;
    a.ntiles = (uint32_t)((n + SH_TILE - 1) / SH_TILE);
    const size_t ncnt = (size_t)world * a.ntiles;
    const size_t need = 2 * ncnt * 4 + 256;
    if (!scratch || scratch_len < need) return SG_ERR_CAPACITY;
    uint32_t* cnt = (uint32_t*)scratch;
    uint32_t* off = cnt + ncnt;
    if (cap && hipMemsetAsync(overflow, 0, 4, s) != hipSuccess) return SG_ERR_DEVICE;
    if (n == 0) {
        if (hipMemsetAsync(dest_counts, 0, world * 8, s) != hipSuccess) return SG_ERR_DEVICE;
        if (cap)
            hipLaunchKernelGGL(k_sh_pad, dim3((unsigned)(((uint64_t)world * cap + 255) / 256)), dim3(256), 0, s, rows,
                               dest_counts, world, cap, 3 + n_cols);
        return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_DEVICE;
    }
    a.counts = cnt;
    hipLaunchKernelGGL(k_sh_count, dim3(a.ntiles), dim3(SH_WAVES * 64), 0, s, a);
    hipLaunchKernelGGL(k_sh_scan, dim3(1), dim3(1024), 0, s, (const uint32_t*)cnt, off, (uint64_t)ncnt);
    a.counts = off;
    a.rows = rows;
    hipLaunchKernelGGL(k_sh_scatter, dim3(a.ntiles), dim3(SH_WAVES * 64), 0, s, a);
    hipLaunchKernelGGL(k_sh_totals, dim3(1), dim3(64), 0, s, off, cnt, world, a.ntiles, n, dest_counts);
    if (cap)
        hipLaunchKernelGGL(k_sh_pad, dim3((unsigned)(((uint64_t)world * cap + 255) / 256)), dim3(256), 0, s, rows,
                           dest_counts, world, cap, 3 + n_cols);
    return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_DEVICE;
}

int sg_shard_pack(uint64_t n, const uint32_t* key, const int64_t* ts, const uint32_t* const* cols, uint32_t n_cols,
                  uint32_t world, uint32_t* rows, unsigned long long* dest_counts, void* scratch, size_t scratch_len,
                  void* stream) {
    return shard_pack(n, key, ts, cols, n_cols, world, 0, rows, dest_counts, nullptr, scratch, scratch_len, stream);
}

int sg_shard_pack_blocks(uint64_t n, const uint32_t* key, const int64_t* ts, const uint32_t* const* cols,
                         uint32_t n_cols, uint32_t world, uint32_t cap, uint32_t* rows, unsigned long long* dest_counts,
                         uint32_t* overflow, void* scratch, size_t scratch_len, void* stream) {
    if (cap == 0 || !overflow) return SG_ERR_INVALID;
    return shard_pack(n, key, ts, cols, n_cols, world, cap, rows, dest_counts, overflow, scratch, scratch_len, stream);
}

}  // extern "C"

// sg_sharded.h: split one device batch by owner shard on the stream's device (all buffers on that device;
// scratch from fan_split_scratch_bytes).  Queues the work only: totals / opos / err are valid once `stream` is.
int fan_split(uint64_t n, const uint32_t* key, uint32_t K, uint32_t world, bool null_keys, const int64_t* ts,
              const void* const* cols, const uint32_t* col_bytes, const uint8_t* const* nulls, uint32_t ncols,
              int64_t* out_ts, void* const* out_cols, uint8_t* const* out_nulls, uint32_t* opos, uint32_t* okey,
              uint32_t* totals, uint32_t* err, void* scratch, size_t scratch_len, hipStream_t s) {
    if (world == 0 || world > SH_MAX_WORLD || n >= (1ull << 32)) return SG_ERR_INVALID;
    FanArgs a{};
    a.n = n;
    a.key = key;
    a.K = K;
    a.world = world;
    a.null_keys = null_keys ? 1u : 0u;
    a.ntiles = (uint32_t)((n + SH_TILE - 1) / SH_TILE);
    const size_t ncnt = (size_t)world * a.ntiles;
    const size_t need = 2 * ncnt * 4 + (size_t)n * 4 + 512;
    if (!scratch || scratch_len < need) return SG_ERR_CAPACITY;
    uint32_t* cnt = (uint32_t*)scratch;
    uint32_t* off = cnt + ncnt;
    a.pos = off + ncnt;
    a.opos = opos;
    a.okey = okey;
    a.err = err;
    if (hipMemsetAsync(err, 0, 4, s) != hipSuccess) return SG_ERR_DEVICE;
    a.counts = cnt;
    hipLaunchKernelGGL(k_fan_count, dim3(a.ntiles), dim3(SH_WAVES * 64), 0, s, a);
    hipLaunchKernelGGL(k_sh_scan, dim3(1), dim3(1024), 0, s, (const uint32_t*)cnt, off, (uint64_t)ncnt);
    a.counts = off;
    hipLaunchKernelGGL(k_fan_rank, dim3(a.ntiles), dim3(SH_WAVES * 64), 0, s, a);
    hipLaunchKernelGGL(k_fan_totals, dim3(1), dim3(64), 0, s, off, world, a.ntiles, cnt, totals);
    const dim3 g((unsigned)((n + 255) / 256)), b(256);
    hipLaunchKernelGGL(k_fan_col<uint64_t>, g, b, 0, s, n, a.pos, (const uint64_t*)ts, (uint64_t*)out_ts);
    for (uint32_t c = 0; c < ncols; ++c) {
        if (col_bytes[c] == 8)
            hipLaunchKernelGGL(k_fan_col<uint64_t>, g, b, 0, s, n, a.pos, (const uint64_t*)cols[c], (uint64_t*)out_cols[c]);
        else if (col_bytes[c] == 4)
            hipLaunchKernelGGL(k_fan_col<uint32_t>, g, b, 0, s, n, a.pos, (const uint32_t*)cols[c], (uint32_t*)out_cols[c]);
        else
            hipLaunchKernelGGL(k_fan_col<uint8_t>, g, b, 0, s, n, a.pos, (const uint8_t*)cols[c], (uint8_t*)out_cols[c]);
        if (nulls && nulls[c])
            hipLaunchKernelGGL(k_fan_col<uint8_t>, g, b, 0, s, n, a.pos, nulls[c], out_nulls[c]);
    }
    return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_DEVICE;
}

size_t fan_split_scratch_bytes(uint64_t n, uint32_t world) {
    const uint32_t ntiles = (uint32_t)((n + SH_TILE - 1) / SH_TILE);
    const size_t ncnt = (size_t)world * ntiles;
    return 2 * ncnt * 4 + (size_t)n * 4 + 512;
}

extern "C" {

size_t sg_shard_scratch_bytes(uint64_t n, uint32_t world) {
    const uint32_t ntiles = (uint32_t)((n + SH_TILE - 1) / SH_TILE);
    const size_t ncnt = (size_t)world * ntiles;
    return 2 * ncnt * 4 + 256;
}

int sg_shard_unpack(uint64_t n, const uint32_t* rows, uint32_t n_cols, uint32_t* key, int64_t* ts,
                    uint32_t* const* cols_dev, void* stream) {
    if (n_cols > SH_MAX_COLS) return SG_ERR_INVALID;
    if (n == 0) return SG_OK;
    hipLaunchKernelGGL(k_sh_unpack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, rows,
                       n_cols, key, ts, cols_dev);
    return hipGetLastError() == hipSuccess ? SG_OK : SG_ERR_DEVICE;
}

}  // extern "C"
