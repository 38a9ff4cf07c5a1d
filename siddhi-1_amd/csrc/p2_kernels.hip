// p2_kernels.hip — ahead-of-time gfx950 kernels around the NFA advance: per-key segment bounds of
// the key-sorted batch, and the ordered scatter of the emitted matches.  The advance kernel itself is
// query-specialised and compiled at engine creation (p2_jit.hip, sg_jit.cpp).
#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu_ir.h"
#include "sg_engine.h"

// ------------------------------------------------------------------------------------------------
// segment bounds of the key-sorted batch: seg_begin[k], seg_end[k]
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_seg_bounds(const uint32_t* __restrict__ skeys, uint32_t n,
                                                    uint32_t n_keys, uint32_t* __restrict__ seg_begin,
                                                    uint32_t* __restrict__ seg_end, uint32_t* __restrict__ err) {
    // every key gets its bounds written (keys without events get an empty [i, i) at the right spot),
    // so no memset of the bound arrays is needed per batch
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t k = skeys[i];
    if (k >= n_keys) {  // key id outside [0, n_keys): reject the batch loudly, never write out of bounds
        atomicOr(err, (uint32_t)SGD_ERR_KEY_RANGE);
        return;
    }
    const uint32_t prev = (i == 0) ? 0xffffffffu : skeys[i - 1];
    if (prev != k) {
        seg_begin[k] = i;
        // keys between the previous run and this one (or before the first run) have no events
        for (uint32_t g = (i == 0) ? 0u : prev + 1; g < k && g < n_keys; ++g) seg_begin[g] = seg_end[g] = i;
    }
    const uint32_t next = (i == n - 1) ? n_keys : skeys[i + 1];
    if (next != k) {
        seg_end[k] = i + 1;
        if (i == n - 1)
            for (uint32_t g = k + 1; g < n_keys; ++g) seg_begin[g] = seg_end[g] = n;
    }
}

// ------------------------------------------------------------------------------------------------
// match ordering: batch event t's matches go to out_count + t_off[t] (t_off = exclusive scan of the
// per-event counts), i.e. ascending trigger seq, then emission order — the reference's callback order
// (MultiProcessStreamReceiver.java:119-121).  Resets t_desc for the next batch.  chain_len is the
// constant 1/1 of a two-state match and was written once at allocation.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_scatter(const ScatterParams s) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= s.n) return;
    const uint64_t d = s.t_desc[t];
    const uint32_t c = (uint32_t)(d >> 32);
    const uint64_t base = *s.out_count;
    if (t == s.n - 1) *s.batch_total = (unsigned long long)s.t_off[t] + c;
    if (c == 0) return;
    s.t_desc[t] = 0;
    const uint64_t o = base + s.t_off[t];
    const uint32_t f = (uint32_t)d;
    const uint64_t trig = s.seq_base + t;
    const uint32_t key = s.key ? s.key[t] : 0u;
    const int64_t ts = s.ts[t];
    if (o + c > s.capacity) {
        atomicOr(s.err, (uint32_t)SGD_ERR_MATCH_CAP);
        return;
    }
    for (uint32_t r = 0; r < c; ++r) {
        const uint64_t q = o + r;
        s.o_trig[q] = trig;
        s.o_slot[2 * q] = s.raw_e1[f + r];
        s.o_slot[2 * q + 1] = trig;
        s.o_key[q] = key;
        s.o_ts[q] = ts;  // StreamPostStateProcessor.java:68: StateEvent ts = ts of the e2 event
    }
}

__global__ void k_bump(unsigned long long* out_count, const unsigned long long* batch_total) {
    *out_count += *batch_total;
}

// per-batch counters of the staged advance pass: one row per wave -> the cumulative totals
__global__ void __launch_bounds__(1024) k_stats_reduce(const unsigned long long* __restrict__ wstats,
                                                       uint32_t n_waves, unsigned long long* __restrict__ stats) {
    __shared__ unsigned long long part[SGD_ST_N][16];
    unsigned long long acc[SGD_ST_N];
    for (int i = 0; i < SGD_ST_N; ++i) acc[i] = 0;
    for (uint32_t w = threadIdx.x; w < n_waves; w += blockDim.x)
        for (int i = 0; i < SGD_ST_N; ++i) acc[i] += wstats[(size_t)w * SGD_ST_N + i];
    for (int i = 0; i < SGD_ST_N; ++i)
        for (int off = 32; off > 0; off >>= 1) acc[i] += __shfl_xor(acc[i], off, 64);
    const int wv = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0)
        for (int i = 0; i < SGD_ST_N; ++i) part[i][wv] = acc[i];
    __syncthreads();
    if (threadIdx.x < SGD_ST_N) {
        unsigned long long t = 0;
        for (int j = 0; j < (int)(blockDim.x / 64); ++j) t += part[threadIdx.x][j];
        stats[threadIdx.x] += t;
    }
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

int sgd_launch_stats_reduce(const unsigned long long* wstats, uint32_t n_waves, unsigned long long* stats,
                            ihipStream_t* stream) {
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(1024), 0, stream, wstats, n_waves, stats);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int sgd_launch_scatter(const ScatterParams& s, ihipStream_t* stream) {
    if (s.n == 0) return 0;
    hipLaunchKernelGGL(k_scatter, dim3((s.n + 255) / 256), dim3(256), 0, stream, s);
    hipLaunchKernelGGL(k_bump, dim3(1), dim3(1), 0, stream, s.out_count, s.batch_total);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
