// scatter64.hip — micro-benchmark: one stable 64-way LSD partition pass of 2^24 (key, 12-B payload)
// elements, the building block of a two-level key-tile grouping.  Per block of BE
// elements: digits ranked in input order (per-wave counters + match-any over 6 bits), the block's
// elements staged in LDS by digit, then written out in runs (avg BE / 64 elements per run).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/scatter64 tools/ubench/scatter64.hip && /tmp/scatter64
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

struct El { uint32_t idx, w, ts; };
constexpr int NT = 256, PER = 16, BE = NT * PER, ND = 64, NWV = NT / 64;

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
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

__global__ void __launch_bounds__(NT) k_hist(const uint32_t* keys, uint32_t n, int shift, uint32_t* mat, uint32_t nblk) {
    __shared__ uint32_t c[ND];
    if (threadIdx.x < ND) c[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t b0 = blockIdx.x * BE;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t i = b0 + j * NT + threadIdx.x;
        if (i < n) atomicAdd(&c[(keys[i] >> shift) & 63u], 1u);
    }
    __syncthreads();
    if (threadIdx.x < ND) mat[threadIdx.x * nblk + blockIdx.x] = c[threadIdx.x];
}

// wave w owns elements [w * BE/4, (w+1) * BE/4) of the block: chunks of 64 consecutive, in order
__global__ void __launch_bounds__(NT) k_scatter(const uint32_t* keys, const El* in, uint32_t n, int shift,
                                                const uint32_t* mscan, uint32_t nblk, uint32_t* okeys, El* out) {
    __shared__ uint32_t wc[NWV][ND];
    __shared__ uint32_t dstart[ND], gbase[ND];
    __shared__ uint32_t skey[BE];
    __shared__ El sel[BE];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x < NWV * ND) (&wc[0][0])[threadIdx.x] = 0;
    constexpr int CPW = BE / NWV / 64;  // chunks per wave
    const uint32_t i0 = blockIdx.x * BE + w * (BE / NWV) + lane;
    uint32_t k[CPW], r[CPW];
    El e[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const uint32_t i = i0 + c * 64;
        k[c] = i < n ? keys[i] : 0xffffffffu;
        if (i < n) e[c] = in[i];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const bool v = k[c] != 0xffffffffu;
        const uint32_t d = (k[c] >> shift) & 63u;
        const uint64_t m = match_any<6>(d, __ballot(v));
        r[c] = 0;
        if (v) {
            const uint32_t before = lane_rank(m), base = wc[w][d];
            if (before == 0) wc[w][d] = base + (uint32_t)__popcll(m);
            r[c] = base + before;
        }
    }
    __syncthreads();
    if (threadIdx.x < ND) {  // per digit: the waves' offsets, the block's total
        uint32_t run = 0;
        for (int q = 0; q < NWV; ++q) { const uint32_t x = wc[q][threadIdx.x]; wc[q][threadIdx.x] = run; run += x; }
        dstart[threadIdx.x] = run;  // (total; scanned below)
        gbase[threadIdx.x] = mscan[threadIdx.x * nblk + blockIdx.x];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int d = 0; d < ND; ++d) { const uint32_t t = dstart[d]; dstart[d] = s; s += t; }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        if (k[c] == 0xffffffffu) continue;
        const uint32_t d = (k[c] >> shift) & 63u;
        const uint32_t p = dstart[d] + wc[w][d] + r[c];
        skey[p] = k[c];
        sel[p] = e[c];
    }
    __syncthreads();
    const uint32_t nb = min((uint32_t)BE, n - blockIdx.x * BE);
    for (uint32_t p = threadIdx.x; p < nb; p += NT) {
        const uint32_t kk = skey[p], d = (kk >> shift) & 63u;
        const uint32_t o = gbase[d] + (p - dstart[d]);
        okeys[o] = kk;
        out[o] = sel[p];
    }
}

int main() {
    const uint32_t n = 1u << 24, K = 1u << 20;
    const uint32_t nblk = (n + BE - 1) / BE;
    std::vector<uint32_t> hk(n);
    uint64_t s = 88172645463325252ull;
    for (uint32_t i = 0; i < n; i++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; hk[i] = (uint32_t)(s % K); }
    uint32_t *keys, *k2, *mat, *mscan;
    El *in, *out;
    CK(hipMalloc(&keys, n * 4)); CK(hipMalloc(&k2, n * 4));
    CK(hipMalloc(&in, n * sizeof(El))); CK(hipMalloc(&out, n * sizeof(El)));
    CK(hipMalloc(&mat, ND * nblk * 4 + 4)); CK(hipMalloc(&mscan, ND * nblk * 4 + 4));
    CK(hipMemcpy(keys, hk.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<El> he(n);
    for (uint32_t i = 0; i < n; i++) he[i] = El{i, hk[i] * 3u, i / 2000u};
    CK(hipMemcpy(in, he.data(), n * sizeof(El), hipMemcpyHostToDevice));
    size_t tb = 0;
    CK(rocprim::exclusive_scan(nullptr, tb, mat, mscan, 0u, (size_t)ND * nblk, rocprim::plus<uint32_t>()));
    void* tmp; CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int shift = 8;
    for (int rep = 0; rep < 6; rep++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_hist, dim3(nblk), dim3(NT), 0, 0, keys, n, shift, mat, nblk);
        CK(rocprim::exclusive_scan(tmp, tb, mat, mscan, 0u, (size_t)ND * nblk, rocprim::plus<uint32_t>()));
        hipEvent_t c; CK(hipEventCreate(&c)); CK(hipEventRecord(c));
        hipLaunchKernelGGL(k_scatter, dim3(nblk), dim3(NT), 0, 0, keys, in, n, shift, mscan, nblk, k2, out);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms = 0, ms2 = 0; CK(hipEventElapsedTime(&ms, a, b)); CK(hipEventElapsedTime(&ms2, c, b));
        printf("hist+scan+scatter %.3f ms (scatter %.3f ms, %.2f TB/s on 32 B/elem)\n", ms, ms2, n * 32.0 / ms2 / 1e9);
    }
    // check: stable and partitioned
    std::vector<uint32_t> ok(n); std::vector<El> oe(n);
    CK(hipMemcpy(ok.data(), k2, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(oe.data(), out, n * sizeof(El), hipMemcpyDeviceToHost));
    uint32_t bad = 0;
    for (uint32_t i = 1; i < n; i++) {
        const uint32_t d0 = (ok[i - 1] >> shift) & 63u, d1 = (ok[i] >> shift) & 63u;
        if (d1 < d0 || (d1 == d0 && oe[i].idx < oe[i - 1].idx) || oe[i].w != ok[i] * 3u) bad++;
    }
    printf("check: %u bad\n", bad);
    return 0;
}
