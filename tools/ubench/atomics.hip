// Microbenchmark: scattered per-key atomics and a counting-sort scatter on the C2 key distribution
// (2^24 events over 2^20 keys), against the rocPRIM 16-B-payload radix sort the engine uses.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_count(const uint32_t* key, uint32_t n, uint32_t* cnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&cnt[key[i]], 1u);
}
struct alignas(16) P16 { uint32_t a, b, c, d; };
__global__ void k_scatter(const uint32_t* key, const int64_t* ts, const float* price, uint32_t n, uint32_t* cur, P16* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t pos = atomicAdd(&cur[key[i]], 1u);
    P16 p; p.a = i; p.b = __float_as_uint(price[i]); p.c = (uint32_t)ts[i]; p.d = (uint32_t)(ts[i] >> 32);
    out[pos] = p;
}
struct PackIt {
    const int64_t* ts; const float* price;
    __host__ __device__ P16 operator()(uint32_t i) const {
        P16 p; p.a = i; p.b = __float_as_uint(price[i]); p.c = (uint32_t)ts[i]; p.d = (uint32_t)(ts[i] >> 32); return p;
    }
};
using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 6>, rocprim::kernel_config<1024, 6>, 10,
                                        rocprim::block_radix_rank_algorithm::match>>;

int main() {
    const uint32_t n = 1u << 24, K = 1u << 20;
    std::vector<uint32_t> hk(n);
    std::mt19937_64 g(42);
    for (auto& x : hk) x = (uint32_t)(g() % K);
    uint32_t *key, *cnt, *cur, *skeys; int64_t* ts; float* price; P16* out;
    CK(hipMalloc(&key, n * 4)); CK(hipMalloc(&cnt, K * 4)); CK(hipMalloc(&cur, K * 4)); CK(hipMalloc(&skeys, n * 4));
    CK(hipMalloc(&ts, n * 8)); CK(hipMalloc(&price, n * 4)); CK(hipMalloc(&out, (size_t)n * 16));
    CK(hipMemcpy(key, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(ts, 0, n * 8)); CK(hipMemset(price, 0, n * 4));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    size_t tmp_bytes = 0;
    auto it = rocprim::make_transform_iterator(rocprim::counting_iterator<uint32_t>(0), PackIt{ts, price});
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tmp_bytes, key, skeys, it, out, n, 0u, 20u));
    void* tmp; CK(hipMalloc(&tmp, tmp_bytes));
    for (int rep = 0; rep < 3; rep++) {
        CK(hipMemset(cnt, 0, K * 4));
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_count, dim3(n / 256), dim3(256), 0, 0, key, n, cnt);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("count atomics: %.1f us\n", ms * 1e3);
        CK(hipMemset(cur, 0, K * 4));
        CK(hipEventRecord(a)); hipLaunchKernelGGL(k_scatter, dim3(n / 256), dim3(256), 0, 0, key, ts, price, n, cur, out);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("scatter (atomic + 16B store): %.1f us\n", ms * 1e3);
        CK(hipEventRecord(a));
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, tmp_bytes, key, skeys, it, out, n, 0u, 20u));
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("rocprim sort pairs 20 bits, 16B payload: %.1f us\n", ms * 1e3);
    }
    return 0;
}
