// Grouping-stage experiment: rocPRIM onesweep configurations for the C2 payload sort with the compact
// 12-B payload (position, price, 32-bit ts offset; pack.h), u32 key ids of 2^20 keys, 2^24 events.
// Prints the mean time per sort of each configuration and checks order + stability.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 sort_sweep12.hip -o sort_sweep12
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>

struct Pay { uint32_t idx; uint32_t w; int32_t ts; };
struct Fn {
    const uint32_t* price; const int64_t* ts;
    __host__ __device__ Pay operator()(uint32_t i) const { Pay o; o.idx = i; o.w = price[i]; o.ts = (int32_t)(ts[i] - ts[0]); return o; }
};
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <unsigned B, unsigned I, unsigned BITS, rocprim::block_radix_rank_algorithm ALG>
using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<B, I>, rocprim::kernel_config<B, I>, BITS, ALG>>;

template <class C, unsigned KB = 20>
void run(const char* name, const uint32_t* keys, uint32_t* skeys, const uint32_t* price, const int64_t* ts, Pay* out,
         uint32_t n) {
    auto it = rocprim::make_transform_iterator(rocprim::counting_iterator<uint32_t>(0), Fn{price, ts});
    size_t tmpb = 0;
    CK(rocprim::radix_sort_pairs<C>(nullptr, tmpb, keys, skeys, it, out, n, 0u, KB, 0));
    void* tmp; CK(hipMalloc(&tmp, tmpb));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) CK(rocprim::radix_sort_pairs<C>(tmp, tmpb, keys, skeys, it, out, n, 0u, KB, 0));
    const int R = 20;
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < R; i++) CK(rocprim::radix_sort_pairs<C>(tmp, tmpb, keys, skeys, it, out, n, 0u, KB, 0));
    CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> hk(n); std::vector<Pay> hp(n);
    CK(hipMemcpy(hk.data(), skeys, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(hp.data(), out, n * sizeof(Pay), hipMemcpyDeviceToHost));
    bool ok = true;
    for (uint32_t i = 1; i < n && ok; i++) ok = hk[i - 1] < hk[i] || (hk[i - 1] == hk[i] && hp[i - 1].idx < hp[i].idx);
    printf("%-28s %8.3f ms/sort  %s\n", name, ms / R, ok ? "ok" : "UNSORTED");
    CK(hipFree(tmp));
}

int main() {
    const uint32_t n = 1u << 24, K = 1u << 20;
    std::vector<uint32_t> hk(n), hpz(n); std::vector<int64_t> ht(n);
    uint64_t x = 0x5EED5EEDull;
    for (uint32_t i = 0; i < n; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; hk[i] = (uint32_t)(x % K); hpz[i] = (uint32_t)(x >> 40); ht[i] = 1700000000000ll + i / 2000; }
    uint32_t *keys, *skeys, *price; int64_t* ts; Pay* out;
    CK(hipMalloc(&keys, n * 4)); CK(hipMalloc(&skeys, n * 4)); CK(hipMalloc(&price, n * 4)); CK(hipMalloc(&ts, n * 8)); CK(hipMalloc(&out, n * 16ull));
    CK(hipMemcpy(keys, hk.data(), n * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(price, hpz.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ts, ht.data(), n * 8, hipMemcpyHostToDevice));
    using M = rocprim::block_radix_rank_algorithm;
    run<Cfg<1024, 16, 10, M::match>>("1024x16 b10 match", keys, skeys, price, ts, out, n);
    // 2^23 keys (C5 per GPU): three passes either way
    for (uint32_t i = 0; i < n; i++) hk[i] = (uint32_t)(((uint64_t)hk[i] * 2654435761u + i) % (1u << 23));
    CK(hipMemcpy(keys, hk.data(), n * 4, hipMemcpyHostToDevice));
    run<rocprim::default_config, 23>("default, 23-bit", keys, skeys, price, ts, out, n);
    run<Cfg<1024, 16, 8, M::match>, 23>("1024x16 b8, 23-bit", keys, skeys, price, ts, out, n);
    run<Cfg<1024, 16, 10, M::match>, 23>("1024x16 b10, 23-bit", keys, skeys, price, ts, out, n);
    run<Cfg<1024, 10, 8, M::match>, 23>("1024x10 b8, 23-bit", keys, skeys, price, ts, out, n);
    run<Cfg<1024, 8, 11, M::match>, 23>("1024x8 b11, 23-bit", keys, skeys, price, ts, out, n);
    return 0;
}
