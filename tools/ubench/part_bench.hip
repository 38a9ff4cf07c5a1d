// part_bench — checks and times the hand-written partition library (csrc/part_kernels.hip) on its own:
//   group_sorted   key-sorted Pay<1> + seg bounds (C3/C4 grouping, every non-fused engine)
//   tiles_fused    the C2 tile pass (the key split happens inside the advance kernel)
//   sort_pairs     u32 ascending / descending, u64 ascending (timer paths)
// against a CPU stable sort of the same input.  Build: make -C tools/ubench part_bench (see Makefile there).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>

#include "../../siddhi-1_amd/csrc/part.h"

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);         \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

static int failures = 0;
#define EXPECT(c, ...)                 \
    do {                               \
        if (!(c)) {                    \
            printf("FAIL: " __VA_ARGS__); \
            printf("\n");              \
            failures++;                \
        }                              \
    } while (0)

struct Batch {
    uint32_t n;
    std::vector<uint32_t> key;
    std::vector<int64_t> ts;
    std::vector<float> price;
    uint32_t *d_key, *d_price;
    int64_t* d_ts;
};

static Batch make_batch(uint32_t n, uint32_t K, int dist, uint32_t seed, bool with_bad) {
    Batch b;
    b.n = n;
    b.key.resize(n);
    b.ts.resize(n);
    b.price.resize(n);
    std::mt19937_64 g(seed);
    std::vector<double> cdf;
    if (dist == 1) {  // Zipf s = 1.1 over K keys
        cdf.resize(K);
        double s = 0;
        for (uint32_t k = 0; k < K; k++) cdf[k] = (s += 1.0 / std::pow(k + 1.0, 1.1));
        for (auto& x : cdf) x /= s;
    }
    std::uniform_real_distribution<double> u(0, 1);
    for (uint32_t i = 0; i < n; i++) {
        uint32_t k;
        if (dist == 1) k = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u(g)) - cdf.begin());
        else k = (uint32_t)(g() % K);
        if (k >= K) k = K - 1;
        if (with_bad && (g() % 1000) == 0) k = (g() & 1) ? 0xffffffffu : K + (uint32_t)(g() % 7);
        b.key[i] = k;
        b.ts[i] = 1000000 + (int64_t)i / 4;
        b.price[i] = (float)(g() % 10000) * 0.01f;
    }
    CK(hipMalloc(&b.d_key, (size_t)n * 4));
    CK(hipMalloc(&b.d_price, (size_t)n * 4));
    CK(hipMalloc(&b.d_ts, (size_t)n * 8));
    CK(hipMemcpy(b.d_key, b.key.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(b.d_price, b.price.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(b.d_ts, b.ts.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    return b;
}

static void free_batch(Batch& b) {
    (void)hipFree(b.d_key);
    (void)hipFree(b.d_price);
    (void)hipFree(b.d_ts);
}

template <class F> static float time_it(F f, int reps = 10) {
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    f();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps; r++) {
        CK(hipEventRecord(a, 0));
        f();
        CK(hipEventRecord(z, 0));
        CK(hipEventSynchronize(z));
        float ms;
        CK(hipEventElapsedTime(&ms, a, z));
        best = std::min(best, ms);
        sum += ms;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(z);
    return sum / reps * 1000.f;  // mean, us
}

static void test_group(const char* name, uint32_t n, uint32_t K, int dist, bool bad, bool drop_null, uint32_t W,
                       void* scratch) {
    Batch b = make_batch(n, K, dist, 1234 + n + K, bad);
    PartScratch s = sgd_part_scratch(scratch, n);
    void* out;
    uint32_t *sb, *se, *err;
    CK(hipMalloc(&out, (size_t)n * 24));
    CK(hipMalloc(&sb, (size_t)K * 4));
    CK(hipMalloc(&se, (size_t)K * 4));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    GroupArgs g{};
    g.n = n;
    g.K = K;
    g.drop_null = drop_null;
    g.W = W;
    g.keys = b.d_key;
    g.src.ts = b.d_ts;
    if (W >= 1) {
        g.src.p[0] = b.d_price;
        g.src.kind[0] = 0;
    }
    g.out = out;
    g.seg_begin = sb;
    g.seg_end = se;
    g.err = err;
    g.s = s;
    const float us = time_it([&] { CK(sgd_group_sorted(g, 0)); });
    // check
    std::vector<uint32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    std::vector<uint32_t> valid;
    bool any_bad = false;
    for (uint32_t i = 0; i < n; i++) {
        if (b.key[i] < K) valid.push_back(i);
        else if (!(drop_null && b.key[i] == 0xffffffffu)) any_bad = true;
    }
    std::stable_sort(valid.begin(), valid.end(), [&](uint32_t x, uint32_t y) { return b.key[x] < b.key[y]; });
    const uint32_t S = W == 0 ? 1 : W + 2;
    std::vector<uint32_t> h((size_t)n * S), hb(K), he(K);
    uint32_t herr = 0;
    CK(hipMemcpy(h.data(), out, (size_t)n * S * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), sb, (size_t)K * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(he.data(), se, (size_t)K * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    size_t wrong = 0;
    for (size_t j = 0; j < valid.size(); j++) {
        const uint32_t i = valid[j];
        if (h[j * S] != i) wrong++;
        else if (W >= 1) {
            uint32_t pw;
            memcpy(&pw, &b.price[i], 4);
            if (h[j * S + 1] != pw || (int32_t)h[j * S + S - 1] != (int32_t)(b.ts[i] - b.ts[0])) wrong++;
        }
    }
    size_t bwrong = 0;
    {
        size_t j = 0;
        for (uint32_t k = 0; k < K; k++) {
            const size_t j0 = j;
            while (j < valid.size() && b.key[valid[j]] == k) j++;
            if (j > j0) {
                if (hb[k] != j0 || he[k] != j) bwrong++;
            } else if (hb[k] != he[k]) bwrong++;
        }
    }
    EXPECT(wrong == 0, "%s: %zu misplaced elements", name, wrong);
    EXPECT(bwrong == 0, "%s: %zu wrong key bounds", name, bwrong);
    EXPECT(((herr & SGD_ERR_KEY_RANGE) != 0) == any_bad, "%s: key range error %u, expected %d", name, herr, (int)any_bad);
    printf("%-48s n=%-9u K=%-9u %9.1f us  %6.2f GB/s-equiv(16B/ev)  %s\n", name, n, K, us, n * 16.0 / us / 1e3,
           (wrong || bwrong) ? "WRONG" : "ok");
    (void)hipFree(out);
    (void)hipFree(sb);
    (void)hipFree(se);
    (void)hipFree(err);
    free_batch(b);
}

static void test_fused(const char* name, uint32_t n, uint32_t K, int dist, void* scratch) {
    Batch b = make_batch(n, K, dist, 99 + n, false);
    PartScratch s = sgd_part_scratch(scratch, n);
    void* out;
    uint32_t *tlo, *err;
    const uint32_t nt = (K + 255) / 256;
    CK(hipMalloc(&out, (size_t)n * 12));
    CK(hipMalloc(&tlo, (size_t)(nt + 1) * 4));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    GroupArgs g{};
    g.n = n;
    g.K = K;
    g.W = 1;
    g.keys = b.d_key;
    g.src.ts = b.d_ts;
    g.src.p[0] = b.d_price;
    g.out = out;
    g.err = err;
    g.s = s;
    const float us = time_it([&] { CK(sgd_group_tiles_fused(g, tlo, 0)); });
    std::vector<uint32_t> v(n);
    std::iota(v.begin(), v.end(), 0u);
    std::stable_sort(v.begin(), v.end(), [&](uint32_t x, uint32_t y) { return (b.key[x] >> 8) < (b.key[y] >> 8); });
    std::vector<uint32_t> h((size_t)n * 3), ht(nt + 1);
    CK(hipMemcpy(h.data(), out, (size_t)n * 12, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ht.data(), tlo, (size_t)(nt + 1) * 4, hipMemcpyDeviceToHost));
    size_t wrong = 0, twrong = 0;
    for (uint32_t j = 0; j < n; j++) {
        const uint32_t i = v[j];
        if (h[(size_t)j * 3] != (i | ((b.key[i] & 255u) << 24))) wrong++;
    }
    {
        uint32_t j = 0;
        for (uint32_t t = 0; t <= nt; t++) {
            if (ht[t] != j) twrong++;
            while (t < nt && j < n && (b.key[v[j]] >> 8) == t) j++;
        }
    }
    EXPECT(wrong == 0, "%s: %zu misplaced", name, wrong);
    EXPECT(twrong == 0, "%s: %zu wrong tile starts", name, twrong);
    printf("%-48s n=%-9u K=%-9u %9.1f us  %6.2f GB/s-equiv(16B/ev)  %s\n", name, n, K, us, n * 16.0 / us / 1e3,
           (wrong || twrong) ? "WRONG" : "ok");
    (void)hipFree(out);
    (void)hipFree(tlo);
    (void)hipFree(err);
    free_batch(b);
}

static void test_pairs(const char* name, uint32_t n, uint32_t bits, bool k64, bool desc, void* scratch) {
    PartScratch s = sgd_part_scratch(scratch, n);
    std::mt19937_64 g(7 + n + bits);
    std::vector<uint64_t> k(n);
    std::vector<uint32_t> v(n);
    const uint64_t mask = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    for (uint32_t i = 0; i < n; i++) {
        k[i] = (g() & mask) >> (g() % 3 == 0 ? 8 : 0);  // (duplicates)
        v[i] = i;
    }
    void *dk, *dko;
    uint32_t *dv, *dvo;
    const size_t kb = k64 ? 8 : 4;
    CK(hipMalloc(&dk, n * kb));
    CK(hipMalloc(&dko, n * kb));
    CK(hipMalloc(&dv, n * 4));
    CK(hipMalloc(&dvo, n * 4));
    if (k64) CK(hipMemcpy(dk, k.data(), n * 8, hipMemcpyHostToDevice));
    else {
        std::vector<uint32_t> k32(k.begin(), k.end());
        CK(hipMemcpy(dk, k32.data(), n * 4, hipMemcpyHostToDevice));
    }
    CK(hipMemcpy(dv, v.data(), n * 4, hipMemcpyHostToDevice));
    const float us = time_it([&] { CK(sgd_sort_pairs(dk, dko, dv, dvo, n, bits, k64, desc, s, 0)); });
    std::vector<uint32_t> ord(n);
    std::iota(ord.begin(), ord.end(), 0u);
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return desc ? k[x] > k[y] : k[x] < k[y]; });
    std::vector<uint32_t> hv(n);
    CK(hipMemcpy(hv.data(), dvo, n * 4, hipMemcpyDeviceToHost));
    size_t wrong = 0;
    for (uint32_t j = 0; j < n; j++) wrong += hv[j] != ord[j];
    EXPECT(wrong == 0, "%s: %zu misplaced", name, wrong);
    printf("%-48s n=%-9u bits=%-6u %9.1f us  %s\n", name, n, bits, us, wrong ? "WRONG" : "ok");
    (void)hipFree(dk);
    (void)hipFree(dko);
    (void)hipFree(dv);
    (void)hipFree(dvo);
}

int main(int argc, char** argv) {
    const uint32_t NMAX = 1u << 24;
    void* scratch;
    CK(hipMalloc(&scratch, sgd_part_scratch_bytes(NMAX)));

    test_fused("fused tile pass, C2 (uniform)", 1u << 24, 1u << 20, 0, scratch);
    test_fused("fused tile pass, C2 (Zipf 1.1)", 1u << 24, 1u << 20, 1, scratch);
    test_fused("fused tile pass, small", 100000, 3000, 0, scratch);
    test_group("sorted W=1, C2 size", 1u << 24, 1u << 20, 0, false, false, 1, scratch);
    test_group("sorted W=1, C3 size, bad keys + nulls", 1u << 22, 1u << 20, 0, true, true, 1, scratch);
    test_group("sorted W=1, bad keys (no drop)", 1u << 20, 1u << 20, 0, true, false, 1, scratch);
    test_group("sorted W=0 (positions), C3 size", 1u << 22, 1u << 20, 0, false, false, 0, scratch);
    test_group("sorted W=1, C5 per GPU (2^23 keys)", 1u << 24, 1u << 23, 0, false, false, 1, scratch);
    test_group("sorted W=1, K=2048 (one pass)", 1u << 16, 2048, 0, false, false, 1, scratch);
    test_group("sorted W=1, K=2048, Zipf", 1u << 22, 2048, 1, false, false, 1, scratch);
    test_group("sorted W=1, K=1", 5000, 1, 0, false, false, 1, scratch);
    test_group("sorted W=1, K=262144, Zipf", 1u << 22, 262144, 1, true, true, 1, scratch);
    test_group("sorted W=1, tiny", 37, 100, 0, false, false, 1, scratch);
    test_pairs("pairs u32 asc 20 bits", 1u << 20, 20, false, false, scratch);
    test_pairs("pairs u32 desc 32 bits", 1u << 20, 32, false, true, scratch);
    test_pairs("pairs u32 desc 7 bits", 3000, 7, false, true, scratch);
    test_pairs("pairs u64 asc 64 bits", 1u << 18, 64, true, false, scratch);
    test_pairs("pairs u64 asc 64 bits, small", 777, 64, true, false, scratch);
    printf("%s (%d failures)\n", failures ? "FAILED" : "ALL OK", failures);
    return failures ? 1 : 0;
}
