// sg_merge.cpp — the host-side merge of per-shard match runs into timestamp order (BASELINE
// north_star: "per-partition output is merged back in timestamp order on the host").
//
// In the reference one receiver thread hands every partition's StateEvents to the QuerySelector in the order
// the events arrived (MultiProcessStreamReceiver.java:119-121), and the stream is in timestamp order.  With
// the keys sharded over GPUs, each shard's matches come out ordered within the shard (its trigger order, so
// its timestamps are nondecreasing); merging the runs by timestamp restores the stream's order.  Equal
// timestamps keep run order (shard 0's first), then the order inside the run: a stable merge.
//
// Parallel merge path: the output is cut into `threads` equal slices; for each cut rank r the smallest
// timestamp v with count(ts <= v) >= r is found by binary search over the timestamp range (each count is one
// std::upper_bound per run), the elements below v are taken from every run and the elements equal to v in
// run order until r is reached.  Each thread then merges its slice of every run with a small tournament over
// the run heads (k = the shard count).
#include <algorithm>
#include <cstdint>
#include <thread>
#include <vector>

#include "../../include/siddhi_gpu.h"

namespace {

struct Runs {
    uint32_t k;
    const int64_t* const* ts;
    const uint64_t* len;
};

// per-run split positions of the first r elements of the stable merge
void split_at(const Runs& R, uint64_t r, uint64_t* pos) {
    uint64_t total = 0;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (uint32_t i = 0; i < R.k; i++) {
        total += R.len[i];
        if (R.len[i]) {
            lo = std::min(lo, R.ts[i][0]);
            hi = std::max(hi, R.ts[i][R.len[i] - 1]);
        }
    }
    if (r == 0 || total == 0) {
        for (uint32_t i = 0; i < R.k; i++) pos[i] = 0;
        return;
    }
    if (r >= total) {
        for (uint32_t i = 0; i < R.k; i++) pos[i] = R.len[i];
        return;
    }
    auto count_le = [&](int64_t v) {
        uint64_t c = 0;
        for (uint32_t i = 0; i < R.k; i++) c += (uint64_t)(std::upper_bound(R.ts[i], R.ts[i] + R.len[i], v) - R.ts[i]);
        return c;
    };
    // smallest v in [lo, hi] with count(ts <= v) >= r
    int64_t a = lo, b = hi;
    while (a < b) {
        const int64_t m = a + (int64_t)(((uint64_t)b - (uint64_t)a) / 2);
        if (count_le(m) >= r) b = m;
        else a = m + 1;
    }
    const int64_t v = a;
    uint64_t below = 0;
    for (uint32_t i = 0; i < R.k; i++) {
        pos[i] = (uint64_t)(std::lower_bound(R.ts[i], R.ts[i] + R.len[i], v) - R.ts[i]);
        below += pos[i];
    }
    uint64_t need = r - below;   // elements equal to v, taken in run order
    for (uint32_t i = 0; i < R.k && need; i++) {
        const uint64_t eq = (uint64_t)(std::upper_bound(R.ts[i] + pos[i], R.ts[i] + R.len[i], v) - (R.ts[i] + pos[i]));
        const uint64_t t = std::min(eq, need);
        pos[i] += t;
        need -= t;
    }
}

// merge the runs' slices [a[i], b[i]) into out (run << 48 | index)
void merge_slice(const Runs& R, const uint64_t* a, const uint64_t* b, uint64_t* out) {
    std::vector<uint64_t> cur(a, a + R.k);
    for (;;) {
        uint32_t best = UINT32_MAX;
        int64_t bv = 0;
        for (uint32_t i = 0; i < R.k; i++) {   // (k is small: a linear tournament; ties go to the lower run)
            if (cur[i] < b[i] && (best == UINT32_MAX || R.ts[i][cur[i]] < bv)) {
                best = i;
                bv = R.ts[i][cur[i]];
            }
        }
        if (best == UINT32_MAX) return;
        // the stretch of `best` that sorts before every other head: (ts, run) order, so an element goes first
        // while ts < the lowest head of a run before `best` and ts <= the lowest head of a run after it
        int64_t lowL = INT64_MAX, lowG = INT64_MAX;
        bool anyL = false, anyG = false;
        for (uint32_t i = 0; i < R.k; i++) {
            if (i == best || cur[i] >= b[i]) continue;
            const int64_t h = R.ts[i][cur[i]];
            if (i < best) { lowL = std::min(lowL, h); anyL = true; }
            else { lowG = std::min(lowG, h); anyG = true; }
        }
        uint64_t end = cur[best] + 1;
        while (end < b[best] && (!anyL || R.ts[best][end] < lowL) && (!anyG || R.ts[best][end] <= lowG)) end++;
        for (uint64_t j = cur[best]; j < end; j++) *out++ = ((uint64_t)best << 48) | j;
        cur[best] = end;
    }
}

}  // namespace

extern "C" int sg_merge_ts(uint32_t n_runs, const int64_t* const* ts, const uint64_t* len, uint32_t threads,
                           uint64_t* out) {
    if (n_runs == 0) return SG_OK;
    if (!ts || !len || !out || n_runs > 65535) return SG_ERR_INVALID;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n_runs; i++) {
        if (len[i] && !ts[i]) return SG_ERR_INVALID;
        if (len[i] >= (1ull << 48)) return SG_ERR_INVALID;
        total += len[i];
    }
    const Runs R{n_runs, ts, len};
    uint32_t T = std::max(1u, std::min<uint32_t>(threads ? threads : 1u, 256u));
    if (total < (1u << 16)) T = 1;
    std::vector<uint64_t> cuts((size_t)(T + 1) * n_runs);
    for (uint32_t t = 0; t <= T; t++) split_at(R, total * t / T, &cuts[(size_t)t * n_runs]);
    auto work = [&](uint32_t t) {
        merge_slice(R, &cuts[(size_t)t * n_runs], &cuts[(size_t)(t + 1) * n_runs], out + total * t / T);
    };
    if (T == 1) {
        work(0);
        return SG_OK;
    }
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < T; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    return SG_OK;
}
