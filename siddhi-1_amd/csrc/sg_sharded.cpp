// sg_sharded.cpp — multi-device fan-out inside one engine (SURVEY §8b "Multi-GPU fan-out is internal to one
// engine", §8e).  An sg_engine created with sg_config.n_devices > 1 owns one engine per listed device and
// forwards every entry point here, so a caller bound to siddhi_gpu.h (the JNI shim of INTEGRATION.md) drives
// several GPUs through the same handle.
//
// Partition keys shard because no processor reads another key's state (PartitionStateHolder.java:43-49;
// PartitionStreamReceiver.java:262-272 routes each event to its key's runtime).  Key ids are dense in first-seen
// order, so consecutive ids are unrelated keys: shard r = key % N owns a key and sees it as local id key / N,
// dense in [0, ceil(n_keys / N)).  A batch is split stably by owner (per key the arrival order is kept); each
// shard numbers its events with its own arrival seqs (dense: 0, 1, 2, ...) and this engine keeps the map back to
// the global seqs, so polls return global trigger / slot seqs and global key ids, merged into the single
// engine's order: batch matches by (trigger seq, emission order) — all matches of one trigger come from the shard
// owning the trigger's key — and the timer matches of an advance key by key in the order of the keys' queue
// heads (the Scheduler listener's TreeMultimap order, Scheduler.java:78-99: each shard reports its emitting keys'
// heads; two keys sharing a due time, on one shard or across two, is the collapse the single engine refuses,
// SURVEY A.10), or by (fire time, key) for the engines that do not order by heads.  Matches are collected from
// the shards before and right after every advance, so batch and timer matches keep the single engine's
// interleaving.  The playback / wall clock is global: every shard gets the same advance_time sequence.  An unpartitioned query
// (n_keys == 1) does not shard: one key's NFA is sequential, it runs on the first device.
//
// Shards are driven concurrently, one host thread per device per call (each sub-engine is used by one thread at
// a time, as siddhi_gpu.h requires).  A device batch stays on the devices: it is split by owner on the device it
// was handed over on (shard_kernels.hip fan_split: stable, one destination-major copy of each column), a shard on
// another device gets its part by a peer copy, and each shard's engine waits for that work on the device
// (sg_wait_stream) — only the per-shard counts and the 4-B batch position of every event (the seq map) come to
// the host.  Host batches are split on the host.  Polls return host memory.
//
// Seq maps are bounded by live state, not by stream length: after a poll (every shard drained: no match is
// pending on any device), a shard whose map has grown past its threshold reports the smallest seq a live partial
// of it still references (sg_internal_min_seq) and its map drops every entry below (SeqMap.trim).
//
// A call that fails part-way (one shard took a sub-batch, another refused it; a poll that lost one shard's
// matches) leaves the shards out of step: the engine then refuses every call but sg_restore / sg_state_import /
// the read-only ones with SG_ERR_STATE (siddhi_gpu.h).
#include "sg_sharded.h"

#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <functional>
#include <future>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu_ir.h"
#include "state_doc.h"

namespace {

// host threads for the fan-out's per-element work (seq maps, merge, gather): SG_FAN_THREADS, else the hardware's
// threads capped at 16 (the GPU boxes give a GPU's process 16 CPUs)
uint32_t fan_threads() {
    static const uint32_t t = [] {
        if (const char* x = getenv("SG_FAN_THREADS")) return std::max(1u, (uint32_t)strtoul(x, nullptr, 0));
        return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    }();
    return t;
}
// the allocator of the fan-out's host staging (seq maps, polled matches, merge codes: tens to hundreds of MB that
// grow with the match rate): value-initialisation is a no-op, so a resize does not zero-fill what is about to be
// overwritten, and blocks of 4 MB and more are mapped with transparent huge pages asked for, so first touching a
// grown buffer costs one fault per 2 MB rather than per 4 KB
template <class T> struct RawAlloc {
    using value_type = T;
    static constexpr size_t kBig = 4u << 20;
    static constexpr int kPopulateWrite = 23;   // MADV_POPULATE_WRITE (Linux 5.14)
    RawAlloc() = default;
    template <class U> RawAlloc(const RawAlloc<U>&) {}
    T* allocate(size_t n) {
        const size_t b = n * sizeof(T);
        if (b < kBig) return std::allocator<T>().allocate(n);
        void* p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(p, b, MADV_HUGEPAGE);
        (void)madvise(p, b, kPopulateWrite);   // (faulted in by one call; kernels before 5.14 fault on first touch)
        return (T*)p;
    }
    void deallocate(T* p, size_t n) {
        const size_t b = n * sizeof(T);
        if (b < kBig) std::allocator<T>().deallocate(p, n);
        else munmap(p, b);
    }
    template <class U> void construct(U* p) { ::new ((void*)p) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
    template <class U> bool operator==(const RawAlloc<U>&) const { return true; }
    template <class U> bool operator!=(const RawAlloc<U>&) const { return false; }
};
template <class T> using RawVec = std::vector<T, RawAlloc<T>>;
// a buffer sized to at least n elements: it only grows (by a quarter more than asked, so a slowly rising match
// count does not regrow it every poll), so a reused buffer is neither re-initialised nor page-faulted again (the
// element count that matters is kept beside it); keep = false: the old contents are not needed (not copied)
template <class V> typename V::value_type* grow_to(V& v, size_t n, bool keep = true) {
    if (v.size() >= n) return v.data();
    const size_t c = n + n / 4;
    if (!keep) V().swap(v);
    v.reserve(c);
    v.resize(c);
    return v.data();
}
// fn(lo, hi) over [0, n) cut into up to T slices of at least 2^15 elements, run on T threads (the caller's included)
template <class F> void par_for(uint64_t n, uint32_t T, const F& fn) {
    T = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(T, n >> 15));
    if (T <= 1) {
        fn((uint64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < T; t++) th.emplace_back([&, t] { fn(n * t / T, n * (t + 1) / T); });
    fn((uint64_t)0, n / T);
    for (auto& x : th) x.join();
}

struct ShardError : std::runtime_error {
    int code;
    ShardError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

size_t tsize(uint32_t t) {
    switch (t) {
    case SG_T_LONG: case SG_T_DOUBLE: return 8;
    case SG_T_BOOL: return 1;
    default: return 4;
    }
}

const uint64_t kMagic = 0x3248534753ull;  // "SGSH2" (v2: seq maps with their base)

}  // namespace

// a shard's local -> global seq map over the live local seqs [base, top): entries below `base` were trimmed (no live
// partial and no pending match references them).  Stored in chunks of 2^20 entries (8 MB, huge pages, faulted in
// when mapped) indexed by local seq >> 20: an append never moves what is there, a trim hands the chunks wholly
// below `base` to a spare list the next appends take from — no copy and no fresh page once the map has reached its
// peak (twice its live span: the trim check runs when it has doubled) (a contiguous vector regrew and re-faulted tens of MB, 10-30 ms, every few pushes)
struct SeqChunkFree {
    void operator()(uint64_t* p) const { munmap(p, 8ull << 20); }
};
using SeqChunk = std::unique_ptr<uint64_t[], SeqChunkFree>;

struct SeqMap {
    static constexpr uint32_t kShift = 20;
    static constexpr uint64_t kMask = (1ull << kShift) - 1;
    static constexpr size_t kSpare = 256;   // spare chunks kept (2 GB; in practice the map's peak less its live span)
    uint64_t base = 0, top = 0;
    uint64_t c0 = 0;                 // chunk number of chunks[0]
    std::vector<SeqChunk> chunks, spare;
    uint64_t trim_at = 1u << 20;     // the size at which the next trim check runs (+ max(2^20, live span) after each)
    uint64_t size() const { return top - base; }
    uint64_t end() const { return top; }
    void reset(uint64_t b) {
        chunks.clear();
        base = top = b;
        c0 = b >> kShift;
    }
    const uint64_t* ptr(uint64_t l) const { return chunks[(l >> kShift) - c0].get() + (l & kMask); }
    uint64_t at(uint64_t l) const { return *ptr(l); }
    static SeqChunk new_chunk() {
        const size_t b = 8ull << 20;
        void* p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(p, b, MADV_HUGEPAGE);
        (void)madvise(p, b, 23);   // MADV_POPULATE_WRITE (Linux 5.14; before it, faulted on first touch)
        return SeqChunk((uint64_t*)p);
    }
    // n more entries at the end: fn(offset, dst, count) fills each contiguous piece of them
    template <class F> void append_with(uint64_t n, const F& fn) {
        if (chunks.empty()) c0 = top >> kShift;
        for (uint64_t done = 0; done < n;) {
            const uint64_t l = top + done, c = l >> kShift;
            while (c - c0 >= chunks.size()) {
                if (!spare.empty()) {
                    chunks.push_back(std::move(spare.back()));
                    spare.pop_back();
                } else {
                    chunks.push_back(new_chunk());
                }
            }
            const uint64_t k = std::min<uint64_t>(n - done, ((c + 1) << kShift) - l);
            fn(done, chunks[c - c0].get() + (l & kMask), k);
            done += k;
        }
        top += n;
    }
    void append(const uint64_t* p, uint64_t n) {
        append_with(n, [&](uint64_t o, uint64_t* d, uint64_t k) { memcpy(d, p + o, 8 * k); });
    }
    // fn(ptr, count) over the live entries in order
    template <class F> void for_pieces(const F& fn) const {
        for (uint64_t l = base; l < top;) {
            const uint64_t k = std::min<uint64_t>(top - l, (((l >> kShift) + 1) << kShift) - l);
            fn(ptr(l), k);
            l += k;
        }
    }
    void trim(uint64_t keep_from) {
        if (keep_from <= base) return;
        base = std::min(keep_from, top);
        size_t d = 0;
        while (d < chunks.size() && ((c0 + d + 1) << kShift) <= base) d++;
        for (size_t i = 0; i < d; i++)
            if (spare.size() < kSpare) spare.push_back(std::move(chunks[i]));
        chunks.erase(chunks.begin(), chunks.begin() + (ptrdiff_t)d);
        c0 += d;
    }
};

struct ShardEngine {
    uint32_t N = 1, K = 1, KL = 1;   // shards, global / local key ranges
    bool null_keys = false;
    std::vector<sg_engine*> sh;
    std::vector<std::vector<uint32_t>> attr_types;   // per stream of the IR
    std::vector<int> dev;                            // per shard: its HIP device
    std::vector<SeqMap> gmap;                        // per shard: global seq of each local seq
    bool failed = false;                             // a call failed part-way (shards out of step)
    uint64_t staged_bytes = 0;                       // batch bytes copied to host memory (host splits of device batches: none)
    uint64_t trims = 0;
    uint64_t host_syncs = 0;   // host waits of the device-batch pushes (sg_stats.host_syncs)
    // device batches: split on their own device (fan_split), two buffer sets used alternately; set j's events
    // done[r] (on shard r's device) are recorded behind what reads set j for shard r — the shard's push, or the
    // peer copy of its part — and the next split into set j waits for them on the device
    struct DevSplit {
        int device = -1;
        hipStream_t stream = nullptr;
        size_t scratch_len = 0;
        uint32_t* totals = nullptr;   // [N] device
        uint32_t* err = nullptr;
        uint32_t* h_totals = nullptr; // pinned [N + 1] (err last)
        uint32_t* h_opos = nullptr;   // pinned [max_batch]
        struct Set {
            void* scratch = nullptr;
            int64_t* ts = nullptr;
            uint32_t* key = nullptr;
            uint32_t* opos = nullptr;
            std::vector<void*> cols;
            std::vector<uint8_t*> nulls;
            std::vector<hipEvent_t> done;  // per shard (created on dev[r])
            std::vector<char> armed;
        } set[2];
        uint32_t next = 0;
    };
    // a shard's staging on its own device for parts split on another device
    struct Peer {
        hipStream_t stream = nullptr;
        struct Set {
            int64_t* ts = nullptr;
            uint32_t* key = nullptr;
            std::vector<void*> cols;
            std::vector<uint8_t*> nulls;
            hipEvent_t done = nullptr;     // recorded behind the shard's push from this set
            bool armed = false;
        } set[2];
        uint32_t next = 0;
    };
    std::vector<DevSplit> splits;   // by source device ordinal (lazily)
    // sg_wait_stream: one event per (caller stream, device), recorded by the call and waited on once by the next
    // device split (then free for reuse by any stream of its device: the list is bounded by the streams named
    // between two pushes, not by every stream ever named)
    struct Wait {
        void* stream;
        int device;
        hipEvent_t ev;
        bool pending;
    };
    std::vector<Wait> waits;
    std::vector<Peer> peers;        // per shard (lazily)
    bool force_peer = false;        // SG_FAN_PEER_COPY (tests): peer-copy every part, even on the source device
    uint64_t max_batch = 0;
    size_t max_attrs = 1;

    ~ShardEngine() { free_device_buffers(); }
    void free_device_buffers() {
        for (auto& w : waits) {
            (void)hipSetDevice(w.device);
            (void)hipEventDestroy(w.ev);
        }
        waits.clear();
        for (size_t r = 0; r < peers.size(); r++) {
            Peer& q = peers[r];
            if (!q.stream) continue;
            (void)hipSetDevice(dev[r]);
            (void)hipStreamSynchronize(q.stream);
            for (auto& st : q.set) {
                if (st.done) (void)hipEventDestroy(st.done);
                for (void* x : {(void*)st.ts, (void*)st.key}) if (x) (void)hipFree(x);
                for (void* x : st.cols) if (x) (void)hipFree(x);
                for (void* x : st.nulls) if (x) (void)hipFree(x);
            }
            (void)hipStreamDestroy(q.stream);
        }
        peers.clear();
        for (DevSplit& p : splits) {
            if (p.device < 0) continue;
            (void)hipSetDevice(p.device);
            if (p.stream) (void)hipStreamSynchronize(p.stream);
            for (auto& st : p.set) {
                for (size_t r = 0; r < st.done.size(); r++)
                    if (st.done[r]) {
                        (void)hipSetDevice(dev[r]);
                        (void)hipEventDestroy(st.done[r]);
                    }
                (void)hipSetDevice(p.device);
                for (void* x : {st.scratch, (void*)st.ts, (void*)st.key, (void*)st.opos}) if (x) (void)hipFree(x);
                for (void* x : st.cols) if (x) (void)hipFree(x);
                for (void* x : st.nulls) if (x) (void)hipFree(x);
            }
            if (p.totals) (void)hipFree(p.totals);   // (err lives in the same allocation)
            if (p.h_totals) (void)hipHostFree(p.h_totals);
            if (p.h_opos) (void)hipHostFree(p.h_opos);
            if (p.stream) (void)hipStreamDestroy(p.stream);
        }
        splits.clear();
        (void)hipGetLastError();
    }

    // matches in host memory, in the single engine's order: `pend` collects them as the shards produce them
    // (batch matches before every advance, timer matches right after it), a poll hands `pend` out as `out`
    struct Out {
        uint64_t n = 0;
        uint32_t ns = 0, mc = 1, ni = 0;
        RawVec<uint64_t> trig, slot;
        RawVec<uint32_t> key, len;
        RawVec<int64_t> ts;
        std::vector<uint64_t> pval;
        std::vector<uint8_t> pnull;
    };
    Out pend, out;
    RawVec<uint64_t> codes;   // collect's output order
    std::vector<Out> parts;   // collect's per-shard staging (kept: its buffers are reused, not page-faulted per poll)
    bool held = false;
    bool proj = false;
    bool heads = false;   // every shard orders its timer matches by the keys' queue heads (and reports them)
    uint32_t nslots = 0, mchain = 1;  // the shards' slot count / chain width (reported by every poll, even empty)

    // run fn(r) for every shard, concurrently when there are several; the first failure is rethrown here
    void each(const std::function<int(uint32_t)>& fn) {
        std::vector<int> rc(N, SG_OK);
        std::vector<std::string> msg(N);
        auto run = [&](uint32_t r) {
            try {
                rc[r] = fn(r);
                if (rc[r] != SG_OK) msg[r] = sg_last_error();   // (the error text is per thread)
            } catch (const ShardError& ex) {
                rc[r] = ex.code;
                msg[r] = ex.what();
            } catch (const std::exception& ex) {
                rc[r] = SG_ERR_DEVICE;
                msg[r] = ex.what();
            }
        };
        if (N == 1) {
            run(0);
        } else {
            std::vector<std::future<void>> fs;
            for (uint32_t r = 1; r < N; r++) fs.push_back(std::async(std::launch::async, run, r));
            run(0);
            for (auto& f : fs) f.get();
        }
        for (uint32_t r = 0; r < N; r++)
            if (rc[r] != SG_OK) throw ShardError(rc[r], "shard " + std::to_string(r) + ": " + msg[r]);
    }


    uint64_t map_seq(uint32_t r, uint64_t local) const {
        if (local >= SG_BLANK_SEQ) return local;   // null / blank / timer markers pass through
        const SeqMap& m = gmap[r];
        if (local < m.base || local >= m.end()) throw ShardError(SG_ERR_DEVICE, "shard seq outside its map");
        return m.at(local);
    }
};

namespace {

int fail_from(const std::exception& ex) {
    if (auto* s = dynamic_cast<const ShardError*>(&ex)) return sg_set_error(s->code, s->what());
    return sg_set_error(SG_ERR_DEVICE, ex.what());
}

void parse_streams(ShardEngine* s, const uint32_t* w, size_t nw) {
    if (nw < SG_IR_HDR_WORDS) throw ShardError(SG_ERR_INVALID, "IR too short");
    const uint32_t ns = w[3];
    size_t p = w[7];
    for (uint32_t i = 0; i < ns; i++) {
        if (p >= nw) throw ShardError(SG_ERR_INVALID, "IR stream table out of range");
        const uint32_t na = w[p++];
        if (p + na > nw) throw ShardError(SG_ERR_INVALID, "IR stream table out of range");
        s->attr_types.emplace_back(w + p, w + p + na);
        p += na;
    }
}

// the staged host copy of a batch (device batches are copied first)
struct HostBatch {
    std::vector<std::vector<uint8_t>> store;
    const int64_t* ts = nullptr;
    const uint32_t* key = nullptr;
    std::vector<const void*> cols;
    std::vector<const uint8_t*> nulls;
};

HostBatch stage(const ShardEngine* s, const sg_batch* b) {
    HostBatch h;
    const uint64_t n = b->n;
    h.cols.assign(b->n_cols, nullptr);
    h.nulls.assign(b->n_cols, nullptr);
    if (b->mem == SG_MEM_HOST) {
        h.ts = b->ts;
        h.key = b->key;
        for (uint32_t c = 0; c < b->n_cols; c++) {
            h.cols[c] = b->cols[c];
            h.nulls[c] = b->nulls ? b->nulls[c] : nullptr;
        }
        return h;
    }
    auto copy = [&](const void* src, size_t bytes) -> const void* {
        h.store.emplace_back(bytes);
        const_cast<ShardEngine*>(s)->staged_bytes += bytes;
        if (bytes && hipMemcpy(h.store.back().data(), src, bytes, hipMemcpyDeviceToHost) != hipSuccess)
            throw ShardError(SG_ERR_DEVICE, "staging a device batch failed");
        return h.store.back().data();
    };
    h.ts = (const int64_t*)copy(b->ts, n * 8);
    if (b->key) h.key = (const uint32_t*)copy(b->key, n * 4);
    const auto& ty = s->attr_types[b->stream];
    for (uint32_t c = 0; c < b->n_cols; c++) {
        h.cols[c] = copy(b->cols[c], n * tsize(ty[c]));
        if (b->nulls && b->nulls[c]) h.nulls[c] = (const uint8_t*)copy(b->nulls[c], n);
    }
    return h;
}

}  // namespace

ShardEngine* shd_create(const void* ir, size_t ir_len, const sg_config* cfg, int* rc) {
    std::unique_ptr<ShardEngine> s(new ShardEngine());
    try {
        parse_streams(s.get(), (const uint32_t*)ir, ir_len / 4);
        s->K = cfg->n_keys ? cfg->n_keys : 1;
        s->N = s->K > 1 ? cfg->n_devices : 1;
        s->KL = (s->K + s->N - 1) / s->N;
        s->null_keys = (cfg->flags & SG_CFG_NULL_KEYS) != 0;
        s->gmap.resize(s->N);
        s->sh.assign(s->N, nullptr);
        s->max_batch = cfg->max_batch ? cfg->max_batch : (1u << 20);
        for (const auto& t : s->attr_types) s->max_attrs = std::max(s->max_attrs, t.size());
        s->force_peer = getenv("SG_FAN_PEER_COPY") != nullptr;
        for (uint32_t r = 0; r < s->N; r++) s->dev.push_back(cfg->devices ? cfg->devices[r] : cfg->device);
        for (uint32_t r = 0; r < s->N; r++) {
            sg_config c = *cfg;
            c.struct_size = sizeof(sg_config);
            c.device = s->dev[r];
            c.n_keys = s->K > 1 ? s->KL : 1;
            c.n_devices = 1;
            c.devices = nullptr;
            const int e = sg_engine_create(ir, ir_len, &c, &s->sh[r]);
            if (e != SG_OK) throw ShardError(e, std::string("shard ") + std::to_string(r) + ": " + sg_last_error());
        }
        s->heads = true;
        for (uint32_t r = 0; r < s->N; r++) s->heads = sg_internal_keep_heads(s->sh[r]) && s->heads;
        *rc = SG_OK;
        return s.release();
    } catch (const std::exception& ex) {
        for (sg_engine* e : s->sh)
            if (e) sg_engine_destroy(e);
        s->sh.clear();
        *rc = fail_from(ex);
        return nullptr;
    }
}

void shd_destroy(ShardEngine* s) {
    if (!s) return;
    for (sg_engine* e : s->sh)
        if (e) sg_engine_destroy(e);
    delete s;
}

namespace {

#define FAN_OK(x)                                                                                         \
    do {                                                                                                  \
        const hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) throw ShardError(SG_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

static double fan_now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static const bool g_fan_prof = getenv("SG_FAN_PROF") != nullptr;   // (experiments: phase times to stderr)

template <class T> T* fan_alloc(size_t n) {
    void* p = nullptr;
    FAN_OK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
    return (T*)p;
}

ShardEngine::DevSplit& split_for(ShardEngine* s, int device) {
    if ((size_t)device >= s->splits.size()) s->splits.resize(device + 1);
    ShardEngine::DevSplit& p = s->splits[device];
    if (p.device >= 0) return p;
    FAN_OK(hipSetDevice(device));
    p.device = device;
    const size_t B = s->max_batch;
    FAN_OK(hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking));
    p.scratch_len = fan_split_scratch_bytes(B, s->N);
    p.totals = fan_alloc<uint32_t>(s->N + 1);
    p.err = p.totals + s->N;
    FAN_OK(hipHostMalloc((void**)&p.h_totals, (s->N + 1) * 4, hipHostMallocDefault));
    FAN_OK(hipHostMalloc((void**)&p.h_opos, B * 4, hipHostMallocDefault));
    for (auto& st : p.set) {
        st.scratch = fan_alloc<uint8_t>(p.scratch_len);
        st.ts = fan_alloc<int64_t>(B);
        st.key = fan_alloc<uint32_t>(B);
        st.opos = fan_alloc<uint32_t>(B);
        for (size_t c = 0; c < s->max_attrs; c++) {
            st.cols.push_back(fan_alloc<uint64_t>(B));
            st.nulls.push_back(fan_alloc<uint8_t>(B));
        }
        st.done.assign(s->N, nullptr);
        st.armed.assign(s->N, 0);
        for (uint32_t r = 0; r < s->N; r++) {
            FAN_OK(hipSetDevice(s->dev[r]));
            FAN_OK(hipEventCreateWithFlags(&st.done[r], hipEventDisableTiming));
        }
        FAN_OK(hipSetDevice(device));
    }
    return p;
}

ShardEngine::Peer& peer_for(ShardEngine* s, uint32_t r) {
    ShardEngine::Peer& q = s->peers[r];
    if (q.stream) return q;
    FAN_OK(hipSetDevice(s->dev[r]));
    const size_t B = s->max_batch;
    FAN_OK(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking));
    for (auto& st : q.set) {
        st.ts = fan_alloc<int64_t>(B);
        st.key = fan_alloc<uint32_t>(B);
        for (size_t c = 0; c < s->max_attrs; c++) {
            st.cols.push_back(fan_alloc<uint64_t>(B));
            st.nulls.push_back(fan_alloc<uint8_t>(B));
        }
        FAN_OK(hipEventCreateWithFlags(&st.done, hipEventDisableTiming));
    }
    return q;
}

// a device batch, split on its device: the shards' parts pushed as device batches (peer-copied to shards on
// other devices), each shard's engine waiting for its part on the device; only the per-shard counts and the
// batch position of every event (the seq maps) are copied to the host
void push_device(ShardEngine* s, const sg_batch* b) {
    hipPointerAttribute_t at{};
    FAN_OK(hipPointerGetAttributes(&at, b->ts));
    const int src = at.device;
    const uint32_t N = s->N;
    const uint64_t n = b->n;
    if (n > s->max_batch) throw ShardError(SG_ERR_INVALID, "batch larger than max_batch");
    const auto& ty = s->attr_types[b->stream];
    const uint32_t nc = b->n_cols;
    ShardEngine::DevSplit& p = split_for(s, src);
    const uint32_t j = p.next;
    auto& st = p.set[j];
    FAN_OK(hipSetDevice(src));
    for (uint32_t r = 0; r < N; r++)   // this set's previous readers are done (on the device)
        if (st.armed[r]) FAN_OK(hipStreamWaitEvent(p.stream, st.done[r], 0));
    for (auto& w : s->waits)           // the producers the caller named since the last push (sg_wait_stream)
        if (w.pending) {
            FAN_OK(hipStreamWaitEvent(p.stream, w.ev, 0));
            w.pending = false;
        }
    std::vector<const void*> cols(nc);
    std::vector<uint32_t> cb(nc);
    std::vector<const uint8_t*> nul(nc, nullptr);
    bool anyNull = false;
    for (uint32_t c = 0; c < nc; c++) {
        cols[c] = b->cols[c];
        cb[c] = (uint32_t)tsize(ty[c]);
        if (b->nulls && b->nulls[c]) {
            nul[c] = b->nulls[c];
            anyNull = true;
        }
    }
    std::vector<void*> ocols(st.cols.begin(), st.cols.begin() + nc);
    std::vector<uint8_t*> onul(st.nulls.begin(), st.nulls.begin() + nc);
    const int rc = fan_split(n, b->key, s->K, N, s->null_keys, b->ts, cols.data(), cb.data(), nul.data(), nc, st.ts,
                             ocols.data(), onul.data(), st.opos, st.key, p.totals, p.err, st.scratch, p.scratch_len,
                             p.stream);
    if (rc != SG_OK) throw ShardError(rc, "device split of the batch failed");
    const double q0 = g_fan_prof ? fan_now() : 0.0;
    FAN_OK(hipMemcpyAsync(p.h_totals, p.totals, (N + 1) * 4, hipMemcpyDeviceToHost, p.stream));
    FAN_OK(hipMemcpyAsync(p.h_opos, st.opos, n * 4, hipMemcpyDeviceToHost, p.stream));
    FAN_OK(hipStreamSynchronize(p.stream));
    s->host_syncs++;
    const double q1 = g_fan_prof ? fan_now() : 0.0;
    if (p.h_totals[N]) throw ShardError(SG_ERR_INVALID, "key id outside [0, n_keys)");
    // validated: nothing has changed yet (a rejected batch leaves every shard as it was)
    std::vector<uint64_t> off(N + 1, 0);
    for (uint32_t r = 0; r < N; r++) off[r + 1] = off[r] + p.h_totals[r];
    hipEvent_t split_done = nullptr;
    FAN_OK(hipEventCreateWithFlags(&split_done, hipEventDisableTiming));
    FAN_OK(hipEventRecord(split_done, p.stream));
    p.next ^= 1u;
    if (s->peers.empty()) s->peers.resize(N);   // (before the shard threads: peer_for touches only peers[r])
    std::vector<char> pushed(N, 0);
    try {
        s->each([&](uint32_t r) -> int {
            const uint64_t m = off[r + 1] - off[r];
            if (m == 0) return SG_OK;
            FAN_OK(hipSetDevice(s->dev[r]));
            sg_batch c{};
            c.struct_size = sizeof(sg_batch);
            c.stream = b->stream;
            c.n = m;
            c.seq_base = s->gmap[r].end();
            c.n_cols = nc;
            c.mem = SG_MEM_DEVICE;
            std::vector<const void*> cp(nc);
            std::vector<const uint8_t*> np(nc, nullptr);
            const bool copy = s->force_peer || s->dev[r] != src;
            ShardEngine::Peer::Set* ps = nullptr;
            hipStream_t wait_on = p.stream;
            if (copy) {   // the part to the shard's device (a peer copy; on one device a device-to-device copy)
                ShardEngine::Peer& q = peer_for(s, r);
                ps = &q.set[q.next];
                q.next ^= 1u;
                if (ps->armed) FAN_OK(hipStreamWaitEvent(q.stream, ps->done, 0));
                FAN_OK(hipStreamWaitEvent(q.stream, split_done, 0));
                const int dd = s->dev[r];
                auto cp_part = [&](void* dst, const void* from, size_t bytes) {
                    if (dd == src) FAN_OK(hipMemcpyAsync(dst, from, bytes, hipMemcpyDeviceToDevice, q.stream));
                    else FAN_OK(hipMemcpyPeerAsync(dst, dd, from, src, bytes, q.stream));
                };
                cp_part(ps->ts, st.ts + off[r], m * 8);
                cp_part(ps->key, st.key + off[r], m * 4);
                for (uint32_t c2 = 0; c2 < nc; c2++) {
                    cp_part(ps->cols[c2], (const uint8_t*)st.cols[c2] + off[r] * cb[c2], m * cb[c2]);
                    if (nul[c2]) cp_part(ps->nulls[c2], st.nulls[c2] + off[r], m);
                }
                (void)hipGetLastError();   // (a stale per-thread error would be picked up by the shard's launches)
                // the split set may be reused once the copies ran
                FAN_OK(hipEventRecord(st.done[r], q.stream));
                st.armed[r] = 1;
                c.ts = ps->ts;
                c.key = ps->key;
                for (uint32_t c2 = 0; c2 < nc; c2++) {
                    cp[c2] = ps->cols[c2];
                    np[c2] = nul[c2] ? ps->nulls[c2] : nullptr;
                }
                wait_on = q.stream;
            } else {
                c.ts = st.ts + off[r];
                c.key = st.key + off[r];
                for (uint32_t c2 = 0; c2 < nc; c2++) {
                    cp[c2] = (const uint8_t*)st.cols[c2] + off[r] * cb[c2];
                    np[c2] = nul[c2] ? st.nulls[c2] + off[r] : nullptr;
                }
            }
            c.cols = cp.data();
            c.nulls = anyNull ? np.data() : nullptr;
            const double v0 = g_fan_prof ? fan_now() : 0.0;
            int rc2 = sg_wait_stream(s->sh[r], wait_on);
            if (rc2 != SG_OK) return rc2;
            rc2 = sg_push_batch(s->sh[r], &c);
            if (rc2 != SG_OK) return rc2;
            const double v1 = g_fan_prof ? fan_now() : 0.0;
            pushed[r] = 1;
            // what reads the part is queued: the buffers it lives in are free once the shard's engine ran it
            if (copy) {
                sg_internal_record(s->sh[r], ps->done);
                ps->armed = true;
            } else {
                sg_internal_record(s->sh[r], st.done[r]);
                st.armed[r] = 1;
            }
            const uint32_t* op = p.h_opos + off[r];
            const uint64_t sb = b->seq_base;
            s->gmap[r].append_with(m, [&](uint64_t o, uint64_t* gv, uint64_t k) {
                par_for(k, std::max(1u, fan_threads() / N), [&](uint64_t lo, uint64_t hi) {
                    for (uint64_t i = lo; i < hi; i++) gv[i] = sb + op[o + i];
                });
            });
            if (g_fan_prof)
                fprintf(stderr, "fan shard %u: push %.2f ms, seq map %.2f ms\n", r, (v1 - v0) * 1e3,
                        (fan_now() - v1) * 1e3);
            return SG_OK;
        });
    } catch (...) {
        (void)hipEventDestroy(split_done);
        for (uint32_t r = 0; r < N; r++)
            if (pushed[r]) s->failed = true;   // some shards took their part: the engine is out of step
        throw;
    }
    (void)hipEventDestroy(split_done);
    if (g_fan_prof)
        fprintf(stderr, "fan push: split + wait %.2f ms, shard pushes + seq maps %.2f ms\n", (q1 - q0) * 1e3,
                (fan_now() - q1) * 1e3);
}

}  // namespace

int shd_push(ShardEngine* s, const sg_batch* b) {
    try {
        if (s->failed) throw ShardError(SG_ERR_STATE, "a previous call failed part-way: restore a snapshot first");
        if (s->held) throw ShardError(SG_ERR_STATE, "release the polled matches before pushing");
        if (b->stream >= s->attr_types.size()) throw ShardError(SG_ERR_INVALID, "stream index out of range");
        if (b->n_cols != s->attr_types[b->stream].size())
            throw ShardError(SG_ERR_INVALID, "column count does not match the stream");
        if (b->n == 0) return SG_OK;
        const uint64_t n = b->n;
        if (s->N == 1) {   // (unpartitioned, or one device): the shard takes the batch as it is
            sg_batch c = *b;
            SeqMap& m = s->gmap[0];
            c.seq_base = m.end();
            const int rc = sg_push_batch(s->sh[0], &c);
            if (rc != SG_OK) return rc;
            const uint64_t sb = b->seq_base;
            m.append_with(n, [&](uint64_t o, uint64_t* mv, uint64_t k) {
                for (uint64_t i = 0; i < k; i++) mv[i] = sb + o + i;
            });
            return SG_OK;
        }
        if (!b->key) throw ShardError(SG_ERR_INVALID, "partitioned query needs key ids");
        // (host and device batches alike: the device split's buffers hold max_batch events)
        if (n > s->max_batch) throw ShardError(SG_ERR_INVALID, "batch larger than max_batch");
        if (b->mem == SG_MEM_DEVICE) {
            push_device(s, b);
            return SG_OK;
        }
        HostBatch h = stage(s, b);
        const uint32_t N = s->N;
        // owner of every event (null keys: dropped with SG_CFG_NULL_KEYS, else an error), per-shard counts
        std::vector<uint32_t> cnt(N, 0);
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t k = h.key[i];
            if (k >= s->K) {
                if (s->null_keys && k == SG_KEY_NULL) continue;
                throw ShardError(SG_ERR_INVALID, "key id outside [0, n_keys)");
            }
            cnt[k % N]++;
        }
        const auto& ty = s->attr_types[b->stream];
        const uint32_t nc = b->n_cols;
        // per shard: the positions of its events (stable: arrival order within the shard), then each column
        // gathered through them with typed loads (one pass per column, no per-byte appends)
        struct Sub {
            std::vector<uint32_t> pos;
            std::vector<int64_t> ts;
            std::vector<uint32_t> key;
            std::vector<std::vector<uint8_t>> cols, nulls;
            std::vector<uint64_t> glob;
        };
        std::vector<Sub> sub(N);
        for (uint32_t r = 0; r < N; r++) sub[r].pos.reserve(cnt[r]);
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t k = h.key[i];
            if (k < s->K) sub[k % N].pos.push_back((uint32_t)i);
        }
        auto gather = [](const void* src, size_t sz, const std::vector<uint32_t>& pos, std::vector<uint8_t>& out) {
            out.resize(pos.size() * sz);
            switch (sz) {
            case 8: { const uint64_t* a = (const uint64_t*)src; uint64_t* o = (uint64_t*)out.data();
                      for (size_t j = 0; j < pos.size(); j++) o[j] = a[pos[j]]; break; }
            case 4: { const uint32_t* a = (const uint32_t*)src; uint32_t* o = (uint32_t*)out.data();
                      for (size_t j = 0; j < pos.size(); j++) o[j] = a[pos[j]]; break; }
            default: { const uint8_t* a = (const uint8_t*)src;
                       for (size_t j = 0; j < pos.size(); j++) memcpy(out.data() + j * sz, a + (size_t)pos[j] * sz, sz); }
            }
        };
        s->each([&](uint32_t r) -> int {   // (the gathers of different shards run side by side)
            Sub& u = sub[r];
            const size_t m = u.pos.size();
            u.ts.resize(m);
            u.key.resize(m);
            u.glob.resize(m);
            for (size_t j = 0; j < m; j++) {
                const uint32_t i = u.pos[j];
                u.ts[j] = h.ts[i];
                u.key[j] = h.key[i] / N;
                u.glob[j] = b->seq_base + i;
            }
            u.cols.resize(nc);
            u.nulls.resize(nc);
            for (uint32_t c = 0; c < nc; c++) {
                gather(h.cols[c], tsize(ty[c]), u.pos, u.cols[c]);
                if (h.nulls[c]) gather(h.nulls[c], 1, u.pos, u.nulls[c]);
            }
            return SG_OK;
        });
        std::vector<char> pushed(N, 0);
        try {
            s->each([&](uint32_t r) -> int {
                Sub& u = sub[r];
                if (u.ts.empty()) return SG_OK;
                std::vector<const void*> cp(nc);
                std::vector<const uint8_t*> np(nc, nullptr);
                bool anyNull = false;
                for (uint32_t c = 0; c < nc; c++) {
                    cp[c] = u.cols[c].data();
                    if (h.nulls[c]) {
                        np[c] = u.nulls[c].data();
                        anyNull = true;
                    }
                }
                SeqMap& m = s->gmap[r];
                sg_batch c{};
                c.struct_size = sizeof(sg_batch);
                c.stream = b->stream;
                c.n = u.ts.size();
                c.seq_base = m.end();
                c.key = u.key.data();
                c.ts = u.ts.data();
                c.cols = cp.data();
                c.nulls = anyNull ? np.data() : nullptr;
                c.n_cols = nc;
                c.mem = SG_MEM_HOST;
                const int rc = sg_push_batch(s->sh[r], &c);
                if (rc == SG_OK) {
                    pushed[r] = 1;
                    m.append(u.glob.data(), u.glob.size());
                }
                return rc;
            });
        } catch (...) {
            for (uint32_t r = 0; r < N; r++)
                if (pushed[r]) s->failed = true;
            throw;
        }
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

int shd_set_projection(ShardEngine* s, const uint32_t* code, uint32_t code_words, const uint32_t* item_pc,
                       const uint32_t* item_len, const uint32_t* item_type, uint32_t n_items, const int32_t* part_attr,
                       uint32_t n_streams) {
    try {
        s->each([&](uint32_t r) {
            return sg_set_projection(s->sh[r], code, code_words, item_pc, item_len, item_type, n_items, part_attr,
                                     n_streams);
        });
        s->proj = true;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

namespace {

// every shard's matches since its last poll, mapped to global seqs / keys, merged and appended to s->pend:
// timers = false: batch matches, by (trigger seq, the shard's emission order) — all matches of one trigger come
// from the shard owning the trigger's key; timers = true: the timer matches of one advance, key by key in the
// order of the keys' queue heads (each shard emitted its keys in that order; two shards' keys sharing a head is
// the Scheduler collapse the single engine refuses), or by (fire time, key) for an engine that does
// not order by heads

void collect(ShardEngine* s, bool timers) {
    const uint32_t N = s->N;
    const double c0 = g_fan_prof ? fan_now() : 0.0;
    std::vector<ShardEngine::Out>& parts = s->parts;
    parts.resize(N);
    std::vector<std::vector<uint32_t>> hk(N);
    std::vector<std::vector<int64_t>> ht(N);
    s->each([&](uint32_t r) -> int {
        sg_match_batch m{};
        const double w0 = g_fan_prof ? fan_now() : 0.0;
        int rc = sg_poll_matches(s->sh[r], SG_MEM_HOST, &m);
        if (rc != SG_OK) return rc;
        const double w1 = g_fan_prof ? fan_now() : 0.0;
        ShardEngine::Out& p = parts[r];
        p.n = m.n;
        p.ns = m.n_slots;
        p.mc = m.max_chain ? m.max_chain : 1;
        grow_to(p.trig, p.n, false);
        grow_to(p.key, p.n, false);
        grow_to(p.ts, p.n, false);
        grow_to(p.len, p.n * p.ns, false);
        grow_to(p.slot, p.n * p.ns * p.mc, false);
        // local -> global seqs (the shard's map), global key ids: sliced over this shard's share of the host threads
        const SeqMap& gm = s->gmap[r];
        const uint64_t mb = gm.base, me = gm.end();
        bool bad = false;
        const uint64_t spm = (uint64_t)p.ns * p.mc;
        par_for(p.n, std::max(1u, fan_threads() / N), [&](uint64_t lo, uint64_t hi) {
            bool b = false;
            auto map = [&](uint64_t l) -> uint64_t {
                if (l >= SG_BLANK_SEQ) return l;   // null / blank / timer markers pass through
                if (l < mb || l >= me) { b = true; return l; }
                return gm.at(l);
            };
            const uint64_t PD = 24;   // (the slot seqs' map entries are scattered: fetched this many matches ahead)
            for (uint64_t i = lo; i < hi; i++) {
                if (i + PD < hi)
                    for (uint64_t q = 0; q < spm; q++) {
                        const uint64_t l = m.slot_seq[(i + PD) * spm + q];
                        if (l >= mb && l < me) __builtin_prefetch(gm.ptr(l));
                    }
                const uint64_t tl = m.trigger_seq[i], tg = tl == SG_TIMER_SEQ ? SG_TIMER_SEQ : map(tl);
                p.trig[i] = tg;
                p.key[i] = N > 1 ? m.key[i] * N + r : m.key[i];
                p.ts[i] = m.ts[i];
                for (uint64_t q = 0; q < p.ns; q++) p.len[i * p.ns + q] = m.chain_len[i * p.ns + q];
                for (uint64_t q = 0; q < spm; q++) {   // (the trigger's own slot is mapped already)
                    const uint64_t l = m.slot_seq[i * spm + q];
                    p.slot[i * spm + q] = l == tl ? tg : map(l);
                }
            }
            if (b) bad = true;   // (a benign race: every writer stores true)
        });
        if (bad) throw ShardError(SG_ERR_DEVICE, "shard seq outside its map");
        if (s->proj) {
            sg_projection pr{};
            rc = sg_get_projection(s->sh[r], SG_MEM_HOST, &pr);
            if (rc != SG_OK) return rc;
            p.ni = pr.n_items;
            p.pval.assign(pr.value, pr.value + (size_t)pr.n_items * p.n);
            p.pnull.assign(pr.null, pr.null + (size_t)pr.n_items * p.n);
        }
        if (timers && s->heads) sg_internal_heads(s->sh[r], hk[r], ht[r]);
        const double w2 = g_fan_prof ? fan_now() : 0.0;
        rc = sg_release_matches(s->sh[r], &m);
        if (g_fan_prof)
            fprintf(stderr, "fan shard %u: poll %.2f ms, map %.2f ms, release %.2f ms\n", r, (w1 - w0) * 1e3,
                    (w2 - w1) * 1e3, (fan_now() - w2) * 1e3);
        return rc;
    });
    const double c1 = g_fan_prof ? fan_now() : 0.0;
    uint64_t total = 0;
    for (uint32_t r = 0; r < N; r++) {
        total += parts[r].n;
        if (parts[r].ns) s->nslots = parts[r].ns;
        s->mchain = std::max(s->mchain, parts[r].mc);
    }
    if (total == 0) return;
    // the output order as (shard << 48 | index) codes
    RawVec<uint64_t>& code = s->codes;
    grow_to(code, total, false);
    // batch matches only (no timer match in any part): each shard's run is already in trigger order (its local
    // seqs map to increasing global ones), and one trigger's matches all come from one shard, so the order is an
    // N-way merge of the runs by trigger seq: the parallel merge path of sg_merge_ts over the host threads
    bool merge = !timers;
    for (uint32_t r = 0; r < N && merge; r++)
        for (uint64_t i = 0; i < parts[r].n; i++)
            if (parts[r].trig[i] >= (1ull << 63) || (i > 0 && parts[r].trig[i] < parts[r].trig[i - 1])) {
                merge = false;   // (a timer match, or a run out of order)
                break;
            }
    if (merge) {
        std::vector<const int64_t*> runs(N);
        std::vector<uint64_t> lens(N);
        for (uint32_t r = 0; r < N; r++) {
            runs[r] = (const int64_t*)parts[r].trig.data();
            lens[r] = parts[r].n;
        }
        if (sg_merge_ts(N, runs.data(), lens.data(), fan_threads(), code.data()) != SG_OK)
            throw ShardError(SG_ERR_DEVICE, "merge of the shards' matches failed");
    } else {
        struct Ref {
            uint32_t r;
            uint64_t i;
            int64_t head;
        };
        std::vector<Ref> ord;
        ord.reserve(total);
        for (uint32_t r = 0; r < N; r++) {
            const ShardEngine::Out& p = parts[r];
            if (timers && s->heads) {
                // the shard's output is its emitting keys' matches, key after key in head order (hk / ht)
                size_t g = 0;
                for (uint64_t i = 0; i < p.n; i++) {
                    const uint32_t lk = N > 1 ? p.key[i] / N : p.key[i];
                    if (i > 0 && p.key[i] != p.key[i - 1]) g++;
                    while (g < hk[r].size() && hk[r][g] != lk) g++;
                    if (g >= hk[r].size()) throw ShardError(SG_ERR_DEVICE, "timer match of a key without a recorded head");
                    ord.push_back({r, i, ht[r][g]});
                }
            } else {
                for (uint64_t i = 0; i < p.n; i++) ord.push_back({r, i, 0});
            }
        }
        std::stable_sort(ord.begin(), ord.end(), [&](const Ref& a, const Ref& b) {
            const ShardEngine::Out &A = parts[a.r], &B = parts[b.r];
            const bool ta = A.trig[a.i] == SG_TIMER_SEQ, tb = B.trig[b.i] == SG_TIMER_SEQ;
            if (ta != tb) return ta;
            if (ta && s->heads) return a.head < b.head;
            if (ta) {
                if (A.ts[a.i] != B.ts[b.i]) return A.ts[a.i] < B.ts[b.i];
                return A.key[a.i] < B.key[b.i];
            }
            return A.trig[a.i] < B.trig[b.i];
        });
        if (timers && s->heads)
            for (size_t x = 1; x < ord.size(); x++)
                if (ord[x].r != ord[x - 1].r && ord[x].head == ord[x - 1].head)
                    throw ShardError(SG_ERR_UNSUPPORTED,
                                     "two partition keys share a timer due time at one clock advance (reference Scheduler "
                                     "collapse quirk, SURVEY A.10): input not supported");
        for (uint64_t x = 0; x < total; x++) code[x] = ((uint64_t)ord[x].r << 48) | ord[x].i;
    }
    const double c2 = g_fan_prof ? fan_now() : 0.0;
    // append to pend (the chain dimension grows to the widest shard's)
    ShardEngine::Out& o = s->pend;
    uint32_t mc = std::max(o.n ? o.mc : 1u, 1u), ns = 0, ni = o.n ? o.ni : 0;
    for (const auto& p : parts)
        if (p.n) {
            mc = std::max(mc, p.mc);
            ns = p.ns;
            ni = std::max(ni, p.ni);
        }
    if (o.n && o.ns != ns) throw ShardError(SG_ERR_DEVICE, "shards disagree on the slot count");
    if (o.n && mc != o.mc) {  // re-pad what is pending
        RawVec<uint64_t> sl(o.n * ns * mc, SG_NULL_SEQ);
        for (uint64_t q = 0; q < o.n * ns; q++)
            for (uint32_t c = 0; c < o.mc; c++) sl[q * mc + c] = o.slot[q * o.mc + c];
        o.slot.swap(sl);
    }
    if (o.n && ni != o.ni) {  // (the item count is the projection's: the same for every shard)
        throw ShardError(SG_ERR_DEVICE, "shards disagree on the projected items");
    }
    const uint64_t n0 = o.n, n1 = n0 + total;
    o.ns = ns;
    o.mc = mc;
    o.ni = ni;
    grow_to(o.trig, n1);
    grow_to(o.key, n1);
    grow_to(o.ts, n1);
    grow_to(o.len, n1 * ns);
    grow_to(o.slot, n1 * ns * mc);
    // projection: item-major over the pending rows -> rebuilt with the new row count
    std::vector<uint64_t> pv((size_t)ni * n1, 0);
    std::vector<uint8_t> pn((size_t)ni * n1, 0);
    for (uint32_t it = 0; it < ni && n0; it++)
        for (uint64_t q = 0; q < n0; q++) {
            pv[(size_t)it * n1 + q] = o.pval[(size_t)it * n0 + q];
            pn[(size_t)it * n1 + q] = o.pnull[(size_t)it * n0 + q];
        }
    par_for(total, fan_threads(), [&](uint64_t lo, uint64_t hi) {
        for (uint64_t x = lo; x < hi; x++) {
            const ShardEngine::Out& p = parts[code[x] >> 48];
            const uint64_t i = code[x] & ((1ull << 48) - 1), d = n0 + x;
            o.trig[d] = p.trig[i];
            o.key[d] = p.key[i];
            o.ts[d] = p.ts[i];
            for (uint32_t sl = 0; sl < ns; sl++) {
                o.len[d * ns + sl] = p.len[i * ns + sl];
                for (uint32_t c = 0; c < mc; c++)
                    o.slot[(d * ns + sl) * mc + c] = c < p.mc ? p.slot[(i * ns + sl) * p.mc + c] : SG_NULL_SEQ;
            }
            for (uint32_t it = 0; it < p.ni; it++) {
                pv[(size_t)it * n1 + d] = p.pval[(size_t)it * p.n + i];
                pn[(size_t)it * n1 + d] = p.pnull[(size_t)it * p.n + i];
            }
        }
    });
    o.pval.swap(pv);
    o.pnull.swap(pn);
    o.n = n1;
    if (g_fan_prof)
        fprintf(stderr, "fan collect: shard polls + seq mapping %.2f ms, order %.2f ms, append %.2f ms (%llu matches)\n",
                (c1 - c0) * 1e3, (c2 - c1) * 1e3, (fan_now() - c2) * 1e3, (unsigned long long)total);
}

}  // namespace

int shd_advance(ShardEngine* s, int64_t now) {
    try {
        if (s->failed) throw ShardError(SG_ERR_STATE, "a previous call failed part-way: restore a snapshot first");
        if (s->held) throw ShardError(SG_ERR_STATE, "release the polled matches first");
        collect(s, false);   // the batch matches so far come before this advance's timer matches
        try {
            s->each([&](uint32_t r) { return sg_advance_time(s->sh[r], now); });
            collect(s, true);
        } catch (...) {
            s->failed = true;   // some shards may have advanced (and emitted) while another failed
            throw;
        }
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

namespace {

// every shard drained (no pending match on any device): a shard whose seq map has grown past its threshold
// drops the entries below the smallest seq its live partials reference; the threshold follows the live span
void trim_maps(ShardEngine* s) {
    std::vector<char> due(s->N, 0);
    bool any = false;
    for (uint32_t r = 0; r < s->N; r++)
        if (s->gmap[r].size() >= s->gmap[r].trim_at) due[r] = any = 1;
    if (!any) return;
    std::vector<uint64_t> lo(s->N, 0);
    s->each([&](uint32_t r) -> int {
        if (due[r]) lo[r] = sg_internal_min_seq(s->sh[r]);
        return SG_OK;
    });
    for (uint32_t r = 0; r < s->N; r++) {
        if (!due[r]) continue;
        SeqMap& m = s->gmap[r];
        m.trim(std::min(lo[r], m.end()));
        // the next check once as many entries again (at least 2^20) were appended: amortised over the pushes
        m.trim_at = m.size() + std::max<uint64_t>(1u << 20, m.size());
        s->trims++;
    }
}

}  // namespace

int shd_poll(ShardEngine* s, uint32_t mem, sg_match_batch* out) {
    try {
        if ((mem & ~(uint32_t)SG_POLL_READY) != SG_MEM_HOST)
            throw ShardError(SG_ERR_INVALID, "a multi-device engine returns matches in host memory");
        if (s->failed) throw ShardError(SG_ERR_STATE, "a previous call failed part-way: restore a snapshot first");
        if (s->held) throw ShardError(SG_ERR_STATE, "release the polled matches first");
        try {
            collect(s, false);
        } catch (...) {
            s->failed = true;   // shards that released their matches before another failed lost them
            throw;
        }
        const double t0 = g_fan_prof ? fan_now() : 0.0;
        trim_maps(s);
        if (g_fan_prof) fprintf(stderr, "fan trim %.2f ms\n", (fan_now() - t0) * 1e3);
        std::swap(s->out, s->pend);   // (pend keeps the old output's buffers, emptied: no fresh pages per poll)
        ShardEngine::Out& e = s->pend;   // (its buffers keep their sizes: only n counts)
        e.n = 0;
        e.ns = 0;
        e.mc = 1;
        e.ni = 0;
        const ShardEngine::Out& o = s->out;
        out->n = o.n;
        out->n_slots = o.n ? o.ns : s->nslots;
        out->max_chain = o.n ? o.mc : s->mchain;
        out->trigger_seq = o.trig.data();
        out->key = o.key.data();
        out->ts = o.ts.data();
        out->slot_seq = o.slot.data();
        out->chain_len = o.len.data();
        out->mem = SG_MEM_HOST;
        out->reserved = 0;
        s->held = true;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

int shd_get_projection(ShardEngine* s, uint32_t mem, sg_projection* out) {
    if (!s->held) return sg_set_error(SG_ERR_STATE, "poll the matches first");
    if (!s->proj) return sg_set_error(SG_ERR_STATE, "no projection set");
    if (mem != SG_MEM_HOST) return sg_set_error(SG_ERR_INVALID, "a multi-device engine returns host memory");
    out->n = s->out.n;
    out->n_items = s->out.ni;
    out->mem = SG_MEM_HOST;
    out->value = s->out.pval.data();
    out->null = s->out.pnull.data();
    return SG_OK;
}

int shd_release(ShardEngine* s, sg_match_batch* m) {
    s->held = false;
    s->out.n = 0;   // (its buffers are kept for the next poll's collect)
    if (m) memset(m, 0, sizeof(*m));
    return SG_OK;
}

int shd_synchronize(ShardEngine* s) {
    try {
        s->each([&](uint32_t r) { return sg_synchronize(s->sh[r]); });
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

int shd_stats(ShardEngine* s, sg_stats* out) {
    try {
        std::vector<sg_stats> st(s->N);
        s->each([&](uint32_t r) { return sg_get_stats(s->sh[r], &st[r]); });
        memset(out, 0, sizeof(*out));
        uint64_t* o = (uint64_t*)out;
        for (const sg_stats& x : st)
            for (size_t i = 0; i < sizeof(sg_stats) / 8; i++) o[i] += ((const uint64_t*)&x)[i];
        // (events / batches: every event reaches exactly one shard, so the sums are the engine's; batches count
        // each shard's sub-batches)
        out->host_staged_bytes = s->staged_bytes;
        out->seq_map_entries = 0;
        for (const SeqMap& m : s->gmap) out->seq_map_entries += m.size();
        out->seq_map_trims = s->trims;
        out->host_syncs = s->host_syncs;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

int shd_reset_keys(ShardEngine* s, const uint32_t* keys, uint64_t n, uint32_t mem) {
    try {
        if (n == 0) return SG_OK;
        std::vector<uint32_t> h(n);
        if (mem == SG_MEM_HOST) {
            memcpy(h.data(), keys, n * 4);
        } else if (hipMemcpy(h.data(), keys, n * 4, hipMemcpyDeviceToHost) != hipSuccess) {
            throw ShardError(SG_ERR_DEVICE, "copying the key ids failed");
        }
        for (uint32_t k : h)
            if (k >= s->K) throw ShardError(SG_ERR_INVALID, "key id outside [0, n_keys)");
        std::vector<std::vector<uint32_t>> per(s->N);
        for (uint32_t k : h) per[k % s->N].push_back(k / s->N);
        s->each([&](uint32_t r) {
            return per[r].empty() ? SG_OK : sg_reset_keys(s->sh[r], per[r].data(), per[r].size(), SG_MEM_HOST);
        });
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

// image: magic u64, N u32, pad u32 | per shard: u64 image bytes, u64 map base, u64 map entries, image, map (u64 each)
int shd_snapshot(ShardEngine* s, void** buf, size_t* len) {
    try {
        if (s->failed) throw ShardError(SG_ERR_STATE, "a previous call failed part-way: the shards are out of step");
        if (s->pend.n || s->held) throw ShardError(SG_ERR_STATE, "poll the matches first");
        std::vector<void*> img(s->N, nullptr);
        std::vector<size_t> il(s->N, 0);
        s->each([&](uint32_t r) { return sg_snapshot(s->sh[r], &img[r], &il[r]); });
        size_t total = 16;
        for (uint32_t r = 0; r < s->N; r++) total += 24 + il[r] + 8 * s->gmap[r].size();
        uint8_t* o = (uint8_t*)malloc(total);
        if (!o) throw ShardError(SG_ERR_CAPACITY, "out of host memory");
        size_t off = 0;
        auto put = [&](const void* p, size_t b) { memcpy(o + off, p, b); off += b; };
        const uint32_t hdr[2] = {s->N, 0};
        put(&kMagic, 8);
        put(hdr, 8);
        for (uint32_t r = 0; r < s->N; r++) {
            const uint64_t a[3] = {il[r], s->gmap[r].base, s->gmap[r].size()};
            put(a, 24);
            put(img[r], il[r]);
            s->gmap[r].for_pieces([&](const uint64_t* q, uint64_t k) { put(q, 8 * k); });
            sg_free_buffer(img[r]);
        }
        *buf = o;
        *len = total;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

int shd_restore(ShardEngine* s, const void* buf, size_t len) {
    try {
        const uint8_t* p = (const uint8_t*)buf;
        size_t off = 0;
        auto need = [&](size_t b) {
            if (off + b > len) throw ShardError(SG_ERR_INVALID, "sharded snapshot truncated");
        };
        need(16);
        uint64_t magic;
        uint32_t hdr[2];
        memcpy(&magic, p, 8);
        memcpy(hdr, p + 8, 8);
        off = 16;
        if (magic != kMagic) throw ShardError(SG_ERR_INVALID, "not a snapshot of a multi-device engine");
        if (hdr[0] != s->N) throw ShardError(SG_ERR_INVALID, "snapshot of a different shard count");
        std::vector<const uint8_t*> img(s->N);
        std::vector<size_t> il(s->N);
        std::vector<SeqMap> maps(s->N);
        for (uint32_t r = 0; r < s->N; r++) {
            need(24);
            uint64_t a[3];
            memcpy(a, p + off, 24);
            off += 24;
            need(a[0]);
            img[r] = p + off;
            il[r] = a[0];
            off += a[0];
            if (a[2] > (len - off) / 8) throw ShardError(SG_ERR_INVALID, "sharded snapshot truncated");
            maps[r].reset(a[1]);
            maps[r].append((const uint64_t*)(const void*)(p + off), a[2]);
            maps[r].trim_at = a[2] + std::max<uint64_t>(1u << 20, a[2]);
            off += 8 * a[2];
        }
        s->each([&](uint32_t r) { return sg_restore(s->sh[r], img[r], il[r]); });
        s->gmap = std::move(maps);
        s->failed = false;
        s->pend = ShardEngine::Out();
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

// one document over every shard: keys and event seqs mapped to global ids, keys in id order
int shd_state_export(ShardEngine* s, void** buf, size_t* len) {
    try {
        if (s->failed) throw ShardError(SG_ERR_STATE, "a previous call failed part-way: the shards are out of step");
        if (s->pend.n || s->held) throw ShardError(SG_ERR_STATE, "poll the matches first");
        std::vector<SdDoc> docs(s->N);
        s->each([&](uint32_t r) -> int {
            void* b = nullptr;
            size_t l = 0;
            const int rc = sg_state_export(s->sh[r], &b, &l);
            if (rc != SG_OK) return rc;
            try {
                docs[r] = sd_read(b, l);
            } catch (...) {
                sg_free_buffer(b);
                throw;
            }
            sg_free_buffer(b);
            return SG_OK;
        });
        SdDoc out;
        out.n_procs = docs[0].n_procs;
        out.n_slots = docs[0].n_slots;
        out.desc = docs[0].desc;
        out.now = docs[0].now;
        out.last_event_ts = docs[0].last_event_ts;
        for (uint32_t r = 0; r < s->N; r++) {
            out.clock_flags = std::max(out.clock_flags, docs[r].clock_flags);
            for (SdKey& k : docs[r].keys) {
                if (s->N > 1) k.key = k.key * s->N + r;
                for (SdStream& ev : k.streams) ev.seq = s->map_seq(r, ev.seq);
                out.keys.push_back(std::move(k));
            }
        }
        std::stable_sort(out.keys.begin(), out.keys.end(), [](const SdKey& a, const SdKey& b) { return a.key < b.key; });
        const std::vector<uint8_t> bytes = sd_write(out);
        void* o = malloc(bytes.size());
        if (!o) throw ShardError(SG_ERR_CAPACITY, "out of host memory");
        memcpy(o, bytes.data(), bytes.size());
        *buf = o;
        *len = bytes.size();
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

// split a document by owner shard; its events get fresh local seqs mapped to their global ones
int shd_state_import(ShardEngine* s, const void* buf, size_t len) {
    try {
        SdDoc d = sd_read(buf, len);
        std::vector<SdDoc> parts(s->N);
        for (SdDoc& p : parts) {
            p.n_procs = d.n_procs;
            p.n_slots = d.n_slots;
            p.desc = d.desc;
            p.now = d.now;
            p.last_event_ts = d.last_event_ts;
            p.clock_flags = d.clock_flags;
        }
        for (SdKey& k : d.keys) {
            if (k.key >= s->K) throw ShardError(SG_ERR_INVALID, "state document key id outside [0, n_keys)");
            const uint32_t r = k.key % s->N;
            k.key /= s->N;
            parts[r].keys.push_back(std::move(k));
        }
        std::vector<std::vector<uint64_t>> add(s->N);
        for (uint32_t r = 0; r < s->N; r++) {
            std::vector<uint64_t> glob;
            for (const SdKey& k : parts[r].keys)
                for (const SdStream& ev : k.streams)
                    if (ev.seq < SG_BLANK_SEQ) glob.push_back(ev.seq);
            std::sort(glob.begin(), glob.end());
            glob.erase(std::unique(glob.begin(), glob.end()), glob.end());
            const uint64_t base = s->gmap[r].end();
            for (SdKey& k : parts[r].keys)
                for (SdStream& ev : k.streams)
                    if (ev.seq < SG_BLANK_SEQ)
                        ev.seq = base + (uint64_t)(std::lower_bound(glob.begin(), glob.end(), ev.seq) - glob.begin());
            add[r] = std::move(glob);
        }
        s->each([&](uint32_t r) -> int {
            const std::vector<uint8_t> bytes = sd_write(parts[r]);
            return sg_state_import(s->sh[r], bytes.data(), bytes.size());
        });
        for (uint32_t r = 0; r < s->N; r++) s->gmap[r].append(add[r].data(), add[r].size());
        s->failed = false;
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

// the fan-out reads a device batch first on its source device's split stream: the next split waits for the work
// queued on `stream` so far (one event per call, taken once by that split; no host wait)
int shd_wait_stream(ShardEngine* s, void* stream) {
    try {
        if (s->N == 1) return sg_wait_stream(s->sh[0], stream);   // (the one shard reads the caller's batch itself)
        int prev = 0, dev = 0;
        FAN_OK(hipGetDevice(&prev));
        if (stream) FAN_OK(hipStreamGetDevice((hipStream_t)stream, &dev));
        else dev = prev;
        // this stream's entry, else a free one of its device (events belong to a device), else a new one
        ShardEngine::Wait* w = nullptr;
        for (auto& x : s->waits)
            if (x.device == dev && x.stream == stream) w = &x;
        for (size_t i = 0; i < s->waits.size() && !w; i++)
            if (s->waits[i].device == dev && !s->waits[i].pending) w = &s->waits[i];
        int rc = SG_OK;
        if (hipSetDevice(dev) != hipSuccess) rc = SG_ERR_DEVICE;
        if (rc == SG_OK && !w) {
            hipEvent_t x = nullptr;
            if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) rc = SG_ERR_DEVICE;
            else {
                s->waits.push_back({stream, dev, x, false});
                w = &s->waits.back();
            }
        }
        if (rc == SG_OK && hipEventRecord(w->ev, (hipStream_t)stream) != hipSuccess) rc = SG_ERR_DEVICE;
        if (rc == SG_OK) {
            w->stream = stream;
            w->pending = true;
        }
        (void)hipSetDevice(prev);   // (the caller's current device is left as it was)
        if (rc != SG_OK) throw ShardError(rc, "sg_wait_stream: event on the caller's stream failed");
        return SG_OK;
    } catch (const std::exception& ex) {
        return fail_from(ex);
    }
}

sg_engine* shd_first(ShardEngine* s) { return s->sh[0]; }
uint32_t shd_count(const ShardEngine* s) { return s->N; }
