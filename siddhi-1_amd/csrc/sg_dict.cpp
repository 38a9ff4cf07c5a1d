// sg_dict.cpp — partition-key dictionary of the C-ABI (include/siddhi_gpu.h).
//
// The reference keys its per-partition state by the String form of the partition attribute
// (ValuePartitionExecutor.execute, partition/executor/ValuePartitionExecutor.java:34-41) in a
// HashMap consulted per event (PartitionStreamReceiver.receive, partition/PartitionStreamReceiver.java:
// 175-260; state created on first sight, PartitionRuntimeImpl.java:346-402).  The device engine wants
// dense key ids instead (its per-key slabs are indexed by key_id), so ingest interns whole batches of
// key strings here: ids are handed out in first-seen order, null keys map to SG_KEY_NULL (the
// reference drops those events).
//
// Layout: every key's bytes are appended to one arena; an open-addressing table (linear probing,
// power-of-two size, load <= 1/2) holds id+1 per slot, and a per-id 64-bit hash makes probe misses a
// single compare.  A batch is interned all-or-nothing: on SG_ERR_CAPACITY the ids it added are
// rolled back by truncating the arena and rebuilding the table.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/siddhi_gpu.h"

int sg_set_error(int code, const char* msg);

struct sg_dict {
    uint32_t max_ids = 0;
    std::vector<uint8_t> arena;     // key bytes, id order
    std::vector<uint64_t> start;    // id -> arena offset; start[size] = arena end
    std::vector<uint64_t> hash;     // id -> hash
    std::vector<uint32_t> table;    // slot -> id + 1 (0 = empty)
    uint64_t mask = 0;

    uint32_t size() const { return (uint32_t)hash.size(); }
};

namespace {

inline uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// 8 bytes per step, length folded in (so "a" and "a\0" differ)
uint64_t hash_bytes(const uint8_t* p, uint64_t n) {
    uint64_t h = 0x9e3779b97f4a7c15ull ^ (n * 0x100000001b3ull);
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, p + i, 8);
        h = mix(h ^ w) + 0x9e3779b97f4a7c15ull;
    }
    uint64_t t = 0;
    for (uint64_t j = 0; i + j < n; j++) t |= (uint64_t)p[i + j] << (8 * j);
    return mix(h ^ t);
}

void rebuild(sg_dict* d, uint64_t want) {
    uint64_t cap = 16;
    while (cap < 2 * want) cap <<= 1;
    d->table.assign(cap, 0u);
    d->mask = cap - 1;
    for (uint32_t id = 0; id < d->size(); id++) {
        uint64_t s = d->hash[id] & d->mask;
        while (d->table[s]) s = (s + 1) & d->mask;
        d->table[s] = id + 1;
    }
}

// slot of the key, or of the empty slot where it would go
uint64_t probe(const sg_dict* d, const uint8_t* p, uint64_t n, uint64_t h) {
    uint64_t s = h & d->mask;
    for (;;) {
        const uint32_t v = d->table[s];
        if (!v) return s;
        const uint32_t id = v - 1;
        if (d->hash[id] == h && d->start[id + 1] - d->start[id] == n &&
            (n == 0 || std::memcmp(d->arena.data() + d->start[id], p, n) == 0))
            return s;
        s = (s + 1) & d->mask;
    }
}

int check_batch(const uint8_t* bytes, const uint64_t* offsets, uint64_t n) {
    if (n && !offsets) return sg_set_error(SG_ERR_INVALID, "null offsets");
    for (uint64_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i]) return sg_set_error(SG_ERR_INVALID, "offsets must not decrease");
    if (n && offsets[n] > offsets[0] && !bytes) return sg_set_error(SG_ERR_INVALID, "null bytes");
    return SG_OK;
}

}  // namespace

extern "C" {

int sg_dict_create(uint32_t max_ids, uint64_t capacity_hint, sg_dict** out) {
    if (!out) return sg_set_error(SG_ERR_INVALID, "null argument");
    if (max_ids == 0 || max_ids == SG_KEY_NULL) return sg_set_error(SG_ERR_INVALID, "max_ids out of range");
    sg_dict* d = new (std::nothrow) sg_dict();
    if (!d) return sg_set_error(SG_ERR_CAPACITY, "out of host memory");
    try {
        d->max_ids = max_ids;
        const uint64_t hint = capacity_hint < max_ids ? capacity_hint : max_ids;
        d->start.reserve(hint + 1);
        d->hash.reserve(hint);
        d->start.push_back(0);
        rebuild(d, hint);
    } catch (...) {
        delete d;
        return sg_set_error(SG_ERR_CAPACITY, "out of host memory");
    }
    *out = d;
    return SG_OK;
}

int sg_dict_intern(sg_dict* d, const uint8_t* bytes, const uint64_t* offsets, const uint8_t* valid, uint64_t n,
                   uint32_t* ids, uint64_t* n_new) {
    if (!d || (n && !ids)) return sg_set_error(SG_ERR_INVALID, "null argument");
    if (int rc = check_batch(bytes, offsets, n)) return rc;
    const uint32_t before = d->size();
    const uint64_t arena_before = d->arena.size();
    try {
        for (uint64_t i = 0; i < n; i++) {
            if (valid && !valid[i]) {
                ids[i] = SG_KEY_NULL;
                continue;
            }
            const uint8_t* p = bytes + offsets[i];
            const uint64_t len = offsets[i + 1] - offsets[i];
            const uint64_t h = hash_bytes(p, len);
            uint64_t s = probe(d, p, len, h);
            if (d->table[s]) {
                ids[i] = d->table[s] - 1;
                continue;
            }
            if (d->size() >= d->max_ids) {
                // all-or-nothing: forget this batch's new keys
                d->hash.resize(before);
                d->start.resize(before + 1);
                d->arena.resize(arena_before);
                rebuild(d, d->size());
                return sg_set_error(SG_ERR_CAPACITY, "more distinct partition keys than max_ids");
            }
            const uint32_t id = d->size();
            d->arena.insert(d->arena.end(), p, p + len);
            d->start.push_back(d->arena.size());
            d->hash.push_back(h);
            if (2 * (uint64_t)d->size() > d->mask + 1) {
                rebuild(d, d->size());
            } else {
                d->table[s] = id + 1;
            }
            ids[i] = id;
        }
    } catch (const std::bad_alloc&) {
        d->hash.resize(before);
        d->start.resize(before + 1);
        d->arena.resize(arena_before);
        rebuild(d, d->size());
        return sg_set_error(SG_ERR_CAPACITY, "out of host memory");
    }
    if (n_new) *n_new = d->size() - before;
    return SG_OK;
}

int sg_dict_lookup(const sg_dict* d, const uint8_t* bytes, const uint64_t* offsets, const uint8_t* valid,
                   uint64_t n, uint32_t* ids) {
    if (!d || (n && !ids)) return sg_set_error(SG_ERR_INVALID, "null argument");
    if (int rc = check_batch(bytes, offsets, n)) return rc;
    for (uint64_t i = 0; i < n; i++) {
        if (valid && !valid[i]) {
            ids[i] = SG_KEY_NULL;
            continue;
        }
        const uint8_t* p = bytes + offsets[i];
        const uint64_t len = offsets[i + 1] - offsets[i];
        const uint32_t v = d->table[probe(d, p, len, hash_bytes(p, len))];
        ids[i] = v ? v - 1 : SG_KEY_NULL;
    }
    return SG_OK;
}

uint32_t sg_dict_size(const sg_dict* d) { return d ? d->size() : 0u; }

int sg_dict_key(const sg_dict* d, uint32_t id, const uint8_t** ptr, uint64_t* len) {
    if (!d || !ptr || !len) return sg_set_error(SG_ERR_INVALID, "null argument");
    if (id >= d->size()) return sg_set_error(SG_ERR_INVALID, "key id not in the dictionary");
    *ptr = d->arena.data() + d->start[id];
    *len = d->start[id + 1] - d->start[id];
    return SG_OK;
}

int sg_dict_clear(sg_dict* d) {
    if (!d) return sg_set_error(SG_ERR_INVALID, "null argument");
    d->arena.clear();
    d->hash.clear();
    d->start.assign(1, 0);
    std::fill(d->table.begin(), d->table.end(), 0u);
    return SG_OK;
}

void sg_dict_destroy(sg_dict* d) { delete d; }

}  // extern "C"
