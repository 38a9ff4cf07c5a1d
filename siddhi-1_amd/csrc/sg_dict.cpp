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
//
// Partition purge (PartitionRuntimeImpl.java:368-401 drops idle keys from its maps) removes keys
// (sg_dict_remove): their ids go to a free list and are handed out again, smallest first, to the next
// new keys, so the live ids stay below max_ids (= the engine's n_keys) under key churn; the removed
// keys' bytes are dropped from the arena once they are most of it.  sg_dict_put binds a key to a given
// id (restoring a snapshot's key map).
#include <algorithm>
#include <cstdint>
#include <functional>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/siddhi_gpu.h"

int sg_set_error(int code, const char* msg);

struct sg_dict {
    uint32_t max_ids = 0;
    std::vector<uint8_t> arena;     // key bytes (a recycled id's new key is appended at the end)
    std::vector<uint64_t> off;      // id -> arena offset
    std::vector<uint64_t> len;      // id -> key length
    std::vector<uint64_t> hash;     // id -> hash
    std::vector<uint8_t> freed;     // id -> 1 once removed (until interned again)
    std::vector<uint32_t> free_ids; // removed ids, descending (back = smallest: reused first)
    uint64_t garbage = 0;           // arena bytes of removed keys
    std::vector<uint32_t> table;    // slot -> id + 1 (0 = empty)
    uint64_t mask = 0;

    uint32_t size() const { return (uint32_t)hash.size(); }  // id bound: ids are < size()
    uint32_t live() const { return size() - (uint32_t)free_ids.size(); }
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
        if (d->freed[id]) continue;
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
        if (d->hash[id] == h && d->len[id] == n && (n == 0 || std::memcmp(d->arena.data() + d->off[id], p, n) == 0))
            return s;
        s = (s + 1) & d->mask;
    }
}

// linear probing delete: close the gap by moving back the entries of the cluster whose home slot is
// not cyclically in (s, j]
void erase_slot(sg_dict* d, uint64_t s) {
    d->table[s] = 0;
    uint64_t j = s;
    for (;;) {
        j = (j + 1) & d->mask;
        const uint32_t v = d->table[j];
        if (!v) return;
        const uint64_t home = d->hash[v - 1] & d->mask;
        const bool stays = (s <= j) ? (home > s && home <= j) : (home > s || home <= j);
        if (!stays) {
            d->table[s] = v;
            d->table[j] = 0;
            s = j;
        }
    }
}

// drop removed keys' bytes from the arena once they are most of it
void compact(sg_dict* d) {
    if (d->garbage < (1u << 20) || 2 * d->garbage < d->arena.size()) return;
    std::vector<uint8_t> a;
    a.reserve(d->arena.size() - d->garbage);
    for (uint32_t id = 0; id < d->size(); id++) {
        if (d->freed[id]) { d->off[id] = 0; d->len[id] = 0; continue; }
        const uint64_t o = a.size();
        a.insert(a.end(), d->arena.begin() + d->off[id], d->arena.begin() + d->off[id] + d->len[id]);
        d->off[id] = o;
    }
    d->arena.swap(a);
    d->garbage = 0;
}

void reset(sg_dict* d) {
    d->arena.clear();
    d->off.clear();
    d->len.clear();
    d->hash.clear();
    d->freed.clear();
    d->free_ids.clear();
    d->garbage = 0;
}

int check_batch(const uint8_t* bytes, const uint64_t* offsets, uint64_t n) {
    if (n && !offsets) return sg_set_error(SG_ERR_INVALID, "null offsets");
    for (uint64_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i]) return sg_set_error(SG_ERR_INVALID, "offsets must not decrease");
    if (n && offsets[n] > offsets[0] && !bytes) return sg_set_error(SG_ERR_INVALID, "null bytes");
    return SG_OK;
}

// bind key bytes to id (fresh: id == size(); recycled: id taken off the free list by the caller)
void bind(sg_dict* d, uint32_t id, const uint8_t* p, uint64_t n, uint64_t h) {
    const uint64_t o = d->arena.size();
    d->arena.insert(d->arena.end(), p, p + n);
    if (id == d->size()) {
        d->off.push_back(o);
        d->len.push_back(n);
        d->hash.push_back(h);
        d->freed.push_back(0);
    } else {
        d->off[id] = o;
        d->len[id] = n;
        d->hash[id] = h;
        d->freed[id] = 0;  // (the removed key's bytes stay counted as garbage until compaction)
    }
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
        d->off.reserve(hint);
        d->len.reserve(hint);
        d->hash.reserve(hint);
        d->freed.reserve(hint);
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
    std::vector<uint32_t> reused;  // ids this batch took off the free list (rolled back on failure)
    uint64_t added = 0;
    auto rollback = [&]() {
        for (uint32_t id : reused) {
            d->freed[id] = 1;
            d->free_ids.push_back(id);
        }
        std::sort(d->free_ids.begin(), d->free_ids.end(), std::greater<uint32_t>());
        d->off.resize(before);
        d->len.resize(before);
        d->hash.resize(before);
        d->freed.resize(before);
        d->arena.resize(arena_before);
        rebuild(d, d->live());
    };
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
            uint32_t id;
            if (!d->free_ids.empty()) {  // a purged key's id is reused, smallest first
                id = d->free_ids.back();
                d->free_ids.pop_back();
                reused.push_back(id);
            } else {
                if (d->size() >= d->max_ids) {
                    rollback();  // all-or-nothing: forget this batch's new keys
                    return sg_set_error(SG_ERR_CAPACITY, "more distinct partition keys than max_ids");
                }
                id = d->size();
            }
            bind(d, id, p, len, h);
            added++;
            if (2 * (uint64_t)d->live() > d->mask + 1) {
                rebuild(d, d->live());
            } else {
                d->table[s] = id + 1;
            }
            ids[i] = id;
        }
    } catch (const std::bad_alloc&) {
        rollback();
        return sg_set_error(SG_ERR_CAPACITY, "out of host memory");
    }
    if (n_new) *n_new = added;
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

int sg_dict_remove(sg_dict* d, const uint32_t* ids, uint64_t n) {
    if (!d || (n && !ids)) return sg_set_error(SG_ERR_INVALID, "null argument");
    std::vector<uint32_t> seen;
    seen.reserve(n);
    for (uint64_t i = 0; i < n; i++) {
        if (ids[i] >= d->size() || d->freed[ids[i]]) return sg_set_error(SG_ERR_INVALID, "key id not in use");
        seen.push_back(ids[i]);
    }
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end())
        return sg_set_error(SG_ERR_INVALID, "key id listed twice");
    for (uint32_t id : seen) {
        const uint64_t s = probe(d, d->arena.data() + d->off[id], d->len[id], d->hash[id]);
        if (d->table[s] == id + 1) erase_slot(d, s);
        d->freed[id] = 1;
        d->garbage += d->len[id];
        d->free_ids.push_back(id);
    }
    std::sort(d->free_ids.begin(), d->free_ids.end(), std::greater<uint32_t>());
    compact(d);
    return SG_OK;
}

int sg_dict_put(sg_dict* d, uint32_t id, const uint8_t* bytes, uint64_t len) {
    if (!d || (len && !bytes)) return sg_set_error(SG_ERR_INVALID, "null argument");
    if (id >= d->max_ids) return sg_set_error(SG_ERR_CAPACITY, "key id not below max_ids");
    if (id < d->size() && !d->freed[id]) return sg_set_error(SG_ERR_INVALID, "key id already in use");
    const uint64_t h = hash_bytes(bytes, len);
    const uint64_t s = probe(d, bytes, len, h);
    if (d->table[s]) return sg_set_error(SG_ERR_INVALID, "key already has an id");
    try {
        while (d->size() < id) {  // ids skipped over are free
            const uint32_t f = d->size();
            bind(d, f, nullptr, 0, 0);
            d->freed[f] = 1;
            d->free_ids.push_back(f);
        }
        if (id < d->size()) d->free_ids.erase(std::find(d->free_ids.begin(), d->free_ids.end(), id));
        std::sort(d->free_ids.begin(), d->free_ids.end(), std::greater<uint32_t>());
        bind(d, id, bytes, len, h);
        rebuild(d, d->live());
    } catch (const std::bad_alloc&) {
        return sg_set_error(SG_ERR_CAPACITY, "out of host memory");
    }
    return SG_OK;
}

uint32_t sg_dict_size(const sg_dict* d) { return d ? d->size() : 0u; }

int sg_dict_key(const sg_dict* d, uint32_t id, const uint8_t** ptr, uint64_t* len) {
    if (!d || !ptr || !len) return sg_set_error(SG_ERR_INVALID, "null argument");
    if (id >= d->size() || d->freed[id]) return sg_set_error(SG_ERR_INVALID, "key id not in the dictionary");
    *ptr = d->arena.data() + d->off[id];
    *len = d->len[id];
    return SG_OK;
}

int sg_dict_clear(sg_dict* d) {
    if (!d) return sg_set_error(SG_ERR_INVALID, "null argument");
    reset(d);
    std::fill(d->table.begin(), d->table.end(), 0u);
    return SG_OK;
}

void sg_dict_destroy(sg_dict* d) { delete d; }

}  // extern "C"
