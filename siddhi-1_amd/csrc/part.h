// part.h — hand-written stable partitioning by key digit for MI355X (part_kernels.hip): the key-run grouping
// of every micro-batch and the engine's other sorts, without a library sort.
//
// Replaces the key-run grouping of PartitionStreamReceiver.receive(Event[])
// (partition/PartitionStreamReceiver.java:175-260: each partition key's events of a batch handed to its state
// in arrival order) and the per-key state lookup (util/snapshot/state/PartitionStateHolder.java:43-80).
//
// One pass = a STABLE partition of n elements by one digit (<= 8 bits) of their key, LSD passes make a sort:
//   k_part_hist     per chunk of 4096 events (XCD-aware chunk order), its events of each digit -> mat
//   k_part_scan     per digit, the exclusive scan of its row of mat over the chunks, and the digit's total
//   k_part_scatter  per chunk: each wave ranks its events among their digit peers in arrival order (wave
//                   ballots, no atomics); the elements are placed digit-sorted in LDS and written out as
//                   runs (~16-64 consecutive elements of one digit per chunk: coalesced stores)
// Uses built on it:
//   - the two-state C2 path (sgd_group_tiles_fused): two 6-bit passes on the key tile (key >> 8: the 256 keys
//     of one advance workgroup), elements tagged with key & 255 in the position's top byte; the split by key
//     happens inside the advance kernel's LDS staging (p2_jit.hip), so a key-sorted payload never goes through
//     HBM;
//   - every other grouping (sgd_group_sorted): LSD passes of <= 8 bits (one pass up to 256 keys), the keys
//     carried along, then per-key bounds — the key-sorted payload (or batch positions) and seg_begin / seg_end
//     every consumer reads;
//   - key / value sorts of the timer paths (sgd_sort_pairs): LSD passes, ascending or descending.
// Elements whose key is out of range (the error word) or the dropped SG_KEY_NULL (SG_CFG_NULL_KEYS) are left
// out; the valid count stays on the device (a later pass reads it).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pack.h"

#define SGD_PT_THREADS 512                 // hist / scatter block: 8 waves
#define SGD_PT_WAVES (SGD_PT_THREADS / 64)
#define SGD_PT_MAX_BITS 8                  // digit bits of one pass (256 digits)
#define SGD_PT_MAX_DIG (1u << SGD_PT_MAX_BITS)
#define SGD_PT_MIN_CE 2048u                // events of the smallest chunk (wide elements)
#define SGD_PT_TILE_BITS 8                 // the fused C2 grouping: one tile per advance workgroup (SGD_BLOCK keys)
#define SGD_PT_MAX_TILES 4096u
#define SGD_PT_FUSED_MAX_BATCH (1u << 24)  // the tile tag rides in position bits 24..31

// device scratch of the passes (sgd_part_scratch_bytes for an upper bound of n)
struct PartScratch {
    uint32_t* mat;       // [SGD_PT_MAX_DIG * nblk]
    uint32_t* tot;       // [SGD_PT_MAX_DIG]
    uint32_t* lo[2];     // [SGD_PT_MAX_DIG + 1] digit starts of a pass (+ the valid count), two alternating
    void* keys[2];       // [n] keys (u32 / u64) or u16 tile codes carried through the passes
    void* el[2];         // [n * 6 words] elements between passes
};
size_t sgd_part_scratch_bytes(uint64_t max_n);
// carve a scratch block of sgd_part_scratch_bytes(max_n) bytes
PartScratch sgd_part_scratch(void* base, uint64_t max_n);

// the grouping of one batch of n events by key id (keys < K; SG_KEY_NULL dropped when drop_null, other ids
// outside [0, K) dropped and reported in *err)
struct GroupArgs {
    uint32_t n, K;
    uint32_t drop_null;
    uint32_t W;              // payload words 1..4 (Pay<W> elements gathered by PackFn<W>), 0: batch positions only
    const uint32_t* keys;    // [n] arrival order
    PackSrc src;             // (W >= 1)
    void* out;               // key-sorted Pay<W>[n], or uint32_t[n] positions (W == 0)
    uint32_t* seg_begin;     // [K]
    uint32_t* seg_end;       // [K]
    uint32_t* err;
    PartScratch s;
    uint32_t tile_bits;      // sgd_group_tiles_fused: keys per tile = 2^tile_bits (0: SGD_PT_TILE_BITS)
    uint32_t pad;
};
hipError_t sgd_group_sorted(const GroupArgs& a, hipStream_t stream);

// the fused C2 grouping: out = Pay<W>[n] grouped by key tile (key >> 8), arrival order within a tile, idx
// bits 24..31 = key & 255; tile_lo[t] = first element of tile t, tile_lo[n_tiles] = the valid count
// (K <= 2^20, n <= 2^24)
hipError_t sgd_group_tiles_fused(const GroupArgs& a, uint32_t* tile_lo, hipStream_t stream);
inline bool sgd_fused_ok(uint64_t K, uint64_t max_batch, uint32_t W, uint32_t tile_bits = SGD_PT_TILE_BITS) {
    // (tile codes travel as u16: at most 65,535 tiles; SGD_PT_MAX_TILES bounds the C2 advance grid)
    const uint64_t max_tiles = tile_bits == SGD_PT_TILE_BITS ? SGD_PT_MAX_TILES : 65535u;
    return K >= 1 && K <= (max_tiles << tile_bits) && max_batch <= SGD_PT_FUSED_MAX_BATCH &&
           W >= 1 && W <= 4;
}

// stable LSD sort of (key, value) pairs on key bits [0, bits): keys u32 (key64 = 0) or u64; descending when
// desc.  The result is in keys_out / vals_out (distinct from the inputs).
hipError_t sgd_sort_pairs(const void* keys_in, void* keys_out, const uint32_t* vals_in, uint32_t* vals_out, uint32_t n,
                          uint32_t bits, bool key64, bool desc, const PartScratch& s, hipStream_t stream);
