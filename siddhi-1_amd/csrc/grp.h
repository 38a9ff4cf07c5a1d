// grp.h — key grouping of a two-state micro-batch by key tile (grp_kernels.hip), the hand-written
// replacement of the two-pass rocPRIM payload sort for up to 2^20 keys:
//   k_grp_hist     per block of SGD_GRP_BLOCK_EVENTS events, the events of each key tile (SGD_BLOCK keys,
//                  one advance workgroup) -> mat[tile * nblk + block]
//   scan           exclusive scan of mat (tile-major): where block b's events of tile t start
//   k_grp_scatter  the payload of every event to its tile's range, stable (arrival order within a tile)
//   k_grp_tile     per tile, in LDS: stable split by key (the low 8 key bits), key-sorted payload out +
//                  seg_begin / seg_end of every key
// The result is what the rocPRIM path produces (key-sorted payload, per-key bounds), so every consumer
// (advance kernels, aggregators) is unchanged.  Events whose key is out of range (error word) or the
// dropped SG_KEY_NULL (SG_CFG_NULL_KEYS) are left out, as k_seg_bounds leaves them out.
#pragma once

#include <hip/hip_runtime.h>

#include "pack.h"

#define SGD_GRP_WAVES 16                                     // scatter / histogram block: 1024 lanes
#define SGD_GRP_WAVE_EVENTS 2048                             // events per wave of a block (32 per lane)
#define SGD_GRP_BLOCK_EVENTS (SGD_GRP_WAVES * SGD_GRP_WAVE_EVENTS)
#define SGD_GRP_MAX_TILES 4096                               // 2^20 keys (12-bit tile ids)
#define SGD_GRP_TILE_WAVES 8                                 // tile sort workgroup: 512 lanes
#define SGD_GRP_MAX_BATCH (1u << 24)                         // the tile sort carries key & 255 in idx bits 24..31

// Ablation knobs that deliberately produce wrong results (timing experiments) exist only in builds made
// with EXTRA=-DSG_EXPERIMENTS; in the shipped library SG_EXP(x) is the constant 0 and their code is gone.
#ifndef SG_EXP
#ifdef SG_EXPERIMENTS
#define SG_EXP(x) (x)
#else
#define SG_EXP(x) 0u
#endif
#endif

struct GrpArgs {
    uint32_t n;          // events in the batch
    uint32_t K;          // n_keys
    uint32_t n_tiles;    // ceil(K / SGD_BLOCK)
    uint32_t nblk;       // ceil(n / SGD_GRP_BLOCK_EVENTS)
    uint32_t drop_null;  // SG_CFG_NULL_KEYS
    uint32_t tile_lds;   // dynamic LDS of the tile sort (bytes); larger tiles are split from HBM
    uint32_t exp;        // grouping ablations (EXTRA=-DSG_EXPERIMENTS builds only: wrong results), 0 otherwise
    uint32_t pad;
    const uint32_t* keys;
    uint32_t* mat;       // [n_tiles * nblk + 1]
    uint32_t* mscan;     // [n_tiles * nblk + 1]
    void* tpay;          // tile-bucketed payload [n]
    void* pay;           // key-sorted payload [n]
    uint32_t* seg_begin; // [K]
    uint32_t* seg_end;   // [K]
    uint32_t* err;
    void* scan_tmp;
    size_t scan_tmp_bytes;
};

// whether a batch of this engine can take the tile grouping
inline bool sgd_group_tiles_ok(uint64_t K, uint64_t max_batch, uint32_t words) {
    return K >= 1 && K <= (uint64_t)SGD_GRP_MAX_TILES * SGD_BLOCK && max_batch <= SGD_GRP_MAX_BATCH && words >= 1 &&
           words <= 4;
}
size_t sgd_group_scan_bytes(uint64_t max_entries);
uint32_t sgd_group_tile_lds(uint64_t n, uint64_t K, uint32_t words);
// queue the grouping of one batch on `stream` (W = payload words 1..4)
hipError_t sgd_group_tiles(const GrpArgs& a, const PackSrc& src, int W, hipStream_t stream);

// ---- the bucket split (grp_kernels.hip): after ONE radix pass on the key bits above SGD_BK_BITS, each bucket
// of 2^SGD_BK_BITS keys is split by key in one workgroup (stable, LDS-staged output) and the per-key bounds are
// written — replacing the radix sort's last pass and k_seg_bounds ----
#define SGD_BK_BITS 10
struct BucketArgs {
    uint32_t n;           // events in the batch
    uint32_t K;           // n_keys
    uint32_t bits;        // key bits the radix pass sorted on (its end bit)
    uint32_t nb;          // buckets: ceil(K / 2^SGD_BK_BITS)
    uint32_t drop_null;   // SG_CFG_NULL_KEYS
    uint32_t stage_bytes; // (set by sgd_bucket_split)
    const uint32_t* skeys;// [n] keys as the radix pass left them
    const void* tpay;     // [n] payload as the radix pass left it
    void* pay;            // [n] key-sorted payload
    uint32_t* blo;        // [nb + 1] first element of each bucket
    uint32_t* seg_begin;  // [K]
    uint32_t* seg_end;    // [K]
    uint32_t* err;
};
// queue the bucket bounds + split of one batch on `stream` (W = payload words 1..4)
hipError_t sgd_bucket_split(const BucketArgs& a, int W, hipStream_t stream);
