// sg_sharded.h — multi-device fan-out inside one sg_engine ("Multi-GPU fan-out is internal to one
// engine"; §8e).  sg_engine_create with sg_config.n_devices > 1 builds one engine per listed device and the
// public entry points forward here.  Host-only C++ (sg_sharded.cpp).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/siddhi_gpu.h"

struct ShardEngine;

// returns nullptr and sets the error (sg_last_error) on failure
ShardEngine* shd_create(const void* ir, size_t ir_len, const sg_config* cfg, int* rc);
void shd_destroy(ShardEngine* s);
int shd_push(ShardEngine* s, const sg_batch* b);
int shd_advance(ShardEngine* s, int64_t now);
int shd_set_projection(ShardEngine* s, const uint32_t* code, uint32_t code_words, const uint32_t* item_pc,
                       const uint32_t* item_len, const uint32_t* item_type, uint32_t n_items, const int32_t* part_attr,
                       uint32_t n_streams);
int shd_get_projection(ShardEngine* s, uint32_t mem, sg_projection* out);
int shd_poll(ShardEngine* s, uint32_t mem, sg_match_batch* out);
int shd_release(ShardEngine* s, sg_match_batch* m);
int shd_synchronize(ShardEngine* s);
int shd_stats(ShardEngine* s, sg_stats* out);
int shd_reset_keys(ShardEngine* s, const uint32_t* keys, uint64_t n, uint32_t mem);
int shd_snapshot(ShardEngine* s, void** buf, size_t* len);
int shd_restore(ShardEngine* s, const void* buf, size_t len);
int shd_state_export(ShardEngine* s, void** buf, size_t* len);
int shd_state_import(ShardEngine* s, const void* buf, size_t len);
int shd_wait_stream(ShardEngine* s, void* stream);
// the first shard's engine and the shard count (sg_engine_describe)
sg_engine* shd_first(ShardEngine* s);
uint32_t shd_count(const ShardEngine* s);

// sg_engine.hip: the error channel of the library
int sg_set_error(int code, const char* msg);
// sg_engine.hip, for the fan-out only: make a shard record, per advance, the keys that emitted timer matches in
// head order with their queue heads (false: the engine does not order timer matches by heads), and read them
bool sg_internal_keep_heads(sg_engine* e);
void sg_internal_heads(sg_engine* e, std::vector<uint32_t>& keys, std::vector<int64_t>& heads);
// sg_engine.hip, for the fan-out only: the smallest event seq a live partial references (UINT64_MAX: none), after
// every queued batch; an event recorded behind everything the engine has queued so far
uint64_t sg_internal_min_seq(sg_engine* e);
void sg_internal_record(sg_engine* e, hipEvent_t ev);

// shard_kernels.hip: split one device batch by owner shard (key % world) on the stream's device — stable, one
// destination-major copy of ts / each column / its nulls (col_bytes 1, 4 or 8), local keys in okey, the batch
// position of every output row in opos, per-shard counts in totals, err != 0 for a key outside [0, K) (an
// SG_KEY_NULL with null_keys is dropped).  Queues the work only.
int fan_split(uint64_t n, const uint32_t* key, uint32_t K, uint32_t world, bool null_keys, const int64_t* ts,
              const void* const* cols, const uint32_t* col_bytes, const uint8_t* const* nulls, uint32_t ncols,
              int64_t* out_ts, void* const* out_cols, uint8_t* const* out_nulls, uint32_t* opos, uint32_t* okey,
              uint32_t* totals, uint32_t* err, void* scratch, size_t scratch_len, hipStream_t s);
size_t fan_split_scratch_bytes(uint64_t n, uint32_t world);
