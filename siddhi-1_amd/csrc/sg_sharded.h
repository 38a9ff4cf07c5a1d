// sg_sharded.h — multi-device fan-out inside one sg_engine ("Multi-GPU fan-out is internal to one
// engine"; §8e).  sg_engine_create with sg_config.n_devices > 1 builds one engine per listed device and the
// public entry points forward here.  Host-only C++ (sg_sharded.cpp).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

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

// sg_engine.hip: the error channel of the library
int sg_set_error(int code, const char* msg);
// sg_engine.hip, for the fan-out only: make a shard record, per advance, the keys that emitted timer matches in
// head order with their queue heads (false: the engine does not order timer matches by heads), and read them
bool sg_internal_keep_heads(sg_engine* e);
void sg_internal_heads(sg_engine* e, std::vector<uint32_t>& keys, std::vector<int64_t>& heads);
