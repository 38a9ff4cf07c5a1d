// gen_host.h — host API of the general NFA engine (gen_host.hip), used by the C-ABI (sg_engine.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/siddhi_gpu.h"

struct GenEngine;
struct GenProgram;

// throws std::runtime_error (unsupported shape / allocation failure)
GenProgram* gen_build_program(const uint32_t* ir, size_t nwords, uint32_t partial_capacity);
GenEngine* gen_create(const uint32_t* ir, size_t nwords, const sg_config& cfg, hipStream_t stream);
void gen_destroy(GenEngine* e);
int gen_push(GenEngine* e, const sg_batch* b, std::string& msg);
int gen_advance(GenEngine* e, int64_t now, std::string& msg);
int gen_poll(GenEngine* e, uint32_t mem, sg_match_batch* out, std::string& msg);
// on-device projection of the select list (sg_set_projection / sg_get_projection)
int gen_set_projection(GenEngine* e, const uint32_t* code, uint32_t words, const uint32_t* pc, const uint32_t* len,
                       const uint32_t* types, uint32_t n, std::string& msg);
int gen_get_projection(GenEngine* e, uint32_t mem, sg_projection* out, std::string& msg);
void gen_release(GenEngine* e);
void gen_stats(GenEngine* e, sg_stats* out);
void gen_synchronize(GenEngine* e);
std::string gen_describe(const GenEngine* e);
// the smallest event seq a live partial references (UINT64_MAX: none); synchronises the engine's stream
uint64_t gen_min_seq(GenEngine* e);
// the multi-device fan-out (sg_sharded.cpp) merges the shards' timer matches in the single engine's order:
// with keep = true every advance records, for each key that emitted, its queue head at that advance (the
// listener's TreeMultimap order, Scheduler.java:78-99), in the key order the engine emitted them.
// false = the engine does not order timer matches by key heads (not partitioned playback with one listener)
bool gen_keep_timer_heads(GenEngine* e, bool keep);
void gen_timer_heads(const GenEngine* e, std::vector<uint32_t>& keys, std::vector<int64_t>& heads);
// device NFA state as a flat image (snapshot/restore, sg_engine.hip): the per-key state blocks plus the
// clock fields.  gen_state_words = words of the block image (blockWords * K).
struct GenClock { int64_t now, last_event_ts; uint32_t advanced, pad; };
uint64_t gen_state_words(const GenEngine* e);
// partition purge: the listed keys' state blocks back to the never-seen (all-zero) state; keys is a
// device array of n ids already range-checked by the caller
int gen_reset_keys(GenEngine* e, const uint32_t* keys, uint32_t n, std::string& msg);
int gen_snapshot(GenEngine* e, uint32_t* words, GenClock* clk, std::string& msg);
int gen_restore(GenEngine* e, const uint32_t* words, const GenClock& clk, std::string& msg);
// the state in the reference's per-state-processor form (state_doc.h)
struct SdDoc;
int gen_state_export(GenEngine* e, SdDoc& d, std::string& msg);
int gen_state_import(GenEngine* e, const SdDoc& d, std::string& msg);
