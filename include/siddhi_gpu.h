/*
 * siddhi_gpu.h — C-ABI of the MI355X pattern/sequence engine.
 *
 * This is the drop-in seam that replaces the reference's per-key NFA advance:
 *
 *   ingest seam   StreamJunction.Receiver.receive(...)
 *                 /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/stream/StreamJunction.java:469-482
 *                 implemented today by PartitionStreamReceiver (partition/PartitionStreamReceiver.java:81-283)
 *                 and the Pattern/Sequence*ProcessStreamReceiver family
 *                 (query/input/MultiProcessStreamReceiver.java:93-241, SingleProcessStreamReceiver.java:55-78)
 *                 -> sg_push_batch()
 *   output seam   QuerySelector.process(ComplexEventChunk<StateEvent>)
 *                 (query/selector/QuerySelector.java:77-100), fed one StateEvent per match
 *                 by StateMultiProcessStreamReceiver.processAndClear (StateMultiProcessStreamReceiver.java:47-68)
 *                 -> sg_poll_matches(): one record per emitted StateEvent, slots given as event seqs
 *   compile seam  StateInputStreamParser.parseInputStream (util/parser/StateInputStreamParser.java:76-146)
 *                 -> sg_engine_create() with the IR of siddhi_gpu_ir.h
 *   playback clock  Scheduler/TimestampGenerator (util/Scheduler.java:65-105) -> sg_advance_time()
 *   persistence   StreamPreStateProcessor.StreamPreState.snapshot/restore (StreamPreStateProcessor.java:450-469)
 *                 -> sg_snapshot()/sg_restore()
 *
 * Threading mirrors the reference's single writer per query (QueryParser.java:169-213 lock,
 * MultiProcessStreamReceiver.java:97 synchronized): one host thread per engine; calls are not re-entrant.
 * Errors: every call returns SG_OK (0) or a negative SG_ERR_*; sg_last_error() gives the message of the
 * calling thread's last failure.  The Java shim maps them to SiddhiAppRuntimeException and routes them
 * through StreamJunction.handleError (StreamJunction.java:372-464).
 */
#ifndef SIDDHI_GPU_H
#define SIDDHI_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_ABI_VERSION 1

#define SG_OK 0
#define SG_ERR_INVALID (-1)     /* bad argument / malformed IR */
#define SG_ERR_UNSUPPORTED (-2) /* query shape not supported by this engine */
#define SG_ERR_DEVICE (-3)      /* HIP runtime failure */
#define SG_ERR_CAPACITY (-4)    /* per-key partial or match buffer capacity exceeded */
#define SG_ERR_STATE (-5)       /* call out of order (e.g. push while matches are held) */

#define SG_MEM_HOST 0u   /* pointers are host memory */
#define SG_MEM_DEVICE 1u /* pointers are device (HBM) memory of the engine's device */
/* or-ed into sg_poll_matches' mem: return the matches of the batches whose processing is complete,
 * without waiting for the batches still in flight (they come with a later poll, in order) */
#define SG_POLL_READY 0x10u

#define SG_NULL_SEQ UINT64_MAX
#define SG_KEY_NULL 0xFFFFFFFFu /* partition key id of an event without a key (null key: dropped) */
/* slot event created by an absent state when it fires (StreamEventFactory.newInstance():
 * no attributes, ts -1; AbsentLogicalPreStateProcessor.java:153-166) */
#define SG_BLANK_SEQ (UINT64_MAX - 1)
/* trigger_seq of a match emitted by a timer (absent state fired by sg_advance_time, delivered at once:
 * AbsentStreamPreStateProcessor.sendEvent, AbsentStreamPreStateProcessor.java:229-246) */
#define SG_TIMER_SEQ UINT64_MAX

/* engine configuration flags */
#define SG_CFG_NO_ORDER 1u /* deliver matches per-key ordered only (skip the global trigger-seq order) */
#define SG_CFG_TIMING 2u   /* record HIP events around every kernel stage (sg_stats *_ns fields) */
/* batches may carry key == SG_KEY_NULL: such events are dropped, as PartitionStreamReceiver drops events
 * whose partition key is null (PartitionStreamReceiver.java:175-205).  Used for fixed-size device batches
 * with padding (the multi-GPU reshard).  Without the flag a SG_KEY_NULL key is out of range. */
#define SG_CFG_NULL_KEYS 4u
/* sg_push_batch with host (SG_MEM_HOST) pointers returns once its copies are queued; the caller keeps
 * the host buffers unchanged until a blocking sg_poll_matches (without SG_POLL_READY), sg_synchronize,
 * or a ready poll that returns that batch's matches (the reference's @async junction hands events over
 * the same way).  Without the flag a host push returns after its copies. */
#define SG_CFG_ASYNC_HOST 8u

typedef struct sg_engine sg_engine;

typedef struct sg_config {
    uint32_t struct_size;      /* sizeof(sg_config) */
    int32_t device;            /* HIP device ordinal */
    uint32_t n_keys;           /* partition key ids are dense in [0, n_keys); 1 when unpartitioned */
    uint32_t max_batch;        /* max events in one sg_push_batch (a multi-device engine: of the whole batch,
                                  host or device, before its split) */
    uint32_t partial_capacity; /* max live partial matches per key */
    uint32_t flags;            /* SG_CFG_* */
    uint64_t match_capacity;   /* max matches held between two polls */
    /* Multi-GPU fan-out inside the engine (replaces the per-key routing of
     * PartitionStreamReceiver.java:262-272 across processes): n_devices > 1 HIP devices listed in devices[]
     * (device above is then ignored).  A partitioned query's keys are sharded key % n_devices (local id
     * key / n_devices) over one engine per device; every entry point keeps its meaning for the whole key
     * range, polls merge the shards' matches into the single engine's order and return host memory
     * (sg_sharded.cpp).  0 or 1: one device.  A caller built against the header without these two fields
     * passes the smaller struct_size and gets one device.  A device batch is split on the device it lives on
     * and reaches other devices by peer copies (never staged to host).  A call that fails after some shards
     * took their part (a push one shard refused, an advance or poll one shard failed) leaves the shards out of
     * step: every later push / advance / poll then fails with SG_ERR_STATE until sg_restore or
     * sg_state_import. */
    uint32_t n_devices;
    uint32_t reserved;
    const int32_t* devices;
} sg_config;

/* One micro-batch of events of ONE input stream, in arrival order (columnar / SoA). */
typedef struct sg_batch {
    uint32_t struct_size;       /* sizeof(sg_batch) */
    uint32_t stream;            /* stream index in the IR stream table */
    uint64_t n;                 /* number of events */
    uint64_t seq_base;          /* arrival sequence number of event 0 (event i has seq_base + i) */
    const uint32_t* key;        /* [n] partition key ids; NULL when the query is not partitioned */
    const int64_t* ts;          /* [n] event timestamps in ms */
    const void* const* cols;    /* [n_cols] attribute columns, typed per the IR stream table */
    const uint8_t* const* nulls;/* [n_cols] per-event null flags (1 = null) or NULL entries */
    uint32_t n_cols;
    uint32_t mem;               /* SG_MEM_HOST or SG_MEM_DEVICE for all pointers above */
} sg_batch;

/* Matches emitted since the previous poll.  Library-owned until sg_release_matches().
 * Order: ascending trigger_seq, then emission order (the reference's callback order for
 * per-event sends, MultiProcessStreamReceiver.java:119-121); per key the order is always the
 * reference's per-partition order. */
typedef struct sg_match_batch {
    uint64_t n;
    uint32_t n_slots;              /* state stream events per match (IR slot count) */
    uint32_t max_chain;            /* max events per slot (count states chain several) */
    const uint64_t* trigger_seq;   /* [n] seq of the event whose processing emitted the match */
    const uint32_t* key;           /* [n] partition key id */
    const int64_t* ts;             /* [n] StateEvent timestamp at emission */
    const uint64_t* slot_seq;      /* [n][n_slots][max_chain] event seqs, SG_NULL_SEQ = none */
    const uint32_t* chain_len;     /* [n][n_slots] events in each slot */
    uint32_t mem;                  /* where the arrays live */
    uint32_t reserved;
} sg_match_batch;

/* On-device projection: QuerySelector.processNoGroupBy (QuerySelector.java:162-206)
 * evaluates the select list on each emitted StateEvent; for a select list of plain expressions (no
 * aggregate, group by or having) the engine does it on the device when the match is emitted, with the
 * Java numerics of the filters (float32 without FMA contraction, null propagation, /0 -> null).
 * code: expression bytecode (siddhi_gpu_ir.h; SG_OP_VAR b = slot, w1 = attribute, w2 = chain index with
 * the selector's default index 0); item i is code[item_pc[i], item_pc[i] + item_len[i]) of result type
 * item_type[i] (SG_T_*).  part_attr[s]: the partition attribute of stream s, or -1 (every event of a match
 * has the match's key, so a slot's partition attribute may be read from the trigger event).  Call once,
 * before the first push; fails with SG_ERR_UNSUPPORTED for items the device cannot evaluate. */
int sg_set_projection(sg_engine* e, const uint32_t* code, uint32_t code_words, const uint32_t* item_pc,
                      const uint32_t* item_len, const uint32_t* item_type, uint32_t n_items, const int32_t* part_attr,
                      uint32_t n_streams);
/* The projected select list of the polled matches (valid from sg_poll_matches to sg_release_matches):
 * value[i * n + m] are item i's bits for match m (int / float / string id / bool in the low 32 bits;
 * long / double 64), null[i * n + m] = 1 when the value is null. */
typedef struct sg_projection {
    uint64_t n;
    uint32_t n_items;
    uint32_t mem;
    const uint64_t* value;
    const uint8_t* null;
} sg_projection;
int sg_get_projection(sg_engine* e, uint32_t mem, sg_projection* out);

/* Exact work counters (the algorithmic-byte model of DESIGN.md is computed from these). */
typedef struct sg_stats {
    uint64_t events;            /* events pushed */
    uint64_t batches;
    uint64_t partials_scanned;  /* partial matches visited by an event */
    uint64_t partials_created;  /* partial matches created */
    uint64_t partials_live;     /* partial matches alive after the last batch */
    uint64_t matches;           /* matches emitted */
    uint64_t keys_touched;      /* sum over batches of keys with >= 1 event */
    uint64_t live_at_batch_start; /* sum over batches of the live partials of the touched keys */
    uint64_t group_ns;          /* SG_CFG_TIMING: device time of key grouping (sort + bounds) */
    uint64_t advance_ns;        /* SG_CFG_TIMING: device time of the NFA advance kernel */
    uint64_t order_ns;          /* SG_CFG_TIMING: device time of match ordering in polls */
    uint64_t advance_launches;  /* NFA advance kernel launches */
    uint64_t window_spills;     /* keys whose live partials outgrew the register window (moved to HBM) */
    uint64_t advance_hbm_ns;    /* SG_CFG_TIMING: part of advance_ns spent in the HBM pass (waves and
                                   keys the LDS-staged pass left to it) */
    uint64_t host_staged_bytes; /* multi-device engine: batch bytes it copied to host memory (device
                                   batches are split on the device: 0) */
    uint64_t seq_map_entries;   /* multi-device engine: local -> global seq map entries it holds (trimmed
                                   below the oldest seq a live partial references after each poll) */
    uint64_t hot_keys;          /* sum over batches of keys the hot-key pipeline advanced (far more events
                                   than the batch's mean per key: all their partials at once, not one lane) */
    uint64_t hot_events;        /* their events */
    uint64_t seq_map_trims;     /* multi-device engine: seq map trims (each a min-seq scan of the due shards) */
    uint64_t host_syncs;        /* multi-device engine: host waits its device-batch pushes made (the split's
                                   per-owner totals and positions read back: one per push) */
} sg_stats;

/* ir/ir_len: an IR blob (siddhi_gpu_ir.h) of one query */
int sg_engine_create(const void* ir, size_t ir_len, const sg_config* cfg, sg_engine** out);
int sg_push_batch(sg_engine* e, const sg_batch* b);
/* The engine clock (TimestampGenerator.currentTime()).  Wall-clock apps (no @app:playback): now_ms is
 * the wall clock; every per-key timer whose scheduled run time is <= now_ms runs, in time order
 * (Scheduler.EventCaller, Scheduler.java:238-298).  Playback apps: now_ms is the event time set by
 * InputHandler.send before the event is processed; timers whose queue head is <= now_ms run
 * (Scheduler time-change listener, Scheduler.java:73-104).  Matches emitted by timers are polled
 * like any other (trigger_seq = SG_TIMER_SEQ). */
int sg_advance_time(sg_engine* e, int64_t now_ms);
/* mem = SG_MEM_HOST copies matches to host memory; SG_MEM_DEVICE returns device pointers into the ring of
 * match_capacity ordered records (a window that wraps the ring comes in two polls, the part up to the
 * ring's end first); | SG_POLL_READY returns only what is complete (a pipelined caller pushes batch i + 1
 * before polling batch i).  A push waits while two batches are in flight, so a caller that ready-polls
 * after every push has at most three batches' matches pending in the ring. */
int sg_poll_matches(sg_engine* e, uint32_t mem, sg_match_batch* out);
int sg_release_matches(sg_engine* e, sg_match_batch* m);
int sg_get_stats(sg_engine* e, sg_stats* out);
/* sg_stats only grows at its end, and sg_get_stats writes the whole struct of this header: a caller built against
 * an older header passes its own sizeof(sg_stats) here and gets exactly that prefix (out_size 0: SG_ERR_INVALID). */
int sg_get_stats_sized(sg_engine* e, sg_stats* out, size_t out_size);
/* Diagnostics: the kernels this engine dispatches per push and per clock advance, in launch order, as a
 * NUL-terminated line of text truncated to out_len (no reference counterpart: the query plan a profiler's
 * kernel names map to, as EXPLAIN would print it). */
int sg_engine_describe(sg_engine* e, char* out, size_t out_len);
int sg_synchronize(sg_engine* e);
/* Device batches produced on another stream (a hipStream_t of the engine's device, NULL = the legacy
 * default stream): the engine's later work waits for everything queued on `stream` so far, without a
 * host synchronisation (the multi-GPU reshard hands its output over this way).  A multi-device engine
 * (n_devices > 1): the next device-batch split waits for it (the stream may be on any of its devices; each
 * call records one event, waited on once by that split; the caller's current device is left unchanged). */
int sg_wait_stream(sg_engine* e, void* stream);
/* Partition purge (@purge(enable, interval, idle.period) on a partition; PartitionRuntimeImpl.java:368-401
 * removes idle keys and cleanGroupByStates() every state holder of the partition's queries, so the
 * key's next event runs initPartition again).  The host tracks last-seen times and picks the idle
 * keys; this resets their NFA state (pending / newAndEvery lists, count chains, absent-state flags and
 * timers) to that of a key never seen.  keys: n key ids in host (SG_MEM_HOST) or device memory;
 * ids outside [0, n_keys) fail with SG_ERR_INVALID. */
int sg_reset_keys(sg_engine* e, const uint32_t* keys, uint64_t n, uint32_t mem);
/* Persistence (SnapshotService.java:91,334 -> StreamPreStateProcessor.java:450-469 per key): an image
 * of the device NFA state (library-owned until sg_free_buffer), restorable into an engine created from
 * the same IR with the same n_keys.  Both fail with SG_ERR_STATE while matches wait to be polled. */
int sg_snapshot(sg_engine* e, void** buf, size_t* len);
int sg_restore(sg_engine* e, const void* buf, size_t len);
int sg_free_buffer(void* buf);
/* The NFA state in the reference's per-state-processor form (PartitionStateHolder: partition key ->
 * each pre-state processor's StreamPreState.snapshot() map {PendingStateEventList,
 * NewAndEveryStateEventList, Initialized, Started} + CountStreamPreState {SuccessCondition,
 * StartStateReset} + absent {IsActive, LastScheduledTime / LastArrivalTime} + the Scheduler's
 * toNotifyQueue; StreamPreStateProcessor.java:450-469, CountPreStateProcessor.java:206-219,
 * AbsentStreamPreStateProcessor.java:328-341, AbsentLogicalPreStateProcessor.java:407-420,
 * Scheduler.java:331-368) as a flat engine-independent document: every initialised key, the StateEvents
 * and StreamEvents its lists reach numbered once (shared references kept) — layout in
 * siddhi-1_amd/csrc/state_doc.h.  Export requires no matches waiting to be polled; the buffer is
 * library-owned until sg_free_buffer.  Import replaces the engine's whole state (keys absent from the
 * document become never-seen); a document exported by any engine of the same query (two-state kernel,
 * general kernel, the oracle) imports into any other, within the target's capacities
 * (SG_ERR_CAPACITY / SG_ERR_UNSUPPORTED otherwise). */
int sg_state_export(sg_engine* e, void** buf, size_t* len);
int sg_state_import(sg_engine* e, const void* buf, size_t len);
void sg_engine_destroy(sg_engine* e);
const char* sg_last_error(void);
int sg_abi_version(void);

/* Multi-GPU ingest (the reshard step in front of PartitionStreamReceiver, whose per-key
 * state never crosses keys: PartitionStateHolder.java:43-49).  sg_shard_pack buckets one rank's slice
 * of the arrival-ordered stream by owning rank (owner = key % world, local key = key / world) into
 * packed rows {local key, ts lo, ts hi, col 0..n_cols-1} of 32-bit words, STABLE (arrival order kept
 * per destination), destinations in rank order; dest_counts[world] (device, u64) receives the rows per
 * destination.  All pointers are device memory of the current HIP device; work is queued on `stream`
 * (a hipStream_t, NULL = default).  scratch: sg_shard_scratch_bytes(n, world) bytes of device memory.
 * sg_shard_unpack turns received rows back into the SoA columns of a batch (cols_dev: a device
 * array of n_cols column pointers). */
int sg_shard_pack(uint64_t n, const uint32_t* key, const int64_t* ts, const uint32_t* const* cols, uint32_t n_cols,
                  uint32_t world, uint32_t* rows, unsigned long long* dest_counts, void* scratch, size_t scratch_len,
                  void* stream);
size_t sg_shard_scratch_bytes(uint64_t n, uint32_t world);
/* The same pack into fixed-size destination blocks, so that the exchange needs no host-side counts (one
 * equal-split all_to_all, no device->host sync per step): destination d's rows go to
 * rows[d * cap, d * cap + count_d), the rest of its block is padding rows whose local key is SG_KEY_NULL
 * (an engine created with SG_CFG_NULL_KEYS drops them).  A destination with more than cap rows sets
 * *overflow (device u32) and its extra rows are not written: the caller must fail the step. */
int sg_shard_pack_blocks(uint64_t n, const uint32_t* key, const int64_t* ts, const uint32_t* const* cols,
                         uint32_t n_cols, uint32_t world, uint32_t cap, uint32_t* rows, unsigned long long* dest_counts,
                         uint32_t* overflow, void* scratch, size_t scratch_len, void* stream);
int sg_shard_unpack(uint64_t n, const uint32_t* rows, uint32_t n_cols, uint32_t* key, int64_t* ts,
                    uint32_t* const* cols_dev, void* stream);

/* Host merge of per-shard match runs (north_star: per-partition output merged back in timestamp
 * order on the host — the order MultiProcessStreamReceiver.java:119-121 hands StateEvents to the selector).
 * Each run i (ts[i], len[i] entries, host memory) is one shard's matches in its own order, timestamps
 * nondecreasing; out[total] receives the stable merge as (run << 48) | index: by timestamp, equal timestamps
 * in run order, then in their run's order.  threads > 1: the output is cut into equal slices merged in
 * parallel (merge path over the runs).  No device needed. */
int sg_merge_ts(uint32_t n_runs, const int64_t* const* ts, const uint64_t* len, uint32_t threads, uint64_t* out);

/* Partition-key dictionary (host ingest; no device needed).  Replaces the
 * String-keyed partition map of PartitionStreamReceiver.receive (partition/PartitionStreamReceiver.java:
 * 175-260), where ValuePartitionExecutor.execute (partition/executor/ValuePartitionExecutor.java:34-41)
 * turns the key attribute into its String form and PartitionRuntimeImpl.initPartition
 * (partition/PartitionRuntimeImpl.java:346-402) creates state the first time a key is seen.  Here each
 * distinct key string gets a dense id in first-seen order (0, 1, 2, ...), the key_id that
 * sg_batch.key carries.  Strings are UTF-8 bytes, batched Arrow-style: string i is
 * bytes[offsets[i], offsets[i+1]) (offsets has n+1 entries).  valid (optional, n bytes): 0 marks a
 * null key, which the reference drops (PartitionStreamReceiver.java:175-205); its id is SG_KEY_NULL.
 * sg_dict_intern assigns ids to new strings; it is all-or-nothing: when the batch would take the
 * dictionary past max_ids it fails with SG_ERR_CAPACITY and assigns nothing.  n_new (optional)
 * receives how many strings were new.  sg_dict_lookup never inserts (absent: SG_KEY_NULL). */
typedef struct sg_dict sg_dict;
int sg_dict_create(uint32_t max_ids, uint64_t capacity_hint, sg_dict** out);
int sg_dict_intern(sg_dict* d, const uint8_t* bytes, const uint64_t* offsets, const uint8_t* valid, uint64_t n,
                   uint32_t* ids, uint64_t* n_new);
int sg_dict_lookup(const sg_dict* d, const uint8_t* bytes, const uint64_t* offsets, const uint8_t* valid,
                   uint64_t n, uint32_t* ids);
/* Partition purge (PartitionRuntimeImpl.java:368-401 drops idle keys from its per-partition maps): the
 * listed ids leave the dictionary and are handed out again, smallest first, to the next new keys (after
 * sg_reset_keys has returned their device state to never-seen), so live ids stay below max_ids under key
 * churn.  All-or-nothing: an id not in use (or listed twice) fails with SG_ERR_INVALID. */
int sg_dict_remove(sg_dict* d, const uint32_t* ids, uint64_t n);
/* bind key bytes to a given free id (restoring a snapshot's key map); ids skipped over become free */
int sg_dict_put(sg_dict* d, uint32_t id, const uint8_t* bytes, uint64_t len);
/* id bound: every id handed out so far is below it (removed ids included) */
uint32_t sg_dict_size(const sg_dict* d);
/* the key string of an id in use (pointer valid until the next intern / put / remove / clear); a removed
 * id fails with SG_ERR_INVALID */
int sg_dict_key(const sg_dict* d, uint32_t id, const uint8_t** ptr, uint64_t* len);
int sg_dict_clear(sg_dict* d);
void sg_dict_destroy(sg_dict* d);

/* Diagnostics (no device needed): generate and compile the query-specialised advance kernel of an IR
 * blob for gfx950.  variant_flags: bit 0 = batches carry null flags, bit 1 = captures carry null bits.
 * out (optional) receives the generated query header, or the compiler log on failure. */
int sg_jit_check(const void* ir, size_t ir_len, uint32_t variant_flags, char* out, size_t out_len);

#ifdef __cplusplus
}
#endif

#endif /* SIDDHI_GPU_H */
