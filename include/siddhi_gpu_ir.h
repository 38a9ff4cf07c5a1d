/*
 * siddhi_gpu_ir.h — binary IR that the host compiler (siddhi-1_amd/compiler.py) emits for one
 * pattern/sequence query and that every engine behind the C-ABI consumes (the HIP engine in
 * siddhi-1_amd/csrc, and the CPU oracle under oracle/ used by the tests).
 *
 * The IR is the lowered form of what the reference builds at
 *   StateInputStreamParser.parseInputStream / parse
 *   (/root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/util/parser/StateInputStreamParser.java:76-408)
 * plus the typed condition executors that ExpressionParser builds
 *   (.../util/parser/ExpressionParser.java:225-1507).
 *
 * It keeps the state-element TREE (stream / next / every / logical / count) rather than a flattened
 * processor graph: each engine performs its own wiring.  Slot numbers are assigned by the compiler in
 * the reference's parse order (next: current then next; logical: element 2 BEFORE element 1, see
 * StateInputStreamParser.java:349-361), because slot ids are semantically visible
 * (CountPreStateProcessor.java:97-103 looks at slot+1 / slot+2).
 *
 * Encoding: a flat little-endian array of uint32 words.
 *
 *   word 0   SG_IR_MAGIC
 *   word 1   SG_IR_VERSION
 *   word 2   query type (SG_Q_PATTERN | SG_Q_SEQUENCE)
 *   word 3   number of input streams  S
 *   word 4   number of slots (state stream events) N
 *   word 5-6 within in ms, int64 (lo, hi); -1 = no within
 *   word 7   offset of the stream table (words)
 *   word 8   offset of the node tree
 *   word 9   number of words in the node tree
 *   word 10  offset of the bytecode
 *   word 11  number of bytecode words
 *   word 12  flags (SG_IR_F_*)
 *   word 13  offset of the slot table (N entries of SG_IR_SLOT_WORDS words)
 *
 *   stream table: for each stream s: n_attrs, then n_attrs type codes (enum sg_type)
 *
 *   slot table (per slot): stream index, multi-value flag (slot belongs to a count state)
 *
 *   node tree, prefix order:
 *     SG_N_STREAM : tag, slot, stream, filter_pc, filter_len, absent, for_lo, for_hi
 *                   (absent = `not S[..] for T`: for = T in ms, -1 when a logical `not` has no `for`)
 *     SG_N_NEXT   : tag, <current>, <next>
 *     SG_N_EVERY  : tag, <child>
 *     SG_N_LOGICAL: tag, logical type (SG_L_AND | SG_L_OR), <element1>, <element2>
 *     SG_N_COUNT  : tag, min, max, <stream node>       (max = SG_COUNT_ANY for unbounded)
 *
 *   bytecode: a typed stack machine, one program per filter (filter_pc .. filter_pc+filter_len).
 *     Values are 64-bit with a null flag.  Every instruction starts with a header word
 *       op | a << 8 | b << 16 | c << 24
 *     SG_OP_VAR    a=type  b=slot          w1=attr index  w2=chain index (int32: k>=0 k-th,
 *                                            -1 last, -2 second to last, ...)  (StateEvent.java:138-182)
 *     SG_OP_CONST  a=type  b=is_null       w1=lo  w2=hi   (int/bool/string id in lo; long/double bits)
 *     SG_OP_CVT    a=from  b=to                           (Java widening primitive conversion)
 *     SG_OP_ADD..SG_OP_MOD  a=result type                 (executor/math: null in -> null,
 *                                                          / and % by zero -> null)
 *     SG_OP_EQ..SG_OP_LE    a=compare domain type         (executor/condition/compare: null -> false,
 *                                                          except NE: null -> true)
 *     SG_OP_AND, SG_OP_OR, SG_OP_NOT                      (never null; not(null) = true)
 *     SG_OP_ISNULL                                        (value is null)
 *     SG_OP_ISNULL_EV   b=slot  w1=chain index            (`e1 is null`: stream event absent)
 *     SG_OP_IFELSE a=result type  pops cond, then, else   (ifThenElse(c, x, y): x iff c is a non-null
 *                                                          true, else y; IfThenElseFunctionExecutor.java)
 *   A filter passes iff the program leaves a non-null true (FilterProcessor.java:48-60).
 */
#ifndef SIDDHI_GPU_IR_H
#define SIDDHI_GPU_IR_H

#include <stdint.h>

#define SG_IR_MAGIC 0x52494753u /* "SGIR" */
#define SG_IR_VERSION 1u

#define SG_IR_HDR_WORDS 14
#define SG_IR_SLOT_WORDS 2

#define SG_IR_F_PARTITIONED 1u
#define SG_IR_F_PLAYBACK 2u    /* @app:playback: the clock is event time (TimestampGeneratorImpl.java:77-122) */

#define SG_COUNT_ANY 0x7fffffffu

enum sg_type {
    SG_T_STRING = 0, /* host dictionary id (uint32); only == / != are defined */
    SG_T_INT = 1,    /* int32  */
    SG_T_LONG = 2,   /* int64  */
    SG_T_FLOAT = 3,  /* float  */
    SG_T_DOUBLE = 4, /* double */
    SG_T_BOOL = 5    /* uint8 0/1 */
};

enum sg_query_type { SG_Q_PATTERN = 0, SG_Q_SEQUENCE = 1 };

enum sg_node_tag {
    SG_N_STREAM = 1,
    SG_N_NEXT = 2,
    SG_N_EVERY = 3,
    SG_N_LOGICAL = 4,
    SG_N_COUNT = 5
};

enum sg_logical_type { SG_L_AND = 1, SG_L_OR = 2 };

/* Projection programs (sg_set_projection): item_type = result type code | aggregator << 8 | role bits.
 * Items come in QuerySelector order: first one item per aggregator (its argument program; empty for
 * count()), then the select list, then at most one `having` condition.  Inside the select items and
 * `having`, VAR b = SG_PROJ_SLOT_AGG reads aggregator w1's current value and b = SG_PROJ_SLOT_OUT reads
 * select item w1 of the same output row (`having` over output attributes, QuerySelector.java:120-160). */
enum sg_proj_agg {
    SG_AGG_NONE = 0,
    SG_AGG_COUNT = 1, /* CountAttributeAggregatorExecutor: LONG, every event */
    SG_AGG_SUM = 2,   /* SumAttributeAggregatorExecutor: LONG for int/long arguments, DOUBLE otherwise */
    SG_AGG_AVG = 3,   /* AvgAttributeAggregatorExecutor: DOUBLE sum / count */
    SG_AGG_MIN = 4,   /* Min(Forever)AttributeAggregatorExecutor: the argument's type */
    SG_AGG_MAX = 5    /* Max(Forever)AttributeAggregatorExecutor */
};
#define SG_PROJ_AGG_ITEM 0x10000u  /* item_type bit: this item is an aggregator's argument */
#define SG_PROJ_HAVING 0x20000u    /* item_type bit: this item is the `having` condition (BOOL) */
#define SG_PROJ_SLOT_AGG 0xFDu
#define SG_PROJ_SLOT_OUT 0xFEu

enum sg_opcode {
    SG_OP_VAR = 1,
    SG_OP_CONST = 2,
    SG_OP_CVT = 3,
    SG_OP_ADD = 10,
    SG_OP_SUB = 11,
    SG_OP_MUL = 12,
    SG_OP_DIV = 13,
    SG_OP_MOD = 14,
    SG_OP_EQ = 20,
    SG_OP_NE = 21,
    SG_OP_GT = 22,
    SG_OP_GE = 23,
    SG_OP_LT = 24,
    SG_OP_LE = 25,
    SG_OP_AND = 30,
    SG_OP_OR = 31,
    SG_OP_NOT = 32,
    SG_OP_ISNULL = 33,
    SG_OP_ISNULL_EV = 34,
    SG_OP_IFELSE = 40
};

/* instruction lengths in words */
static inline int sg_op_len(uint32_t op) {
    switch (op & 0xffu) {
    case SG_OP_VAR: return 3;
    case SG_OP_CONST: return 3;
    case SG_OP_ISNULL_EV: return 2;
    default: return 1;
    }
}

#endif /* SIDDHI_GPU_IR_H */
