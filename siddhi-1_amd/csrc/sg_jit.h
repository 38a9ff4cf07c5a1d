// sg_jit.h — query specialisation of the advance kernel (host side, internal).
//
// The two-state plan of a query (pattern mode, stream roles, column types, the lowered filters and
// the capture layout) is turned into a header "sgq_query.h" of typed HIP code, compiled together
// with p2_jit.hip by hipRTC for gfx950.  Filter constants are kernel arguments (P2Params::cst), so
// queries that differ only in constants share one code object; code objects are cached in memory
// and on disk ($SG_JIT_CACHE, default ~/.cache/siddhi_gpu).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "sg_engine.h"

struct JitQuery {
    int mode = 0;                         // SGD_P2_* bits
    bool multi = false;                   // both states read the same stream
    bool within = false;
    uint32_t reg_slots = 12;              // SGQ_R
    uint32_t reg_slots_hbm = 0;           // SGQ_RH (0: SGQ_R)
    std::vector<uint32_t> coltypes[2];    // types of the filter columns of stream s0 / s1
    const DProg* f0 = nullptr;
    const DProg* f1 = nullptr;
    std::vector<uint8_t> cap_col;         // capture c = column cap_col[c] of stream s0
    std::vector<uint8_t> cap_type;
    bool evnull = false;                  // this variant's batches carry null flags
    bool capnull = false;                 // captures carry null bits
    bool proj = false;                    // on-device projection: matches carry the partial's captures
};

// payload words of a stream: [batch position][column words][null word?][pad][ts lo, ts hi]
uint32_t sgj_col_words(const std::vector<uint32_t>& types);
uint32_t sgj_stride(uint32_t words);      // words = column words (+1 null word)

// generate sgq_query.h; the filter constants are appended to `consts` (P2Params::cst order)
std::string sgj_generate(const JitQuery& q, std::vector<uint64_t>& consts);

// compile p2_jit.hip + the query header for gfx950 (no device needed); cached
bool sgj_compile(const std::string& query_header, std::vector<char>& code, std::string& log);

// Java widening conversion of a constant's bits (JLS 5.1.2)
uint64_t sgj_fold_cvt(uint64_t bits, uint32_t from, uint32_t to);
