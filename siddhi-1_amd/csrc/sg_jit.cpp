// sg_jit.cpp — code generation and hipRTC compilation of the query-specialised advance kernel.
//
// The reference evaluates a filter by walking an ExpressionExecutor tree per event and partial
// (query/processor/filter/FilterProcessor.java:48-60 -> executor/condition/compare/*,
// executor/math/*).  Here the lowered filter program becomes straight-line typed HIP over the
// Java value model of p2_jit.hip (JV<T>: value + null flag), compiled once per query shape.
#include "sg_jit.h"

#include <hip/hiprtc.h>

#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <unordered_map>

#include "../../include/siddhi_gpu_ir.h"

namespace {

#include "../lib/jit_src.inc"  // kJitKernel (p2_jit.hip), kJitEngineH (sg_engine.h), kJitIrH (siddhi_gpu_ir.h)

const char* ctype(uint32_t t) {
    switch (t) {
    case SG_T_INT: return "int32_t";
    case SG_T_LONG: return "int64_t";
    case SG_T_FLOAT: return "float";
    case SG_T_DOUBLE: return "double";
    case SG_T_STRING: return "uint32_t";
    case SG_T_BOOL: return "bool";
    default: throw std::runtime_error("unknown attribute type");
    }
}

bool wide(uint32_t t) { return t == SG_T_LONG || t == SG_T_DOUBLE; }

// value of type t from 32-bit words lo (and hi)
std::string from_words(uint32_t t, const std::string& lo, const std::string& hi) {
    switch (t) {
    case SG_T_INT: return "(int32_t)" + lo;
    case SG_T_LONG: return "sg_i64(" + lo + ", " + hi + ")";
    case SG_T_FLOAT: return "sg_f32(" + lo + ")";
    case SG_T_DOUBLE: return "sg_f64(" + lo + ", " + hi + ")";
    case SG_T_STRING: return "(uint32_t)" + lo;
    default: return "(" + lo + " != 0u)";
    }
}

// value of type t from the 64-bit constant word c
std::string from_const(uint32_t t, const std::string& c) {
    switch (t) {
    case SG_T_INT: return "(int32_t)(uint32_t)" + c;
    case SG_T_LONG: return "(int64_t)" + c;
    case SG_T_FLOAT: return "__uint_as_float((uint32_t)" + c + ")";
    case SG_T_DOUBLE: return "__longlong_as_double((long long)" + c + ")";
    case SG_T_STRING: return "(uint32_t)" + c;
    default: return "((" + c + " & 1ull) != 0ull)";
    }
}

// the 32-bit words of a value expression v of type t
void to_words(uint32_t t, const std::string& v, std::string& lo, std::string& hi) {
    switch (t) {
    case SG_T_INT: lo = "(uint32_t)" + v; break;
    case SG_T_LONG: lo = "(uint32_t)(uint64_t)" + v; hi = "(uint32_t)((uint64_t)" + v + " >> 32)"; break;
    case SG_T_FLOAT: lo = "__float_as_uint(" + v + ")"; break;
    case SG_T_DOUBLE:
        lo = "(uint32_t)(uint64_t)__double_as_longlong(" + v + ")";
        hi = "(uint32_t)((uint64_t)__double_as_longlong(" + v + ") >> 32)";
        break;
    case SG_T_STRING: lo = v; break;
    default: lo = "(" + v + " ? 1u : 0u)";
    }
}

struct Val {
    std::string e;   // expression of type JV<ctype(t)>
    uint32_t t = 0;
    bool cst = false;
    uint64_t bits = 0;
    bool cnull = false;
};

struct FilterGen {
    std::ostringstream& o;
    std::vector<uint64_t>& consts;
    const JitQuery& q;
    int tmp = 0;

    std::string jv(uint32_t t) { return std::string("JV<") + ctype(t) + ">"; }

    std::string mat(const Val& v) {
        if (!v.cst) return v.e;
        if (v.cnull) return jv(v.t) + "{" + ctype(v.t) + "(), true}";
        if (consts.size() >= SGD_MAX_CONST) throw std::runtime_error("too many filter constants for the device");
        const size_t i = consts.size();
        consts.push_back(v.bits);
        return jv(v.t) + "{" + from_const(v.t, "p.cst[" + std::to_string(i) + "]") + ", false}";
    }

    std::string emit(uint32_t t, const std::string& rhs) {
        const std::string n = "v" + std::to_string(tmp++);
        o << "    const " << jv(t) << " " << n << " = " << rhs << ";\n";
        return n;
    }

    // capture c of the partial (words cw[], null bits cn)
    std::string capture(uint32_t c) {
        uint32_t word = 0;
        for (uint32_t i = 0; i < c; i++) word += wide(q.cap_type[i]) ? 2 : 1;
        const uint32_t t = q.cap_type[c];
        const std::string v = from_words(t, "cw[" + std::to_string(word) + "]", "cw[" + std::to_string(word + 1) + "]");
        const std::string nul = q.capnull ? "((cn >> " + std::to_string(c) + ") & 1u) != 0u" : "false";
        return jv(t) + "{" + v + ", " + nul + "}";
    }

    void gen(const DProg& f, bool is_f1) {
        std::vector<Val> st;
        auto pop = [&]() {
            if (st.empty()) throw std::runtime_error("filter program stack underflow");
            Val v = st.back();
            st.pop_back();
            return v;
        };
        for (uint32_t pc = 0; pc < f.len; pc++) {
            const DInst& I = f.ins[pc];
            switch (I.op) {
            case SG_OP_VAR: {
                Val v;
                v.t = I.t;
                if (I.src == SGD_SRC_EV) {
                    v.e = "e.a" + std::to_string(I.arg);
                } else if (I.src == SGD_SRC_CAP) {
                    if (!is_f1) throw std::runtime_error("start-state filter reads a capture");
                    v.e = capture((uint32_t)I.arg);
                } else {
                    v.cst = true;
                    v.cnull = true;
                }
                st.push_back(v);
                break;
            }
            case SG_OP_CONST: {
                Val v;
                v.t = I.t;
                v.cst = true;
                v.cnull = I.t2 != 0;
                v.bits = I.imm;
                st.push_back(v);
                break;
            }
            case SG_OP_CVT: {
                Val v = pop();
                if (v.t != I.t) throw std::runtime_error("conversion of a value of the wrong type");
                if (v.cst) {
                    if (!v.cnull) v.bits = sgj_fold_cvt(v.bits, I.t, I.t2);
                    v.t = I.t2;
                } else {
                    v.e = emit(I.t2, std::string("jcvt<") + ctype(I.t2) + ">(" + v.e + ")");
                    v.t = I.t2;
                }
                st.push_back(v);
                break;
            }
            case SG_OP_ADD: case SG_OP_SUB: case SG_OP_MUL: case SG_OP_DIV: case SG_OP_MOD: {
                Val r = pop(), l = pop();
                if (l.t != I.t || r.t != I.t || I.t == SG_T_STRING || I.t == SG_T_BOOL)
                    throw std::runtime_error("arithmetic operand types do not match");
                Val v;
                v.t = I.t;
                v.e = emit(I.t, "jarith(" + std::to_string(I.op) + ", " + mat(l) + ", " + mat(r) + ")");
                st.push_back(v);
                break;
            }
            case SG_OP_EQ: case SG_OP_NE: case SG_OP_GT: case SG_OP_GE: case SG_OP_LT: case SG_OP_LE: {
                Val r = pop(), l = pop();
                if (l.t != I.t || r.t != I.t) throw std::runtime_error("comparison operand types do not match");
                Val v;
                v.t = SG_T_BOOL;
                v.e = emit(SG_T_BOOL, "jcmp<" + std::to_string(I.op) + ">(" + mat(l) + ", " + mat(r) + ")");
                st.push_back(v);
                break;
            }
            case SG_OP_AND: case SG_OP_OR: {
                Val r = pop(), l = pop();
                if (l.t != SG_T_BOOL || r.t != SG_T_BOOL) throw std::runtime_error("logical operand is not bool");
                Val v;
                v.t = SG_T_BOOL;
                v.e = emit(SG_T_BOOL, "JV<bool>{jtrue(" + mat(l) + ") " + (I.op == SG_OP_AND ? "&&" : "||") +
                                          " jtrue(" + mat(r) + "), false}");
                st.push_back(v);
                break;
            }
            case SG_OP_NOT: {
                Val a = pop();
                if (a.t != SG_T_BOOL) throw std::runtime_error("not of a non-bool");
                Val v;
                v.t = SG_T_BOOL;
                v.e = emit(SG_T_BOOL, "JV<bool>{!jtrue(" + mat(a) + "), false}");
                st.push_back(v);
                break;
            }
            case SG_OP_ISNULL: {
                Val a = pop();
                Val v;
                v.t = SG_T_BOOL;
                v.e = emit(SG_T_BOOL, "JV<bool>{" + mat(a) + ".n, false}");
                st.push_back(v);
                break;
            }
            default: throw std::runtime_error("unknown filter op");
            }
        }
        if (f.len == 0) {
            o << "    return true;\n";
            return;
        }
        if (st.size() != 1 || st.back().t != SG_T_BOOL) throw std::runtime_error("filter does not yield one bool");
        o << "    return jtrue(" << mat(st.back()) << ");\n";
    }
};

void gen_stream(std::ostringstream& o, int s, const std::vector<uint32_t>& types, bool evnull) {
    const uint32_t words = sgj_col_words(types);
    const uint32_t nw = 1 + words;  // null word
    o << "struct SgEv" << s << " {";
    for (size_t c = 0; c < types.size(); c++) o << " JV<" << ctype(types[c]) << "> a" << c << ";";
    o << " };\n";
    o << "__device__ __forceinline__ SgEv" << s << " sgq_ev" << s << "(const uint32_t* w) {\n    SgEv" << s << " e;\n";
    uint32_t off = 1;
    for (size_t c = 0; c < types.size(); c++) {
        const std::string lo = "w[" + std::to_string(off) + "]", hi = "w[" + std::to_string(off + 1) + "]";
        o << "    e.a" << c << ".v = " << from_words(types[c], lo, hi) << ";\n";
        if (evnull)
            o << "    e.a" << c << ".n = ((w[" << nw << "] >> " << c << ") & 1u) != 0u;\n";
        else
            o << "    e.a" << c << ".n = false;\n";
        off += wide(types[c]) ? 2 : 1;
    }
    o << "    return e;\n}\n";
    o << "__device__ __forceinline__ void sgq_pack" << s << "(const PackParams& q, uint32_t j, uint32_t* w) {\n";
    off = 1;
    for (size_t c = 0; c < types.size(); c++) {
        const uint32_t t = types[c];
        if (wide(t)) {
            o << "    { const uint64_t v = ((const uint64_t*)q.col[" << c << "])[j]; w[" << off << "] = (uint32_t)v; w["
              << off + 1 << "] = (uint32_t)(v >> 32); }\n";
        } else if (t == SG_T_BOOL) {
            o << "    w[" << off << "] = ((const uint8_t*)q.col[" << c << "])[j] ? 1u : 0u;\n";
        } else {
            o << "    w[" << off << "] = ((const uint32_t*)q.col[" << c << "])[j];\n";
        }
        off += wide(t) ? 2 : 1;
    }
    if (evnull) {
        o << "    uint32_t nb = 0;\n";
        for (size_t c = 0; c < types.size(); c++)
            o << "    if (q.nul[" << c << "]) nb |= (q.nul[" << c << "][j] != 0 ? 1u : 0u) << " << c << ";\n";
        o << "    w[" << nw << "] = nb;\n";
    }
    o << "}\n";
}

uint64_t fnv1a(const void* d, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* p = (const unsigned char*)d;
    for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; }
    return h;
}

const char* const kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                             "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"};

std::string cache_dir() {
    if (const char* d = getenv("SG_JIT_CACHE")) return d;
    if (const char* x = getenv("XDG_CACHE_HOME")) return std::string(x) + "/siddhi_gpu";
    if (const char* hm = getenv("HOME")) return std::string(hm) + "/.cache/siddhi_gpu";
    return "";
}

void mkdirs(const std::string& path) {
    for (size_t i = 1; i <= path.size(); i++)
        if (i == path.size() || path[i] == '/') (void)mkdir(path.substr(0, i).c_str(), 0755);
}

std::mutex g_mu;
std::unordered_map<std::string, std::vector<char>> g_cache;  // full source -> code object

}  // namespace

uint32_t sgj_col_words(const std::vector<uint32_t>& types) {
    uint32_t w = 0;
    for (uint32_t t : types) w += wide(t) ? 2 : 1;
    return w;
}

uint32_t sgj_stride(uint32_t words) {
    const uint32_t w = words ? words : 1;
    return w + 2;  // == sizeof(Pay<w>) / 4 of the sorted-payload path (pack.h): position, words, ts offset
}

uint64_t sgj_fold_cvt(uint64_t b, uint32_t from, uint32_t to) {
    if (from == to) return b;
    if (from == SG_T_INT) {
        int32_t x = (int32_t)(uint32_t)b;
        if (to == SG_T_LONG) return (uint64_t)(int64_t)x;
        if (to == SG_T_FLOAT) { float f = (float)x; uint32_t u; memcpy(&u, &f, 4); return u; }
        double d = (double)x; uint64_t u; memcpy(&u, &d, 8); return u;
    }
    if (from == SG_T_LONG) {
        int64_t x = (int64_t)b;
        if (to == SG_T_FLOAT) { float f = (float)x; uint32_t u; memcpy(&u, &f, 4); return u; }
        double d = (double)x; uint64_t u; memcpy(&u, &d, 8); return u;
    }
    if (from == SG_T_FLOAT && to == SG_T_DOUBLE) {
        uint32_t u = (uint32_t)b; float f; memcpy(&f, &u, 4); double d = (double)f; uint64_t o; memcpy(&o, &d, 8);
        return o;
    }
    throw std::runtime_error("bad constant conversion");
}

std::string sgj_generate(const JitQuery& q, std::vector<uint64_t>& consts) {
    if (q.reg_slots < 1 || q.reg_slots > SGD_MAX_REG) throw std::runtime_error("register window out of range");
    std::ostringstream o;
    uint32_t ncapw = 0;
    for (uint8_t t : q.cap_type) ncapw += wide(t) ? 2 : 1;
    const int ns = q.multi ? 1 : 2;
    uint32_t stride[2];
    for (int s = 0; s < 2; s++)
        stride[s] = sgj_stride(sgj_col_words(q.coltypes[q.multi ? 0 : s]) + (q.evnull ? 1 : 0));
    o << "// generated by sg_jit.cpp: one two-state pattern query\n#pragma once\n";
    // tuning experiments (tools/exp_c2.py): SG_JIT_EXTRA="NAME=VALUE,..." prepends #defines
#ifdef SG_EXPERIMENTS
    if (const char* x = getenv("SG_JIT_EXTRA")) {
        std::string defs(x), item;
        std::istringstream ds(defs);
        while (std::getline(ds, item, ',')) {
            const size_t eq = item.find('=');
            if (item.empty()) continue;
            o << "#define " << (eq == std::string::npos ? item : item.substr(0, eq) + " " + item.substr(eq + 1)) << "\n";
        }
    }
#endif
    o << "#define SGQ_R " << q.reg_slots << "\n";
    const uint32_t rh = q.reg_slots_hbm ? q.reg_slots_hbm : q.reg_slots;
    if (rh > SGD_MAX_REG_HBM) throw std::runtime_error("HBM-pass register window out of range");
    o << "#define SGQ_RH " << rh << "\n";
    o << "#define SGQ_MODE " << q.mode << "\n";
    o << "#define SGQ_MULTI " << (q.multi ? 1 : 0) << "\n";
    o << "#define SGQ_WITHIN " << (q.within ? 1 : 0) << "\n";
    o << "#define SGQ_NCAPW " << ncapw << "\n";
    o << "#define SGQ_CAPNULL " << (q.capnull ? 1 : 0) << "\n";
    o << "#define SGQ_PROJ " << (q.proj ? 1 : 0) << "\n";
    o << "#define SGQ_STRIDE0 " << stride[0] << "\n";
    o << "#define SGQ_STRIDE1 " << stride[1] << "\n";
    for (int s = 0; s < ns; s++) gen_stream(o, s, q.coltypes[s], q.evnull);
    if (q.multi) o << "typedef SgEv0 SgEv1;\n#define sgq_ev1 sgq_ev0\n#define sgq_pack1 sgq_pack0\n";
    FilterGen g{o, consts, q};
    o << "__device__ __forceinline__ bool sgq_f0(const SgEv0& e, const P2Params& p) {\n";
    g.gen(*q.f0, false);
    o << "}\n";
    o << "__device__ __forceinline__ bool sgq_f1(const SgEv1& e, const uint32_t* cw, uint32_t cn, "
         "const P2Params& p) {\n";
    g.gen(*q.f1, true);
    o << "}\n";
    o << "__device__ __forceinline__ void sgq_capture(const SgEv0& e, uint32_t* cw, uint32_t& cn) {\n";
    uint32_t word = 0;
    for (size_t c = 0; c < q.cap_type.size(); c++) {
        const uint32_t t = q.cap_type[c];
        std::string lo, hi;
        to_words(t, "e.a" + std::to_string(q.cap_col[c]) + ".v", lo, hi);
        o << "    cw[" << word << "] = " << lo << ";\n";
        if (wide(t)) o << "    cw[" << word + 1 << "] = " << hi << ";\n";
        o << "    cn |= (e.a" << (int)q.cap_col[c] << ".n ? 1u : 0u) << " << c << ";\n";
        word += wide(t) ? 2 : 1;
    }
    o << "}\n";
    return o.str();
}

bool sgj_compile(const std::string& qh, std::vector<char>& code, std::string& log) {
    std::string key = qh;
    key += '\x01';
    key += kJitKernel;
    key += kJitEngineH;
    key += kJitIrH;
    for (const char* opt : kOpts) key += opt;
    if (getenv("SG_JIT_ATOMIC_OPT")) key += "+atomicopt";
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(key);
    if (it != g_cache.end()) {
        code = it->second;
        return true;
    }
    char name[64];
    snprintf(name, sizeof(name), "%016llx.co", (unsigned long long)fnv1a(key.data(), key.size()));
    const std::string dir = cache_dir();
    const std::string path = dir.empty() ? "" : dir + "/" + name;
    if (!path.empty()) {
        std::ifstream f(path, std::ios::binary);
        if (f) {
            std::vector<char> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
            if (!buf.empty()) {
                g_cache[key] = buf;
                code = std::move(buf);
                return true;
            }
        }
    }
    hiprtcProgram prog;
    const char* headers[] = {kJitIrH, kJitEngineH, qh.c_str()};
    const char* names[] = {"siddhi_gpu_ir.h", "sg_engine.h", "sgq_query.h"};
    if (hiprtcCreateProgram(&prog, kJitKernel, "p2_jit.hip", 3, headers, names) != HIPRTC_SUCCESS) {
        log = "hiprtcCreateProgram failed";
        return false;
    }
    std::vector<const char*> opts(kOpts, kOpts + sizeof(kOpts) / sizeof(kOpts[0]));
    if (getenv("SG_JIT_ATOMIC_OPT")) opts.resize(opts.size() - 2);  // experiments: default atomic optimizer
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    log.assign(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    bool ok = rc == HIPRTC_SUCCESS;
    if (ok) {
        size_t cs = 0;
        hiprtcGetCodeSize(prog, &cs);
        code.resize(cs);
        hiprtcGetCode(prog, code.data());
        g_cache[key] = code;
        if (!path.empty()) {  // best effort: write-then-rename so concurrent processes never see a torn file
            mkdirs(dir);
            const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
            std::ofstream f(tmp, std::ios::binary);
            if (f && f.write(code.data(), (std::streamsize)code.size())) {
                f.close();
                (void)rename(tmp.c_str(), path.c_str());
            } else {
                (void)unlink(tmp.c_str());
            }
        }
    } else {
        log = std::string(hiprtcGetErrorString(rc)) + "\n" + log;
    }
    hiprtcDestroyProgram(&prog);
    return ok;
}
