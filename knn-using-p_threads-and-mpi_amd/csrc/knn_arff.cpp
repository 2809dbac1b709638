// knn_arff.cpp -- clean-room ARFF ingestion + the reference's C++ API on the GPU path.
//
// Parsing follows libarff's observable behaviour (srna99/KNN-using-p_threads-and-MPI,
// libarff/arff_lexer.cpp:87-203, arff_parser.cpp:23-153, arff_value.cpp:33-48,
// arff_utils.h:56-63, arff_data.cpp:117-165):
//   * tokens are separated by ' ', '\t', '\n' and ','; '\r' is NOT a separator;
//     '%' starts a comment only as the first character of a line; '{' '}' are tokens;
//     '?' is a missing value; quoted strings keep their spaces
//   * the instance reader consumes exactly num_attributes tokens per instance
//     (newlines are not row delimiters) and drops a partial instance at EOF
//   * NUMERIC fields are parsed like `istringstream >> float`: the longest prefix
//     [+-]digits[.digits][e[+-]digits] is converted by strtof and must convert
//     completely; overflow (inf) fails; anything else stays a STRING value, which the
//     cross-check then rejects for a NUMERIC attribute
//   * attribute types: numeric|real, string, date, {nominal}; anything else throws
// The whole file is read at once (libarff reads one byte per fread call).  When every
// attribute is NUMERIC (the KNN case) the data section is parsed by several threads
// (parse_numeric_parallel): tokens are counted per chunk, a prefix sum gives every
// token its instance/attribute, and each thread converts its own tokens straight into
// the [n][na] buffer.  Anything the fast path does not model exactly -- '?', quotes,
// braces, '%', a ',' that does not directly follow a token (libarff's lexer reads an
// empty token there and stops), a field that does not parse -- sends the whole data
// section back to the serial lexer, which reproduces libarff's result or error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/knn_amd.h"
#include "../../include/knn_arff.hpp"
#include "../../include/knn_compat_threads.hpp"

// multi-thread.cpp:15 -- the driver's own definition wins over this weak one
__attribute__((weak)) int* predictions = nullptr;

namespace {

[[noreturn]] void throwf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void throwf(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    throw std::runtime_error(buf);
}

bool icase_eq(const std::string& a, const char* b) {
    size_t n = std::strlen(b);
    if (a.size() != n) return false;
    for (size_t i = 0; i < n; i++)
        if (std::tolower((unsigned char)a[i]) != std::tolower((unsigned char)b[i])) return false;
    return true;
}

// libstdc++ num_get<float> as used by `istringstream >> float` (libarff/arff_utils.h:56-63)
bool parse_float_like_istream(const char* s, size_t n, float* out) {
    char acc[128];
    size_t m = 0, i = 0;
    auto push = [&](char c) { if (m + 1 < sizeof(acc)) acc[m++] = c; };
    if (i < n && (s[i] == '+' || s[i] == '-')) push(s[i++]);
    bool mantissa = false, dot = false;
    while (i < n) {
        char c = s[i];
        if (c >= '0' && c <= '9') { push(c); mantissa = true; i++; }
        else if (c == '.' && !dot) { push(c); dot = true; i++; }
        else break;
    }
    if (i < n && (s[i] == 'e' || s[i] == 'E') && mantissa) {
        push(s[i++]);
        if (i < n && (s[i] == '+' || s[i] == '-')) push(s[i++]);
        while (i < n && s[i] >= '0' && s[i] <= '9') push(s[i++]);
    }
    acc[m] = '\0';
    if (m == 0) return false;
    char* end = nullptr;
    float v = std::strtof(acc, &end);
    if (end == acc || *end != '\0') return false;
    if (std::isinf(v)) return false;
    *out = v;
    return true;
}

enum Kind : uint8_t { K_FLOAT = 0, K_STRING = 1, K_NOMINAL = 2, K_MISSING = 3 };

struct ParsedAttr {
    std::string name;
    ArffValueEnum type;
    std::vector<std::string> nominal;
};

struct ParsedArff {
    std::string relation;
    std::vector<ParsedAttr> attrs;
    int64_t n = 0;
    std::vector<float> values;   // [n][nattr]
    std::vector<uint8_t> kinds;  // [n][nattr]
    std::unordered_map<int64_t, std::string> strs;
};

enum Tok { T_RELATION, T_ATTRIBUTE, T_DATA, T_NUMERIC, T_STRING, T_DATE, T_BOPEN, T_BCLOSE, T_MISSING, T_EOF, T_VALUE };

class Lexer {
public:
    explicit Lexer(std::vector<char>&& buf) : b_(std::move(buf)) {}
    size_t pos() const { return p_; }
    const std::vector<char>& buffer() const { return b_; }
    Tok next(std::string& s) {
        if (pend_close_) { pend_close_ = false; s = "}"; return T_BCLOSE; }
        for (;;) {
            while (p_ < b_.size() && is_space(b_[p_])) p_++;
            if (p_ < b_.size() && b_[p_] == '%' && (p_ == 0 || b_[p_ - 1] == '\n')) {
                while (p_ < b_.size() && b_[p_] != '\n') p_++;
                continue;
            }
            break;
        }
        s.clear();
        if (p_ >= b_.size()) return T_EOF;
        char c = b_[p_];
        if (c == '{') { p_++; s = "{"; return T_BOPEN; }
        if (c == '}') { p_++; s = "}"; return T_BCLOSE; }
        if (c == '?') {
            while (p_ < b_.size() && b_[p_] != ',' && b_[p_] != '\n') p_++;
            if (p_ < b_.size() && b_[p_] == ',') p_++;
            s = "?";
            return T_MISSING;
        }
        if (c == '\'' || c == '"') {
            p_++;
            while (p_ < b_.size() && b_[p_] != c) {
                if (b_[p_] == '}') { pend_close_ = true; p_++; return classify(s); }
                s += b_[p_++];
            }
            if (p_ < b_.size()) p_++;
            skip_sep();
            return classify(s);
        }
        while (p_ < b_.size() && !is_space(b_[p_]) && b_[p_] != ',') {
            if (b_[p_] == '}') { pend_close_ = true; p_++; return classify(s); }
            s += b_[p_++];
        }
        skip_sep();
        return classify(s);
    }

private:
    static bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n'; }
    void skip_sep() { if (p_ < b_.size() && (b_[p_] == ',' || is_space(b_[p_]))) p_++; }
    static Tok classify(const std::string& s) {
        if (icase_eq(s, "@relation")) return T_RELATION;
        if (icase_eq(s, "@attribute")) return T_ATTRIBUTE;
        if (icase_eq(s, "@data")) return T_DATA;
        if (icase_eq(s, "numeric") || icase_eq(s, "real")) return T_NUMERIC;
        if (icase_eq(s, "string")) return T_STRING;
        if (icase_eq(s, "date")) return T_DATE;
        if (s.empty()) return T_EOF;
        return T_VALUE;
    }
    std::vector<char> b_;
    size_t p_ = 0;
    bool pend_close_ = false;
};

inline bool is_sep(char c) { return c == ' ' || c == '\t' || c == '\n' || c == ','; }

int arff_threads() {
    if (const char* e = std::getenv("KNN_ARFF_THREADS")) {
        int t = std::atoi(e);
        if (t >= 1) return t;
    }
    unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hw, 16u));
}

// All-NUMERIC data section [beg, end) of b -> P->values/kinds/n.  Returns false (P
// untouched) when the section holds anything outside the plain grammar "token (',' |
// whitespace) whitespace*" with every token a number; the caller then runs the lexer.
bool parse_numeric_parallel(const std::vector<char>& b, size_t beg, ParsedArff* P) {
    const size_t end = b.size(), na = P->attrs.size();
    const int T = arff_threads();
    if (T < 2 || na == 0 || end <= beg) return false;
    const char* d = b.data();
    // chunk c owns the tokens that START in [cut[c], cut[c+1])
    std::vector<size_t> cut(T + 1);
    for (int c = 0; c <= T; c++) cut[c] = beg + (end - beg) * (size_t)c / (size_t)T;
    std::vector<int64_t> count(T, 0);
    std::vector<char> bad(T, 0);
    auto token_start = [&](size_t i) { return !is_sep(d[i]) && (i == beg || is_sep(d[i - 1])); };
    auto scan = [&](int c) {
        int64_t n = 0;
        for (size_t i = cut[c]; i < cut[c + 1]; i++) {
            const char ch = d[i];
            if (ch == '?' || ch == '\'' || ch == '"' || ch == '{' || ch == '}' || ch == '%' || ch == '\0') { bad[c] = 1; return; }
            if (ch == ',' && (i == beg || is_sep(d[i - 1]))) { bad[c] = 1; return; }
            if (token_start(i)) n++;
        }
        count[c] = n;
    };
    {
        std::vector<std::thread> th;
        for (int c = 1; c < T; c++) th.emplace_back(scan, c);
        scan(0);
        for (auto& t : th) t.join();
    }
    for (int c = 0; c < T; c++) if (bad[c]) return false;
    std::vector<int64_t> first(T + 1, 0);
    for (int c = 0; c < T; c++) first[c + 1] = first[c] + count[c];
    const int64_t n = first[T] / (int64_t)na;  // a partial last instance is dropped (libarff)
    std::vector<float> values((size_t)(n * (int64_t)na));
    auto conv = [&](int c) {
        int64_t g = first[c];
        for (size_t i = cut[c]; i < cut[c + 1] && g < n * (int64_t)na; i++) {
            if (!token_start(i)) continue;
            size_t j = i;
            while (j < end && !is_sep(d[j])) j++;
            float v;
            if (!parse_float_like_istream(d + i, j - i, &v)) { bad[c] = 1; return; }
            values[(size_t)g++] = v;
            i = j - 1;
        }
    };
    {
        std::vector<std::thread> th;
        for (int c = 1; c < T; c++) th.emplace_back(conv, c);
        conv(0);
        for (auto& t : th) t.join();
    }
    for (int c = 0; c < T; c++) if (bad[c]) return false;
    P->values = std::move(values);
    P->kinds.assign(P->values.size(), (uint8_t)K_FLOAT);
    P->n = n;
    return true;
}

std::unique_ptr<ParsedArff> parse_file(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throwf("ArffScanner: failed to open the file '%s'!", path.c_str());
    std::vector<char> buf;
    if (std::fseek(f, 0, SEEK_END) == 0) {
        const long sz = std::ftell(f);
        if (sz > 0) buf.resize((size_t)sz);
        std::rewind(f);
    }
    size_t got = buf.empty() ? 0 : std::fread(buf.data(), 1, buf.size(), f);
    buf.resize(got);
    char chunk[1 << 16];
    size_t r;
    while ((r = std::fread(chunk, 1, sizeof(chunk), f)) > 0) buf.insert(buf.end(), chunk, chunk + r);
    std::fclose(f);
    Lexer lx(std::move(buf));
    auto P = std::make_unique<ParsedArff>();
    std::string s;
    if (lx.next(s) != T_RELATION) throwf("ArffParser::_read_relation: First token must be of 'RELATION'!");
    if (lx.next(s) != T_VALUE) throwf("ArffParser::_read_relation: RELATION token must be followed by VALUE_TOKEN!");
    P->relation = s;
    for (;;) {
        Tok t = lx.next(s);
        if (t == T_DATA || t == T_EOF) break;
        if (t != T_ATTRIBUTE) throwf("ArffParser::_read_attrs: First token must be of 'ATTRIBUTE'!");
        ParsedAttr a;
        if (lx.next(a.name) != T_VALUE) throwf("ArffParser::_read_attr: 'ATTRIBUTE' must be followed by a 'VALUE_TOKEN'!");
        Tok ty = lx.next(s);
        switch (ty) {
            case T_NUMERIC: a.type = NUMERIC; break;
            case T_STRING: a.type = STRING; break;
            case T_DATE: a.type = DATE; break;
            case T_BOPEN: a.type = NOMINAL; break;
            default: throwf("ArffParser::_read_attr: Bad attribute type for name=%s attr-type=%s!", a.name.c_str(), s.c_str());
        }
        if (a.type == NOMINAL) {
            for (;;) {
                Tok v = lx.next(s);
                if (v == T_VALUE) a.nominal.push_back(s);
                else if (v == T_BCLOSE) break;
                else throwf("ArffParser::_read_attr: For nominal values expecting 'VALUE_TOKEN'!");
            }
        }
        P->attrs.push_back(std::move(a));
    }
    const size_t na = P->attrs.size();
    bool all_numeric = na > 0;
    for (auto& a : P->attrs) all_numeric = all_numeric && a.type == NUMERIC;
    if (all_numeric && parse_numeric_parallel(lx.buffer(), lx.pos(), P.get())) return P;
    std::vector<float> rv(na);
    std::vector<uint8_t> rk(na);
    std::vector<std::pair<size_t, std::string>> rs;
    for (;;) {
        rs.clear();
        bool eof = false;
        for (size_t i = 0; i < na; i++) {
            Tok t = lx.next(s);
            if (t == T_EOF) { eof = true; break; }
            if (t != T_VALUE && t != T_MISSING)
                throwf("ArffParser::_read_instances expects 'VALUE_TOKEN' or 'MISSING_TOKEN'!");
            const ParsedAttr& a = P->attrs[i];
            if (t == T_MISSING) { rk[i] = K_MISSING; rv[i] = 0.f; continue; }
            if (a.type == NUMERIC) {
                float v;
                if (parse_float_like_istream(s.data(), s.size(), &v)) { rk[i] = K_FLOAT; rv[i] = v; }
                else throwf("ArffData: attr-name=%s attr-type=NUMERIC, but inst-type=STRING!", a.name.c_str());
            } else if (a.type == STRING || a.type == NOMINAL) {
                if (a.type == NOMINAL) {
                    bool found = false;
                    for (auto& nv : a.nominal) if (nv == s) { found = true; break; }
                    if (!found) throwf("ArffData: attr:(name=%s type=NOMINAL) inst-val=%s not found!", a.name.c_str(), s.c_str());
                }
                rk[i] = a.type == STRING ? K_STRING : K_NOMINAL;
                rv[i] = 0.f;
                rs.emplace_back(i, s);
            } else {
                // libarff adds no value for DATE fields, then the cross-check indexes past the end
                throwf("ArffInstance::get Index out of bounds! (DATE attribute '%s' is not supported by libarff)", a.name.c_str());
            }
        }
        if (eof) break;
        P->values.insert(P->values.end(), rv.begin(), rv.end());
        P->kinds.insert(P->kinds.end(), rk.begin(), rk.end());
        for (auto& e : rs) P->strs.emplace(P->n * (int64_t)na + (int64_t)e.first, std::move(e.second));
        P->n++;
    }
    return P;
}

const char* kind_name(uint8_t k) {
    return k == K_STRING ? "STRING" : k == K_NOMINAL ? "NOMINAL" : k == K_MISSING ? "NUMERIC" : "FLOAT";
}

}  // namespace

uint64_t knn_flat_view_uid() {
    static std::atomic<uint64_t> next{1};
    return next.fetch_add(1, std::memory_order_relaxed);
}

int knn_ctx_device(const knn_ctx* c);  // (knn_capi.cpp: the device a context drives)
void* knn_ctx_stream(const knn_ctx* c);  // (knn_capi.cpp: its stream)

namespace {

// Flatten features [0, na-1) and the class attribute with operator float semantics.
void flatten(const ParsedArff& P, KnnFlatView* out) {
    const int na = (int)P.attrs.size();
    if (na < 1) throwf("ArffData: no attributes");
    out->n = P.n;
    out->d = na - 1;
    out->ld = (out->d + 3) & ~3;
    if (out->ld == 0) out->ld = 4;
    out->feat.assign((size_t)out->n * out->ld, 0.f);
    out->labels.assign((size_t)out->n, 0);
    for (int64_t r = 0; r < P.n; r++) {
        for (int c = 0; c < na; c++) {
            uint8_t k = P.kinds[(size_t)r * na + c];
            if (k != K_FLOAT) throwf("operator float cannot work on type '%s'!", kind_name(k));
            float v = P.values[(size_t)r * na + c];
            if (c < na - 1) out->feat[(size_t)r * out->ld + c] = v;
            else out->labels[(size_t)r] = (int32_t)v;
        }
    }
}

// ---------------------------------------------------------------------------------
// device contexts for the C++ API: one per visible GPU, created once
// ---------------------------------------------------------------------------------
struct Devices {
    std::vector<knn_ctx*> ctx;
    // a knn_ctx serves one call at a time: the reference's pthreads driver calls KNN from
    // numThreads threads at once (multi-thread.cpp:170-192), so calls that land on the same
    // device queue here (the device runs them back to back either way)
    std::vector<std::unique_ptr<std::mutex>> busy;
    std::mutex mu;
};
Devices& devices() {
    static Devices* D = new Devices();  // intentionally leaked: no HIP teardown at exit
    return *D;
}

std::vector<knn_ctx*>& contexts() {
    Devices& D = devices();
    std::lock_guard<std::mutex> g(D.mu);
    if (D.ctx.empty()) {
        int n = knn_amd_num_devices();
        int phys = 0;
        if (hipGetDeviceCount(&phys) != hipSuccess || phys < 1) phys = 1;
        for (int i = 0; i < n; i++) {
            knn_opts o{i % phys, KNN_ALGO_AUTO, 0, 0, KNN_OPT_CACHE_TRAIN};  // ArffData is immutable once parsed
            knn_ctx* c = nullptr;
            knn_status s = knn_create(&c, &o);
            if (s != KNN_OK) {
                if (i == 0) throwf("KNN: no usable gfx950 device (knn_create status %d)", (int)s);
                break;
            }
            D.ctx.push_back(c);
            D.busy.emplace_back(new std::mutex());
        }
    }
    return D.ctx;
}

// The partition KNN() uses over G devices: KNN_AMD_SHARD = test (default: the reference's rule,
// queries split, train replicated), train (train rows split, per-shard top-k merged) or auto
// (knn_shard_policy: train-sharded when one copy of train does not fit a device)
int shard_mode(int64_t nt, int64_t nq, int d, int G) {
    const char* e = std::getenv("KNN_AMD_SHARD");
    if (G <= 1 || !e || !std::strcmp(e, "test")) return KNN_SHARD_TEST;
    if (!std::strcmp(e, "train")) return KNN_SHARD_TRAIN;
    if (std::strcmp(e, "auto")) throwf("KNN: KNN_AMD_SHARD=%s (test, train or auto)", e);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) tot = 0;
    int32_t p = KNN_SHARD_TEST;
    if (knn_shard_policy(nt, nq, d, KNN_F32, G, (int64_t)tot, &p) != KNN_OK) p = KNN_SHARD_TEST;
    return p;
}

// device buffer of one call (freed on every exit path)
struct DevMem {
    void* p = nullptr;
    int dev = 0;
    DevMem(int device, size_t bytes) : dev(device) {
        if (hipSetDevice(dev) != hipSuccess || hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) p = nullptr;
    }
    ~DevMem() {
        if (p) { (void)hipSetDevice(dev); (void)hipFree(p); }
    }
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
};

// Train-sharded KNN() over G devices (the reference only splits the test set):
// device g holds train rows shard_range(n, G, g) and the queries [q0, q1), and computes its
// shard's exact top-k of every query as (distance bits, global index, label) records
// (knn_shard_topk_device); device 0 gathers the G record blocks and merges them by (distance,
// global index) -- the reference's lower-index tie rule over the whole train set -- and votes
// (knn_merge_vote_device).  Bit-identical to the test-sharded result.
void predict_range_train_sharded(const KnnFlatView& tr, const KnnFlatView& te, int k, int C, int64_t q0, int64_t q1,
                                 int* out, std::vector<knn_ctx*>& cs, int G) {
    const int64_t nq = q1 - q0;
    const size_t recb = sizeof(int32_t) * 3 * (size_t)k * (size_t)nq;
    std::vector<std::unique_ptr<DevMem>> rec(G);
    std::vector<knn_status> st(G, KNN_OK);
    std::vector<std::string> why(G);
    std::vector<std::thread> th;
    for (int g = 0; g < G; g++) {
        auto job = [&, g]() {
            std::lock_guard<std::mutex> busy(*devices().busy[g]);
            int64_t t0 = 0, t1 = 0;
            knn_shard_range(tr.n, G, g, &t0, &t1);
            const size_t tb = sizeof(float) * (size_t)tr.ld * (size_t)(t1 - t0), qb = sizeof(float) * (size_t)te.ld * (size_t)nq;
            const int dev = knn_ctx_device(cs[g]);
            DevMem dt(dev, tb), dl(dev, sizeof(int32_t) * (size_t)(t1 - t0)), dq(dev, qb);
            rec[g].reset(new DevMem(dev, recb));
            if (!dt.p || !dl.p || !dq.p || !rec[g]->p) { st[g] = KNN_ENOMEM; why[g] = "device allocation"; return; }
            // uploads on the context's own stream, so the shard pass is ordered after them (a
            // null-stream hipMemcpy may return before its DMA lands, and the context's stream
            // does not wait for the null stream)
            hipStream_t sg = (hipStream_t)knn_ctx_stream(cs[g]);
            if (hipMemcpyAsync(dt.p, tr.feat.data() + (size_t)t0 * tr.ld, tb, hipMemcpyHostToDevice, sg) != hipSuccess ||
                hipMemcpyAsync(dl.p, tr.labels.data() + t0, sizeof(int32_t) * (size_t)(t1 - t0), hipMemcpyHostToDevice,
                               sg) != hipSuccess ||
                hipMemcpyAsync(dq.p, te.feat.data() + (size_t)q0 * te.ld, qb, hipMemcpyHostToDevice, sg) != hipSuccess) {
                st[g] = KNN_EHIP; why[g] = "upload"; return;
            }
            knn_dataset dtr{dt.p, (const int32_t*)dl.p, t1 - t0, tr.d, tr.ld, KNN_F32};
            knn_dataset dte{dq.p, nullptr, nq, te.d, te.ld, KNN_F32};
            st[g] = knn_shard_topk_device(cs[g], &dtr, &dte, k, C, t0, (int32_t*)rec[g]->p, sg);
            if (st[g] != KNN_OK) why[g] = knn_last_error(cs[g]);
        };
        th.emplace_back(job);
    }
    for (auto& t : th) t.join();
    for (int g = 0; g < G; g++)
        if (st[g] != KNN_OK) throwf("KNN (train-sharded, device %d): %s (status %d)", g, why[g].c_str(), (int)st[g]);
    // the exchange: every shard's records to device 0, [G][nq][3][k]
    std::lock_guard<std::mutex> busy(*devices().busy[0]);
    const int dev0 = knn_ctx_device(cs[0]);
    DevMem all(dev0, recb * (size_t)G), pred(dev0, sizeof(int32_t) * (size_t)nq);
    if (!all.p || !pred.p) throwf("KNN (train-sharded): device allocation failed");
    // the gather on device 0's context stream, ahead of the merge on the same stream (round 5: a
    // null-stream hipMemcpyPeer returned before its copy landed and the merge, on the context's
    // non-blocking stream, read half-copied records -- "a train label is outside [0, C)")
    (void)hipSetDevice(dev0);
    hipStream_t s0 = (hipStream_t)knn_ctx_stream(cs[0]);
    for (int g = 0; g < G; g++)
        if (hipMemcpyPeerAsync((char*)all.p + recb * (size_t)g, dev0, rec[g]->p, rec[g]->dev, recb, s0) != hipSuccess)
            throwf("KNN (train-sharded): copy of shard %d's lists failed", g);
    const knn_status s = knn_merge_vote_device(cs[0], G, nq, k, C, (const int32_t*)all.p, (int32_t*)pred.p, nullptr,
                                               nullptr, s0);
    if (s != KNN_OK) throwf("KNN (train-sharded merge): %s (status %d)", knn_last_error(cs[0]), (int)s);
    if (hipMemcpy(out, pred.p, sizeof(int32_t) * (size_t)nq, hipMemcpyDeviceToHost) != hipSuccess)
        throwf("KNN (train-sharded): download failed");
}

// predictions for test rows [q0, q1), sharded over the devices by the reference rule
void predict_range(ArffData* train, ArffData* test, int k, int64_t q0, int64_t q1, int* out) {
    const int64_t nq = q1 - q0;
    if (nq <= 0) return;
    if (k <= 0) {  // main.cpp:65-76 with no candidates: every argmax is class 0
        std::memset(out, 0, sizeof(int) * (size_t)nq);
        return;
    }
    const KnnFlatView& tr = train->flat();
    const KnnFlatView& te = test->flat();
    const int C = (int)train->num_classes();
    if (tr.d != te.d) throwf("KNN: train has %d features, test has %d", tr.d, te.d);
    if (k > tr.n) throwf("KNN: k=%d exceeds the %lld train instances", k, (long long)tr.n);
    knn_dataset dtr{tr.feat.data(), tr.labels.data(), tr.n, tr.d, tr.ld, KNN_F32};
    knn_dataset dte{te.feat.data(), nullptr, te.n, te.d, te.ld, KNN_F32};
    std::vector<knn_ctx*>& cs = contexts();
    if (cs.size() > 1 && shard_mode(tr.n, nq, tr.d, (int)std::min<int64_t>((int64_t)cs.size(), tr.n)) == KNN_SHARD_TRAIN)
        return predict_range_train_sharded(tr, te, k, C, q0, q1, out, cs, (int)std::min<int64_t>((int64_t)cs.size(), tr.n));
    const int G = (int)std::min<int64_t>((int64_t)cs.size(), nq);
    std::vector<knn_status> st(G, KNN_OK);
    std::vector<std::thread> th;
    const int64_t per = nq / G, left = nq % G;
    int64_t s = q0;
    for (int g = 0; g < G; g++) {
        const int64_t e = s + per + (g == G - 1 ? left : 0);
        int32_t* dst = reinterpret_cast<int32_t*>(out) + (s - q0);
        auto job = [&, g, s, e, dst]() {
            std::lock_guard<std::mutex> busy(*devices().busy[g]);
            // the train cache hits only for this very flat view (a freed ArffData's buffers can
            // be handed to the next one at the same address)
            st[g] = knn_set_generation(cs[g], tr.uid);
            if (st[g] == KNN_OK) st[g] = knn_predict(cs[g], &dtr, &dte, k, C, s, e, dst, nullptr, nullptr);
        };
        if (G == 1) job(); else th.emplace_back(job);
        s = e;
    }
    for (auto& t : th) t.join();
    for (int g = 0; g < G; g++)
        if (st[g] != KNN_OK) throwf("KNN: %s (status %d)", knn_last_error(cs[g]), (int)st[g]);
}

}  // namespace

// ---------------------------------------------------------------------------------
// libarff-compatible classes
// ---------------------------------------------------------------------------------
std::string arff_value2str(ArffValueEnum e) {
    switch (e) {
        case INTEGER: return "INTEGER";
        case FLOAT: return "FLOAT";
        case DATE: return "DATE";
        case STRING: return "STRING";
        case NUMERIC: return "NUMERIC";
        case NOMINAL: return "NOMINAL";
        default: return "UNKNOWN";
    }
}

ArffValue::ArffValue(int32 i) : m_float(0.f), m_int(i), m_type(INTEGER), m_missing(false) {}
ArffValue::ArffValue(float f) : m_float(f), m_int(0), m_type(FLOAT), m_missing(false) {}
ArffValue::ArffValue(const std::string& str) : m_float(0.f), m_int(0), m_type(STRING), m_missing(false), m_str(str) {
    float v;
    if (parse_float_like_istream(str.data(), str.size(), &v)) { m_type = FLOAT; m_float = v; }
}
ArffValue::ArffValue(const std::string& str, ArffValueEnum t) : m_float(0.f), m_int(0), m_type(t), m_missing(false), m_str(str) {}
ArffValue::ArffValue(ArffValueEnum t) : m_float(0.f), m_int(0), m_type(t), m_missing(true) {}
void ArffValue::set(int32 i) { m_type = INTEGER; m_int = i; }
void ArffValue::set(float f) { m_type = FLOAT; m_float = f; }
void ArffValue::set(const std::string& str, ArffValueEnum e) {
    if (e != DATE && e != STRING && e != NOMINAL)
        throwf("ArffValue::set expects 'DATE' or 'STRING', you've passed '%s'!", arff_value2str(e).c_str());
    m_type = e;
    m_str = str;
}
bool ArffValue::missing() const { return m_missing; }
ArffValueEnum ArffValue::type() const { return m_type; }
ArffValue::operator int32() const {
    if (m_type == INTEGER) return m_int;
    if (m_type == FLOAT) return (int32)m_float;
    throwf("operator int32 cannot work on type '%s'!", arff_value2str(m_type).c_str());
}
ArffValue::operator float() const {
    if (m_type == INTEGER) return (float)m_int;
    if (m_type == FLOAT) return m_float;
    throwf("operator float cannot work on type '%s'!", arff_value2str(m_type).c_str());
}
ArffValue::operator std::string() const {
    if (m_type == INTEGER) return std::to_string(m_int);
    if (m_type == FLOAT) {
        char b[64];
        std::snprintf(b, sizeof(b), "%g", (double)m_float);
        return b;
    }
    return m_str;
}

ArffAttr::ArffAttr(const std::string& name, ArffValueEnum type) : m_name(name), m_enum(type) {}
std::string ArffAttr::name() const { return m_name; }
ArffValueEnum ArffAttr::type() const { return m_enum; }

ArffInstance::ArffInstance() {}
ArffInstance::~ArffInstance() { for (ArffValue* v : m_data) delete v; }
int32 ArffInstance::size() const { return (int32)m_data.size(); }
void ArffInstance::add(ArffValue* val) { m_data.push_back(val); }
ArffValue* ArffInstance::get(int idx) const {
    if (idx < 0 || (size_t)idx >= m_data.size())
        throwf("ArffInstance::get Index out of bounds! idx=%d size=%d", idx, (int)m_data.size());
    return m_data[idx];
}

ArffData::ArffData() {}
ArffData::~ArffData() {
    for (ArffAttr* a : m_attrs) delete a;
    for (ArffInstance* i : m_instances) delete i;
}
void ArffData::set_relation_name(const std::string& name) { m_rel = name; }
std::string ArffData::get_relation_name() const { return m_rel; }
int32 ArffData::num_attributes() const { return (int32)m_attrs.size(); }
int32 ArffData::num_classes() {
    if (m_num_classes >= 0) return m_num_classes;
    int32 mx = 0;
    const int32 last = num_attributes() - 1;
    for (ArffInstance* in : m_instances) {
        int32 c = (int32)(*in->get((int)last));
        if (c > mx) mx = c;
    }
    m_num_classes = mx + 1;
    return m_num_classes;
}
void ArffData::add_attr(ArffAttr* attr) { m_attrs.push_back(attr); }
ArffAttr* ArffData::get_attr(int32 idx) const {
    if (idx < 0 || (size_t)idx >= m_attrs.size())
        throwf("ArffData::get_attr index out of bounds! idx=%ld size=%d", idx, (int)m_attrs.size());
    return m_attrs[idx];
}
int32 ArffData::num_instances() const { return (int32)m_instances.size(); }
void ArffData::cross_check(const ArffInstance* inst) {
    if (!inst) throwf("ArffData: input instance pointer is null!");
    for (size_t i = 0; i < m_attrs.size(); i++) {
        ArffValue* v = inst->get((int)i);
        ArffValueEnum vt = v->type(), at = m_attrs[i]->type();
        bool bad_num = at == NUMERIC && vt != INTEGER && vt != FLOAT && vt != NUMERIC;
        bool bad_nom = at == NOMINAL && vt != STRING && vt != NOMINAL;
        if (bad_num || bad_nom || (at != NUMERIC && at != NOMINAL && at != vt))
            throwf("ArffData: attr-name=%s attr-type=%s, but inst-type=%s!", m_attrs[i]->name().c_str(),
                   arff_value2str(at).c_str(), arff_value2str(vt).c_str());
    }
}
void ArffData::add_instance(ArffInstance* inst) {
    cross_check(inst);
    m_instances.push_back(inst);
    m_num_classes = -1;
}
ArffInstance* ArffData::get_instance(int32 idx) const {
    if (idx < 0 || (size_t)idx >= m_instances.size())
        throwf("ArffData::get_instance index out of bounds! idx=%ld size=%d", idx, (int)m_instances.size());
    return m_instances[idx];
}
void ArffData::add_nominal_val(const std::string& name, const std::string& val) { m_nominals[name].push_back(val); }
std::vector<std::string> ArffData::get_nominal(const std::string& name) {
    auto it = m_nominals.find(name);
    if (it == m_nominals.end()) throwf("ArffData::get_nominal list named '%s' does not exist!", name.c_str());
    return it->second;
}

const KnnFlatView& ArffData::flat() const {
    std::call_once(m_flat_once, [this]() {
        auto v = std::make_unique<KnnFlatView>();
        const int na = (int)m_attrs.size();
        if (na < 1) throwf("ArffData: no attributes");
        v->n = (int64_t)m_instances.size();
        v->d = na - 1;
        v->ld = std::max(4, (v->d + 3) & ~3);
        v->feat.assign((size_t)v->n * v->ld, 0.f);
        v->labels.assign((size_t)v->n, 0);
        for (int64_t r = 0; r < v->n; r++) {
            const ArffInstance* in = m_instances[(size_t)r];
            for (int c = 0; c < na - 1; c++) v->feat[(size_t)r * v->ld + c] = (float)(*in->get(c));
            v->labels[(size_t)r] = (int32_t)(float)(*in->get(na - 1));  // main.cpp:57,66
        }
        m_flat = std::move(v);
    });
    return *m_flat;
}

ArffParser::ArffParser(const std::string& file) : m_file(file), m_data(nullptr) {}
ArffParser::~ArffParser() { delete m_data; }
ArffData* ArffParser::parse() {
    if (m_data) return m_data;
    std::unique_ptr<ParsedArff> P = parse_file(m_file);
    std::unique_ptr<ArffData> D(new ArffData());
    D->m_rel = P->relation;
    const size_t na = P->attrs.size();
    for (auto& a : P->attrs) {
        D->m_attrs.push_back(new ArffAttr(a.name, a.type));
        for (auto& nv : a.nominal) D->m_nominals[a.name].push_back(nv);
    }
    D->m_instances.reserve((size_t)P->n);
    bool all_float = true;
    for (int64_t r = 0; r < P->n; r++) {
        ArffInstance* in = new ArffInstance();
        for (size_t c = 0; c < na; c++) {
            const int64_t o = r * (int64_t)na + (int64_t)c;
            switch (P->kinds[(size_t)o]) {
                case K_FLOAT: in->add(new ArffValue(P->values[(size_t)o])); break;
                case K_MISSING: in->add(new ArffValue(P->attrs[c].type)); all_float = false; break;
                default: in->add(new ArffValue(P->strs[o], P->attrs[c].type)); all_float = false; break;
            }
        }
        D->m_instances.push_back(in);
    }
    if (all_float && na >= 1) {
        // pre-build the flat view straight from the parse buffers
        auto v = std::make_unique<KnnFlatView>();
        flatten(*P, v.get());
        D->m_flat = std::move(v);
        std::call_once(D->m_flat_once, []() {});
    }
    if (na >= 1) {
        // num_classes once, here (libarff/arff_data.cpp:41-57 caches it lazily and racily)
        try { D->num_classes(); } catch (...) {}
    }
    m_data = D.release();
    return m_data;
}

// ---------------------------------------------------------------------------------
// KNN entry points
// ---------------------------------------------------------------------------------
int knn_amd_num_devices() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (const char* e = std::getenv("KNN_AMD_DEVICES")) {
        int want = std::atoi(e);
        if (want > 0 && want < n) n = want;
        // KNN_AMD_SHARE_GPU=1: more workers than GPUs, worker w on GPU w % n (rehearses an
        // N-GPU partition, the train-sharded exchange included, on fewer devices)
        const char* sh = std::getenv("KNN_AMD_SHARE_GPU");
        if (want > n && n > 0 && sh && !std::strcmp(sh, "1")) n = std::min(want, 64);
    }
    return n;
}

void knn_amd_init() { (void)contexts(); }

int* KNN(ArffData* train, ArffData* test, int k) {
    const int64_t nq = test->num_instances();
    int* pred = (int*)std::malloc(sizeof(int) * (size_t)(nq > 0 ? nq : 1));
    if (!pred) throwf("KNN: out of memory");
    try {
        predict_range(train, test, k, 0, nq, pred);
    } catch (...) {
        std::free(pred);
        throw;
    }
    return pred;
}

int* KNN(ArffData* train, ArffData* test, int k, int start, int end) {
    if (start < 0 || end < start || end > test->num_instances()) throwf("KNN: bad range [%d, %d)", start, end);
    int* pred = (int*)std::malloc(sizeof(int) * (size_t)((end - start) > 0 ? (end - start) : 1));
    if (!pred) throwf("KNN: out of memory");
    try {
        predict_range(train, test, k, start, end, pred);
    } catch (...) {
        std::free(pred);
        throw;
    }
    return pred;
}

void* KNN(void* params) {
    arguments* a = static_cast<arguments*>(params);
    predict_range(a->train, a->test, a->k, a->start, a->end, predictions + a->start);
    return nullptr;
}

int* computeConfusionMatrix(int* pred, ArffData* dataset) {
    const int32 C = dataset->num_classes();
    int* cm = (int*)std::calloc((size_t)(C * C), sizeof(int));
    const int32 last = dataset->num_attributes() - 1;
    for (int32 i = 0; i < dataset->num_instances(); i++) {
        int t = (int)(int32)(*dataset->get_instance(i)->get((int)last));  // main.cpp:93
        cm[t * C + pred[i]]++;
    }
    return cm;
}

float computeAccuracy(int* cm, ArffData* dataset) {
    const int32 C = dataset->num_classes();
    int ok = 0;
    for (int32 i = 0; i < C; i++) ok += cm[i * C + i];
    return ok / (float)dataset->num_instances();
}

// ---------------------------------------------------------------------------------
// C ABI: ARFF loader (flat, no per-value objects)
// ---------------------------------------------------------------------------------
struct knn_arff {
    std::unique_ptr<ParsedArff> P;
    int32_t num_classes = 0;
};

extern "C" {

knn_status knn_arff_open(const char* path, knn_arff** out, char* err, int32_t err_len) {
    if (!path || !out) return KNN_EINVAL;
    *out = nullptr;
    try {
        auto h = std::make_unique<knn_arff>();
        h->P = parse_file(path);
        const size_t na = h->P->attrs.size();
        int32_t mx = 0;
        bool ok = na >= 1;
        for (int64_t r = 0; ok && r < h->P->n; r++) {
            size_t o = (size_t)r * na + na - 1;
            if (h->P->kinds[o] != K_FLOAT) { ok = false; break; }
            int32_t c = (int32_t)(int64_t)h->P->values[o];
            if (c > mx) mx = c;
        }
        h->num_classes = mx + 1;
        *out = h.release();
        return KNN_OK;
    } catch (const std::exception& e) {
        if (err && err_len > 0) std::snprintf(err, (size_t)err_len, "%s", e.what());
        return KNN_EIO;
    }
}

void knn_arff_shape(const knn_arff* h, int64_t* n, int32_t* na, int32_t* C) {
    if (n) *n = h ? h->P->n : 0;
    if (na) *na = h ? (int32_t)h->P->attrs.size() : 0;
    if (C) *C = h ? h->num_classes : 0;
}

knn_status knn_arff_copy(const knn_arff* h, float* feat, int32_t ld, int32_t* labels) {
    if (!h) return KNN_EINVAL;
    const int na = (int)h->P->attrs.size();
    if (na < 1 || ld < na - 1) return KNN_EINVAL;
    for (int64_t r = 0; r < h->P->n; r++) {
        for (int c = 0; c < na; c++) {
            size_t o = (size_t)r * na + c;
            if (h->P->kinds[o] != K_FLOAT) return KNN_EINVAL;
            float v = h->P->values[o];
            if (c < na - 1) { if (feat) feat[r * ld + c] = v; }
            else if (labels) labels[r] = (int32_t)v;
        }
        if (feat) for (int c = na - 1; c < ld; c++) feat[r * ld + c] = 0.f;
    }
    return KNN_OK;
}

void knn_arff_close(knn_arff* h) { delete h; }

}  // extern "C"
