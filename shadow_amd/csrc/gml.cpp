// gml.cpp — GML text -> srg_graph (host side of the ingest step in front of the routing path).
//
// Restates, for the MI355X routing builder's host code:
//   * gml_parser::parse         src/lib/gml-parser/src/lib.rs:55-60 (trailing input ignored)
//   * the nom grammar           src/lib/gml-parser/src/parser.rs:44-281
//       key        [A-Za-z_][A-Za-z0-9_]*                          :45-51
//       gml        multispace0 "graph" space0 "[" newline items* "]" multispace0   :68-150
//       node/edge  space0 "[" newline (key value)* "]" newline     :153-212
//       value      space0 ( int newline | float newline | string newline )          :214-224
//       int        digit1 -> i32 (overflow falls through to float)  :226-229
//       float      nom recognize_float -> f32 (cut after the exponent marker)        :231-234
//       string     '"' escaped_transform(is_not("\""), ...) '"'  == '"' [^"]+ '"'     :237-250
//       newline    space0 multispace1 space0                        :252-254
//   * NetworkGraph::parse       src/main/network/graph/mod.rs:134-181
//   * ShadowNode::try_from      mod.rs:28-60 (bandwidths: BitsPerSec<SiPrefixUpper>)
//   * ShadowEdge::try_from      mod.rs:72-111 (latency/jitter Time<TimePrefix>, packet_loss)
//   * units FromStr / convert   src/main/utility/units.rs:377-439 (regex ^([+-]?[0-9\.]*)\s*(.*)$)
//     TimePrefix                units.rs:218-280, SiPrefixUpper units.rs:140-200
//
// Error strings follow the reference's wording so the Rust wrapper can forward them.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <thread>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/shadow_routing.h"

struct srg_graph {
    bool directed = false;
    std::vector<uint32_t> node_id;
    std::vector<uint64_t> bw_down, bw_up;
    std::vector<int> has_down, has_up;
    std::unordered_map<uint32_t, uint32_t> id_to_index;
    std::vector<uint32_t> src, dst;
    std::vector<uint64_t> lat_ns;
    std::vector<float> loss;
    uint32_t parse_chunks = 1;
};

namespace {

// ----------------------------------------------------------------------------------------
// Zero-copy views into the GML text: one pass over the text, no allocation per key/value.
struct SV {
    const char* p = nullptr;
    uint32_t n = 0;
    bool eq(const char* s) const {
        const size_t m = std::strlen(s);
        return m == n && std::memcmp(p, s, n) == 0;
    }
    bool same(const SV& o) const { return n == o.n && std::memcmp(p, o.p, n) == 0; }
    std::string str() const { return std::string(p, n); }
};

// nom-like result: OK, ERR (recoverable: alt/many_till may try something else), FAIL (fatal)
enum class R { OK, ERR, FAIL };

struct Value {
    enum Kind { INT, FLOAT, STR } kind = INT;
    int32_t i = 0;
    float f = 0.0f;
    SV s;
};

struct KV {
    SV k;
    Value v;
};

struct Parser {
    const char* begin;
    const char* end;
    std::string fail_msg;  // for FAIL
    const char* fail_at = nullptr;

    static bool is_space(char c) { return c == ' ' || c == '\t'; }
    static bool is_mspace(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
    static bool is_alpha(unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
    static bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

    const char* space0(const char* p) const {
        while (p < end && is_space(*p)) ++p;
        return p;
    }
    const char* multispace0(const char* p) const {
        while (p < end && is_mspace(*p)) ++p;
        return p;
    }
    // newline = space0 multispace1 space0  (parser.rs:252-254)
    R newline(const char*& p) const {
        const char* q = space0(p);
        const char* r = multispace0(q);
        if (r == q) return R::ERR;  // multispace1 needs >= 1 char
        p = space0(r);
        return R::OK;
    }
    R tag(const char*& p, const char* t) const {
        size_t n = std::strlen(t);
        if ((size_t)(end - p) < n || std::memcmp(p, t, n) != 0) return R::ERR;
        p += n;
        return R::OK;
    }
    R fail(const char* at, const std::string& m) {
        fail_msg = m;
        fail_at = at;
        return R::FAIL;
    }
    // key (parser.rs:45-51): take(1) alphabetic-or-'_' (chr as u8), take_while alnum-or-'_'
    R key(const char*& p, SV& out) const {
        if (p >= end) return R::ERR;
        // take(1) takes one *char*; `chr as u8` truncates multibyte chars -> never a letter
        unsigned char c = (unsigned char)*p;
        if (!(is_alpha(c) || c == '_')) return R::ERR;
        const char* q = p + 1;
        while (q < end) {
            unsigned char d = (unsigned char)*q;
            if (is_alpha(d) || is_digit(d) || d == '_') {
                ++q;
                continue;
            }
            if (d >= 0x80) {
                // multibyte char: (chr as u8) of the code point -> check its low byte
                int len = (d >= 0xF0) ? 4 : (d >= 0xE0) ? 3 : (d >= 0xC0) ? 2 : 1;
                if (q + len > end) break;
                uint32_t cp = 0;
                if (len == 2) cp = ((d & 0x1F) << 6) | (q[1] & 0x3F);
                else if (len == 3) cp = ((d & 0x0F) << 12) | ((q[1] & 0x3F) << 6) | (q[2] & 0x3F);
                else if (len == 4)
                    cp = ((d & 0x07) << 18) | ((q[1] & 0x3F) << 12) | ((q[2] & 0x3F) << 6) | (q[3] & 0x3F);
                unsigned char lo = (unsigned char)(cp & 0xFF);
                if (len > 1 && (is_alpha(lo) || is_digit(lo) || lo == '_')) {
                    q += len;
                    continue;
                }
            }
            break;
        }
        out.p = p;
        out.n = (uint32_t)(q - p);
        p = q;
        return R::OK;
    }
    // int (parser.rs:226-229)
    R int_(const char*& p, Value& v) const {
        const char* q = p;
        int64_t acc = 0;
        bool ovf = false;
        while (q < end && is_digit((unsigned char)*q)) {
            acc = acc * 10 + (*q - '0');
            ovf |= acc > INT32_MAX;
            if (ovf) acc = INT32_MAX + 1ll;
            ++q;
        }
        if (q == p) return R::ERR;
        if (ovf) return R::ERR;  // str::parse::<i32>: overflow -> map_res error (ERR)
        v.kind = Value::INT;
        v.i = (int32_t)acc;
        p = q;
        return R::OK;
    }
    // float = recognize_float (nom 7.1.3) -> str::parse::<f32> (parser.rs:231-234)
    R float_(const char*& p, Value& v) {
        const char* q = p;
        if (q < end && (*q == '+' || *q == '-')) ++q;
        if (q < end && is_digit((unsigned char)*q)) {
            while (q < end && is_digit((unsigned char)*q)) ++q;
            if (q < end && *q == '.') {
                ++q;
                while (q < end && is_digit((unsigned char)*q)) ++q;
            }
        } else if (q < end && *q == '.' && q + 1 < end && is_digit((unsigned char)q[1])) {
            q += 1;
            while (q < end && is_digit((unsigned char)*q)) ++q;
        } else {
            return R::ERR;
        }
        if (q < end && (*q == 'e' || *q == 'E')) {
            const char* e = q + 1;
            if (e < end && (*e == '+' || *e == '-')) ++e;
            const char* d = e;
            while (e < end && is_digit((unsigned char)*e)) ++e;
            if (e == d) return fail(d, "expected exponent digits in float");  // cut(digit1)
            q = e;
        }
        // Rust's f32 parse is correctly rounded.  Fast path (Clinger): a mantissa < 2^24 and a
        // power of ten <= 10^10 are both exact floats, so one IEEE division rounds correctly.
        {
            const char* c = p;
            const bool neg = *c == '-';
            if (*c == '+' || *c == '-') ++c;
            uint32_t m = 0;
            int digits = 0, frac = 0;
            bool ok = true, dot = false;
            for (; c < q; ++c) {
                if (*c == '.') { dot = true; continue; }
                if (*c == 'e' || *c == 'E') { ok = false; break; }
                if (m == 0 && *c == '0') { if (dot) ++frac; continue; }  // leading zeros
                if (++digits > 7) { ok = false; break; }
                m = m * 10 + (uint32_t)(*c - '0');
                if (dot) ++frac;
            }
            if (ok && frac <= 10) {
                static const float p10[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
                const float f = (float)m / p10[frac];
                v.kind = Value::FLOAT;
                v.f = neg ? -f : f;
                p = q;
                return R::OK;
            }
        }
        const size_t len = (size_t)(q - p);
        char small[64];
        std::string big;
        char* txt = small;
        if (len < sizeof small) {
            std::memcpy(small, p, len);
            small[len] = 0;
        } else {
            big.assign(p, q);
            txt = &big[0];
        }
        char* ep = nullptr;
        const float f = std::strtof(txt, &ep);
        if (ep != txt + len) return R::ERR;
        v.kind = Value::FLOAT;
        v.f = f;
        p = q;
        return R::OK;
    }
    // string (parser.rs:237-250): '"' then a NON-EMPTY run of non-quote bytes then '"'
    R string_(const char*& p, Value& v) const {
        if (p >= end || *p != '"') return R::ERR;
        const char* s = p + 1;
        const char* q = static_cast<const char*>(std::memchr(s, '"', (size_t)(end - s)));
        if (!q) return R::ERR;        // Eof
        if (q == s) return R::ERR;    // escaped_transform at index 0 -> Error
        v.kind = Value::STR;
        v.s.p = s;
        v.s.n = (uint32_t)(q - s);
        p = q + 1;
        return R::OK;
    }
    // value (parser.rs:214-224): int newline | float newline | string newline
    R value(const char*& p, Value& v) {
        const char* start = space0(p);
        if (start < end && *start == '"') {  // int_ and float_ both fail on '"'
            const char* q = start;
            if (string_(q, v) == R::OK && newline(q) == R::OK) {
                p = q;
                return R::OK;
            }
            return R::ERR;
        }
        {
            const char* q = start;
            if (int_(q, v) == R::OK && newline(q) == R::OK) {
                p = q;
                return R::OK;
            }
        }
        {
            const char* q = start;
            R r = float_(q, v);
            if (r == R::FAIL) return r;
            if (r == R::OK && newline(q) == R::OK) {
                p = q;
                return R::OK;
            }
        }
        {
            const char* q = start;
            if (string_(q, v) == R::OK && newline(q) == R::OK) {
                p = q;
                return R::OK;
            }
        }
        return R::ERR;
    }

    // many_till(tuple((key, value)), tag("]")) + duplicate check + newline (kvs reused: no alloc)
    R block(const char*& p, std::vector<KV>& kvs) {
        kvs.clear();
        const char* q = space0(p);
        if (tag(q, "[") != R::OK) return R::ERR;
        if (newline(q) != R::OK) return R::ERR;
        for (;;) {
            if (tag(q, "]") == R::OK) break;
            KV kv;
            if (key(q, kv.k) != R::OK) return R::ERR;
            R r = value(q, kv.v);
            if (r != R::OK) return r;
            kvs.push_back(kv);
        }
        for (size_t a = 1; a < kvs.size(); ++a)
            for (size_t b = 0; b < a; ++b)
                if (kvs[a].k.same(kvs[b].k)) return fail(q, "Duplicate keys are not supported");
        if (newline(q) != R::OK) return R::ERR;
        p = q;
        return R::OK;
    }
};

// ---------------- units (units.rs), on views --------------------------------------------
bool is_unicode_ws(const char*& p, const char* end) {
    unsigned char c = (unsigned char)*p;
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) {
        p += 1;
        return true;
    }
    // U+0085, U+00A0 (2 bytes), U+1680, U+2000-200A, U+2028, U+2029, U+202F, U+205F, U+3000
    if (c == 0xC2 && p + 1 < end && ((unsigned char)p[1] == 0x85 || (unsigned char)p[1] == 0xA0)) {
        p += 2;
        return true;
    }
    if (p + 2 < end) {
        unsigned char b1 = (unsigned char)p[1], b2 = (unsigned char)p[2];
        uint32_t cp = ((c & 0x0F) << 12) | ((b1 & 0x3F) << 6) | (b2 & 0x3F);
        if ((c & 0xF0) == 0xE0 &&
            (cp == 0x1680 || (cp >= 0x2000 && cp <= 0x200A) || cp == 0x2028 || cp == 0x2029 ||
             cp == 0x202F || cp == 0x205F || cp == 0x3000)) {
            p += 3;
            return true;
        }
    }
    return false;
}

SV utrim(SV s) {
    const char* b = s.p;
    const char* e = s.p + s.n;
    {  // ASCII fast path: no byte >= 0x80 at either end after trimming ASCII white space
        const char* fb = b;
        const char* fe = e;
        auto ws = [](char c) { return c == ' ' || (c >= 0x09 && c <= 0x0D); };
        while (fb < fe && ws(*fb)) ++fb;
        while (fe > fb && ws(fe[-1])) --fe;
        if ((fb == fe || (unsigned char)*fb < 0x80) && (fe == fb || (unsigned char)fe[-1] < 0x80)) {
            SV r;
            r.p = fb;
            r.n = (uint32_t)(fe - fb);
            return r;
        }
    }
    while (b < e) {
        const char* q = b;
        if (!is_unicode_ws(q, e)) break;
        b = q;
    }
    // trim end: scan forward remembering the last non-ws end
    const char* last = b;
    const char* p = b;
    while (p < e) {
        const char* q = p;
        if (is_unicode_ws(q, e)) {
            p = q;
        } else {
            unsigned char c = (unsigned char)*p;
            int len = (c >= 0xF0) ? 4 : (c >= 0xE0) ? 3 : (c >= 0xC0) ? 2 : 1;
            p += len;
            last = p;
        }
    }
    SV r;
    r.p = b;
    r.n = (uint32_t)((last > e ? e : last) - b);
    return r;
}

// regex ^([+-]?[0-9\.]*)\s*(.*)$  -> (value, unit), both trimmed (units.rs:409-417)
bool split_value_unit(SV s, SV& val, SV& unit) {
    const char* p = s.p;
    const char* e = s.p + s.n;
    const char* v0 = p;
    if (p < e && (*p == '+' || *p == '-')) ++p;
    while (p < e && ((*p >= '0' && *p <= '9') || *p == '.')) ++p;
    val.p = v0;
    val.n = (uint32_t)(p - v0);
    while (p < e) {
        const char* q = p;
        if (!is_unicode_ws(q, e)) break;
        p = q;
    }
    if (std::memchr(p, '\n', (size_t)(e - p))) return false;  // `.` does not match '\n'
    unit.p = p;
    unit.n = (uint32_t)(e - p);
    val = utrim(val);
    unit = utrim(unit);
    return true;
}

// Rust u64::from_str: optional '+', then >= 1 ASCII digit, no overflow.
bool parse_u64(SV s, uint64_t& out, const char*& err) {
    size_t i = 0;
    if (i < s.n && s.p[i] == '+') ++i;
    if (i == s.n) {
        err = s.n == 0 ? "cannot parse integer from empty string" : "invalid digit found in string";
        return false;
    }
    unsigned __int128 acc = 0;
    for (; i < s.n; ++i) {
        if (s.p[i] < '0' || s.p[i] > '9') {
            err = "invalid digit found in string";
            return false;
        }
        acc = acc * 10 + (unsigned)(s.p[i] - '0');
        if (acc > UINT64_MAX) {
            err = "number too large to fit in target type";
            return false;
        }
    }
    out = (uint64_t)acc;
    return true;
}

const char* kTimeUnitErr =
    "Unit was not one of (ns|nanosecond|nanoseconds|us|μs|microsecond|microseconds"
    "|ms|millisecond|milliseconds|s|sec|secs|second|seconds|m|min|mins|minute|minutes"
    "|h|hr|hrs|hour|hours)";

// Time<TimePrefix>::from_str + convert(Nano) magnitude (units.rs:236-280, 377-388, 405-439).
// Returns false with `err` on a parse error; `ns_overflow` set if the ns value overflows u64.
bool parse_time_ns(SV s, uint64_t& value, uint64_t& ns, bool& ns_overflow, const char*& err) {
    SV v, u;
    if (!split_value_unit(s, v, u)) {
        err = "Unable to identify value and unit";
        return false;
    }
    // Time suffixes = [""]: strip_suffix("") always succeeds -> prefix = unit
    uint64_t mag;
    if (u.n == 0 || u.eq("s") || u.eq("sec") || u.eq("secs") || u.eq("second") || u.eq("seconds"))
        mag = 1000000000ull;
    else if (u.eq("ns") || u.eq("nanosecond") || u.eq("nanoseconds"))
        mag = 1;
    else if (u.eq("us") || u.eq("μs") || u.eq("microsecond") || u.eq("microseconds"))
        mag = 1000ull;
    else if (u.eq("ms") || u.eq("millisecond") || u.eq("milliseconds"))
        mag = 1000000ull;
    else if (u.eq("m") || u.eq("min") || u.eq("mins") || u.eq("minute") || u.eq("minutes"))
        mag = 60000000000ull;
    else if (u.eq("h") || u.eq("hr") || u.eq("hrs") || u.eq("hour") || u.eq("hours"))
        mag = 3600000000000ull;
    else {
        err = kTimeUnitErr;
        return false;
    }
    if (!parse_u64(v, value, err)) return false;
    unsigned __int128 p = (unsigned __int128)value * mag;  // checked_mul
    ns_overflow = p > UINT64_MAX;
    ns = ns_overflow ? UINT64_MAX : (uint64_t)p;
    return true;
}

// BitsPerSec<SiPrefixUpper>::from_str (suffixes ["bit","bits"], units.rs:140-200, 571-578)
bool parse_bits(SV s, uint64_t& bits, const char*& err) {
    SV v, u;
    if (!split_value_unit(s, v, u)) {
        err = "Unable to identify value and unit";
        return false;
    }
    SV prefix = u;
    for (const char* suf : {"bit", "bits"}) {
        const uint32_t n = (uint32_t)std::strlen(suf);
        if (u.n >= n && std::memcmp(u.p + u.n - n, suf, n) == 0) {
            prefix.n = u.n - n;
            break;
        }
    }
    uint64_t mag;
    if (prefix.n == 0) mag = 1;
    else if (prefix.eq("K") || prefix.eq("kilo")) mag = 1000ull;
    else if (prefix.eq("Ki") || prefix.eq("kibi")) mag = 1024ull;
    else if (prefix.eq("M") || prefix.eq("mega")) mag = 1000000ull;
    else if (prefix.eq("Mi") || prefix.eq("mebi")) mag = 1048576ull;
    else if (prefix.eq("G") || prefix.eq("giga")) mag = 1000000000ull;
    else if (prefix.eq("Gi") || prefix.eq("gibi")) mag = 1073741824ull;
    else if (prefix.eq("T") || prefix.eq("tera")) mag = 1000000000000ull;
    else if (prefix.eq("Ti") || prefix.eq("tebi")) mag = 1099511627776ull;
    else {
        err = "Unit prefix was not one of (K|kilo|Ki|kibi|M|mega|Mi|mebi"
              "|G|giga|Gi|gibi|T|tera|Ti|tebi)";
        return false;
    }
    uint64_t val;
    if (!parse_u64(v, val, err)) return false;
    unsigned __int128 p = (unsigned __int128)val * mag;
    bits = p > UINT64_MAX ? UINT64_MAX : (uint64_t)p;
    return true;
}

void set_err(char* buf, size_t len, const std::string& m) {
    if (buf && len) std::snprintf(buf, len, "%s", m.c_str());
}

int line_of(const char* begin, const char* at) {
    int line = 1;
    for (const char* p = begin; p < at; ++p)
        if (*p == '\n') ++line;
    return line;
}

// ---- one pass over a run of top-level items -------------------------------------------
// Syntax (gml_parser::parse) is checked as the items are read; each node / edge is converted
// right away (ShadowNode / ShadowEdge::try_from, mod.rs:28-111), but a conversion error is only
// RECORDED (first one, in order) and reported after the whole text parsed -- the reference
// parses all of the text before it converts anything (mod.rs:135).
struct NodeRec {
    uint32_t id;
    uint64_t down, up;
    uint8_t has_down, has_up;
};
struct EdgeRec {
    uint32_t src_id, dst_id;
    uint64_t lat_ns;
    float loss;
};
struct Items {
    std::vector<NodeRec> nodes;
    std::vector<EdgeRec> edges;
    int64_t node_err = -1, edge_err = -1;  // first conversion error (index within this run)
    std::string node_err_msg, edge_err_msg;
    std::vector<int32_t> directed;          // values of every `directed` key, in order
    std::vector<SV> other_keys;
    bool syntax_ok = true;
    const char* err_at = nullptr;           // syntax error position (sequential run)
    std::string fail_msg;
    const char* stop = nullptr;             // where the run stopped
    bool saw_close = false;                 // the graph's closing "]" was read
};

const char* node_conv(const std::vector<KV>& kvs, NodeRec& n, std::string& msg) {
    (void)msg;
    n = NodeRec{0, 0, 0, 0, 0};
    bool has_id = false;
    for (auto& kv : kvs)
        if (kv.k.eq("id")) {
            n.id = (uint32_t)kv.v.i;
            has_id = true;
        }
    if (!has_id) return "Node 'id' was not provided";
    // host_bandwidth_down is converted before host_bandwidth_up (mod.rs:34-57)
    for (int pass = 0; pass < 2; ++pass) {
        const char* name = pass == 0 ? "host_bandwidth_down" : "host_bandwidth_up";
        for (auto& kv : kvs) {
            if (!kv.k.eq(name)) continue;
            if (kv.v.kind != Value::STR) {
                msg = std::string("Node '") + name + "' is not a string";
                return msg.c_str();
            }
            uint64_t bits;
            const char* e = nullptr;
            if (!parse_bits(kv.v.s, bits, e)) {
                msg = std::string("Node '") + name + "' is not a valid unit: " + e;
                return msg.c_str();
            }
            if (pass == 0) { n.down = bits; n.has_down = 1; }
            else { n.up = bits; n.has_up = 1; }
        }
    }
    return nullptr;
}

// ShadowEdge::try_from (mod.rs:75-110), in the reference's check order
const char* edge_conv(const std::vector<KV>& kvs, EdgeRec& r, std::string& msg) {
    const Value* lat = nullptr;
    const Value* jit = nullptr;
    const Value* pl = nullptr;
    r = EdgeRec{0, 0, 0, 0.0f};
    for (auto& kv : kvs) {
        if (kv.k.eq("latency")) lat = &kv.v;
        else if (kv.k.eq("jitter")) jit = &kv.v;
        else if (kv.k.eq("packet_loss")) pl = &kv.v;
        else if (kv.k.eq("source")) r.src_id = (uint32_t)kv.v.i;
        else if (kv.k.eq("target")) r.dst_id = (uint32_t)kv.v.i;
    }
    if (!lat) return "Edge 'latency' was not provided";
    if (lat->kind != Value::STR) return "Edge 'latency' is not a string";
    uint64_t lat_val = 0, lat_ns = 0;
    bool ovf = false;
    const char* ue = nullptr;
    if (!parse_time_ns(lat->s, lat_val, lat_ns, ovf, ue)) {
        msg = std::string("Edge 'latency' is not a valid unit: ") + ue;
        return msg.c_str();
    }
    if (jit) {
        if (jit->kind != Value::STR) return "Edge 'jitter' is not a string";
        uint64_t jv, jns;
        bool jo;
        if (!parse_time_ns(jit->s, jv, jns, jo, ue)) {
            msg = std::string("Edge 'jitter' is not a valid unit: ") + ue;
            return msg.c_str();
        }
    }
    float loss = 0.0f;
    if (pl) {
        if (pl->kind != Value::FLOAT) return "Edge 'packet_loss' is not a float";
        loss = pl->f;
    }
    if (loss < 0.0f || loss > 1.0f) return "Edge 'packet_loss' is not in the range [0,1]";
    if (lat_val == 0) return "Edge 'latency' must not be 0";
    // an overflowing ns conversion panics later in the reference (mod.rs:336 unwrap);
    // UINT64_MAX makes the routing entry points fail with SRG_ERR_LATENCY_RANGE.
    r.lat_ns = ovf ? UINT64_MAX : lat_ns;
    r.loss = loss;
    return nullptr;
}

// Items from p until `stop_at` (a chunk boundary) or, when stop_at == nullptr, until the
// graph's closing "]".  A chunked run that meets the closing "]", a syntax error, or an item
// ending past its boundary reports syntax_ok = false (the caller then parses sequentially).
void parse_items(const char* text, const char* p, const char* text_end, const char* stop_at, Items& out) {
    Parser P{text, text_end};
    std::vector<KV> kvs;
    kvs.reserve(16);
    std::string msg;
    if (stop_at) {  // address space only: pages are touched as the records are written
        const size_t bytes = (size_t)(stop_at - p);
        out.edges.reserve(bytes / 40 + 16);
        out.nodes.reserve(bytes / 16 + 16);
    }
    auto syntax = [&](const char* at) {
        out.syntax_ok = false;
        out.err_at = at;
        out.fail_msg = P.fail_msg;
    };
    for (;;) {
        if (stop_at && p >= stop_at) {
            if (p != stop_at) out.syntax_ok = false;
            break;
        }
        if (P.tag(p, "]") == R::OK) {
            out.saw_close = true;
            if (stop_at) out.syntax_ok = false;
            break;
        }
        SV k;
        const char* item_at = p;
        if (P.key(p, k) != R::OK) return syntax(item_at);
        const bool is_node = k.eq("node"), is_edge = k.eq("edge");
        if (is_node || is_edge) {
            R r = P.block(p, kvs);
            if (r == R::FAIL) return syntax(P.fail_at);
            if (r != R::OK) return syntax(item_at);
            if (is_node) {
                // node(): id must be an Int (parser.rs:171-175)
                for (auto& kv : kvs)
                    if (kv.k.eq("id") && kv.v.kind != Value::INT) {
                        P.fail_msg = "Incorrect 'id' type";
                        return syntax(p);
                    }
                NodeRec n;
                const char* e = node_conv(kvs, n, msg);
                if (e && out.node_err < 0) {
                    out.node_err = (int64_t)out.nodes.size();
                    out.node_err_msg = e;
                }
                out.nodes.push_back(n);
            } else {
                // edge(): source / target required Ints (parser.rs:199-211)
                const Value* s = nullptr;
                const Value* t = nullptr;
                for (auto& kv : kvs) {
                    if (kv.k.eq("source")) s = &kv.v;
                    if (kv.k.eq("target")) t = &kv.v;
                }
                if (s && s->kind != Value::INT) { P.fail_msg = "Incorrect 'source' type"; return syntax(p); }
                if (!s) { P.fail_msg = "'source' doesn't exist"; return syntax(p); }
                if (t && t->kind != Value::INT) { P.fail_msg = "Incorrect 'target' type"; return syntax(p); }
                if (!t) { P.fail_msg = "'target' doesn't exist"; return syntax(p); }
                EdgeRec er;
                const char* e = edge_conv(kvs, er, msg);
                if (e && out.edge_err < 0) {
                    out.edge_err = (int64_t)out.edges.size();
                    out.edge_err_msg = e;
                }
                out.edges.push_back(er);
            }
        } else if (k.eq("directed")) {
            // int_as_bool (parser.rs:264-273)
            Value v;
            R r = P.value(p, v);
            if (r == R::FAIL) return syntax(P.fail_at);
            if (r != R::OK) return syntax(item_at);
            if (v.kind != Value::INT) { P.fail_msg = "Value was not an integer"; return syntax(p); }
            if (v.i != 0 && v.i != 1) { P.fail_msg = "Bool must be 0 or 1"; return syntax(p); }
            out.directed.push_back(v.i);
        } else {
            Value v;
            R r = P.value(p, v);
            if (r == R::FAIL) return syntax(P.fail_at);
            if (r != R::OK) return syntax(item_at);
            out.other_keys.push_back(k);
        }
    }
    out.stop = p;
}

int parse_threads() {
    int n = (int)std::thread::hardware_concurrency();
    if (const char* s = std::getenv("OMP_NUM_THREADS")) {
        const int v = std::atoi(s);
        if (v > 0) n = std::min(n > 0 ? n : v, v);
    }
    return std::max(1, std::min(n, 64));
}

// Chunk boundaries: the start of a line "<spaces>node [" or "<spaces>edge [" near each cut
// point.  A wrong guess (e.g. inside a multi-line string) makes a chunk's run fail its boundary
// check and the whole text is parsed sequentially instead -- the result never depends on it.
std::vector<const char*> chunk_starts(const char* p0, const char* end, size_t chunks) {
    std::vector<const char*> cuts{p0};
    const size_t len = (size_t)(end - p0);
    for (size_t i = 1; i < chunks; ++i) {
        const char* q = p0 + len * i / chunks;
        if (q <= cuts.back()) continue;
        const char* found = nullptr;
        while (q < end) {
            const char* nl = static_cast<const char*>(std::memchr(q, '\n', (size_t)(end - q)));
            if (!nl) break;
            const char* a = nl + 1;
            while (a < end && (*a == ' ' || *a == '\t')) ++a;
            if (end - a >= 6 && (std::memcmp(a, "node", 4) == 0 || std::memcmp(a, "edge", 4) == 0)) {
                const char* b = a + 4;
                while (b < end && (*b == ' ' || *b == '\t')) ++b;
                if (b < end && *b == '[') {
                    found = a;
                    break;
                }
            }
            q = a;
        }
        if (!found) break;
        if (found > cuts.back()) cuts.push_back(found);
    }
    return cuts;
}

int parse_impl(const char* text, size_t len, srg_graph* g, std::string& err) {
    const char* end = text + len;
    Parser P{text, end};
    const char* p = P.multispace0(text);
    auto syntax_at = [&](const char* at, const std::string& fm) {
        err = "GML syntax error at line " + std::to_string(line_of(text, at));
        if (!fm.empty()) err += ": " + fm;
        return SRG_ERR_PARSE;
    };
    if (P.tag(p, "graph") != R::OK) return syntax_at(p, "");
    p = P.space0(p);
    if (P.tag(p, "[") != R::OK) return syntax_at(p, "");
    if (P.newline(p) != R::OK) return syntax_at(p, "");

    // ---- gml_parser::parse: chunked in parallel when large, else (and on any doubt) sequential
    const size_t min_chunk = []() {
        const char* s = std::getenv("SRG_GML_MIN_CHUNK");  // testing aid: force small chunks
        return s ? (size_t)std::max(1ll, std::atoll(s)) : (size_t)32 << 20;
    }();
    const size_t want = std::min<size_t>((size_t)parse_threads(), std::max<size_t>(1, (size_t)(end - p) / min_chunk));
    std::vector<Items> parts;
    bool ok = false;
    if (want > 1) {
        std::vector<const char*> cuts = chunk_starts(p, end, want);
        if (cuts.size() > 1) {
            parts.resize(cuts.size());
            std::vector<std::thread> th;
            for (size_t i = 0; i < cuts.size(); ++i)
                th.emplace_back([&, i]() {
                    try {
                        Items local;  // not parts[i] in place: neighbouring Items share cache lines
                        parse_items(text, cuts[i], end, i + 1 < cuts.size() ? cuts[i + 1] : nullptr, local);
                        parts[i] = std::move(local);
                    } catch (...) {
                        parts[i].syntax_ok = false;
                    }
                });
            for (auto& t : th) t.join();
            ok = true;
            for (size_t i = 0; i < parts.size(); ++i)
                ok &= parts[i].syntax_ok && (i + 1 < parts.size() || parts[i].saw_close);
        }
    }
    if (!ok) {
        parts.assign(1, Items{});
        parse_items(text, p, end, nullptr, parts[0]);
        if (!parts[0].syntax_ok) return syntax_at(parts[0].err_at, parts[0].fail_msg);
        if (!parts[0].saw_close) return syntax_at(parts[0].stop ? parts[0].stop : end, "");
    }
    g->parse_chunks = (uint32_t)parts.size();
    const char* close_at = parts.back().stop;
    std::vector<int32_t> directed;
    std::vector<SV> other;
    size_t V = 0, E = 0;
    for (auto& it : parts) {
        directed.insert(directed.end(), it.directed.begin(), it.directed.end());
        other.insert(other.end(), it.other_keys.begin(), it.other_keys.end());
        V += it.nodes.size();
        E += it.edges.size();
    }
    if (directed.size() > 1) return syntax_at(close_at, "The 'directed' key must only be specified once");
    for (size_t a = 1; a < other.size(); ++a)
        for (size_t b = 0; b < a; ++b)
            if (other[a].same(other[b])) return syntax_at(close_at, "Duplicate keys are not supported");
    g->directed = !directed.empty() && directed[0] == 1;

    // ---- NetworkGraph::parse (mod.rs:134-181): nodes, then edges, in order -------------------
    g->node_id.resize(V);
    g->bw_down.resize(V);
    g->bw_up.resize(V);
    g->has_down.resize(V);
    g->has_up.resize(V);
    size_t off = 0;
    for (auto& it : parts) {
        if (it.node_err >= 0) {
            err = it.node_err_msg;
            return SRG_ERR_PARSE;
        }
        for (size_t i = 0; i < it.nodes.size(); ++i) {
            const NodeRec& n = it.nodes[i];
            g->node_id[off + i] = n.id;
            g->bw_down[off + i] = n.down;
            g->bw_up[off + i] = n.up;
            g->has_down[off + i] = n.has_down;
            g->has_up[off + i] = n.has_up;
        }
        off += it.nodes.size();
    }
    g->id_to_index.reserve(V);
    for (uint32_t i = 0; i < (uint32_t)V; ++i) g->id_to_index[g->node_id[i]] = i;  // later duplicates win
    g->src.resize(E);
    g->dst.resize(E);
    g->lat_ns.resize(E);
    g->loss.resize(E);
    // dense id -> index table when the ids allow it (the common 0..V-1 case)
    uint32_t max_id = 0;
    for (uint32_t id : g->node_id) max_id = std::max(max_id, id);
    std::vector<uint32_t> direct;
    if (V && (uint64_t)max_id < 4ull * V + 1024) {
        direct.assign((size_t)max_id + 1, UINT32_MAX);
        for (uint32_t i = 0; i < (uint32_t)V; ++i) direct[g->node_id[i]] = i;
    }
    auto lookup = [&](uint32_t id) -> uint32_t {
        if (!direct.empty()) return id < direct.size() ? direct[id] : UINT32_MAX;
        auto f = g->id_to_index.find(id);
        return f == g->id_to_index.end() ? UINT32_MAX : f->second;
    };
    off = 0;
    for (auto& it : parts) {
        const size_t stop = it.edge_err >= 0 ? (size_t)it.edge_err : it.edges.size();
        for (size_t e = 0; e < stop; ++e) {
            const EdgeRec& r = it.edges[e];
            const uint32_t si = lookup(r.src_id);
            if (si == UINT32_MAX) { err = "Edge source " + std::to_string(r.src_id) + " doesn't exist"; return SRG_ERR_PARSE; }
            const uint32_t ti = lookup(r.dst_id);
            if (ti == UINT32_MAX) { err = "Edge target " + std::to_string(r.dst_id) + " doesn't exist"; return SRG_ERR_PARSE; }
            g->src[off + e] = si;
            g->dst[off + e] = ti;
            g->lat_ns[off + e] = r.lat_ns;
            g->loss[off + e] = r.loss;
        }
        if (it.edge_err >= 0) {
            err = it.edge_err_msg;
            return SRG_ERR_PARSE;
        }
        off += it.edges.size();
    }
    return SRG_OK;
}

}  // namespace

extern "C" {

int srg_graph_parse_gml(const char* text, size_t len, srg_graph** out, char* errbuf, size_t errlen) {
    if (!out || (!text && len)) {
        set_err(errbuf, errlen, "null argument");
        return SRG_ERR_ARG;
    }
    *out = nullptr;
    try {
        srg_graph* g = new srg_graph();
        std::string err;
        int rc = parse_impl(text ? text : "", len, g, err);
        if (rc != SRG_OK) {
            delete g;
            set_err(errbuf, errlen, err);
            return rc;
        }
        *out = g;
        return SRG_OK;
    } catch (const std::bad_alloc&) {
        set_err(errbuf, errlen, "out of host memory while parsing GML");
        return SRG_ERR_OOM;
    } catch (...) {
        set_err(errbuf, errlen, "internal error while parsing GML");
        return SRG_ERR_INTERNAL;
    }
}

void srg_graph_free(srg_graph* g) { delete g; }

void srg_graph_edge_list(const srg_graph* g, srg_edge_list* out) {
    if (!g || !out) return;
    out->num_vertices = (uint32_t)g->node_id.size();
    out->directed = g->directed ? 1 : 0;
    out->num_edges = g->src.size();
    out->src = g->src.data();
    out->dst = g->dst.data();
    out->latency_ns = g->lat_ns.data();
    out->packet_loss = g->loss.data();
    out->node_ids = g->node_id.data();
}

uint32_t srg_graph_num_vertices(const srg_graph* g) { return g ? (uint32_t)g->node_id.size() : 0; }
uint64_t srg_graph_num_edges(const srg_graph* g) { return g ? g->src.size() : 0; }
int srg_graph_directed(const srg_graph* g) { return g && g->directed ? 1 : 0; }

int srg_graph_node_index(const srg_graph* g, uint32_t gml_id, uint32_t* out_index) {
    if (!g || !out_index) return SRG_ERR_ARG;
    auto f = g->id_to_index.find(gml_id);
    if (f == g->id_to_index.end()) return SRG_ERR_ARG;
    *out_index = f->second;
    return SRG_OK;
}

uint32_t srg_graph_node_id(const srg_graph* g, uint32_t index) {
    if (!g || index >= g->node_id.size()) return UINT32_MAX;
    return g->node_id[index];
}

void srg_graph_node_bandwidth(const srg_graph* g, uint32_t index, uint64_t* down_bits, int* has_down,
                              uint64_t* up_bits, int* has_up) {
    if (!g || index >= g->node_id.size()) return;
    if (down_bits) *down_bits = g->bw_down[index];
    if (has_down) *has_down = g->has_down[index];
    if (up_bits) *up_bits = g->bw_up[index];
    if (has_up) *has_up = g->has_up[index];
}

void srg_graph_node_bandwidths(const srg_graph* g, uint64_t* down_bits, int* has_down, uint64_t* up_bits,
                               int* has_up) {
    if (!g) return;
    const size_t V = g->node_id.size();
    if (down_bits) std::copy(g->bw_down.begin(), g->bw_down.end(), down_bits);
    if (has_down) std::copy(g->has_down.begin(), g->has_down.begin() + V, has_down);
    if (up_bits) std::copy(g->bw_up.begin(), g->bw_up.end(), up_bits);
    if (has_up) std::copy(g->has_up.begin(), g->has_up.begin() + V, has_up);
}

uint32_t srg_graph_parse_chunks(const srg_graph* g) { return g ? g->parse_chunks : 0; }

}  // extern "C"
