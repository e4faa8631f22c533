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
#include <map>
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
};

namespace {

// ----------------------------------------------------------------------------------------
// nom-like result: OK, ERR (recoverable: alt/many_till may try something else), FAIL (fatal)
enum class R { OK, ERR, FAIL };

struct Value {
    enum Kind { INT, FLOAT, STR } kind = INT;
    int32_t i = 0;
    float f = 0.0f;
    std::string s;
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
    R key(const char*& p, std::string& out) const {
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
        out.assign(p, q);
        p = q;
        return R::OK;
    }
    // int (parser.rs:226-229)
    R int_(const char*& p, Value& v) const {
        const char* q = p;
        while (q < end && is_digit((unsigned char)*q)) ++q;
        if (q == p) return R::ERR;
        // str::parse::<i32>: overflow -> map_res error (ERR)
        int64_t acc = 0;
        for (const char* r = p; r < q; ++r) {
            acc = acc * 10 + (*r - '0');
            if (acc > INT32_MAX) return R::ERR;
        }
        v.kind = Value::INT;
        v.i = (int32_t)acc;
        p = q;
        return R::OK;
    }
    // float = recognize_float (nom 7.1.3) -> str::parse::<f32> (parser.rs:231-234)
    R float_(const char*& p, Value& v) {
        const char* q = p;
        if (q < end && (*q == '+' || *q == '-')) ++q;
        const char* m = q;
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
        (void)m;
        if (q < end && (*q == 'e' || *q == 'E')) {
            const char* e = q + 1;
            if (e < end && (*e == '+' || *e == '-')) ++e;
            const char* d = e;
            while (e < end && is_digit((unsigned char)*e)) ++e;
            if (e == d) return fail(d, "expected exponent digits in float");  // cut(digit1)
            q = e;
        }
        std::string txt(p, q);
        // Rust's f32 parse is correctly rounded, as glibc strtof (C locale numerics).
        errno = 0;
        char* ep = nullptr;
        float f = std::strtof(txt.c_str(), &ep);
        if (ep != txt.c_str() + txt.size()) return R::ERR;
        v.kind = Value::FLOAT;
        v.f = f;
        p = q;
        return R::OK;
    }
    // string (parser.rs:237-250): '"' then a NON-EMPTY run of non-quote bytes then '"'
    R string_(const char*& p, Value& v) const {
        if (p >= end || *p != '"') return R::ERR;
        const char* q = p + 1;
        const char* s = q;
        while (q < end && *q != '"') ++q;
        if (q == s) return R::ERR;      // escaped_transform at index 0 -> Error
        if (q >= end) return R::ERR;    // Eof
        v.kind = Value::STR;
        v.s.assign(s, q);
        p = q + 1;
        return R::OK;
    }
    // value (parser.rs:214-224)
    R value(const char*& p, Value& v) {
        const char* start = space0(p);
        {
            const char* q = start;
            Value t;
            if (int_(q, t) == R::OK && newline(q) == R::OK) {
                v = t;
                p = q;
                return R::OK;
            }
        }
        {
            const char* q = start;
            Value t;
            R r = float_(q, t);
            if (r == R::FAIL) return r;
            if (r == R::OK && newline(q) == R::OK) {
                v = t;
                p = q;
                return R::OK;
            }
        }
        {
            const char* q = start;
            Value t;
            if (string_(q, t) == R::OK && newline(q) == R::OK) {
                v = t;
                p = q;
                return R::OK;
            }
        }
        return R::ERR;
    }

    struct KV {
        std::string k;
        Value v;
    };
    // many_till(tuple((key, value)), tag("]")) + duplicate check + newline
    R block(const char*& p, std::vector<KV>& kvs) {
        const char* q = space0(p);
        if (tag(q, "[") != R::OK) return R::ERR;
        if (newline(q) != R::OK) return R::ERR;
        for (;;) {
            if (tag(q, "]") == R::OK) break;
            KV kv;
            if (key(q, kv.k) != R::OK) return R::ERR;
            R r = value(q, kv.v);
            if (r != R::OK) return r;
            kvs.push_back(std::move(kv));
        }
        std::map<std::string, int> seen;
        for (auto& kv : kvs)
            if (seen[kv.k]++) return fail(q, "Duplicate keys are not supported");
        if (newline(q) != R::OK) return R::ERR;
        p = q;
        return R::OK;
    }
};

// ---------------- units (units.rs) ----------------------------------------------------
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

std::string utrim(const std::string& s) {
    const char* b = s.data();
    const char* e = s.data() + s.size();
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
    return std::string(b, last > e ? e : last);
}

// regex ^([+-]?[0-9\.]*)\s*(.*)$  -> (value, unit), both trimmed (units.rs:409-417)
bool split_value_unit(const std::string& s, std::string& val, std::string& unit) {
    const char* p = s.data();
    const char* e = s.data() + s.size();
    const char* v0 = p;
    if (p < e && (*p == '+' || *p == '-')) ++p;
    while (p < e && ((*p >= '0' && *p <= '9') || *p == '.')) ++p;
    val.assign(v0, p);
    while (p < e) {
        const char* q = p;
        if (!is_unicode_ws(q, e)) break;
        p = q;
    }
    if (std::memchr(p, '\n', e - p)) return false;  // `.` does not match '\n'
    unit.assign(p, e);
    val = utrim(val);
    unit = utrim(unit);
    return true;
}

// Rust u64::from_str: optional '+', then >= 1 ASCII digit, no overflow.
bool parse_u64(const std::string& s, uint64_t& out, std::string& err) {
    size_t i = 0;
    if (i < s.size() && s[i] == '+') ++i;
    if (i == s.size()) {
        err = s.empty() ? "cannot parse integer from empty string" : "invalid digit found in string";
        return false;
    }
    unsigned __int128 acc = 0;
    for (; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9') {
            err = "invalid digit found in string";
            return false;
        }
        acc = acc * 10 + (unsigned)(s[i] - '0');
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
bool parse_time_ns(const std::string& s, uint64_t& value, uint64_t& ns, bool& ns_overflow,
                   std::string& err) {
    std::string v, u;
    if (!split_value_unit(s, v, u)) {
        err = "Unable to identify value and unit";
        return false;
    }
    // Time suffixes = [""]: strip_suffix("") always succeeds -> prefix = unit
    uint64_t mag;
    if (u.empty() || u == "s" || u == "sec" || u == "secs" || u == "second" || u == "seconds")
        mag = 1000000000ull;
    else if (u == "ns" || u == "nanosecond" || u == "nanoseconds")
        mag = 1;
    else if (u == "us" || u == "μs" || u == "microsecond" || u == "microseconds")
        mag = 1000ull;
    else if (u == "ms" || u == "millisecond" || u == "milliseconds")
        mag = 1000000ull;
    else if (u == "m" || u == "min" || u == "mins" || u == "minute" || u == "minutes")
        mag = 60000000000ull;
    else if (u == "h" || u == "hr" || u == "hrs" || u == "hour" || u == "hours")
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
bool parse_bits(const std::string& s, uint64_t& bits, std::string& err) {
    std::string v, u;
    if (!split_value_unit(s, v, u)) {
        err = "Unable to identify value and unit";
        return false;
    }
    std::string prefix = u;
    for (const char* suf : {"bit", "bits"}) {
        size_t n = std::strlen(suf);
        if (u.size() >= n && u.compare(u.size() - n, n, suf) == 0) {
            prefix = u.substr(0, u.size() - n);
            break;
        }
    }
    uint64_t mag;
    if (prefix.empty()) mag = 1;
    else if (prefix == "K" || prefix == "kilo") mag = 1000ull;
    else if (prefix == "Ki" || prefix == "kibi") mag = 1024ull;
    else if (prefix == "M" || prefix == "mega") mag = 1000000ull;
    else if (prefix == "Mi" || prefix == "mebi") mag = 1048576ull;
    else if (prefix == "G" || prefix == "giga") mag = 1000000000ull;
    else if (prefix == "Gi" || prefix == "gibi") mag = 1073741824ull;
    else if (prefix == "T" || prefix == "tera") mag = 1000000000000ull;
    else if (prefix == "Ti" || prefix == "tebi") mag = 1099511627776ull;
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

struct RawNode {
    std::vector<Parser::KV> kvs;
};

int parse_impl(const char* text, size_t len, srg_graph* g, std::string& err) {
    Parser P{text, text + len};
    const char* p = P.multispace0(text);
    auto syntax = [&](const char* at) {
        err = "GML syntax error at line " + std::to_string(line_of(text, at));
        if (!P.fail_msg.empty()) err += ": " + P.fail_msg;
        return SRG_ERR_PARSE;
    };
    if (P.tag(p, "graph") != R::OK) return syntax(p);
    p = P.space0(p);
    if (P.tag(p, "[") != R::OK) return syntax(p);
    if (P.newline(p) != R::OK) return syntax(p);

    std::vector<RawNode> nodes, edges;
    int directed_count = 0;
    bool directed = false;
    std::vector<std::string> other_keys;
    for (;;) {
        if (P.tag(p, "]") == R::OK) break;
        std::string k;
        const char* item_at = p;
        if (P.key(p, k) != R::OK) return syntax(item_at);
        if (k == "node" || k == "edge") {
            RawNode rn;
            R r = P.block(p, rn.kvs);
            if (r == R::FAIL) return syntax(P.fail_at);
            if (r != R::OK) return syntax(item_at);
            // node(): id must be Int; edge(): source/target required Ints (parser.rs:171-211)
            if (k == "node") {
                for (auto& kv : rn.kvs)
                    if (kv.k == "id" && kv.v.kind != Value::INT) {
                        P.fail_msg = "Incorrect 'id' type";
                        return syntax(p);
                    }
                nodes.push_back(std::move(rn));
            } else {
                const Value* s = nullptr;
                const Value* t = nullptr;
                for (auto& kv : rn.kvs) {
                    if (kv.k == "source") s = &kv.v;
                    if (kv.k == "target") t = &kv.v;
                }
                if (s && s->kind != Value::INT) { P.fail_msg = "Incorrect 'source' type"; return syntax(p); }
                if (!s) { P.fail_msg = "'source' doesn't exist"; return syntax(p); }
                if (t && t->kind != Value::INT) { P.fail_msg = "Incorrect 'target' type"; return syntax(p); }
                if (!t) { P.fail_msg = "'target' doesn't exist"; return syntax(p); }
                edges.push_back(std::move(rn));
            }
        } else if (k == "directed") {
            // int_as_bool (parser.rs:264-273)
            Value v;
            R r = P.value(p, v);
            if (r == R::FAIL) return syntax(P.fail_at);
            if (r != R::OK) return syntax(item_at);
            if (v.kind != Value::INT) { P.fail_msg = "Value was not an integer"; return syntax(p); }
            if (v.i != 0 && v.i != 1) { P.fail_msg = "Bool must be 0 or 1"; return syntax(p); }
            directed = v.i == 1;
            ++directed_count;
            if (directed_count == 1) g->directed = directed;
        } else {
            Value v;
            R r = P.value(p, v);
            if (r == R::FAIL) return syntax(P.fail_at);
            if (r != R::OK) return syntax(item_at);
            other_keys.push_back(k);
        }
    }
    if (directed_count > 1) {
        P.fail_msg = "The 'directed' key must only be specified once";
        return syntax(p);
    }
    {
        std::map<std::string, int> seen;
        for (auto& k : other_keys)
            if (seen[k]++) {
                P.fail_msg = "Duplicate keys are not supported";
                return syntax(p);
            }
    }

    // ---- NetworkGraph::parse (mod.rs:134-181) ----
    const uint32_t V = (uint32_t)nodes.size();
    g->node_id.resize(V);
    g->bw_down.assign(V, 0);
    g->bw_up.assign(V, 0);
    g->has_down.assign(V, 0);
    g->has_up.assign(V, 0);
    for (uint32_t i = 0; i < V; ++i) {
        bool has_id = false;
        for (auto& kv : nodes[i].kvs) {
            if (kv.k == "id") {
                g->node_id[i] = (uint32_t)kv.v.i;
                has_id = true;
            }
        }
        if (!has_id) {
            err = "Node 'id' was not provided";
            return SRG_ERR_PARSE;
        }
        for (auto& kv : nodes[i].kvs) {
            const bool down = kv.k == "host_bandwidth_down";
            const bool up = kv.k == "host_bandwidth_up";
            if (!down && !up) continue;
            const char* name = down ? "host_bandwidth_down" : "host_bandwidth_up";
            if (kv.v.kind != Value::STR) {
                err = std::string("Node '") + name + "' is not a string";
                return SRG_ERR_PARSE;
            }
            uint64_t bits;
            std::string e;
            if (!parse_bits(kv.v.s, bits, e)) {
                err = std::string("Node '") + name + "' is not a valid unit: " + e;
                return SRG_ERR_PARSE;
            }
            if (down) { g->bw_down[i] = bits; g->has_down[i] = 1; }
            else { g->bw_up[i] = bits; g->has_up[i] = 1; }
        }
        // the reference validates down before up (mod.rs:34-57); both checked above in
        // key order -- re-check order for a node with two bad bandwidths is immaterial
        // to success/failure.
        g->id_to_index[g->node_id[i]] = i;  // HashMap::insert: later duplicates win
    }
    const size_t E = edges.size();
    g->src.reserve(E);
    g->dst.reserve(E);
    g->lat_ns.reserve(E);
    g->loss.reserve(E);
    for (size_t e = 0; e < E; ++e) {
        const Value* lat = nullptr;
        const Value* jit = nullptr;
        const Value* pl = nullptr;
        uint32_t s = 0, t = 0;
        for (auto& kv : edges[e].kvs) {
            if (kv.k == "latency") lat = &kv.v;
            else if (kv.k == "jitter") jit = &kv.v;
            else if (kv.k == "packet_loss") pl = &kv.v;
            else if (kv.k == "source") s = (uint32_t)kv.v.i;
            else if (kv.k == "target") t = (uint32_t)kv.v.i;
        }
        // ShadowEdge::try_from (mod.rs:75-110), in the reference's check order
        if (!lat) { err = "Edge 'latency' was not provided"; return SRG_ERR_PARSE; }
        if (lat->kind != Value::STR) { err = "Edge 'latency' is not a string"; return SRG_ERR_PARSE; }
        uint64_t lat_val = 0, lat_ns = 0;
        bool ovf = false;
        std::string ue;
        if (!parse_time_ns(lat->s, lat_val, lat_ns, ovf, ue)) {
            err = "Edge 'latency' is not a valid unit: " + ue;
            return SRG_ERR_PARSE;
        }
        if (jit) {
            if (jit->kind != Value::STR) { err = "Edge 'jitter' is not a string"; return SRG_ERR_PARSE; }
            uint64_t jv, jns;
            bool jo;
            if (!parse_time_ns(jit->s, jv, jns, jo, ue)) {
                err = "Edge 'jitter' is not a valid unit: " + ue;
                return SRG_ERR_PARSE;
            }
        }
        float loss = 0.0f;
        if (pl) {
            if (pl->kind != Value::FLOAT) { err = "Edge 'packet_loss' is not a float"; return SRG_ERR_PARSE; }
            loss = pl->f;
        }
        if (loss < 0.0f || loss > 1.0f) {
            err = "Edge 'packet_loss' is not in the range [0,1]";
            return SRG_ERR_PARSE;
        }
        if (lat_val == 0) { err = "Edge 'latency' must not be 0"; return SRG_ERR_PARSE; }
        auto si = g->id_to_index.find(s);
        if (si == g->id_to_index.end()) { err = "Edge source " + std::to_string(s) + " doesn't exist"; return SRG_ERR_PARSE; }
        auto ti = g->id_to_index.find(t);
        if (ti == g->id_to_index.end()) { err = "Edge target " + std::to_string(t) + " doesn't exist"; return SRG_ERR_PARSE; }
        g->src.push_back(si->second);
        g->dst.push_back(ti->second);
        // an overflowing ns conversion panics later in the reference (mod.rs:336 unwrap);
        // UINT64_MAX makes the routing entry points fail with SRG_ERR_LATENCY_RANGE.
        g->lat_ns.push_back(ovf ? UINT64_MAX : lat_ns);
        g->loss.push_back(loss);
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

}  // extern "C"
