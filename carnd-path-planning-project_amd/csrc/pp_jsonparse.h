// pp_jsonparse.h — the telemetry frame parser and the control message writer, written once for
// the host codec (pp_codec.cpp) and the device codec kernels (pp_eval.hip): byte access goes
// through a Reader (host: a pointer; device: a 16-byte register window over global memory) and
// the results through a Sink; numbers use pp_numfmt.h's exact conversions. Numbers outside those
// conversions' domains call Sink::slow_number, which the host answers with libc and the device by
// flagging the frame for the host (PP_MSG_HOST).
//
// Semantics (src/main.cpp:1217-1252, 1325-1333, helpers.h:15-25, json.hpp 2.1) — see pp_codec.cpp.
#pragma once
#include <stdint.h>

#include "pp_numfmt.h"

namespace ppjson {

constexpr int kMsgOk = 0, kMsgManual = 1, kMsgTooManyCars = 2, kMsgIgnore = 3, kMsgHost = 4, kMsgBad = -1;
constexpr int kMaxDepth = 64;

// A parsed JSON number: kind 0 unsigned integer, 1 signed integer, 2 float (json.hpp lexer)
struct Num {
    double d;
    int64_t i;
    uint64_t u;
    int kind;
};

// nlohmann get<int>: static_cast from the stored type
PP_HD inline int num_to_int(const Num& x) {
    if (x.kind == 0) return (int)x.u;
    if (x.kind == 1) return (int)x.i;
    if (!(x.d > -2147483649.0 && x.d < 2147483648.0)) return INT32_MIN;   // UB in the reference
    return (int)x.d;
}

template <class R, class K>
struct Parser {
    const R& r;
    K& sink;
    int64_t p, e;
    PP_HD Parser(const R& r_, K& k_, int64_t b, int64_t e_) : r(r_), sink(k_), p(b), e(e_) {}
    PP_HD int at(int64_t i) const { return r.at(i); }
    PP_HD void ws() {
        while (p < e) {
            const int c = at(p);
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r') p++;
            else break;
        }
    }
    PP_HD bool eat(int c) {
        ws();
        if (p < e && at(p) == c) { p++; return true; }
        return false;
    }
    // string; the first 31 bytes go to key (NUL-terminated), *klen = full length
    PP_HD bool str(char* key, int* klen) {
        if (!eat('"')) return false;
        int n = 0;
        while (p < e && at(p) != '"') {
            int c = at(p);
            if (c == '\\') { p++; if (p >= e) return false; c = 256; }     // escaped: never a plain key
            if (key && n < 31) key[n] = (char)(c == 256 ? 1 : c);
            n++;
            p++;
        }
        if (p >= e) return false;
        p++;
        if (key) key[n < 31 ? n : 31] = 0;
        if (klen) *klen = n;
        return true;
    }
    PP_HD bool lit(const char* w) {
        int n = 0;
        while (w[n]) n++;
        if (e - p < n) return false;
        for (int i = 0; i < n; i++) if (at(p + i) != w[i]) return false;
        p += n;
        return true;
    }
    PP_HD bool number(Num& out) {
        ws();
        uint64_t M;
        int e10;
        bool neg, is_int, fast;
        // scan through the reader
        const int64_t s = p;
        int64_t q = p;
        neg = false; is_int = true; fast = true;
        uint64_t m = 0;
        int nd = 0, ex = 0;
        bool lead = true;
        if (q < e && at(q) == '-') { neg = true; q++; }
        if (q >= e || at(q) < '0' || at(q) > '9') return false;
        if (at(q) == '0') {
            q++;
        } else {
            while (q < e && at(q) >= '0' && at(q) <= '9') {
                lead = false;
                if (nd < 19) { m = m * 10 + (uint64_t)(at(q) - '0'); nd++; }
                else { fast = false; ex++; }
                q++;
            }
        }
        if (q < e && at(q) == '.') {
            q++;
            is_int = false;
            if (q >= e || at(q) < '0' || at(q) > '9') return false;
            while (q < e && at(q) >= '0' && at(q) <= '9') {
                if (lead && at(q) == '0') { ex--; q++; continue; }
                lead = false;
                if (nd < 19) { m = m * 10 + (uint64_t)(at(q) - '0'); nd++; ex--; }
                else fast = false;
                q++;
            }
        }
        if (q < e && (at(q) == 'e' || at(q) == 'E')) {
            q++;
            is_int = false;
            bool en = false;
            if (q < e && (at(q) == '+' || at(q) == '-')) { en = at(q) == '-'; q++; }
            if (q >= e || at(q) < '0' || at(q) > '9') return false;
            int v = 0;
            while (q < e && at(q) >= '0' && at(q) <= '9') {
                if (v < 100000) v = v * 10 + (at(q) - '0');
                else fast = false;
                q++;
            }
            ex += en ? -v : v;
        }
        M = m;
        e10 = ex;
        p = q;
        if (is_int && fast && e10 == 0) {
            // json.hpp:2600-2630 strtoull / strtoll: <= 19 digits fit a uint64; a negative value fits
            // an int64 when M <= 2^63 ("-0" -> +0.0)
            if (!neg) { out.kind = 0; out.u = M; out.d = (double)M; return true; }
            if (M <= (1ull << 63)) {
                out.kind = 1;
                out.i = M == (1ull << 63) ? INT64_MIN : -(int64_t)M;
                out.d = (double)out.i;
                return true;
            }
        }
        if (!is_int && fast) {
            out.kind = 2;
            if (ppnum::dec_to_double(M, e10, neg, &out.d)) return true;
        }
        return sink.slow_number(r, s, q, is_int, neg, out);
    }
    // validating skip of any value (iterative; nesting <= kMaxDepth)
    PP_HD bool skip() {
        uint64_t stack = 0;          // bit d: container at depth d is an object
        int depth = 0;
        for (;;) {
            ws();
            if (p >= e) return false;
            const int c = at(p);
            bool value_done = false;
            if (c == '{' || c == '[') {
                if (depth >= kMaxDepth) return false;
                p++;
                const bool obj = c == '{';
                if (obj) stack |= (1ull << depth); else stack &= ~(1ull << depth);
                depth++;
                if (eat(obj ? '}' : ']')) { depth--; value_done = true; }
                else if (obj) { if (!str(nullptr, nullptr) || !eat(':')) return false; continue; }
                else continue;
            } else if (c == '"') {
                if (!str(nullptr, nullptr)) return false;
                value_done = true;
            } else if (c == 't') { if (!lit("true")) return false; value_done = true; }
            else if (c == 'f') { if (!lit("false")) return false; value_done = true; }
            else if (c == 'n') { if (!lit("null")) return false; value_done = true; }
            else { Num x; if (!number(x)) return false; value_done = true; }
            // after a value: close containers or continue with the next element
            while (value_done) {
                if (depth == 0) return true;
                const bool obj = (stack >> (depth - 1)) & 1;
                if (eat(',')) {
                    if (obj && (!str(nullptr, nullptr) || !eat(':'))) return false;
                    value_done = false;
                } else if (eat(obj ? '}' : ']')) {
                    depth--;
                } else {
                    return false;
                }
            }
        }
    }
    PP_HD bool num_array(int which) {
        if (!eat('[')) return false;
        int n = 0;
        if (!eat(']')) {
            do {
                Num x;
                if (!number(x)) return false;
                sink.prev(which, n, x.d);
                n++;
            } while (eat(','));
            if (!eat(']')) return false;
        }
        sink.prev_count(which, n);
        return true;
    }
    PP_HD bool sensor_fusion() {
        if (!eat('[')) return false;
        if (eat(']')) return true;
        do {
            if (!eat('[')) return false;
            Num v[5];
            int n = 0;
            if (!eat(']')) {
                do {
                    Num x;
                    if (!number(x)) return false;
                    if (n < 5) v[n] = x;
                    n++;
                } while (eat(','));
                if (!eat(']')) return false;
            }
            if (n < 5) return false;          // car_data[1..4] must exist
            sink.row(num_to_int(v[0]), v[1].d, v[2].d, v[3].d, v[4].d);
        } while (eat(','));
        return eat(']');
    }
};

PP_HD inline bool key_is(const char* k, int klen, const char* w) {
    int i = 0;
    for (; w[i]; i++) if (i >= klen || k[i] != w[i]) return false;
    return i == klen;
}

// One frame [0, len) of reader r. Returns a kMsg* code; the sink holds the fields.
template <class R, class K>
PP_HD int parse_frame(const R& r, int64_t len, K& sink) {
    // src/main.cpp:1220: length > 2 and the "42" prefix
    if (!(len > 2 && r.at(0) == '4' && r.at(1) == '2')) return kMsgIgnore;
    // helpers.h:15-25 hasData: "null" anywhere -> no data; payload [first '[', first '}' + 1]
    int64_t b1 = -1, b2 = -1;
    for (int64_t i = 0; i < len; i++) {
        const int c = r.at(i);
        if (c == 'n' && i + 3 < len && r.at(i + 1) == 'u' && r.at(i + 2) == 'l' && r.at(i + 3) == 'l') return kMsgManual;
        if (c == '[' && b1 < 0) b1 = i;
        if (c == '}' && b2 < 0) b2 = i;
    }
    if (b1 < 0 || b2 < 0) return kMsgManual;
    int64_t end = b2 + 2;
    if (end > len) end = len;
    if (end < b1) return kMsgBad;
    Parser<R, K> P(r, sink, b1, end);
    char ev[32];
    int evl;
    if (!P.eat('[') || !P.str(ev, &evl) || !P.eat(',')) return kMsgBad;
    if (!key_is(ev, evl, "telemetry")) return P.skip() && P.eat(']') ? kMsgIgnore : kMsgBad;
    if (!P.eat('{')) return kMsgBad;
    bool has[7] = {false, false, false, false, false, false, false};
    if (!P.eat('}')) {
        do {
            char k[32];
            int kl;
            if (!P.str(k, &kl) || !P.eat(':')) return kMsgBad;
            // a repeated key keeps its first value (json.hpp:3084 object emplace)
            const int f = key_is(k, kl, "x") ? 0 : key_is(k, kl, "y") ? 1 : key_is(k, kl, "yaw") ? 2
                        : key_is(k, kl, "speed") ? 3 : key_is(k, kl, "previous_path_x") ? 4
                        : key_is(k, kl, "previous_path_y") ? 5 : key_is(k, kl, "sensor_fusion") ? 6 : -1;
            if (f < 0 || has[f]) { if (!P.skip()) return kMsgBad; continue; }
            if (f < 4) { Num x; if (!P.number(x)) return kMsgBad; sink.scalar(f, x.d); }
            else if (f < 6) { if (!P.num_array(f - 4)) return kMsgBad; }
            else { if (!P.sensor_fusion()) return kMsgBad; }
            has[f] = true;
        } while (P.eat(','));
        if (!P.eat('}')) return kMsgBad;
    }
    if (!P.eat(']')) return kMsgBad;
    for (int f = 0; f < 6; f++) if (!has[f]) return kMsgBad;
    if (sink.host_needed()) return kMsgHost;
    return kMsgOk;
}

// Cars in std::map<int, Car> order (ascending id, the last row of an id wins), in place over
// parallel arrays of n rows (row i at element i * st); returns the number of distinct ids. Stable
// insertion sort (n small).
PP_HD inline int map_order(int* id, double* x, double* y, double* vx, double* vy, int n, int64_t st = 1) {
    for (int i = 1; i < n; i++) {
        const int ki = id[i * st];
        const double a = x[i * st], b = y[i * st], c = vx[i * st], d = vy[i * st];
        int j = i - 1;
        while (j >= 0 && id[j * st] > ki) {
            const int64_t p = (j + 1) * st, q = j * st;
            id[p] = id[q]; x[p] = x[q]; y[p] = y[q]; vx[p] = vx[q]; vy[p] = vy[q];
            j--;
        }
        const int64_t p = (j + 1) * st;
        id[p] = ki; x[p] = a; y[p] = b; vx[p] = c; vy[p] = d;
    }
    int u = 0;
    for (int i = 0; i < n; i++) {
        if (i + 1 < n && id[(i + 1) * st] == id[i * st]) continue;        // a later row of the same id wins
        const int64_t p = u * st, q = i * st;
        id[p] = id[q]; x[p] = x[q]; y[p] = y[q]; vx[p] = vx[q]; vy[p] = vy[q];
        u++;
    }
    return u;
}

// ---- control message (json.hpp dump_float + the msgJson object, src/main.cpp:1461-1464) ----
// W provides put(char) and put(const char*, int). Returns false if a number needs the host
// (outside fmt15g's domain and the writer cannot format it).
template <class W>
PP_HD inline bool dump_number(W& w, double x) {
    if (!(x == x) || x - x != 0.0) { w.put("null", 4); return true; }     // NaN / inf
    char b[40];
    int n;
    if (x == 0.0) {
        const bool sn = __builtin_signbit(x);
        if (sn) { w.put("-0.0", 4); } else { w.put("0.0", 3); }
        return true;
    }
    n = ppnum::fmt15g(x, b);
    if (n == 0) return w.slow_number(x);
    w.put(b, n);
    bool int_like = true;
    for (int i = 0; i < n; i++) if (b[i] == '.' || b[i] == 'e') { int_like = false; break; }
    if (int_like) w.put(".0", 2);
    return true;
}

template <class W>
PP_HD inline void put_str(W& w, const char* t) {
    int n = 0;
    while (t[n]) n++;
    w.put(t, n);
}

template <class W>
PP_HD inline bool control_message(W& w, const double* nx, const double* ny, int64_t stride, int n) {
    bool ok = true;
    put_str(w, "42[\"control\",{\"next_x\":[");
    for (int i = 0; i < n; i++) { if (i) w.put(','); ok &= dump_number(w, nx[(int64_t)i * stride]); }
    put_str(w, "],\"next_y\":[");
    for (int i = 0; i < n; i++) { if (i) w.put(','); ok &= dump_number(w, ny[(int64_t)i * stride]); }
    put_str(w, "]}]");
    return ok;
}

}  // namespace ppjson
