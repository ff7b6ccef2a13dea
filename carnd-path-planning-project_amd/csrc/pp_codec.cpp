// pp_codec.cpp — the simulator wire codec, host C++.
//
// Telemetry in: a batch of socket.io text frames `42["telemetry",{...}]` (src/main.cpp:1217-1252)
// -> the SoA scene batch of include/pp.h. Control out: next_x/next_y -> `42["control",{...}]`
// (src/main.cpp:1461-1466). Byte-for-byte and bit-for-bit what the reference's helpers.h:15-25
// hasData + nlohmann::json 2.1 parse/dump produce:
//   - hasData: a frame containing "null" anywhere is "no data" (manual mode); otherwise the
//     payload is [first '[', first '}' + 1];
//   - numbers (json.hpp:2600-2650): an integer literal is read by strtoull / strtoll and
//     converted to double (so "-0" gives +0.0, and a 20-digit integer rounds once); any other
//     literal by strtod. A short-digit fast path (<= 15 significant digits, |exp10| <= 22:
//     one exactly rounded IEEE operation on exact operands, Clinger 1990) gives the same bits;
//     everything else calls strtod;
//   - `int id = car_data[0]`: static_cast<int> of the stored integer or double;
//   - sensor_fusion rows go into std::map<int, Car> order: ascending id, a repeated id keeps
//     the last row (src/main.cpp:1329);
//   - dump (json.hpp:6680-6730): "%.15g" (digits10), ".0" appended when the text has neither
//     '.' nor 'e', non-finite -> null; object keys in std::map order (next_x < next_y).
// Batches are split over host threads; the product path stays the HIP kernels.
#include <errno.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pp.h"

namespace {

struct Cur {
    const char* p;
    const char* e;
    bool ok = true;
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
    }
    bool eat(char c) {
        ws();
        if (p < e && *p == c) { p++; return true; }
        return false;
    }
    bool peek(char c) {
        ws();
        return p < e && *p == c;
    }
};

// 10^k, k <= 22: exact doubles
const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                           1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// A JSON number as nlohmann 2.1 reads it. kind: 0 unsigned integer, 1 signed integer, 2 float
struct Num {
    double d;
    int64_t i;
    uint64_t u;
    int kind;
};

bool parse_number(Cur& c, Num& out) {
    c.ws();
    const char* s = c.p;
    const char* p = s;
    const char* e = c.e;
    bool neg = false;
    if (p < e && *p == '-') { neg = true; p++; }
    if (p >= e || *p < '0' || *p > '9') return false;
    const char* int_b = p;
    if (*p == '0') p++;
    else while (p < e && *p >= '0' && *p <= '9') p++;
    const char* int_e = p;
    const char* frac_b = nullptr;
    const char* frac_e = nullptr;
    bool is_float = false;
    if (p < e && *p == '.') {
        p++;
        frac_b = p;
        if (p >= e || *p < '0' || *p > '9') return false;
        while (p < e && *p >= '0' && *p <= '9') p++;
        frac_e = p;
        is_float = true;
    }
    int exp10 = 0;
    bool exp_big = false;
    if (p < e && (*p == 'e' || *p == 'E')) {
        p++;
        bool eneg = false;
        if (p < e && (*p == '+' || *p == '-')) { eneg = *p == '-'; p++; }
        if (p >= e || *p < '0' || *p > '9') return false;
        while (p < e && *p >= '0' && *p <= '9') {
            if (exp10 < 100000) exp10 = exp10 * 10 + (*p - '0');
            else exp_big = true;
            p++;
        }
        if (eneg) exp10 = -exp10;
        is_float = true;
    }
    c.p = p;
    const size_t len = (size_t)(p - s);
    char small[72];
    std::string big;
    const char* z;                  // NUL-terminated copy for the libc conversions
    if (len < sizeof(small)) { memcpy(small, s, len); small[len] = 0; z = small; }
    else { big.assign(s, len); z = big.c_str(); }
    if (!is_float) {
        // json.hpp:2600-2630: strtoull / strtoll first; on overflow fall through to strtod
        char* endp = nullptr;
        errno = 0;
        if (!neg) {
            const unsigned long long x = strtoull(z, &endp, 10);
            if (errno == 0) { out.kind = 0; out.u = (uint64_t)x; out.d = (double)out.u; return true; }
        } else {
            const long long x = strtoll(z, &endp, 10);
            if (errno == 0) { out.kind = 1; out.i = (int64_t)x; out.d = (double)out.i; return true; }
        }
    }
    out.kind = 2;
    // fast path: <= 15 significant digits, |effective exponent| <= 22 -> one exact IEEE op
    if (!exp_big) {
        uint64_t m = 0;
        int nd = 0;                 // significant digits accumulated
        bool lead = true;
        bool fits = true;
        for (const char* q = int_b; q < int_e; q++) {
            if (lead && *q == '0') continue;
            lead = false;
            if (++nd > 15) { fits = false; break; }
            m = m * 10 + (uint64_t)(*q - '0');
        }
        int e10 = exp10;
        if (fits && frac_b) {
            for (const char* q = frac_b; q < frac_e; q++) {
                e10--;
                if (lead && *q == '0') continue;
                lead = false;
                if (++nd > 15) { fits = false; break; }
                m = m * 10 + (uint64_t)(*q - '0');
            }
        }
        if (fits && e10 >= -22 && e10 <= 22) {
            double v = (double)m;
            v = e10 >= 0 ? v * kPow10[e10] : v / kPow10[-e10];
            out.d = neg ? -v : v;
            return true;
        }
    }
    out.d = strtod(z, nullptr);
    return true;
}

bool parse_string(Cur& c, std::string* out) {
    if (!c.eat('"')) return false;
    const char* b = c.p;
    while (c.p < c.e && *c.p != '"') {
        if (*c.p == '\\') { c.p++; if (c.p >= c.e) return false; }
        c.p++;
    }
    if (c.p >= c.e) return false;
    if (out) out->assign(b, (size_t)(c.p - b));
    c.p++;
    return true;
}

bool skip_value(Cur& c, int depth = 0) {
    if (depth > 64) return false;
    c.ws();
    if (c.p >= c.e) return false;
    const char ch = *c.p;
    if (ch == '"') return parse_string(c, nullptr);
    if (ch == '{') {
        c.p++;
        if (c.eat('}')) return true;
        do {
            if (!parse_string(c, nullptr) || !c.eat(':') || !skip_value(c, depth + 1)) return false;
        } while (c.eat(','));
        return c.eat('}');
    }
    if (ch == '[') {
        c.p++;
        if (c.eat(']')) return true;
        do {
            if (!skip_value(c, depth + 1)) return false;
        } while (c.eat(','));
        return c.eat(']');
    }
    auto lit = [&](const char* w) {
        const size_t n = strlen(w);
        if ((size_t)(c.e - c.p) >= n && memcmp(c.p, w, n) == 0) { c.p += n; return true; }
        return false;
    };
    if (ch == 't') return lit("true");
    if (ch == 'f') return lit("false");
    if (ch == 'n') return lit("null");
    Num x;
    return parse_number(c, x);
}

// array of numbers; the first `keep` values are stored
bool parse_num_array(Cur& c, double* dst, int keep, int32_t* count) {
    if (!c.eat('[')) return false;
    int n = 0;
    if (!c.eat(']')) {
        do {
            Num x;
            if (!parse_number(c, x)) return false;
            if (n < keep) dst[n] = x.d;
            n++;
        } while (c.eat(','));
        if (!c.eat(']')) return false;
    }
    *count = n;
    return true;
}

int to_int(const Num& x) {                // nlohmann get<int>: static_cast from the stored type
    if (x.kind == 0) return (int)x.u;
    if (x.kind == 1) return (int)x.i;
    if (!(x.d > -2147483649.0 && x.d < 2147483648.0)) return INT32_MIN;   // UB in the reference
    return (int)x.d;
}

struct Row { int id; double x, y, vx, vy; };

struct Parsed {
    double x = 0, y = 0, yaw = 0, speed = 0;
    double px[PP_PREV_KEEP], py[PP_PREV_KEEP];
    int32_t npx = 0, npy = 0;
    std::vector<Row> rows;
    bool has[6] = {false, false, false, false, false, false};
    bool has_sf = false;
};

bool parse_sensor_fusion(Cur& c, std::vector<Row>& rows) {
    if (!c.eat('[')) return false;
    if (c.eat(']')) return true;
    do {
        if (!c.eat('[')) return false;
        Num v[5];
        int n = 0;
        if (!c.eat(']')) {
            do {
                Num x;
                if (!parse_number(c, x)) return false;
                if (n < 5) v[n] = x;
                n++;
            } while (c.eat(','));
            if (!c.eat(']')) return false;
        }
        if (n < 5) return false;          // car_data[1..4] must exist
        rows.push_back({to_int(v[0]), v[1].d, v[2].d, v[3].d, v[4].d});
    } while (c.eat(','));
    return c.eat(']');
}

// 0: telemetry parsed; 1: no data (the reference answers "manual", src/main.cpp:1468-1471);
// 3: not a "42" event frame or another event (no answer); -1: the reference would throw
int parse_frame(const char* msg, size_t len, Parsed& P) {
    // src/main.cpp:1220: length > 2 and "42" prefix
    if (!(len > 2 && msg[0] == '4' && msg[1] == '2')) return 3;
    // helpers.h:15-25 hasData
    const std::string_view sv(msg, len);
    if (sv.find("null") != std::string_view::npos) return 1;
    const size_t b1 = sv.find_first_of('['), b2 = sv.find_first_of('}');
    if (b1 == std::string_view::npos || b2 == std::string_view::npos) return 1;
    size_t end = b2 + 2;
    if (end > len) end = len;
    if (end < b1) return -1;
    Cur c{msg + b1, msg + end};
    std::string event;
    if (!c.eat('[') || !parse_string(c, &event) || !c.eat(',')) return -1;
    if (event != "telemetry") { return skip_value(c) && c.eat(']') ? 3 : -1; }
    if (!c.eat('{')) return -1;
    if (!c.eat('}')) {
        do {
            std::string key;
            if (!parse_string(c, &key) || !c.eat(':')) return -1;
            // a repeated key keeps its first value (json.hpp:3084 object emplace)
            Num x;
            double* scal[4] = {&P.x, &P.y, &P.yaw, &P.speed};
            const int k = key == "x" ? 0 : key == "y" ? 1 : key == "yaw" ? 2 : key == "speed" ? 3
                        : key == "previous_path_x" ? 4 : key == "previous_path_y" ? 5
                        : key == "sensor_fusion" ? 6 : -1;
            if (k >= 0 && k < 6 && P.has[k]) { if (!skip_value(c)) return -1; continue; }
            if (k == 6 && P.has_sf) { if (!skip_value(c)) return -1; continue; }
            if (k >= 0 && k < 4) { if (!parse_number(c, x)) return -1; *scal[k] = x.d; P.has[k] = true; }
            else if (k == 4) { if (!parse_num_array(c, P.px, PP_PREV_KEEP, &P.npx)) return -1; P.has[4] = true; }
            else if (k == 5) { if (!parse_num_array(c, P.py, PP_PREV_KEEP, &P.npy)) return -1; P.has[5] = true; }
            else if (k == 6) { if (!parse_sensor_fusion(c, P.rows)) return -1; P.has_sf = true; }
            else if (!skip_value(c)) return -1;
        } while (c.eat(','));
        if (!c.eat('}')) return -1;
    }
    if (!c.eat(']')) return -1;
    for (bool h : P.has) if (!h) return -1;
    if (P.npx != P.npy) return -1;
    return 0;
}

// "%.15g" + ".0" when int-like; null when not finite (json.hpp:6680-6730)
inline void dump_float(std::string& o, double x) {
    if (!std::isfinite(x)) { o += "null"; return; }
    char b[64];
    const int n = snprintf(b, sizeof(b), "%.15g", x);
    o.append(b, (size_t)n);
    bool int_like = true;
    for (int i = 0; i < n; i++) if (b[i] == '.' || b[i] == 'e') { int_like = false; break; }
    if (int_like) o += ".0";
}

template <class F>
void parallel_for(int64_t n, int threads, F f) {
    if (threads <= 1 || n < 64) { f(0, n); return; }
    if (threads > 256) threads = 256;
    std::vector<std::thread> ts;
    const int64_t chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        const int64_t b = t * chunk, e = std::min(n, b + chunk);
        if (b >= e) break;
        ts.emplace_back([=] { f(b, e); });
    }
    for (auto& t : ts) t.join();
}

}  // namespace

extern "C" {

int32_t pp_telemetry_parse(const char* buf, const int64_t* offsets, int64_t n_msgs, pp_scene_batch* out,
                           int32_t* msg_status, int32_t n_threads) {
    if (!buf || !offsets || !out || !msg_status || n_msgs < 0 || out->n_scenes < n_msgs ||
        out->car_stride < 0 || out->car_stride > PP_MAX_CARS || !out->ego_x || !out->ego_y ||
        !out->ego_yaw_deg || !out->ego_speed_mph || !out->prev_x || !out->prev_y || !out->n_prev ||
        !out->n_cars || (out->car_stride > 0 && (!out->car_id || !out->car_x || !out->car_y ||
                                                 !out->car_vx || !out->car_vy)))
        return PP_ERR_ARG;
    const int64_t S = out->n_scenes;
    const int stride = out->car_stride;
    parallel_for(n_msgs, n_threads, [&](int64_t b, int64_t e) {
        Parsed P;
        for (int64_t s = b; s < e; s++) {
            P.rows.clear();
            for (bool& h : P.has) h = false;
            P.has_sf = false;
            P.npx = P.npy = 0;
            const int64_t o0 = offsets[s], o1 = offsets[s + 1];
            int st = o1 >= o0 ? parse_frame(buf + o0, (size_t)(o1 - o0), P) : -1;
            // std::map<int, Car> order: ascending id, the last row of an id wins
            std::stable_sort(P.rows.begin(), P.rows.end(), [](const Row& a, const Row& c) { return a.id < c.id; });
            std::vector<Row> u;
            for (size_t k = 0; k < P.rows.size(); k++) {
                if (k + 1 < P.rows.size() && P.rows[k + 1].id == P.rows[k].id) continue;
                u.push_back(P.rows[k]);
            }
            if (st == 0 && (int)u.size() > stride) st = 2;     // more distinct cars than columns
            msg_status[s] = st;
            double* ex = (double*)out->ego_x;
            ex[s] = st >= 0 ? P.x : 0;
            ((double*)out->ego_y)[s] = st >= 0 ? P.y : 0;
            ((double*)out->ego_yaw_deg)[s] = st >= 0 ? P.yaw : 0;
            ((double*)out->ego_speed_mph)[s] = st >= 0 ? P.speed : 0;
            const int np = st >= 0 ? P.npx : 0;
            ((int32_t*)out->n_prev)[s] = np;
            for (int i = 0; i < PP_PREV_KEEP; i++) {
                ((double*)out->prev_x)[(int64_t)i * S + s] = i < np ? P.px[i] : 0.0;
                ((double*)out->prev_y)[(int64_t)i * S + s] = i < np ? P.py[i] : 0.0;
            }
            const int nc = st >= 0 ? std::min((int)u.size(), stride) : 0;
            ((int32_t*)out->n_cars)[s] = nc;
            for (int j = 0; j < stride; j++) {
                const int64_t ix = (int64_t)j * S + s;
                const bool ok = j < nc;
                ((int32_t*)out->car_id)[ix] = ok ? u[j].id : 0;
                ((double*)out->car_x)[ix] = ok ? u[j].x : 0.0;
                ((double*)out->car_y)[ix] = ok ? u[j].y : 0.0;
                ((double*)out->car_vx)[ix] = ok ? u[j].vx : 0.0;
                ((double*)out->car_vy)[ix] = ok ? u[j].vy : 0.0;
            }
        }
    });
    return PP_OK;
}

int32_t pp_control_format(const double* next_x, const double* next_y, const int32_t* n_out, int64_t n_scenes,
                          int64_t stride, char* out, int64_t out_cap, int64_t* offsets, int32_t n_threads) {
    if (!next_x || !next_y || !n_out || !offsets || n_scenes < 0 || stride < n_scenes || out_cap < 0 ||
        (out_cap > 0 && !out))
        return PP_ERR_ARG;
    std::vector<std::string> parts((size_t)n_scenes);
    parallel_for(n_scenes, n_threads, [&](int64_t b, int64_t e) {
        for (int64_t s = b; s < e; s++) {
            std::string& o = parts[(size_t)s];
            o.reserve(2048);
            o = "42[\"control\",{\"next_x\":[";
            const int n = n_out[s] < 0 ? 0 : n_out[s];
            for (int i = 0; i < n; i++) { if (i) o += ','; dump_float(o, next_x[(int64_t)i * stride + s]); }
            o += "],\"next_y\":[";
            for (int i = 0; i < n; i++) { if (i) o += ','; dump_float(o, next_y[(int64_t)i * stride + s]); }
            o += "]}]";
        }
    });
    int64_t total = 0;
    for (int64_t s = 0; s < n_scenes; s++) { offsets[s] = total; total += (int64_t)parts[(size_t)s].size(); }
    offsets[n_scenes] = total;
    if (total > out_cap) return PP_ERR_NOMEM;   // offsets hold the sizes needed
    for (int64_t s = 0; s < n_scenes; s++) memcpy(out + offsets[s], parts[(size_t)s].data(), parts[(size_t)s].size());
    return PP_OK;
}

}  // extern "C"
