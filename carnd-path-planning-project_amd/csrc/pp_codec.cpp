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
//     literal by strtod — here the exact integer algorithm of pp_numfmt.h for <= 19 significant
//     digits and |exp10| <= 27 (the same bits), strtod beyond;
//   - `int id = car_data[0]`: static_cast<int> of the stored integer or double;
//   - sensor_fusion rows go into std::map<int, Car> order: ascending id, a repeated id keeps
//     the last row (src/main.cpp:1329);
//   - dump (json.hpp:6680-6730): "%.15g" (digits10; pp_numfmt.h fmt15g for 1e-13 <= |x| < 1e18,
//     snprintf beyond), ".0" appended when the text has neither '.' nor 'e', non-finite -> null;
//     object keys in std::map order (next_x < next_y).
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
#define PP_HD
#include "pp_jsonparse.h"

namespace {

struct HostReader {
    const char* b;
    int at(int64_t i) const { return (unsigned char)b[i]; }
};

// fields of one frame; numbers outside pp_numfmt's domain go through libc like nlohmann's
struct HostSink {
    double x = 0, y = 0, yaw = 0, speed = 0;
    double px[PP_PREV_KEEP], py[PP_PREV_KEEP];
    int32_t npx = 0, npy = 0;
    std::vector<int> id;
    std::vector<double> cx, cy, cvx, cvy;
    void reset() { npx = npy = 0; id.clear(); cx.clear(); cy.clear(); cvx.clear(); cvy.clear(); }
    void scalar(int f, double v) { (f == 0 ? x : f == 1 ? y : f == 2 ? yaw : speed) = v; }
    void prev(int which, int i, double v) { if (i < PP_PREV_KEEP) (which ? py : px)[i] = v; }
    void prev_count(int which, int n) { (which ? npy : npx) = n; }
    void row(int i, double a, double b, double c, double d) { id.push_back(i); cx.push_back(a); cy.push_back(b); cvx.push_back(c); cvy.push_back(d); }
    bool host_needed() const { return false; }
    // json.hpp:2600-2650: strtoull / strtoll for integer tokens (then strtod on overflow), strtod
    bool slow_number(const HostReader& r, int64_t s, int64_t q, bool is_int, bool neg, ppjson::Num& out) {
        std::string z(r.b + s, (size_t)(q - s));
        if (is_int) {
            char* endp = nullptr;
            errno = 0;
            if (!neg) {
                const unsigned long long v = strtoull(z.c_str(), &endp, 10);
                if (errno == 0) { out.kind = 0; out.u = (uint64_t)v; out.d = (double)out.u; return true; }
            } else {
                const long long v = strtoll(z.c_str(), &endp, 10);
                if (errno == 0) { out.kind = 1; out.i = (int64_t)v; out.d = (double)out.i; return true; }
            }
        }
        out.kind = 2;
        out.d = strtod(z.c_str(), nullptr);
        return true;
    }
};

struct HostWriter {
    std::string& o;
    void put(char c) { o += c; }
    void put(const char* p, int n) { o.append(p, (size_t)n); }
    bool slow_number(double x) {
        char b[64];
        const int n = snprintf(b, sizeof(b), "%.15g", x);
        o.append(b, (size_t)n);
        bool int_like = true;
        for (int i = 0; i < n; i++) if (b[i] == '.' || b[i] == 'e') { int_like = false; break; }
        if (int_like) o += ".0";
        return true;
    }
};

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
        HostSink K;
        for (int64_t s = b; s < e; s++) {
            K.reset();
            const int64_t o0 = offsets[s], o1 = offsets[s + 1];
            int st = ppjson::kMsgBad;
            if (o1 >= o0) {
                HostReader R{buf + o0};
                st = ppjson::parse_frame(R, o1 - o0, K);
                if (st == ppjson::kMsgOk && K.npx != K.npy) st = ppjson::kMsgBad;
            }
            int u = 0;
            if (st == ppjson::kMsgOk) {
                u = ppjson::map_order(K.id.data(), K.cx.data(), K.cy.data(), K.cvx.data(), K.cvy.data(), (int)K.id.size());
                if (u > stride) st = ppjson::kMsgTooManyCars;
            }
            const bool ok = st == ppjson::kMsgOk || st == ppjson::kMsgTooManyCars;
            msg_status[s] = st;
            ((double*)out->ego_x)[s] = ok ? K.x : 0;
            ((double*)out->ego_y)[s] = ok ? K.y : 0;
            ((double*)out->ego_yaw_deg)[s] = ok ? K.yaw : 0;
            ((double*)out->ego_speed_mph)[s] = ok ? K.speed : 0;
            const int np = ok ? K.npx : 0;
            ((int32_t*)out->n_prev)[s] = np;
            for (int i = 0; i < PP_PREV_KEEP; i++) {
                ((double*)out->prev_x)[(int64_t)i * S + s] = i < np ? K.px[i] : 0.0;
                ((double*)out->prev_y)[(int64_t)i * S + s] = i < np ? K.py[i] : 0.0;
            }
            const int nc = ok ? std::min(u, stride) : 0;
            ((int32_t*)out->n_cars)[s] = nc;
            for (int j = 0; j < stride; j++) {
                const int64_t ix = (int64_t)j * S + s;
                const bool on = j < nc;
                ((int32_t*)out->car_id)[ix] = on ? K.id[j] : 0;
                ((double*)out->car_x)[ix] = on ? K.cx[j] : 0.0;
                ((double*)out->car_y)[ix] = on ? K.cy[j] : 0.0;
                ((double*)out->car_vx)[ix] = on ? K.cvx[j] : 0.0;
                ((double*)out->car_vy)[ix] = on ? K.cvy[j] : 0.0;
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
            o.clear();
            o.reserve(2048);
            HostWriter W{o};
            ppjson::control_message(W, next_x + s, next_y + s, stride, n_out[s] < 0 ? 0 : n_out[s]);
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
