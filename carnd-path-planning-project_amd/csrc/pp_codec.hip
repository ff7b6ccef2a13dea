// pp_codec.hip — the wire codec on the MI355X (include/pp.h pp_telemetry_parse_device /
// pp_control_format_device). The same parser and writer as the host codec (pp_jsonparse.h,
// pp_numfmt.h) instantiated for the device: one lane per frame, bytes read through a 16-byte
// register window (one global_load_dwordx4 per 16 bytes of the frame), control text assembled in
// a 16-byte register and stored as aligned dwordx4 into a per-frame slot. The first kDevRows
// sensor_fusion rows are held in registers; a frame with more moves them into its output columns
// and takes the rest there (ordered in place, std::map order). A frame or message that needs libc
// (a number outside the exact conversions' domain, more rows than the batch's car columns, a slot
// overflow) is flagged for the host instead: status PP_MSG_HOST / len -1.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pp.h"
#include "pp_jsonparse.h"

namespace {

constexpr int kDevRows = 24;

struct DevReader {
    const uint4* base;               // 16-byte aligned buffer
    int64_t off;                     // frame start (bytes)
    mutable int64_t chunk;
    mutable uint4 w;
    __device__ int at(int64_t i) const {
        const int64_t a = off + i;
        const int64_t c = a >> 4;
        if (c != chunk) { w = base[c]; chunk = c; }
        const int k = (int)(a & 15);
        const uint32_t word = k < 4 ? w.x : k < 8 ? w.y : k < 12 ? w.z : w.w;
        return (int)((word >> (8 * (k & 3))) & 0xFFu);
    }
};

struct DevSink {
    double x, y, yaw, speed;
    double px[PP_PREV_KEEP], py[PP_PREV_KEEP];
    int32_t npx, npy;
    int n;
    bool host;
    int id[kDevRows];
    double cx[kDevRows], cy[kDevRows], cvx[kDevRows], cvy[kDevRows];
    // the frame's output columns (row j at [j * S + s]), used once it has more than kDevRows rows
    int32_t* oid;
    double *ox, *oy, *ovx, *ovy;
    int64_t S;
    int stride;
    __device__ void scalar(int f, double v) {
        if (f == 0) x = v; else if (f == 1) y = v; else if (f == 2) yaw = v; else speed = v;
    }
    __device__ void prev(int which, int i, double v) {
        if (i < PP_PREV_KEEP) { if (which) py[i] = v; else px[i] = v; }
    }
    __device__ void prev_count(int which, int k) { if (which) npy = k; else npx = k; }
    __device__ void row(int i, double a, double b, double c, double d) {
        if (n < kDevRows) {
            id[n] = i; cx[n] = a; cy[n] = b; cvx[n] = c; cvy[n] = d;
        } else if (n < stride) {
            if (n == kDevRows) {                       // move the register rows into the columns
#pragma unroll
                for (int j = 0; j < kDevRows; j++) {
                    oid[j * S] = id[j]; ox[j * S] = cx[j]; oy[j * S] = cy[j]; ovx[j * S] = cvx[j]; ovy[j * S] = cvy[j];
                }
            }
            oid[n * S] = i; ox[n * S] = a; oy[n * S] = b; ovx[n * S] = c; ovy[n * S] = d;
        } else {
            host = true;                               // more rows than the batch has columns
        }
        n++;
    }
    __device__ bool host_needed() const { return host; }
    __device__ bool slow_number(const DevReader&, int64_t, int64_t, bool, bool, ppjson::Num& out) {
        host = true;
        out.kind = 2;
        out.d = 0;
        return true;
    }
};

__global__ __launch_bounds__(256) void k_tel_parse(const uint4* buf, const int64_t* off, int64_t n_msgs,
                                                   pp_scene_batch out, int32_t* status) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_msgs) return;
    const int64_t S = out.n_scenes;
    const int stride = out.car_stride;
    DevSink K;
    K.npx = K.npy = 0;
    K.n = 0;
    K.host = false;
    K.x = K.y = K.yaw = K.speed = 0;
    K.oid = (int32_t*)out.car_id + s; K.ox = (double*)out.car_x + s; K.oy = (double*)out.car_y + s;
    K.ovx = (double*)out.car_vx + s; K.ovy = (double*)out.car_vy + s;
    K.S = S;
    K.stride = stride;
    const int64_t o0 = off[s], o1 = off[s + 1];
    int st = ppjson::kMsgBad;
    if (o1 >= o0) {
        DevReader R;
        R.base = buf; R.off = o0; R.chunk = -1;
        st = ppjson::parse_frame(R, o1 - o0, K);
        if (st == ppjson::kMsgOk && K.npx != K.npy) st = ppjson::kMsgBad;
    }
    int u = 0;
    const bool cols = K.n > kDevRows;                  // the rows are in the output columns
    if (st == ppjson::kMsgOk) {
        u = cols ? ppjson::map_order(K.oid, K.ox, K.oy, K.ovx, K.ovy, K.n, S)
                 : ppjson::map_order(K.id, K.cx, K.cy, K.cvx, K.cvy, K.n);
        if (u > stride) st = ppjson::kMsgTooManyCars;
    }
    const bool ok = st == ppjson::kMsgOk || st == ppjson::kMsgTooManyCars;
    status[s] = st;
    ((double*)out.ego_x)[s] = ok ? K.x : 0;
    ((double*)out.ego_y)[s] = ok ? K.y : 0;
    ((double*)out.ego_yaw_deg)[s] = ok ? K.yaw : 0;
    ((double*)out.ego_speed_mph)[s] = ok ? K.speed : 0;
    const int np = ok ? K.npx : 0;
    ((int32_t*)out.n_prev)[s] = np;
    for (int i = 0; i < PP_PREV_KEEP; i++) {
        ((double*)out.prev_x)[(int64_t)i * S + s] = i < np ? K.px[i] : 0.0;
        ((double*)out.prev_y)[(int64_t)i * S + s] = i < np ? K.py[i] : 0.0;
    }
    const int nc = ok ? (u < stride ? u : stride) : 0;
    ((int32_t*)out.n_cars)[s] = nc;
    for (int j = 0; j < stride; j++) {
        const int64_t ix = (int64_t)j * S + s;
        const bool on = j < nc;
        if (cols && on) continue;                      // already in place
        ((int32_t*)out.car_id)[ix] = on ? K.id[j] : 0;
        ((double*)out.car_x)[ix] = on ? K.cx[j] : 0.0;
        ((double*)out.car_y)[ix] = on ? K.cy[j] : 0.0;
        ((double*)out.car_vx)[ix] = on ? K.cvx[j] : 0.0;
        ((double*)out.car_vy)[ix] = on ? K.cvy[j] : 0.0;
    }
}

// 16 bytes assembled in registers, stored aligned into the frame's slot
struct DevWriter {
    uint4* dst;
    int64_t cap;                    // slot bytes (multiple of 16)
    int64_t n;
    uint32_t w[4];
    bool host;
    __device__ void put(char c) {
        const int k = (int)(n & 15);
        const uint32_t b = (uint32_t)(unsigned char)c << (8 * (k & 3));
        if ((k & 3) == 0) w[k >> 2] = b; else w[k >> 2] |= b;
        n++;
        if ((n & 15) == 0) {
            if (n <= cap) dst[(n >> 4) - 1] = make_uint4(w[0], w[1], w[2], w[3]);
            else host = true;
        }
    }
    __device__ void put(const char* p, int k) { for (int i = 0; i < k; i++) put(p[i]); }
    __device__ bool slow_number(double) { host = true; return false; }
    __device__ void finish() {
        const int k = (int)(n & 15);
        if (k == 0) return;
        for (int i = k; i < 16; i++) {        // zero the rest of the last chunk
            if ((i & 3) == 0) w[i >> 2] = 0;
        }
        if (n <= cap) dst[n >> 4] = make_uint4(w[0], w[1], w[2], w[3]);
        else host = true;
    }
};

__global__ __launch_bounds__(256) void k_ctl_format(const double* nx, const double* ny, const int32_t* n_out,
                                                    int64_t S, int64_t stride, uint4* slots, int64_t slot_bytes,
                                                    int32_t* len) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    DevWriter W;
    W.dst = slots + s * (slot_bytes >> 4);
    W.cap = slot_bytes;
    W.n = 0;
    W.host = false;
    W.w[0] = W.w[1] = W.w[2] = W.w[3] = 0;
    const int n = n_out[s] < 0 ? 0 : n_out[s];
    const bool ok = ppjson::control_message(W, nx + s, ny + s, stride, n);
    W.finish();
    len[s] = (ok && !W.host) ? (int32_t)W.n : -1;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) { if (hipGetDevice(&prev) != hipSuccess) prev = -1; (void)hipSetDevice(d); }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

}  // namespace

extern "C" {

int32_t pp_telemetry_parse_device(const char* d_buf, const int64_t* d_offsets, int64_t n_msgs, pp_scene_batch* d_out,
                                  int32_t* d_status, int32_t device, void* hip_stream) {
    if (!d_buf || !d_offsets || !d_out || !d_status || n_msgs < 0 || d_out->n_scenes < n_msgs ||
        d_out->car_stride < 0 || d_out->car_stride > PP_MAX_CARS || ((uintptr_t)d_buf & 15) != 0)
        return PP_ERR_ARG;
    if (n_msgs == 0) return PP_OK;
    DeviceGuard g(device);
    const int64_t blocks = (n_msgs + 255) / 256;
    hipLaunchKernelGGL(k_tel_parse, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)hip_stream,
                       (const uint4*)d_buf, d_offsets, n_msgs, *d_out, d_status);
    return hipGetLastError() == hipSuccess ? PP_OK : PP_ERR_HIP;
}

int32_t pp_control_format_device(const double* d_next_x, const double* d_next_y, const int32_t* d_n_out,
                                 int64_t n_scenes, int64_t stride, char* d_slots, int64_t slot_bytes,
                                 int32_t* d_len, int32_t device, void* hip_stream) {
    if (!d_next_x || !d_next_y || !d_n_out || !d_slots || !d_len || n_scenes < 0 || stride < n_scenes ||
        slot_bytes < 16 || (slot_bytes & 15) != 0 || ((uintptr_t)d_slots & 15) != 0)
        return PP_ERR_ARG;
    if (n_scenes == 0) return PP_OK;
    DeviceGuard g(device);
    const int64_t blocks = (n_scenes + 255) / 256;
    hipLaunchKernelGGL(k_ctl_format, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)hip_stream, d_next_x,
                       d_next_y, d_n_out, n_scenes, stride, (uint4*)d_slots, slot_bytes, d_len);
    return hipGetLastError() == hipSuccess ? PP_OK : PP_ERR_HIP;
}

}  // extern "C"
