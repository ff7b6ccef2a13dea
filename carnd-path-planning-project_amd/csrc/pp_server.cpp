// pp_server.cpp — the simulator shim: a WebSocket server speaking what the
// reference's uWS hub speaks (src/main.cpp:1214-1494: text frames carrying socket.io events,
// `42["telemetry",{...}]` in, `42["control",{...}]` or `42["manual",{}]` out), that batches the
// frames of every connected client per tick into one pp_plan_batch_host call.
//
// RFC 6455 subset: HTTP/1.1 upgrade (Sec-WebSocket-Accept = base64(SHA-1(key + GUID))), masked
// client frames, fragmented text messages, ping -> pong, close -> close. Per connection the
// planner's cross-frame state is kept like the reference's lambda captures: the std::map car table
// and target_lane (= 1 at start, src/main.cpp:1194-1195); the reference holds one set per process,
// the server one per connection. Replies per frame exactly as the lambda: telemetry -> control,
// "42" without data -> manual, anything else -> nothing; a frame the reference could not parse
// (its json::parse / field reads would throw and end the process) closes that connection.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdint.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "../../include/pp.h"
#include "pp_cartable.h"
#include "pp_wsproto.h"

namespace {

using ppws::handshake;
using ppws::ws_accept;
using ppws::ws_frame;
using ppws::ws_read;

struct Conn : ppws::WsConn {
    // the reference lambda's captures (src/main.cpp:1194-1195)
    int32_t target_lane = 1;
    pptab::CarTable table;          // std::map<int, Car> sensor_fusion_cars (any ids)
};

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

}  // namespace

extern "C" int32_t pp_serve(pp_map* M, const pp_server_opts* o, volatile int32_t* stop, int32_t* bound_port,
                            int64_t* stats) {
    if (!M || !o || o->max_clients < 1 || o->max_clients > 65536 || o->n_speeds < 1 || o->n_speeds > PP_MAX_SPEEDS)
        return PP_ERR_ARG;
    const int lfd = socket(AF_INET, SOCK_STREAM, 0);
    if (lfd < 0) return PP_ERR_ARG;
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)o->port);
    if (inet_pton(AF_INET, o->host ? o->host : "127.0.0.1", &a.sin_addr) != 1 ||
        bind(lfd, (sockaddr*)&a, sizeof(a)) != 0 || listen(lfd, 128) != 0) {
        close(lfd);
        return PP_ERR_ARG;
    }
    socklen_t al = sizeof(a);
    getsockname(lfd, (sockaddr*)&a, &al);
    if (bound_port) *bound_port = ntohs(a.sin_port);
    set_nonblock(lfd);
    pp_params prm;
    pp_params_default(&prm);
    prm.n_speeds = o->n_speeds;                  // reference decision: winner = (T, max_speed)
    std::vector<std::unique_ptr<Conn>> conns;
    int64_t frames = 0, ticks = 0, accepted = 0, replies = 0;
    int32_t rc = PP_OK;
    const int cap = o->max_clients;
    const int N = prm.n_points, C = PP_NUM_LANES * prm.n_speeds;
    // sensor_fusion columns of the host batch: grown (up to PP_MAX_CARS) when a frame reports more
    // distinct cars than it holds, then the tick's frames are parsed again
    int J = 16;
    // host batch (SoA) + results, sized per tick
    std::vector<double> ego, pxy, cars, tabd;
    std::vector<int32_t> ints, cid, tabi, mst;
    std::vector<double> nxy(2 * N * cap), cost(C * cap);
    std::vector<int32_t> win(cap), nout(cap);
    std::vector<uint32_t> status(cap);
    std::string obuf;
    std::vector<int64_t> ooff(cap + 1);
    while (!(stop && *stop) && rc == PP_OK && !(o->max_frames > 0 && frames >= o->max_frames)) {
        // poll: listener + connections
        std::vector<pollfd> pf;
        pf.push_back({lfd, POLLIN, 0});
        for (auto& c : conns) pf.push_back({c->fd, (short)(POLLIN | (c->out.empty() ? 0 : POLLOUT)), 0});
        if (poll(pf.data(), pf.size(), 2) < 0 && errno != EINTR) { rc = PP_ERR_ARG; break; }
        if (pf[0].revents & POLLIN) {
            for (;;) {
                const int fd = accept(lfd, nullptr, nullptr);
                if (fd < 0) break;
                if ((int)conns.size() >= cap) { close(fd); continue; }
                set_nonblock(fd);
                setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                auto c = std::make_unique<Conn>();
                c->fd = fd;
                conns.push_back(std::move(c));
                accepted++;
            }
        }
        for (size_t k = 0; k < conns.size() && k + 1 < pf.size(); k++) {
            Conn& c = *conns[k];
            if (pf[k + 1].revents & (POLLIN | POLLHUP | POLLERR)) {
                char b[65536];
                for (;;) {
                    const ssize_t r = recv(c.fd, b, sizeof(b), 0);
                    if (r > 0) { c.in.append(b, (size_t)r); continue; }
                    if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) c.closing = true;
                    break;
                }
                if (!c.upgraded) handshake(c);
                if (c.upgraded) ws_read(c);
            }
        }
        // one pending text message per connection per tick
        std::vector<int> who;
        std::vector<std::string> batch;
        for (size_t k = 0; k < conns.size(); k++) {
            Conn& c = *conns[k];
            if (!c.msgs.empty() && !c.closing) {
                who.push_back((int)k);
                batch.push_back(std::move(c.msgs.front()));
                c.msgs.pop_front();
            }
        }
        if (!batch.empty()) {
            ticks++;
            const int A = (int)batch.size();
            std::string buf;
            std::vector<int64_t> off(A + 1, 0);
            for (int i = 0; i < A; i++) { buf += batch[i]; off[i + 1] = (int64_t)buf.size(); }
            pp_scene_batch B;
            mst.resize(A);
            for (;;) {
                ego.resize(4 * (size_t)A); pxy.resize(2 * PP_PREV_KEEP * (size_t)A); cars.resize(4 * (size_t)J * A);
                ints.resize(3 * (size_t)A); cid.resize((size_t)J * A);
                memset(&B, 0, sizeof(B));
                B.n_scenes = A; B.car_stride = J;
                B.ego_x = ego.data(); B.ego_y = ego.data() + A; B.ego_yaw_deg = ego.data() + 2 * A; B.ego_speed_mph = ego.data() + 3 * A;
                B.prev_x = pxy.data(); B.prev_y = pxy.data() + PP_PREV_KEEP * A;
                B.n_prev = ints.data(); B.prev_target_lane = ints.data() + A; B.n_cars = ints.data() + 2 * A;
                B.car_id = cid.data();
                B.car_x = cars.data(); B.car_y = cars.data() + J * A; B.car_vx = cars.data() + 2 * J * A; B.car_vy = cars.data() + 3 * J * A;
                rc = pp_telemetry_parse(buf.data(), off.data(), A, &B, mst.data(), o->threads);
                if (rc != PP_OK || J >= PP_MAX_CARS) break;
                bool more = false;
                for (int i = 0; i < A; i++) more |= mst[i] == 2;
                if (!more) break;
                J = std::min(2 * J, PP_MAX_CARS);
            }
            if (rc != PP_OK) break;
            // dense batch of the telemetry frames, with each connection's state
            // status 2 (more distinct cars than PP_MAX_CARS) is not planned: the reference would
            // use every car, the batch holds PP_MAX_CARS; such a connection is closed
            std::vector<int> tel;
            for (int i = 0; i < A; i++) {
                if (mst[i] == 0) tel.push_back(i);
                else if (mst[i] == 2) conns[who[i]]->closing = true;
            }
            // a frame whose car table would exceed PP_MAX_CARS distinct cars: closed the same way
            {
                std::vector<int> keep;
                for (int i : tel) {
                    Conn& c = *conns[who[i]];
                    const int nc = ((const int32_t*)B.n_cars)[i];
                    std::vector<int32_t> ids(nc);
                    for (int j = 0; j < nc; j++) ids[j] = B.car_id[(size_t)j * A + i];
                    if (c.table.union_size(ids.data(), nc) > PP_MAX_CARS) c.closing = true;
                    else keep.push_back(i);
                }
                tel.swap(keep);
            }
            const int T = (int)tel.size();
            if (T) {
                // compact in place (tel is increasing, so i <= tel[i])
                auto mvD = [&](double* base, int rows) {
                    for (int r = 0; r < rows; r++) for (int i = 0; i < T; i++) base[(size_t)r * T + i] = base[(size_t)r * A + tel[i]];
                };
                auto mvI = [&](int32_t* base, int rows) {
                    for (int r = 0; r < rows; r++) for (int i = 0; i < T; i++) base[(size_t)r * T + i] = base[(size_t)r * A + tel[i]];
                };
                mvD(ego.data(), 4); mvD(pxy.data(), 2 * PP_PREV_KEEP); mvD(cars.data(), 4 * J);
                mvI(ints.data(), 3); mvI(cid.data(), J);
                pp_scene_batch D = B;
                D.n_scenes = T;
                D.ego_x = ego.data(); D.ego_y = ego.data() + T; D.ego_yaw_deg = ego.data() + 2 * T; D.ego_speed_mph = ego.data() + 3 * T;
                D.prev_x = pxy.data(); D.prev_y = pxy.data() + PP_PREV_KEEP * T;
                D.n_prev = ints.data(); D.prev_target_lane = ints.data() + T; D.n_cars = ints.data() + 2 * T;
                D.car_x = cars.data(); D.car_y = cars.data() + J * T; D.car_vx = cars.data() + 2 * J * T; D.car_vy = cars.data() + 3 * J * T;
                // each connection's car table laid out over the union of its ids and its frame's
                // ids (pp_cartable.h), padded to the batch's largest union
                int TSl = 0;
                std::vector<int> used(T);
                for (int i = 0; i < T; i++) {
                    const int nc = D.n_cars[i];
                    std::vector<int32_t> ids(nc);
                    for (int j = 0; j < nc; j++) ids[j] = D.car_id[(size_t)j * T + i];
                    used[i] = conns[who[tel[i]]]->table.union_size(ids.data(), nc);
                    TSl = std::max(TSl, used[i]);
                }
                D.tab_slots = TSl;
                tabi.resize(3 * (size_t)TSl * T);
                tabd.resize(6 * (size_t)TSl * T);
                D.tab_id = tabi.data() + 2 * (size_t)TSl * T;
                D.tab_valid = tabi.data(); D.tab_lane = tabi.data() + (size_t)TSl * T;
                D.tab_s = tabd.data(); D.tab_d = tabd.data() + (size_t)TSl * T; D.tab_vs = tabd.data() + 2 * (size_t)TSl * T;
                D.tab_vd = tabd.data() + 3 * (size_t)TSl * T; D.tab_vx = tabd.data() + 4 * (size_t)TSl * T;
                D.tab_vy = tabd.data() + 5 * (size_t)TSl * T;
                const pptab::Slots sl = {T, D.tab_id, D.tab_valid, D.tab_lane, D.tab_s, D.tab_d, D.tab_vs, D.tab_vd,
                                         D.tab_vx, D.tab_vy};
                for (int i = 0; i < T; i++) {
                    Conn& c = *conns[who[tel[i]]];
                    ((int32_t*)D.prev_target_lane)[i] = c.target_lane;
                    const int nc = D.n_cars[i];
                    std::vector<int32_t> ids(nc);
                    for (int j = 0; j < nc; j++) ids[j] = D.car_id[(size_t)j * T + i];
                    c.table.layout(ids.data(), nc, sl, i, TSl, pp_debug_get(PP_DBG_POISON) == 1);
                }
                pp_result R;
                memset(&R, 0, sizeof(R));
                R.winner = win.data(); R.n_out = nout.data(); R.next_x = nxy.data(); R.next_y = nxy.data() + (size_t)N * T;
                R.cost = cost.data(); R.status = status.data();
                rc = pp_plan_batch_host(M, o->device, &D, &prm, &R, nullptr);
                if (rc != PP_OK) break;
                for (int i = 0; i < T; i++) {
                    Conn& c = *conns[who[tel[i]]];
                    c.target_lane = win[i] / prm.n_speeds;
                    c.table.take_back(sl, i, used[i]);
                }
                int64_t need = 0;
                ooff.assign(T + 1, 0);
                int frc = pp_control_format(R.next_x, R.next_y, R.n_out, T, T, nullptr, 0, ooff.data(), o->threads);
                need = ooff[T];
                obuf.resize((size_t)need);
                frc = pp_control_format(R.next_x, R.next_y, R.n_out, T, T, &obuf[0], need, ooff.data(), o->threads);
                if (frc != PP_OK) { rc = frc; break; }
                for (int i = 0; i < T; i++) {
                    Conn& c = *conns[who[tel[i]]];
                    ws_frame(c.out, 1, obuf.data() + ooff[i], (size_t)(ooff[i + 1] - ooff[i]));
                    replies++;
                }
                frames += T;
            }
            for (int i = 0; i < A; i++) {
                Conn& c = *conns[who[i]];
                if (mst[i] == 1) { static const char m[] = "42[\"manual\",{}]"; ws_frame(c.out, 1, m, sizeof(m) - 1); replies++; }
                else if (mst[i] == -1) c.closing = true;
            }
        }
        // flush, drop closed
        for (auto& c : conns) {
            while (!c->out.empty()) {
                const ssize_t w = send(c->fd, c->out.data(), c->out.size(), MSG_NOSIGNAL);
                if (w > 0) { c->out.erase(0, (size_t)w); continue; }
                if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
                c->closing = true;
                c->out.clear();
            }
        }
        for (size_t k = 0; k < conns.size();) {
            if (conns[k]->closing && conns[k]->out.empty()) { close(conns[k]->fd); conns.erase(conns.begin() + k); }
            else k++;
        }
    }
    for (auto& c : conns) close(c->fd);
    close(lfd);
    if (stats) { stats[0] = frames; stats[1] = ticks; stats[2] = accepted; stats[3] = replies; }
    return rc;
}

extern "C" int32_t pp_ws_accept_key(const char* key, char* out, int32_t cap) {
    if (!key || !out || cap < 29) return PP_ERR_ARG;
    const std::string a = ws_accept(key);
    memcpy(out, a.c_str(), a.size() + 1);
    return PP_OK;
}
