// plan_frames.cpp — a compiled C++11 caller of the C-ABI (include/pp.h), written exactly as the
// INTEGRATION.md patch tells a maintainer to change the reference's src/main.cpp: the map is made
// once after the CSV load (replacing Map::Init, :1193), and each telemetry frame's planning block
// (:1254-1457) becomes one pp_plan_frame call with the cross-frame target_lane (:1195) passed in
// and updated. Test infrastructure (tests/test_abi_caller.py): g++ -std=c++11, linked against
// libppamd.so like the reference would be.
//
// Usage: plan_frames MAP.bin FRAMES.bin OUT.bin   (GPU: plans every frame)
//        plan_frames MAP.bin --host                (no GPU: the map and the ABI's host entry points)
// MAP.bin: int32 n, n doubles x, n doubles y. FRAMES.bin: int32 count, then per frame: int32 reset
// (1: pp_plan_reset before it, a new episode), int32 target_lane, doubles x, y, yaw, speed,
// int32 n_prev, n_prev x, n_prev y, int32 n_cars, n_cars rows of (int32 id, doubles x, y, vx, vy,
// s, d) — the simulator's sensor_fusion rows. OUT.bin: per frame int32 rc, int32 target_lane,
// int32 n, n x, n y.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "pp.h"

namespace {

struct Reader {
    FILE* f;
    template <typename T> T get() {
        T v;
        if (fread(&v, sizeof(T), 1, f) != 1) { fprintf(stderr, "short read\n"); exit(2); }
        return v;
    }
};

struct Car { int32_t id; double x, y, vx, vy, s, d; };   // a sensor_fusion row [id, x, y, vx, vy, s, d]

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s MAP.bin FRAMES.bin OUT.bin | MAP.bin --host\n", argv[0]); return 2; }
    FILE* mf = fopen(argv[1], "rb");
    if (!mf) { perror(argv[1]); return 2; }
    Reader mr{mf};
    const int32_t n = mr.get<int32_t>();
    std::vector<double> map_waypoints_x(n), map_waypoints_y(n);
    for (int i = 0; i < n; i++) map_waypoints_x[i] = mr.get<double>();
    for (int i = 0; i < n; i++) map_waypoints_y[i] = mr.get<double>();
    fclose(mf);

    // in main(), after the CSV load (replaces map.Init at :1193)
    pp_map* pm = nullptr;
    int32_t rc = pp_map_create(map_waypoints_x.data(), map_waypoints_y.data(), (int32_t)map_waypoints_x.size(), &pm);
    if (rc != PP_OK) { fprintf(stderr, "pp_map_create %d\n", rc); return 1; }
    if (strcmp(argv[2], "--host") == 0) {
        std::vector<double> geo((size_t)n * (4 + 2 * PP_NUM_LANES));
        const int ok = pp_map_geometry(pm, geo.data(), n) == PP_OK && pp_num_lanes() == PP_NUM_LANES &&
                       pp_map_create(nullptr, nullptr, 0, nullptr) == PP_ERR_ARG;
        printf("%s %s lanes=%d\n", ok ? "host-ok" : "host-FAILED", pp_version(), pp_num_lanes());
        pp_map_destroy(pm);
        return ok ? 0 : 1;
    }
    if (argc < 4) return 2;
    rc = pp_reserve(pm, /*device=*/0, /*max_scenes=*/1);
    if (rc != PP_OK) { fprintf(stderr, "pp_reserve %d\n", rc); return 1; }

    FILE* ff = fopen(argv[2], "rb");
    FILE* of = fopen(argv[3], "wb");
    if (!ff || !of) { perror("frames/out"); return 2; }
    Reader fr{ff};
    const int32_t frames = fr.get<int32_t>();
    int failures = 0;
    for (int k = 0; k < frames; k++) {
        const int32_t reset = fr.get<int32_t>();
        int32_t target_lane = fr.get<int32_t>();                 // the lambda's capture (:1195)
        const double x = fr.get<double>(), y = fr.get<double>(), yaw = fr.get<double>(), speed = fr.get<double>();
        const int32_t npv = fr.get<int32_t>();
        std::vector<double> previous_path_x(npv), previous_path_y(npv);
        for (int i = 0; i < npv; i++) previous_path_x[i] = fr.get<double>();
        for (int i = 0; i < npv; i++) previous_path_y[i] = fr.get<double>();
        const int32_t nc = fr.get<int32_t>();
        std::vector<Car> sensor_fusion(nc);
        for (int j = 0; j < nc; j++) {
            Car& c = sensor_fusion[j];
            c.id = fr.get<int32_t>();
            c.x = fr.get<double>(); c.y = fr.get<double>(); c.vx = fr.get<double>(); c.vy = fr.get<double>();
            c.s = fr.get<double>(); c.d = fr.get<double>();
        }
        if (reset) pp_plan_reset(pm, 0);

        // in onMessage, replacing :1254-1457 (as written there)
        std::vector<double> px(previous_path_x.begin(), previous_path_x.end());
        std::vector<double> py(previous_path_y.begin(), previous_path_y.end());
        std::vector<int32_t> ids; std::vector<double> cx, cy, cvx, cvy;
        for (auto& car : sensor_fusion) {                 // rows [id, x, y, vx, vy, s, d]
            ids.push_back(car.id); cx.push_back(car.x); cy.push_back(car.y);
            cvx.push_back(car.vx); cvy.push_back(car.vy);
        }
        double nx[50], ny[50]; int32_t nn = 0;
        rc = pp_plan_frame(pm, 0, x, y, yaw, speed,
                           px.data(), py.data(), (int32_t)px.size(),
                           ids.data(), cx.data(), cy.data(), cvx.data(), cvy.data(),
                           (int32_t)ids.size(), &target_lane, nx, ny, &nn);
        std::vector<double> next_x_vals(nx, nx + (rc == PP_OK ? nn : 0)), next_y_vals(ny, ny + (rc == PP_OK ? nn : 0));

        failures += rc != PP_OK;
        const int32_t m = (int32_t)next_x_vals.size();
        fwrite(&rc, 4, 1, of);
        fwrite(&target_lane, 4, 1, of);
        fwrite(&m, 4, 1, of);
        fwrite(next_x_vals.data(), 8, m, of);
        fwrite(next_y_vals.data(), 8, m, of);
    }
    fclose(ff);
    fclose(of);
    pp_map_destroy(pm);
    printf("planned %d frames, %d failed calls\n", frames, failures);
    return failures ? 1 : 0;
}
