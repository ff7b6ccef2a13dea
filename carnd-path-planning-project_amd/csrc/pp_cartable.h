// pp_cartable.h — the reference's cross-frame car table on the host (pp_plan_frame, pp_serve).
//
// The reference keeps `std::map<int, Car> sensor_fusion_cars` across frames (src/main.cpp:1194):
// a car reported in a frame is (re)created and matched — its entry overwritten, or erased when
// matching fails (:1325-1350) — and a car absent from the frame keeps its stale entry, which the
// planner still visits in ascending id order. CarTable holds exactly that map. Before a frame it
// lays the union of its ids and the frame's ids out as pp_scene_batch table slots (include/pp.h
// tab_*: ascending ids, stored state or "empty"); after the frame it takes the slots back (valid:
// the entry is set; invalid: the id is erased). The kernel only ever sees slots, so car ids can be
// any ints; the union is limited to PP_MAX_CARS distinct cars.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <climits>
#include <map>
#include <vector>

#include "../../include/pp.h"

namespace pptab {

struct Entry { int32_t lane; double s, d, vs, vd, vx, vy; };

// slot arrays of one batch: slot k of scene i at [k * stride + i]
struct Slots {
    int64_t stride;
    int32_t *id, *valid, *lane;
    double *s, *d, *vs, *vd, *vx, *vy;
};

struct CarTable {
    std::map<int32_t, Entry> cars;

    // ids of the frame, ascending and distinct (the rows of a parsed/sorted frame)
    int union_size(const int32_t* ids, int n) const {
        int u = (int)cars.size();
        for (int j = 0; j < n; j++)
            if (!cars.count(ids[j]) && (j == 0 || ids[j] != ids[j - 1])) u++;
        return u;
    }
    // writes slots [0, n_slots) of scene i: the union in ascending id order, then padding
    // (id INT32_MAX, empty) up to n_slots. Returns the union size, or -1 if it exceeds n_slots.
    // poison (PP_DBG_POISON): the state of every slot that holds no entry is NaN / INT32_MAX
    // instead of 0 (the kernels must write a reported car's slot before anything reads it).
    int layout(const int32_t* ids, int n, const Slots& t, int64_t i, int n_slots, bool poison = false) const {
        std::vector<int32_t> u;
        u.reserve(cars.size() + n);
        for (const auto& kv : cars) u.push_back(kv.first);
        for (int j = 0; j < n; j++) u.push_back(ids[j]);
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end()), u.end());
        if ((int)u.size() > n_slots) return -1;
        for (int k = 0; k < n_slots; k++) {
            const int64_t x = (int64_t)k * t.stride + i;
            if (k < (int)u.size()) {
                t.id[x] = u[k];
                auto it = cars.find(u[k]);
                if (it != cars.end()) {
                    const Entry& e = it->second;
                    t.valid[x] = 1; t.lane[x] = e.lane;
                    t.s[x] = e.s; t.d[x] = e.d; t.vs[x] = e.vs; t.vd[x] = e.vd; t.vx[x] = e.vx; t.vy[x] = e.vy;
                    continue;
                }
            } else {
                t.id[x] = INT32_MAX;
            }
            const double z = poison ? __builtin_nan("") : 0.0;
            t.valid[x] = 0; t.lane[x] = poison ? INT32_MAX : 0;
            t.s[x] = t.d[x] = t.vs[x] = t.vd[x] = t.vx[x] = t.vy[x] = z;
        }
        return (int)u.size();
    }
    // takes back the n_used slots of scene i after the frame
    void take_back(const Slots& t, int64_t i, int n_used) {
        for (int k = 0; k < n_used; k++) {
            const int64_t x = (int64_t)k * t.stride + i;
            if (t.valid[x]) cars[t.id[x]] = Entry{t.lane[x], t.s[x], t.d[x], t.vs[x], t.vd[x], t.vx[x], t.vy[x]};
            else cars.erase(t.id[x]);
        }
    }
};

}  // namespace pptab
