// ---- oracle/ref_json.cpp — TEST INFRASTRUCTURE ONLY ------------------------------------------
// The reference's wire codec as the reference itself runs it: helpers.h hasData and the
// vendored nlohmann::json (src/json.hpp), both compiled from /root/reference by oracle/Makefile
// into oracle/_ref/libppref_json.so. The glue below restates src/main.cpp:1217-1252 (message
// filter, parse, field reads), :1325-1333 (sensor_fusion rows into std::map<int, Car>) and
// :1461-1464 (control message dump).
#include <array>
#include <map>
#include <string>
#include <vector>

#include "Eigen-3.3/Eigen/Core"   // helpers.h uses Eigen (main.cpp:5-15 include order)
#include "Eigen-3.3/Eigen/QR"
#include "Eigen-3.3/Eigen/LU"
#include "json.hpp"
#include "helpers.h"

using nlohmann::json;

// 0: telemetry; 1: no data (manual answer); 3: not a "42" frame / other event (no answer);
// -1: the reference would throw
extern "C" int ref_json_parse(const char* msg, double* ego4, double* prev_x, double* prev_y, int cap_prev,
                              int* n_prev, int* ids, double* cars4, int cap_cars, int* n_cars) {
    std::string data(msg);
    const size_t length = data.size();
    if (!(length && length > 2 && data[0] == '4' && data[1] == '2')) return 3;
    auto s = hasData(data);
    if (s == "") return 1;
    try {
        auto j = json::parse(s);
        std::string event = j[0].get<std::string>();
        if (event != "telemetry") return 3;
        double ego_x = j[1]["x"];
        double ego_y = j[1]["y"];
        double ego_yaw = j[1]["yaw"];
        double ego_speed = j[1]["speed"];
        ego4[0] = ego_x; ego4[1] = ego_y; ego4[2] = ego_yaw; ego4[3] = ego_speed;
        auto previous_path_x = j[1]["previous_path_x"];
        auto previous_path_y = j[1]["previous_path_y"];
        const int n = (int)previous_path_x.size();
        *n_prev = n;
        for (int i = 0; i < n && i < cap_prev; i++) {
            double px = previous_path_x[i], py = previous_path_y[i];
            prev_x[i] = px;
            prev_y[i] = py;
        }
        auto sensor_fusion = j[1]["sensor_fusion"];
        std::map<int, std::array<double, 4>> cars;
        for (int i = 0; i < (int)sensor_fusion.size(); i++) {
            auto car_data = sensor_fusion[i];
            int id = car_data[0];
            auto& c = cars[id];
            double x = car_data[1], y = car_data[2], vx = car_data[3], vy = car_data[4];
            c = {x, y, vx, vy};
        }
        int k = 0;
        for (auto& p : cars) {
            if (k < cap_cars) {
                ids[k] = p.first;
                for (int q = 0; q < 4; q++) cars4[4 * k + q] = p.second[q];
            }
            k++;
        }
        *n_cars = k;
    } catch (...) {
        return -1;
    }
    return 0;
}

// returns the message length (bytes written if <= cap)
extern "C" long ref_json_dump(const double* x, const double* y, int n, char* out, long cap) {
    json msgJson;
    msgJson["next_x"] = std::vector<double>(x, x + n);
    msgJson["next_y"] = std::vector<double>(y, y + n);
    auto msg = "42[\"control\"," + msgJson.dump() + "]";
    if ((long)msg.size() <= cap) memcpy(out, msg.data(), msg.size());
    return (long)msg.size();
}
