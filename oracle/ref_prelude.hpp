// oracle/ref_prelude.hpp — TEST INFRASTRUCTURE ONLY (parity checker build).
//
// Prepended to the reference's own src/main.cpp lines 22-1154 (constants, Car, Map,
// LaneChangePlanner, SpeedController, TrajectoryBuilder, LimitSpeed, jump_to_waypoint) when
// oracle/Makefile builds oracle/_ref/libppref.so. It includes exactly the reference headers that
// main.cpp:5-15 includes for that code (vendored Eigen, helpers.h, spline.h) and the std headers;
// main.cpp:4 (uWebSockets, absent from the image) and json.hpp are only used by main() at
// :1156-1495, which is not compiled. No reference source is copied into the repository: the
// Makefile streams the line range from /root/reference straight into g++.
#include <fstream>
#include <iostream>
#include <map>
#include <string>
#include <vector>
#include <stdio.h>
#include <math.h>
#include "Eigen-3.3/Eigen/Core"
#include "Eigen-3.3/Eigen/QR"
#include "Eigen-3.3/Eigen/LU"
#include "helpers.h"
#include "spline.h"
using std::string;
using std::vector;

// The horizon's point count. The reference hard-codes it as the literal 50 at src/main.cpp:854
// (`result_points.size() < 50`) and :1039 (`>= 50`); _ref/libppref_n.so is built with exactly those
// two literals replaced by this variable (oracle/Makefile), so ref_set_params can pin horizons other
// than 50 to the reference's own code. The 50 m reach at :911 is a distance and stays as it lies.
// In the builds without the substitution the variable only sizes the harness's output arrays.
int ref_n_points = 50;
