// cmpc_abi_latency — latency of the drop-in single-instance interface, driven exactly as the
// reference's caller drives it once per MPC step (ConvexMPCLocomotion.cpp:807-836):
//   setup_problem -> update_x_drag -> update_solver_settings -> update_problem_data_floats
//   (synchronous solve) -> get_solution(0..11)
// Links libcmpc_hip.so through include/cmpc_solver.h only. A1 trot instances at every phase of
// the 18-segment gait, body state and command varied per call.
// usage: cmpc_abi_latency [horizon=10] [calls=2000] [use_jcqp=0]  -> one JSON line
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../../include/cmpc_solver.h"

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 10;
  const int calls = argc > 2 ? std::atoi(argv[2]) : 2000;
  const double use_jcqp = argc > 3 ? std::atof(argv[3]) : 0.0;
  const int warm = 50;
  // ConvexMPCLocomotion.cpp:617, :623, :806-807
  float weights[12] = {0.25f, 0.25f, 10, 10, 2, 50, 0, 0, 0.3f, 0.2f, 0.2f, 0.1f};
  const float alpha = 4e-5f, dt = 0.026f, h = 0.29f;
  const float hipx[4] = {0.1805f, 0.1805f, -0.1805f, -0.1805f};
  const float hipy[4] = {-0.1308f, 0.1308f, -0.1308f, 0.1308f};
  std::vector<float> traj(12 * N);
  std::vector<int> gait(4 * N);
  std::vector<double> us;
  us.reserve(calls);
  double fsum = 0.0;
  for (int c = 0; c < warm + calls; c++) {
    const float ph = 0.37f * c;
    const float yaw = 0.3f * std::sin(ph), roll = 0.02f * std::sin(1.3f * ph), pitch = 0.02f * std::cos(ph);
    const float cy = std::cos(yaw / 2), sy = std::sin(yaw / 2), cr = std::cos(roll / 2),
                sr = std::sin(roll / 2), cp = std::cos(pitch / 2), sp = std::sin(pitch / 2);
    float q[4] = {cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy,
                  cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy};
    float p[3] = {0.01f * c, 0.0f, h + 0.01f * std::sin(ph)};
    float v[3] = {0.5f + 0.1f * std::sin(ph), 0.05f * std::cos(ph), 0.0f};
    float w[3] = {0.1f * std::sin(ph), 0.1f * std::cos(ph), 0.2f * std::sin(0.5f * ph)};
    float r[12];
    for (int l = 0; l < 4; l++) {
      r[0 * 4 + l] = std::cos(yaw) * hipx[l] - std::sin(yaw) * hipy[l];
      r[1 * 4 + l] = std::sin(yaw) * hipx[l] + std::cos(yaw) * hipy[l];
      r[2 * 4 + l] = -h;
    }
    const int it = c % 18;  // trot, P = 18, offsets (0, 9, 9, 0), durations 9 (Gait.cpp:159-188)
    const int off[4] = {0, 9, 9, 0};
    for (int i = 0; i < N; i++) {
      const int row = (i + it + 1) % 18;
      for (int l = 0; l < 4; l++) gait[4 * i + l] = ((row - off[l] + 18) % 18) < 9;
      float* t = &traj[12 * i];
      for (int j = 0; j < 12; j++) t[j] = 0.f;
      t[2] = yaw + dt * i * 0.2f;
      t[3] = p[0] + dt * i * 0.5f;
      t[4] = p[1];
      t[5] = h;
      t[8] = 0.2f;
      t[9] = 0.5f;
    }
    // the ROS node's inputs of the periodic-disturbance estimator (SolverMPC.cpp:692-798):
    // simulation time and the measured vertical disturbance, a 1.3 Hz sine here
    simulation_time = dt * c;
    f_ext[3] = 5.f * std::sin(2.f * 3.14159265f * 1.3f * simulation_time);
    const auto t0 = std::chrono::steady_clock::now();
    setup_problem(dt, N, 0.4, 120);
    update_x_drag(0.1f);
    update_solver_settings(10000, 1e-7, 1e-8, 1.5, 0.1, use_jcqp);
    update_problem_data_floats(p, v, q, w, r, roll, pitch, yaw, weights, traj.data(), alpha,
                               gait.data());
    double f = 0.0;
    for (int j = 0; j < 12; j++) f += get_solution(j);
    const auto t1 = std::chrono::steady_clock::now();
    fsum += f;
    if (c >= warm) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  std::sort(us.begin(), us.end());
  auto pct = [&](double x) { return us[std::min(us.size() - 1, (size_t)(x * us.size()))]; };
  std::printf("{\"horizon\": %d, \"use_jcqp\": %g, \"calls\": %d, \"p50_us\": %.1f, \"p90_us\": %.1f, "
              "\"p99_us\": %.1f, \"min_us\": %.1f, \"force_sum\": %.3f}\n",
              N, use_jcqp, calls, pct(0.5), pct(0.9), pct(0.99), us.front(), fsum);
  return 0;
}
