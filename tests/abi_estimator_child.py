"""Child process of tests/test_gpu_estimator.py::test_abi_estimator_sequence (the reference
ABI's estimator state is process-global, as the reference's, so each driven instance needs a
fresh process). Drives instance `i` of the n20_config5 fixture through the single-instance ABI
the way ConvexMPCLocomotion::solveDenseMPC does every MPC step (:639-836): the caller-owned
globals f_ext (residual, component 3 = the disturbance sample) and simulation_time, then
setup_problem -> update_x_drag -> update_solver_settings -> update_problem_data_floats ->
get_solution. Writes per call f_est, f_est_smoothed, f_est_static and the last call's forces.

usage: python tests/abi_estimator_child.py <instance> <out.npz>
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    i, out = int(sys.argv[1]), sys.argv[2]
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    R = importlib.import_module("quad-periodic-mpc_amd.records")
    g = np.load(os.path.join(ROOT, "tests", "golden", "n20_config5.npz"), allow_pickle=False)
    N = int(g["horizon"])
    rec = g["records"][i]
    gait = cm.unpack_gait(rec[None], N)[0].astype(np.int32)
    wts = np.asarray(g["weights"], np.float32)
    T = g["f3"].shape[1]
    fest = np.zeros((T, 6), np.float32)
    smooth = np.zeros((T, 6), np.float32)
    static = np.zeros((T, 6), np.float32)
    for k in range(T):
        sm.set_f_ext([0.0, 0.0, 0.0, float(g["f3"][i, k]), 0.0, 0.0])
        sm.set_simulation_time(float(g["t"][k]))
        sm.setup_problem(float(g["dt"]), N, float(g["mu"]), float(g["f_max"]))
        sm.update_x_drag(float(rec[R.REC_XDRAG]))
        sm.update_solver_settings(100, 1e-7, 1e-8, 1.5, 1e-5, 0)
        sm.update_problem_data_floats(rec[R.REC_P:R.REC_P + 3], rec[R.REC_V:R.REC_V + 3],
                                      rec[R.REC_Q:R.REC_Q + 4], rec[R.REC_W:R.REC_W + 3],
                                      rec[R.REC_R:R.REC_R + 12], rec[R.REC_RPY], rec[R.REC_RPY + 1],
                                      rec[R.REC_RPY + 2], wts, rec[32:32 + 12 * N],
                                      float(g["alpha"]), gait)
        fest[k] = sm.get_f_est("f_est")
        smooth[k] = sm.get_f_est("f_est_smoothed")
        static[k] = sm.get_f_est("f_est_static")
    forces = np.array([sm.get_solution(j) for j in range(12 * N)])
    np.savez(out, fest=fest, smooth=smooth, static=static, forces=forces)


if __name__ == "__main__":
    main()
