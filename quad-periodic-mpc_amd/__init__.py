"""MI355X-native batched convex-MPC solver (drop-in for SolverMPC's C interface)."""
from .records import (CmpcParams, make_params, pack_records, record_words, unpack_gait,  # noqa: F401
                      DEFAULT_WEIGHTS, STATUS_NAMES)
from .instances import make_disturbance, make_instances, make_logs, trot_table  # noqa: F401
