"""ttmpc -- MI355X-native batched truck-trailer NMPC (drop-in for the reference's mpc_control*.py).

Reference: Avan1ko/car-trailer-mpc python-files/{mpc_control, mpc_control_nmpc, mpc_control_fuzzy,
trajectory_planning, truck_trailer_model}.py.  All solves run in libttmpc.so on a gfx950 GPU.
"""
from ._lib import (STATUS_NAMES, TT_ACCEPTABLE, TT_CONVERGED, TT_HANDOFF_TIMEOUT, TT_INFEASIBLE, TT_MAX_ITER,  # noqa: F401
                   TT_NONFINITE, TT_STEP_FAILED,
                   TT_VARIANT_FUZZY, TT_VARIANT_NMPC, TT_VARIANT_OBCA_PLAN, TT_VARIANT_TRACK, TT_VARIANT_TRACK_OBCA,
                   BatchSolver, ObcaSolver, TTError, lib, obca_n)
from .mpc_control import MPCTrackingControl  # noqa: F401
from .mpc_control_fuzzy import MPCTrackingControlFuzzy, fuzzy_weights  # noqa: F401
from .mpc_control_nmpc import TruckTrailerNMPC  # noqa: F401
from .mpc_control_obs import MPCTrackingControlObs  # noqa: F401
from .trajectory_optimization import TrajectoryOptimization  # noqa: F401
from .truck_trailer_model import TruckTrailerModel  # noqa: F401

__all__ = ["MPCTrackingControl", "MPCTrackingControlObs", "TrajectoryOptimization", "TruckTrailerNMPC", "MPCTrackingControlFuzzy", "TruckTrailerModel", "BatchSolver", "ObcaSolver",
           "fuzzy_weights", "TTError", "lib"]
