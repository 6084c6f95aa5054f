"""Batched closed-loop simulation on the GPU -- the receding-horizon loop of python-files/simulation.py
(and simulation_nmpc.py) for B Monte-Carlo instances at once, with every per-step array in HBM.

Reference loop (simulation.py:484-531), per instance, per step t = 0, dt, 2dt, ... <= T_sim:
    k = floor(t / dt)                                   (t accumulated with +=, as the reference does)
    window  = reference window at k with end padding                         486-501
    collide = check_trajectory_collision(previous prediction or window)       503-506
    x_meas  = state + N(0, process_noise_std)  (ENABLE_DISTURBANCES)          509-513
    X, U    = controller.solve(x_meas, window)                                516
    state   = update(state, U[:, 0], params, DISTURBANCE_PARAMS)              524-527
Here one step = sim_window_kernel -> collision_kernel -> [warm_kernel] -> track_kernel -> [record_kernel]
-> plant_kernel, all enqueued on one stream (libttmpc.so: tt_sim.hip + tt_track.hip).  With a switch
solver (USE_SWITCH_MPC, simulation.py:23, 433-441) the instances whose check collides are re-solved by
MPCTrackingControlObs (the OBCA kernel) and their results replace the tracking solution.

The reference draws the measurement noise with np.random.normal; pass ``noise`` (steps, B, 6) to
reproduce a given draw, else it is drawn on the device with a seeded torch generator.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np
import torch

from ._lib import TT_ACCEPTABLE, TT_VARIANT_FUZZY, TTError, TTPlant, lib

# closed-loop failure policies (include/ttmpc.h TT_POLICY_*): what a driver does after a failed solve
POLICIES = {"track": 0, "nmpc": 1, "fuzzy": 2}

# simulation.py:26-32
DISTURBANCE_PARAMS = {"friction_coeff": 0.9, "slippage_coeff": 0.9, "process_noise_std": 0.02,
                      "lateral_slip_gain": 0.01, "slip_angle_max": 0.0}
# simulation_nmpc.py:21-27 (there ENABLE_DISTURBANCES = False)
DISTURBANCE_PARAMS_NMPC = {"friction_coeff": 1.0, "slippage_coeff": 1.0, "process_noise_std": 0.02,
                           "lateral_slip_gain": 0.0, "slip_angle_max": 0.0}


def plant(params, disturbance_params=None) -> TTPlant:
    """tt_plant from the reference's params dict (+ DISTURBANCE_PARAMS, or None = nominal update)."""
    p = TTPlant()
    p.dt, p.L1, p.L2, p.Mh = float(params["dt"]), float(params["L1"]), float(params["L2"]), float(params["M"])
    p.W1, p.W2 = float(params.get("W1", 0.0)), float(params.get("W2", 0.0))
    d = disturbance_params
    p.enable = int(d is not None)
    d = d or {}
    # apply_disturbances / apply_slippage_to_dynamics / apply_lateral_slip skip a missing key
    p.friction_coeff = float(d.get("friction_coeff", 1.0))
    p.slippage_coeff = float(d.get("slippage_coeff", 1.0))
    p.process_noise_std = float(d.get("process_noise_std", 0.0))
    p.lateral_slip_gain = float(d.get("lateral_slip_gain", 0.0))
    p.slip_angle_max = float(d.get("slip_angle_max", 0.0))
    return p


def _stream(stream, dev):
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    return C.c_void_p(s.cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise TTError(f"{what} failed ({rc})")


def _dev(a, dev, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a) if not torch.is_tensor(a) else a, dtype=dtype).to(dev).contiguous()


# ---------------------------------------------------------------- single-kernel device entry points
def window(plan_x, plan_u, k, N, state=None, noise=None, x_meas=None, xref=None, uref=None, stream=None):
    """Reference window (simulation.py:486-501) for every instance: plan_x (P,Np+1,6), plan_u (P,Np,2) device
    tensors with P = 1 (shared plan) or B; state (B,6) -> x_meas = state + noise (509-513)."""
    dev = plan_x.device
    Np = plan_u.shape[-2]
    B = state.shape[0] if state is not None else plan_x.shape[0]
    xref = torch.empty((B, N + 1, 6), dtype=torch.float64, device=dev) if xref is None else xref
    uref = torch.empty((B, N, 2), dtype=torch.float64, device=dev) if uref is None else uref
    if state is not None and x_meas is None:
        x_meas = torch.empty((B, 6), dtype=torch.float64, device=dev)
    per = int(plan_x.shape[0] != 1)
    if per and plan_x.shape[0] != B:
        raise ValueError("per-instance plans need one plan per instance")
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    _check(lib().tt_sim_window_device(B, int(N), int(k), int(Np), plan_x.data_ptr(), plan_u.data_ptr(), per,
                                      ptr(state), ptr(noise), ptr(x_meas), xref.data_ptr(), uref.data_ptr(),
                                      _stream(stream, dev)), "tt_sim_window_device")
    return x_meas, xref, uref


def collision_flags(poses, obstacles, params, flag=None, stream=None):
    """check_trajectory_collision (simulation.py:363-385) per instance: poses (B,K,>=4) device tensor with
    contiguous rows; obstacles (M,4) device tensor.  -> int32 flag (B,)."""
    dev = poses.device
    B, K, w = poses.shape
    flag = torch.empty(B, dtype=torch.int32, device=dev) if flag is None else flag
    p = plant(params)
    M = 0 if obstacles is None else int(obstacles.shape[0])
    if poses.stride(-1) != 1:
        raise ValueError("pose rows must be contiguous")
    sk = poses.stride(1) if K > 1 else w          # a size-1 dim may carry any stride (numpy gives 0)
    _check(lib().tt_collision_device(B, K, poses.data_ptr(), poses.stride(0), sk,
                                     None if M == 0 else obstacles.data_ptr(), M, C.byref(p), flag.data_ptr(),
                                     _stream(stream, dev)), "tt_collision_device")
    return flag


def plant_update(state, u, params, disturbance_params=None, status=None, zero_on_fail=False, u_applied=None,
                 stream=None, state_noise=None):
    """update(q, u, params, disturbance_params) (simulation.py:167-199) in place on state (B,6); u is
    (B,2) or a solve's U (B,N,2) (applies U[:, 0]).  state_noise (B,6): the NMPC / fuzzy drivers' update
    (simulation_nmpc.py:94-105), which adds state_noise * dt right after the Euler step."""
    dev = state.device
    p = plant(params, disturbance_params)
    stride = u.stride(0)
    if state_noise is not None and (state_noise.shape != state.shape or not state_noise.is_contiguous()):
        raise ValueError("state_noise must be a contiguous (B, 6) tensor")
    _check(lib().tt_plant_update_noise_device(state.shape[0], C.byref(p), state.data_ptr(), u.data_ptr(), stride,
                                              None if status is None else status.data_ptr(), int(bool(zero_on_fail)),
                                              None if state_noise is None else state_noise.data_ptr(),
                                              None if u_applied is None else u_applied.data_ptr(), _stream(stream, dev)),
           "tt_plant_update_noise_device")
    return state


def update(q, u, params, disturbance_params=None, device=0, state_noise=None):
    """Host convenience with the reference's signature (simulation.py:167): one state, numpy in / out.
    state_noise (6,): simulation_nmpc.py / simulation_fuzzy.py's update, with the process noise the reference
    draws inside apply_disturbances given explicitly."""
    dev = torch.device("cuda", device)
    s = _dev(np.asarray(q, dtype=np.float64).reshape(1, 6), dev)
    sn = None if state_noise is None else _dev(np.asarray(state_noise, dtype=np.float64).reshape(1, 6), dev)
    plant_update(s, _dev(np.asarray(u, dtype=np.float64).reshape(1, 2), dev), params, disturbance_params,
                 state_noise=sn)
    return s.cpu().numpy()[0]


def interpolate(state_traj, input_traj, dt_1, dt_2, stream=None):
    """do_interpolation (simulation.py:201-218) of B plans on the device: (B,Np+1,6), (B,Np,2) ->
    (B,nNp+1,6), (B,nNp,2), n = floor(dt_1/dt_2)."""
    dev = state_traj.device
    B, Np = input_traj.shape[0], input_traj.shape[1]
    n = math.floor(dt_1 / dt_2)
    so = torch.empty((B, n * Np + 1, 6), dtype=torch.float64, device=dev)
    uo = torch.empty((B, n * Np, 2), dtype=torch.float64, device=dev)
    _check(lib().tt_interpolate_device(B, Np, n, state_traj.data_ptr(), input_traj.data_ptr(), so.data_ptr(),
                                       uo.data_ptr(), _stream(stream, dev)), "tt_interpolate_device")
    return so, uo


def step_indices(T_sim, dt):
    """The reference's step sequence: t = 0; while t <= T_sim: k = floor(t/dt); ...; t += dt."""
    ks, t = [], 0.0
    while t <= T_sim:
        ks.append(math.floor(t / dt))
        t += dt
    return ks


class ClosedLoop:
    """B independent closed loops driven by one tracking solver (a ttmpc.BatchSolver of horizon N).

    plan_x / plan_u: one shared plan in the reference's (6,Np+1) / (2,Np) orientation (e.g.
    do_interpolation(state_traj.txt, ...)), or (B,Np+1,6) / (B,Np,2) per-instance plans.  warm_start=True
    is TruckTrailerNMPC's shifted warm start (NMPC / fuzzy solvers).

    policy: the driver's reaction to a failed solve, on the device per instance (tt_policy_plant_device):
      "track" (simulation.py:519-527) applies the returned inputs; "nmpc" (simulation_nmpc.py:206-216)
      applies zero control and stops the instance after 20 consecutive failures; "fuzzy"
      (simulation_fuzzy.py:207-221) re-applies the last successful control, zero after 15 consecutive
      failures, stops after 30.  Default: "fuzzy" for a TT_VARIANT_FUZZY solver, "nmpc" when
      zero_on_fail=True, else "track".  A TT_VARIANT_FUZZY solver gets per-instance fuzzy weights each step
      (tt_fuzzy_weights_device, mpc_control_fuzzy.py:90-119) and its failed instances are re-solved once
      with unit weights from the same guess (145-159).

    noise_in_plant=True is the NMPC / fuzzy drivers' disturbance model (simulation_nmpc.py:94-105,
    simulation_fuzzy.py): the solver sees the exact state and, with disturbances on, the process noise
    N(0, process_noise_std) enters the plant as q_ += noise * dt (tt_policy_plant_noise_device); the default is
    simulation.py's (noise on the measured state, simulation.py:509-513).  Default: True for the "nmpc" and
    "fuzzy" policies."""

    def __init__(self, solver, plan_x, plan_u, params, disturbance_params=None, measurement_noise=None,
                 obstacles=None, check_collision=True, switch_solver=None, warm_start=False, bug_compatible=True,
                 zero_on_fail=False, device=None, seed=0, policy=None, noise_in_plant=None):
        self.solver = solver
        self.N = solver.N
        self.dev = torch.device("cuda", solver.device if device is None else device)
        px, pu = np.asarray(plan_x, dtype=np.float64), np.asarray(plan_u, dtype=np.float64)
        if px.ndim == 2:   # one shared plan in the reference's orientation: (6, Np+1), (2, Np)
            px, pu = px.T[None], pu.T[None]
        self.plan_x, self.plan_u = _dev(px, self.dev), _dev(pu, self.dev)
        self.params = dict(params)
        self.dist = disturbance_params
        # simulation.py:509-513: noisy measurement iff disturbances are on
        self.measurement_noise = (disturbance_params is not None) if measurement_noise is None else measurement_noise
        self.obstacles = None if obstacles is None else _dev(np.asarray(obstacles, dtype=np.float64).reshape(-1, 4),
                                                             self.dev)
        self.check_collision = check_collision and self.obstacles is not None
        self.switch = switch_solver
        self.warm, self.bug_compatible, self.zero_on_fail = warm_start, bug_compatible, zero_on_fail
        self.fuzzy = getattr(solver, "variant", None) == TT_VARIANT_FUZZY
        if policy is None:
            policy = "fuzzy" if self.fuzzy else ("nmpc" if zero_on_fail else "track")
        if policy not in POLICIES:
            raise ValueError(f"policy must be one of {sorted(POLICIES)}")
        self.policy = policy
        self.noise_in_plant = (policy in ("nmpc", "fuzzy")) if noise_in_plant is None else bool(noise_in_plant)
        if self.noise_in_plant and measurement_noise:
            raise ValueError("noise_in_plant: the NMPC / fuzzy drivers measure the exact state")
        if self.noise_in_plant:
            self.measurement_noise = False
        self.gen = torch.Generator(device=self.dev)
        self.gen.manual_seed(int(seed))
        self.stream = torch.cuda.Stream(self.dev)

    def _alloc(self, B):
        N, d, f = self.N, self.dev, torch.float64
        self.B = B
        self.state = torch.empty((B, 6), dtype=f, device=d)
        self.x_meas = torch.empty((B, 6), dtype=f, device=d)
        self.xref = torch.empty((B, N + 1, 6), dtype=f, device=d)
        self.uref = torch.empty((B, N, 2), dtype=f, device=d)
        self.X = torch.empty((B, N + 1, 6), dtype=f, device=d)
        self.U = torch.empty((B, N, 2), dtype=f, device=d)
        self.st = torch.empty(B, dtype=torch.int32, device=d)
        self.it = torch.empty(B, dtype=torch.int32, device=d)
        self.kkt = torch.empty(B, dtype=f, device=d)
        self.flag = torch.zeros(B, dtype=torch.int32, device=d)
        self.u_applied = torch.empty((B, 2), dtype=f, device=d)
        # failure-policy state (tt_policy_plant_device)
        self.u_last = torch.zeros((B, 2), dtype=f, device=d)
        self.consec = torch.zeros(B, dtype=torch.int32, device=d)
        self.fails = torch.zeros(B, dtype=torch.int32, device=d)
        self.active = torch.ones(B, dtype=torch.int32, device=d)
        if self.fuzzy:
            self.wq = torch.empty((B, 8), dtype=f, device=d)
        if self.warm:
            self.zg = torch.empty((B, 8 * N + 6), dtype=f, device=d)
            self.last = torch.zeros((B, 8 * N + 6), dtype=f, device=d)
            self.have = torch.zeros(B, dtype=torch.int32, device=d)

    def reset(self, x_init):
        x = np.asarray(x_init, dtype=np.float64).reshape(-1, 6)
        self._alloc(x.shape[0])
        self.state.copy_(_dev(x, self.dev))
        self.first = True
        # the buffers were allocated and filled on the current stream; step() works on self.stream
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))

    def _check_noise(self, noise, shape):
        """noise must be a float64 tensor of exactly `shape` on the loop's device (the kernels index it as such)."""
        if not (isinstance(noise, torch.Tensor) and noise.dtype == torch.float64 and noise.device == self.dev and
                tuple(noise.shape) == tuple(shape)):
            got = (tuple(noise.shape), noise.dtype, noise.device) if isinstance(noise, torch.Tensor) else type(noise)
            raise ValueError(f"noise must be a float64 tensor of shape {tuple(shape)} on {self.dev}, got {got}")

    def step(self, k, noise=None):
        """Enqueue one closed-loop step at window index k (noise: (B,6) float64 device tensor or None: the measurement
        noise, or with noise_in_plant -- the default of the "nmpc" / "fuzzy" policies -- the plant's process noise
        before its dt factor)."""
        L, s, B, N = lib(), self.stream, self.B, self.N
        sp = C.c_void_p(s.cuda_stream)
        if noise is not None:
            self._check_noise(noise, (B, 6))
        with torch.cuda.stream(s):
            if (self.measurement_noise or self.noise_in_plant) and noise is None and self.dist is not None:
                noise = torch.randn((B, 6), generator=self.gen, dtype=torch.float64, device=self.dev)
                noise.mul_(float(self.dist.get("process_noise_std", 0.0)))
            window(self.plan_x, self.plan_u, k, N, self.state, noise if self.measurement_noise else None,
                   self.x_meas, self.xref, self.uref, stream=s)
            if self.check_collision:
                collision_flags(self.xref if self.first else self.X, self.obstacles, self.params, self.flag, stream=s)
            zg = 0
            if self.warm:
                _check(L.tt_warm_start_device(B, N, self.last.data_ptr(), self.have.data_ptr(), self.xref.data_ptr(),
                                              self.uref.data_ptr(), int(self.bug_compatible), self.zg.data_ptr(), sp),
                       "tt_warm_start_device")
                zg = self.zg.data_ptr()
            wq = 0
            if self.fuzzy:
                _check(L.tt_fuzzy_weights_device(B, N, self.x_meas.data_ptr(), self.xref.data_ptr(), self.wq.data_ptr(),
                                                 sp), "tt_fuzzy_weights_device")
                wq = self.wq.data_ptr()
            self.solver.solve_device(B, self.x_meas.data_ptr(), self.xref.data_ptr(), self.uref.data_ptr(),
                                     self.X.data_ptr(), self.U.data_ptr(), self.st.data_ptr(), self.it.data_ptr(),
                                     self.kkt.data_ptr(), wq_wr=wq, z_guess=zg, stream=s.cuda_stream)
            if self.fuzzy:
                self._fuzzy_retry(s)
            if self.switch is not None and self.check_collision:
                self._switch_solve(s)
            if self.warm:
                _check(L.tt_record_solution_device(B, N, self.X.data_ptr(), self.U.data_ptr(), self.st.data_ptr(),
                                                   self.last.data_ptr(), self.have.data_ptr(), sp),
                       "tt_record_solution_device")
            self._policy_plant(sp, noise if self.noise_in_plant else None)
        self.first = False

    def _policy_plant(self, sp, state_noise=None):
        p = plant(self.params, self.dist)
        sn = None
        if state_noise is not None:
            self._check_noise(state_noise, (self.B, 6))
            state_noise = state_noise.contiguous()
            self._sn = state_noise    # keep it alive until the stream has consumed it
            sn = state_noise.data_ptr()
        _check(lib().tt_policy_plant_noise_device(self.B, C.byref(p), POLICIES[self.policy], self.state.data_ptr(),
                                                  self.U.data_ptr(), self.U.stride(0), self.st.data_ptr(),
                                                  self.u_last.data_ptr(), self.consec.data_ptr(), self.fails.data_ptr(),
                                                  self.active.data_ptr(), sn, self.u_applied.data_ptr(), sp),
               "tt_policy_plant_noise_device")

    def _fuzzy_retry(self, s):
        """mpc_control_fuzzy.py:145-159: failed instances re-solve once with unit weights, same guess."""
        idx = torch.nonzero((self.st > TT_ACCEPTABLE) & (self.active != 0), as_tuple=True)[0]
        n = int(idx.numel())          # host sync: the compaction size decides the retry launch
        if n == 0:
            return
        N = self.N
        x0, xr, ur = self.x_meas[idx].contiguous(), self.xref[idx].contiguous(), self.uref[idx].contiguous()
        w = torch.ones((n, 8), dtype=torch.float64, device=self.dev)
        zg = self.zg[idx].contiguous() if self.warm else None
        X = torch.empty((n, N + 1, 6), dtype=torch.float64, device=self.dev)
        U = torch.empty((n, N, 2), dtype=torch.float64, device=self.dev)
        st = torch.empty(n, dtype=torch.int32, device=self.dev)
        it = torch.empty(n, dtype=torch.int32, device=self.dev)
        kk = torch.empty(n, dtype=torch.float64, device=self.dev)
        self.solver.solve_device(n, x0.data_ptr(), xr.data_ptr(), ur.data_ptr(), X.data_ptr(), U.data_ptr(),
                                 st.data_ptr(), it.data_ptr(), kk.data_ptr(), wq_wr=w.data_ptr(),
                                 z_guess=0 if zg is None else zg.data_ptr(), stream=s.cuda_stream)
        self.X[idx], self.U[idx], self.st[idx], self.it[idx], self.kkt[idx] = X, U, st, it, kk

    # ---------------- hipGraph replay of the closed loop ----------------
    def _graph_step(self, first, d_ks, d_step, noise_all, logs):
        """Enqueue one closed-loop step whose step index lives on the device (replayable)."""
        L, s, B, N = lib(), self.stream, self.B, self.N
        sp = C.c_void_p(s.cuda_stream)
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        Np = self.plan_u.shape[-2]
        per = int(self.plan_x.shape[0] != 1)
        meas_all = None if self.noise_in_plant else noise_all
        _check(L.tt_sim_window_indexed_device(B, N, d_ks.data_ptr(), d_step.data_ptr(), int(Np),
                                              self.plan_x.data_ptr(), self.plan_u.data_ptr(), per,
                                              self.state.data_ptr(), ptr(meas_all), self.x_meas.data_ptr(),
                                              self.xref.data_ptr(), self.uref.data_ptr(), sp),
               "tt_sim_window_indexed_device")
        if self.check_collision:
            collision_flags(self.xref if first else self.X, self.obstacles, self.params, self.flag, stream=s)
        zg = 0
        if self.warm:
            _check(L.tt_warm_start_device(B, N, self.last.data_ptr(), self.have.data_ptr(), self.xref.data_ptr(),
                                          self.uref.data_ptr(), int(self.bug_compatible), self.zg.data_ptr(), sp),
                   "tt_warm_start_device")
            zg = self.zg.data_ptr()
        self.solver.solve_device(B, self.x_meas.data_ptr(), self.xref.data_ptr(), self.uref.data_ptr(),
                                 self.X.data_ptr(), self.U.data_ptr(), self.st.data_ptr(), self.it.data_ptr(),
                                 self.kkt.data_ptr(), z_guess=zg, stream=s.cuda_stream)
        if self.warm:
            _check(L.tt_record_solution_device(B, N, self.X.data_ptr(), self.U.data_ptr(), self.st.data_ptr(),
                                               self.last.data_ptr(), self.have.data_ptr(), sp),
                   "tt_record_solution_device")
        sn = None
        if self.noise_in_plant and noise_all is not None:  # this step's process noise, selected on the device
            sn = self._sn_buf
            sn.copy_(torch.index_select(noise_all, 0, d_step.long()).view(B, 6))
        self._policy_plant(sp, sn)
        S, Ua, Ss, Si, Sc = logs
        _check(L.tt_sim_log_advance_device(B, d_step.data_ptr(), self.state.data_ptr(), self.u_applied.data_ptr(),
                                           self.st.data_ptr(), self.it.data_ptr(),
                                           self.flag.data_ptr() if self.check_collision else None, S.data_ptr(),
                                           Ua.data_ptr(), Ss.data_ptr(), Si.data_ptr(), Sc.data_ptr(), sp),
               "tt_sim_log_advance_device")

    def run_graph(self, x_init, T_sim, noise=None):
        """run() with the per-step launches captured once into a hipGraph (torch.cuda.CUDAGraph on this
        loop's stream) and replayed: step 0 runs eagerly (its collision check looks at the first window,
        simulation.py:503-506), steps 1.. replay the captured step.  The step index, the reference's k
        sequence and the measurement noise of every step are device-resident.  Not available with a switch
        solver (its compaction needs the host).  Same logs as run()."""
        if self.switch is not None or self.fuzzy:
            raise ValueError("run_graph supports neither the switch solver nor the fuzzy retry (host compaction); "
                             "use run()")
        ks = step_indices(T_sim, float(self.params["dt"]))
        self.reset(x_init)
        B, K, d, s = self.B, len(ks), self.dev, self.stream
        d_ks = torch.tensor(ks, dtype=torch.int32, device=d)
        d_step = torch.zeros(1, dtype=torch.int32, device=d)
        noise_all = None
        self._sn_buf = torch.empty((B, 6), dtype=torch.float64, device=d)
        if (self.measurement_noise or self.noise_in_plant) and self.dist is not None:
            if noise is None:
                noise_all = torch.randn((K, B, 6), generator=self.gen, dtype=torch.float64, device=d)
                noise_all.mul_(float(self.dist.get("process_noise_std", 0.0)))
            else:
                arr = noise if isinstance(noise, torch.Tensor) else np.asarray(noise, dtype=np.float64)
                if tuple(arr.shape) != (K, B, 6):
                    raise ValueError(f"noise must have shape (steps, B, 6) = {(K, B, 6)}, got {tuple(arr.shape)}")
                noise_all = _dev(arr, d)
        logs = (torch.empty((K + 1, B, 6), dtype=torch.float64, device=d),
                torch.empty((K, B, 2), dtype=torch.float64, device=d),
                torch.zeros((K, B), dtype=torch.int32, device=d), torch.zeros((K, B), dtype=torch.int32, device=d),
                torch.zeros((K, B), dtype=torch.int32, device=d))
        logs[0][0].copy_(self.state)
        torch.cuda.synchronize(d)
        with torch.cuda.stream(s):
            self._graph_step(True, d_ks, d_step, noise_all, logs)
        if K > 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                self._graph_step(False, d_ks, d_step, noise_all, logs)
            with torch.cuda.stream(s):  # replay() launches on the current stream
                for _ in range(K - 1):
                    g.replay()
        torch.cuda.synchronize(d)
        self.first = False
        S, Ua, Ss, Si, Sc = (t.cpu().numpy() for t in logs)
        return dict(self._policy_logs(), k=np.array(ks), states=S, controls=Ua, status=Ss, iters=Si,
                    collide=Sc.astype(bool), success=Ss <= TT_ACCEPTABLE)

    def _switch_solve(self, s):
        """USE_SWITCH_MPC: instances whose check collided use MPCTrackingControlObs (simulation.py:506-512)."""
        idx = torch.nonzero(self.flag, as_tuple=True)[0]
        n = int(idx.numel())          # host sync: the compaction size decides the OBCA launch
        if n == 0:
            return
        o, N = self.switch, self.N
        x0, xr, ur = self.x_meas[idx].contiguous(), self.xref[idx].contiguous(), self.uref[idx].contiguous()
        X = torch.empty((n, N + 1, 6), dtype=torch.float64, device=self.dev)
        U = torch.empty((n, N, 2), dtype=torch.float64, device=self.dev)
        st = torch.empty(n, dtype=torch.int32, device=self.dev)
        it = torch.empty(n, dtype=torch.int32, device=self.dev)
        kk = torch.empty(n, dtype=torch.float64, device=self.dev)
        o.solve_device(n, x0.data_ptr(), 0, xr.data_ptr(), ur.data_ptr(), 0, X.data_ptr(), U.data_ptr(), 0,
                       st.data_ptr(), it.data_ptr(), kk.data_ptr(), stream=s.cuda_stream)
        self.X[idx], self.U[idx], self.st[idx], self.it[idx], self.kkt[idx] = X, U, st, it, kk

    def run(self, x_init, T_sim, noise=None, record=True):
        """Run the reference's loop to T_sim.  noise: optional (steps, B, 6) measurement-noise draws (with
        noise_in_plant: the plant's process-noise draws).
        Returns numpy logs: states (steps+1,B,6), controls (steps,B,2) as applied, status / iters /
        collide (steps,B), and the step indices k."""
        ks = step_indices(T_sim, float(self.params["dt"]))
        self.reset(x_init)
        B, K = self.B, len(ks)
        if record:
            S = torch.empty((K + 1, B, 6), dtype=torch.float64, device=self.dev)
            Ua = torch.empty((K, B, 2), dtype=torch.float64, device=self.dev)
            Ss = torch.empty((K, B), dtype=torch.int32, device=self.dev)
            Si = torch.empty((K, B), dtype=torch.int32, device=self.dev)
            Sc = torch.empty((K, B), dtype=torch.int32, device=self.dev)
            Sa = torch.empty((K, B), dtype=torch.int32, device=self.dev)
            S[0].copy_(self.state)
        nz = None if noise is None else _dev(noise, self.dev)
        if nz is not None and tuple(nz.shape) != (K, B, 6):
            raise ValueError(f"noise must have shape (steps, B, 6) = {(K, B, 6)}, got {tuple(nz.shape)}")
        for j, k in enumerate(ks):
            self.step(k, None if nz is None else nz[j])
            if record:
                with torch.cuda.stream(self.stream):
                    S[j + 1].copy_(self.state)
                    Ua[j].copy_(self.u_applied)
                    Ss[j].copy_(self.st)
                    Si[j].copy_(self.it)
                    Sc[j].copy_(self.flag)
                    Sa[j].copy_(self.active)
        torch.cuda.synchronize(self.dev)
        pol = self._policy_logs()
        if not record:
            return dict(pol, k=np.array(ks), state=self.state.cpu().numpy())
        act = Sa.cpu().numpy()
        stop = np.where((act == 0).any(axis=0), (act == 0).argmax(axis=0), -1)
        return dict(pol, k=np.array(ks), states=S.cpu().numpy(), controls=Ua.cpu().numpy(), status=Ss.cpu().numpy(),
                    iters=Si.cpu().numpy(), collide=Sc.cpu().numpy().astype(bool),
                    success=Ss.cpu().numpy() <= TT_ACCEPTABLE, active=act.astype(bool), stop_step=stop)

    def _policy_logs(self):
        """failure_count / consecutive_failures of the reference drivers, per instance, and whether the
        instance is still running (False = stopped by the policy)."""
        return {"failures": self.fails.cpu().numpy(), "consecutive_failures": self.consec.cpu().numpy(),
                "running": self.active.cpu().numpy().astype(bool)}
