"""Host-side mirror of python-files/truck_trailer_model.py (numpy instead of CasADi SX).

The GPU kernel evaluates the same kinematics (truck_trailer_model.py:8-24) itself; this class
only carries the dimensions / params the controller constructors read, as in the reference.
"""
from __future__ import annotations

import numpy as np


class TruckTrailerModel:
    def __init__(self, params):
        self.num_state = 6  # (x, y, theta, psi, phi, v)
        self.num_input = 2  # (a, omega)
        self._params = params

    def f(self, q, u):
        """truck_trailer_model.py:8-24."""
        p = self._params
        x, y, th, psi, phi, v = np.asarray(q, dtype=np.float64).reshape(6)
        a, om = np.asarray(u, dtype=np.float64).reshape(2)
        t = np.tan(phi)
        return np.array([v * np.cos(th), v * np.sin(th), v * t / p["L1"],
                         -v * t / p["L1"] * (1 + p["M"] / p["L2"] * np.cos(psi)) - v * np.sin(psi) / p["L2"], om, a])

    def compute_next_state(self, x_k, u_k):
        """truck_trailer_model.py:26-29 (forward Euler)."""
        return np.asarray(x_k, dtype=np.float64).reshape(6) + self.f(x_k, u_k) * self._params["dt"]

    def get_vehicle_Hrep(self):
        G = np.array([[1.0, 0.0], [0.0, 1.0], [-1.0, 0.0], [0.0, -1.0]])
        L, W = self._params["L1"], self._params["W1"]
        return G, np.array([[L / 2], [W / 2], [L / 2], [W / 2]])

    def get_trailer_Hrep(self):
        G = np.array([[1.0, 0.0], [0.0, 1.0], [-1.0, 0.0], [0.0, -1.0]])
        L, W = self._params["L2"], self._params["W2"]
        return G, np.array([[L / 2], [W / 2], [L / 2], [W / 2]])

    def get_vehicle_center(self, x_rear, y_rear, heading):
        return (x_rear + np.cos(heading) * self._params["L1"] / 2, y_rear + np.sin(heading) * self._params["L1"] / 2)

    def get_trailer_center(self, x_rear, y_rear, heading, psi):
        xh = x_rear - np.cos(heading) * self._params["M"]
        yh = y_rear - np.sin(heading) * self._params["M"]
        return (xh - np.cos(heading + psi) * self._params["L2"] / 2, yh - np.sin(heading + psi) * self._params["L2"] / 2)
