"""Flight recorder with the reference ``Logger``'s API and on-disk format
(``gym_pybullet_drones/utils/Logger.py``).

The arrays live in device memory ([T][D][16] time-major, so one log call for all drones is
one contiguous write) and only ``save()`` / ``save_as_csv()`` / the array properties bring them
to the host in the reference's layout: ``timestamps`` (D, T), ``states`` (D, 16, T) with the
16-state reorder [pos, vel, rpy, ang_v, rpm] of the 20-float state vector, ``controls``
(D, 12, T).  ``log()`` keeps the reference's per-drone counter semantics (:83-127), including
its grow-by-one-column and not-preallocated rules; ``log_batch()`` logs every drone of a
``BatchedAviarySim`` at once from the device-resident state (``sim.state20()``).
Plotting is out of scope (matplotlib is not part of the path).
"""
import os
from datetime import datetime

import numpy as np
import torch

# Logger.log: np.hstack([state[0:3], state[10:13], state[7:10], state[13:20]])   (:125)
REORDER = (0, 1, 2, 10, 11, 12, 7, 8, 9, 13, 14, 15, 16, 17, 18, 19)


class Logger:
    def __init__(self, logging_freq_hz, output_folder="results", num_drones=1, duration_sec=0, colab=False,
                 device=None, dtype=torch.float64):
        self.COLAB = colab
        self.OUTPUT_FOLDER = output_folder
        if not os.path.exists(self.OUTPUT_FOLDER):
            os.mkdir(self.OUTPUT_FOLDER)
        self.LOGGING_FREQ_HZ = logging_freq_hz
        self.NUM_DRONES = int(num_drones)
        self.PREALLOCATED_ARRAYS = False if duration_sec == 0 else True
        self.counters = np.zeros(self.NUM_DRONES)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.dtype = dtype
        self._width = int(duration_sec * self.LOGGING_FREQ_HZ)     # logical number of columns
        self._alloc(max(self._width, 16))
        self._idx = torch.tensor(REORDER, device=self.device)

    # ------------------------------------------------------------------ storage
    def _alloc(self, cap):
        D = self.NUM_DRONES
        ts = torch.zeros((cap, D), dtype=self.dtype, device=self.device)
        st = torch.zeros((cap, D, 16), dtype=self.dtype, device=self.device)
        ct = torch.zeros((cap, D, 12), dtype=self.dtype, device=self.device)
        if hasattr(self, "_ts"):
            n = self._ts.shape[0]
            ts[:n], st[:n], ct[:n] = self._ts, self._st, self._ct
        self._ts, self._st, self._ct = ts, st, ct

    def _grow_one(self):
        if self._width >= self._ts.shape[0]:
            self._alloc(2 * self._ts.shape[0])
        self._width += 1

    def _as_dev(self, x, n):
        t = torch.as_tensor(x, dtype=self.dtype).to(self.device)
        return t.reshape(-1)[:n] if t.dim() <= 1 else t

    # ------------------------------------------------------------------ reference API
    def log(self, drone, timestamp, state, control=np.zeros(12)):
        """Logger.log (:83-127) for one drone."""
        if drone < 0 or drone >= self.NUM_DRONES or timestamp < 0 or len(state) != 20 or len(control) != 12:
            print("[ERROR] in Logger.log(), invalid data")
        current_counter = int(self.counters[drone])
        if current_counter >= self._width:
            self._grow_one()
        elif not self.PREALLOCATED_ARRAYS and self._width > current_counter:
            current_counter = self._width - 1
        s = self._as_dev(state, 20)
        self._ts[current_counter, drone] = float(timestamp)
        self._st[current_counter, drone] = s.index_select(0, self._idx)
        self._ct[current_counter, drone] = self._as_dev(control, 12)
        self.counters[drone] = current_counter + 1

    def log_batch(self, timestamp, states, controls=None):
        """Equivalent to ``log(d, timestamp, states[d], controls[d])`` for d = 0..D-1, as one
        device write: ``states`` [D, 20] (e.g. ``sim.state20()``), ``controls`` [D, 12] or None."""
        c = int(self.counters[0])
        if not np.all(self.counters == c):
            for d in range(self.NUM_DRONES):
                self.log(d, timestamp, states[d], np.zeros(12) if controls is None else controls[d])
            return
        if c >= self._width:
            self._grow_one()
        elif not self.PREALLOCATED_ARRAYS and self._width > c:
            c = self._width - 1
        s = torch.as_tensor(states).to(device=self.device, dtype=self.dtype).reshape(self.NUM_DRONES, 20)
        self._ts[c] = float(timestamp)
        self._st[c] = s.index_select(1, self._idx)
        if controls is None:
            self._ct[c] = 0
        else:
            self._ct[c] = torch.as_tensor(controls).to(device=self.device, dtype=self.dtype).reshape(self.NUM_DRONES, 12)
        self.counters[:] = c + 1

    @property
    def timestamps(self):
        return self._ts[:self._width].transpose(0, 1).cpu().numpy()

    @property
    def states(self):
        return self._st[:self._width].permute(1, 2, 0).cpu().numpy()

    @property
    def controls(self):
        return self._ct[:self._width].permute(1, 2, 0).cpu().numpy()

    def save(self):
        """Logger.save (:131-135): np.savez(timestamps, states, controls) into
        ``save-flight-<date>.npy``; returns the path."""
        path = os.path.join(self.OUTPUT_FOLDER, "save-flight-" + datetime.now().strftime("%m.%d.%Y_%H.%M.%S") + ".npy")
        with open(path, 'wb') as out_file:
            np.savez(out_file, timestamps=self.timestamps, states=self.states, controls=self.controls)
        return path

    def save_as_csv(self, comment=""):
        """Logger.save_as_csv (:139-207): one two-column (t, value) CSV per quantity and drone."""
        csv_dir = os.path.join(self.OUTPUT_FOLDER, "save-flight-" + comment + "-" + datetime.now().strftime("%m.%d.%Y_%H.%M.%S"))
        if not os.path.exists(csv_dir):
            os.makedirs(csv_dir + '/')
        st = self.states
        T = st.shape[2]
        t = np.arange(0, T / self.LOGGING_FREQ_HZ, 1 / self.LOGGING_FREQ_HZ)

        def dump(name, v):
            with open(os.path.join(csv_dir, name), 'wb') as out_file:
                np.savetxt(out_file, np.transpose(np.vstack([t, v])), delimiter=",")

        for i in range(self.NUM_DRONES):
            for name, row in (("x", 0), ("y", 1), ("z", 2), ("r", 6), ("p", 7), ("ya", 8)):
                dump(f"{name}{i}.csv", st[i, row, :])
            for name, row in (("rr", 6), ("pr", 7), ("yar", 8)):
                dump(f"{name}{i}.csv", np.hstack([0, (st[i, row, 1:] - st[i, row, 0:-1]) * self.LOGGING_FREQ_HZ]))
            for name, row in (("vx", 3), ("vy", 4), ("vz", 5), ("wx", 9), ("wy", 10), ("wz", 11)):
                dump(f"{name}{i}.csv", st[i, row, :])
            for k in range(4):
                dump(f"rpm{k}-{i}.csv", st[i, 12 + k, :])
            for k in range(4):
                dump(f"pwm{k}-{i}.csv", (st[i, 12 + k, :] - 4070.3) / 0.2685)
        return csv_dir

    def plot(self, pwm=False):
        raise NotImplementedError("Logger.plot needs matplotlib (plotting is out of scope); use save() / save_as_csv()")
