"""Restatement of the reference's Logger bookkeeping (TEST INFRASTRUCTURE ONLY - only
``tests/`` may import it).

Follows ``gym_pybullet_drones/utils/Logger.py``:
  * ``:19-79``   __init__: counters, timestamps (D, T), states (D, 16, T), controls (D, 12, T),
                 preallocated when duration_sec > 0
  * ``:83-127``  log(): grow-by-one-column when a counter runs past the arrays, the
                 not-preallocated counter rule, the 16-state reorder
                 [pos(0:3), vel(10:13), rpy(7:10), ang_v + rpm (13:20)]
  * ``:131-135`` save(): np.savez(timestamps, states, controls)
Plotting (matplotlib) is not restated.
"""
import numpy as np


class RefLogger:
    def __init__(self, logging_freq_hz, num_drones=1, duration_sec=0):
        self.LOGGING_FREQ_HZ = logging_freq_hz
        self.NUM_DRONES = num_drones
        self.PREALLOCATED_ARRAYS = False if duration_sec == 0 else True
        self.counters = np.zeros(num_drones)
        self.timestamps = np.zeros((num_drones, duration_sec * self.LOGGING_FREQ_HZ))
        self.states = np.zeros((num_drones, 16, duration_sec * self.LOGGING_FREQ_HZ))
        self.controls = np.zeros((num_drones, 12, duration_sec * self.LOGGING_FREQ_HZ))

    def log(self, drone, timestamp, state, control=np.zeros(12)):
        current_counter = int(self.counters[drone])
        if current_counter >= self.timestamps.shape[1]:
            self.timestamps = np.concatenate((self.timestamps, np.zeros((self.NUM_DRONES, 1))), axis=1)
            self.states = np.concatenate((self.states, np.zeros((self.NUM_DRONES, 16, 1))), axis=2)
            self.controls = np.concatenate((self.controls, np.zeros((self.NUM_DRONES, 12, 1))), axis=2)
        elif not self.PREALLOCATED_ARRAYS and self.timestamps.shape[1] > current_counter:
            current_counter = self.timestamps.shape[1] - 1
        self.timestamps[drone, current_counter] = timestamp
        self.states[drone, :, current_counter] = np.hstack([state[0:3], state[10:13], state[7:10], state[13:20]])
        self.controls[drone, :, current_counter] = control
        self.counters[drone] = current_counter + 1

    def arrays(self):
        return dict(timestamps=self.timestamps, states=self.states, controls=self.controls)
