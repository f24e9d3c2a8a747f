"""Enumerations with the reference's names and values (``gym_pybullet_drones/utils/enums.py:3-48``)."""
from enum import Enum


class DroneModel(Enum):
    """Drone models enumeration class (enums.py:3-8)."""
    CF2X = "cf2x"   # Bitcraze Crazyflie 2.0 in the X configuration
    CF2P = "cf2p"   # Bitcraze Crazyflie 2.0 in the + configuration
    RACE = "racer"  # Racer drone in the X configuration


class Physics(Enum):
    """Physics implementations enumeration class (enums.py:13-21)."""
    PYB = "pyb"
    DYN = "dyn"
    PYB_GND = "pyb_gnd"
    PYB_DRAG = "pyb_drag"
    PYB_DW = "pyb_dw"
    PYB_GND_DRAG_DW = "pyb_gnd_drag_dw"


class ImageType(Enum):
    """Camera capture image type enumeration class (enums.py:25-31)."""
    RGB = 0
    DEP = 1
    SEG = 2
    BW = 3


class ActionType(Enum):
    """Action type enumeration class (enums.py:35-41)."""
    RPM = "rpm"
    PID = "pid"
    VEL = "vel"
    ONE_D_RPM = "one_d_rpm"
    ONE_D_PID = "one_d_pid"


class ObservationType(Enum):
    """Observation type enumeration class (enums.py:45-48)."""
    KIN = "kin"
    RGB = "rgb"
