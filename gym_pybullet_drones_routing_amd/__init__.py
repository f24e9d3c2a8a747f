"""MI355X-native batched quadrotor DYN path with the HoverAviary / MultiHoverAviary surface.

Hot path: ``csrc/`` (HIP kernels for gfx950 behind the C ABI in ``include/gpd.h``), driven
from Python through ``sim.BatchedAviarySim``; ``envs`` mirrors the reference's Gymnasium
surface (reference: komxun/gym-pybullet-drones-routing, ``gym_pybullet_drones/envs``).
"""
from .enums import ActionType, DroneModel, ImageType, ObservationType, Physics  # noqa: F401

__all__ = ["ActionType", "DroneModel", "ImageType", "ObservationType", "Physics"]
