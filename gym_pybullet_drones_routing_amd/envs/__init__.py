"""Gymnasium-surface mirrors of the reference's RL envs (``gym_pybullet_drones/envs``)."""
from .BaseRLAviary import BaseRLAviary  # noqa: F401
from .HoverAviary import HoverAviary  # noqa: F401
from .MultiHoverAviary import MultiHoverAviary  # noqa: F401
from .vec_env import AviaryVecEnv, ShardedAviaryVecEnv, make_vec_env  # noqa: F401

try:  # register the reference's gymnasium ids when gymnasium is present (__init__.py:1-21)
    from gymnasium.envs.registration import register, registry
    for _id, _ep in (("hover-aviary-v0", "gym_pybullet_drones_routing_amd.envs:HoverAviary"),
                     ("multihover-aviary-v0", "gym_pybullet_drones_routing_amd.envs:MultiHoverAviary")):
        if _id not in registry:
            register(id=_id, entry_point=_ep)
except Exception:  # gymnasium not installed
    pass
