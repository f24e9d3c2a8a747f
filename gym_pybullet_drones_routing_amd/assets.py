"""Drone model parameters: built-in table + URDF parser.

``parse_urdf`` mirrors ``BaseAviary._parseURDFParameters`` (``envs/BaseAviary.py:982-1014``):
it reads the same ``<properties>`` attributes, the base link's mass/inertia, the collision
cylinder and — additionally, because the explicit integrator needs them for the PYB force
placement and ground effect — the four prop links' inertial origins
(``assets/cf2x.urdf:42,54,66,78``).  The built-in values used when no URDF path is given are
read from the C library (``gpd_default_params``), so Python and kernels share one table.
"""
import xml.etree.ElementTree as etxml

from . import _lib
from .enums import DroneModel

_MODEL_ID = {DroneModel.CF2X: _lib.GPD_MODEL_CF2X, DroneModel.CF2P: _lib.GPD_MODEL_CF2P,
             DroneModel.RACE: _lib.GPD_MODEL_RACE}


def model_id(drone_model):
    return _MODEL_ID[DroneModel(drone_model)]


def default_params(drone_model=DroneModel.CF2X):
    """Built-in parameters of cf2x / cf2p / racer (the values of the reference's URDFs)."""
    return _lib.default_params(model_id(drone_model))


def parse_urdf(path, drone_model=DroneModel.CF2X):
    """Parse a drone URDF the way BaseAviary._parseURDFParameters does (:989-1012)."""
    root = etxml.parse(str(path)).getroot()
    props = root[0].attrib
    base = root[1]
    p = _lib.DroneParams()
    p.model = model_id(drone_model)
    p.m = float(base[0][1].attrib["value"])
    p.arm = float(props["arm"])
    p.thrust2weight = float(props["thrust2weight"])
    p.ixx = float(base[0][2].attrib["ixx"])
    p.iyy = float(base[0][2].attrib["iyy"])
    p.izz = float(base[0][2].attrib["izz"])
    p.kf = float(props["kf"])
    p.km = float(props["km"])
    p.collision_h = float(base[2][1][0].attrib["length"])
    p.collision_r = float(base[2][1][0].attrib["radius"])
    p.collision_z_offset = [float(s) for s in base[2][0].attrib["xyz"].split(" ")][2]
    p.max_speed_kmh = float(props["max_speed_kmh"])
    p.gnd_eff_coeff = float(props["gnd_eff_coeff"])
    p.prop_radius = float(props["prop_radius"])
    p.drag_coeff_xy = float(props["drag_coeff_xy"])
    p.drag_coeff_z = float(props["drag_coeff_z"])
    p.dw_coeff_1 = float(props["dw_coeff_1"])
    p.dw_coeff_2 = float(props["dw_coeff_2"])
    p.dw_coeff_3 = float(props["dw_coeff_3"])
    links = {ln.attrib.get("name"): ln for ln in root.findall("link")}
    for k in range(4):
        origin = links[f"prop{k}_link"].find("inertial").find("origin")
        xyz = [float(s) for s in origin.attrib["xyz"].split()]
        for j in range(3):
            p.prop_pos[k][j] = xyz[j]
    return p


def params_dict(p):
    """ctypes DroneParams -> plain dict (for printing / tests)."""
    d = {name: getattr(p, name) for name, _ in p._fields_ if name != "prop_pos"}
    d["prop_pos"] = [[p.prop_pos[k][j] for j in range(3)] for k in range(4)]
    return d
