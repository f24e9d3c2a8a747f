"""Drone parameters: C library table == oracle table == URDF parser on equivalent XML."""
import math

import pytest

from oracle.params import RAW, derived

MODELS = [("cf2x", 0), ("cf2p", 1), ("racer", 2)]


@pytest.mark.parametrize("name,mid", MODELS)
def test_builtin_table_matches_oracle(name, mid):
    from gym_pybullet_drones_routing_amd import _lib
    from gym_pybullet_drones_routing_amd.assets import params_dict
    p = params_dict(_lib.default_params(mid))
    o = RAW[name]
    for k in ("m", "arm", "thrust2weight", "ixx", "iyy", "izz", "kf", "km", "collision_h", "collision_r",
              "collision_z_offset", "max_speed_kmh", "gnd_eff_coeff", "prop_radius", "drag_coeff_xy",
              "drag_coeff_z", "dw_coeff_1", "dw_coeff_2", "dw_coeff_3"):
        assert p[k] == o[k], k
    assert p["prop_pos"] == [list(x) for x in o["prop_pos"]]


def _urdf_text(o):
    """A URDF with the reference's element structure, generated from the parameter table."""
    props = " ".join(f'{k}="{o[v]}"' for k, v in (
        ("arm", "arm"), ("kf", "kf"), ("km", "km"), ("thrust2weight", "thrust2weight"),
        ("max_speed_kmh", "max_speed_kmh"), ("gnd_eff_coeff", "gnd_eff_coeff"), ("prop_radius", "prop_radius"),
        ("drag_coeff_xy", "drag_coeff_xy"), ("drag_coeff_z", "drag_coeff_z"), ("dw_coeff_1", "dw_coeff_1"),
        ("dw_coeff_2", "dw_coeff_2"), ("dw_coeff_3", "dw_coeff_3")))
    links = "".join(
        f'<link name="prop{k}_link"><inertial><origin rpy="0 0 0" xyz="{x} {y} {z}"/><mass value="0"/>'
        f'<inertia ixx="0" ixy="0" ixz="0" iyy="0" iyz="0" izz="0"/></inertial></link>'
        for k, (x, y, z) in enumerate(o["prop_pos"]))
    return (f'<?xml version="1.0" ?><robot name="t"><properties {props} />'
            f'<link name="base_link"><inertial><origin rpy="0 0 0" xyz="0 0 0"/><mass value="{o["m"]}"/>'
            f'<inertia ixx="{o["ixx"]}" ixy="0" ixz="0" iyy="{o["iyy"]}" iyz="0" izz="{o["izz"]}"/></inertial>'
            f'<visual><origin rpy="0 0 0" xyz="0 0 0"/></visual>'
            f'<collision><origin rpy="0 0 0" xyz="0 0 {o["collision_z_offset"]}"/>'
            f'<geometry><cylinder radius="{o["collision_r"]}" length="{o["collision_h"]}"/></geometry></collision>'
            f'</link>{links}</robot>')


@pytest.mark.parametrize("name,mid", MODELS)
def test_urdf_parser(tmp_path, name, mid):
    from gym_pybullet_drones_routing_amd.assets import params_dict, parse_urdf
    from gym_pybullet_drones_routing_amd.enums import DroneModel
    f = tmp_path / f"{name}.urdf"
    f.write_text(_urdf_text(RAW[name]))
    p = params_dict(parse_urdf(f, DroneModel(name)))
    assert p["model"] == mid
    for k in ("m", "arm", "kf", "km", "ixx", "izz", "collision_h", "dw_coeff_3", "prop_radius"):
        assert p[k] == RAW[name][k], k
    assert p["prop_pos"] == [list(x) for x in RAW[name]["prop_pos"]]


def test_hover_rpm_formula():
    p = derived("cf2x")
    assert p["hover_rpm"] == math.sqrt(9.8 * 0.027 / (4 * 3.16e-10))
