"""bipedal_rescue_env on MI355X (BASELINE configs[3]): model loader and capacities.

The composed model is the output of the reference's own composition code
(bipedal_rescue_env/rescue_env.py:121-277, tests/golden/make_fixtures.py): RK4 integrator
(rescue_env.py:148), PGS, nq = nv = 63, 41 bodies, 89 geoms, 3185 candidate pairs including
static cylinders. Under random actions it holds up to ~130 contacts / ~520 constraint rows
(oracle rollouts), so its rows live in global scratch (Layout.gB) rather than LDS.
"""
from __future__ import annotations

import functools
import os

from .. import mjcf

ASSET = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "bipedal_rescue.xml")
EFC_CAPACITY = 512
CON_CAPACITY = 128


@functools.lru_cache(maxsize=None)
def bipedal_model() -> mjcf.Model:
    with open(ASSET) as f:
        m = mjcf.compile_xml(f.read())
    m.efc_capacity = EFC_CAPACITY
    m.con_capacity = CON_CAPACITY
    return m
