"""humanoid_dancing_env on MI355X (BASELINE configs[4] member): model loader (env classes below)."""
from __future__ import annotations

import functools
import os

from .. import mjcf

ASSET = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "humanoid_dancing.xml")


@functools.lru_cache(maxsize=None)
def dancing_model() -> mjcf.Model:
    with open(ASSET) as f:
        return mjcf.compile_xml(f.read())
