import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


@pytest.fixture(scope="session")
def soccer_xml():
    with open(os.path.join(ROOT, "mujoco_gymnasium_environments_amd", "assets", "humanoid_soccer.xml")) as f:
        return f.read()


@pytest.fixture(scope="session")
def soccer_model(soccer_xml):
    from mujoco_gymnasium_environments_amd import mjcf
    return mjcf.compile_xml(soccer_xml)


@pytest.fixture(scope="session")
def soccer_packed(soccer_model):
    from mujoco_gymnasium_environments_amd import cabi
    return cabi.pack_model(soccer_model)


@pytest.fixture(scope="session")
def parkour_model():
    from mujoco_gymnasium_environments_amd import mjcf
    with open(os.path.join(ROOT, "mujoco_gymnasium_environments_amd", "assets", "quadruped_parkour.xml")) as f:
        return mjcf.compile_xml(f.read())


@pytest.fixture(scope="session")
def parkour_packed(parkour_model):
    from mujoco_gymnasium_environments_amd import cabi
    return cabi.pack_model(parkour_model)


@pytest.fixture(scope="session")
def bipedal_model():
    from mujoco_gymnasium_environments_amd.envs.bipedal import bipedal_model as load
    return load()


@pytest.fixture(scope="session")
def bipedal_packed(bipedal_model):
    from mujoco_gymnasium_environments_amd import cabi
    return cabi.pack_model(bipedal_model)


@pytest.fixture(scope="session")
def dancing_model():
    from mujoco_gymnasium_environments_amd.envs.dancing import dancing_model as load
    return load()


@pytest.fixture(scope="session")
def dancing_packed(dancing_model):
    from mujoco_gymnasium_environments_amd import cabi
    return cabi.pack_model(dancing_model)


@pytest.fixture(scope="session")
def martial_model():
    from mujoco_gymnasium_environments_amd.envs.martial import martial_model as load
    return load()


@pytest.fixture(scope="session")
def martial_packed(martial_model):
    from mujoco_gymnasium_environments_amd import cabi
    return cabi.pack_model(martial_model)
