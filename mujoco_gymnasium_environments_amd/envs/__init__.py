"""Task environments. humanoid_soccer is the headline task (BASELINE.json); quadruped_parkour is
the low-DoF bring-up task (BASELINE configs 1-2); bipedal_rescue is the RK4 scaling task (config 4);
humanoid_dancing is a config-5 task (RK4, cylinder floor); humanoid_construction (RK4 + Newton,
nv 99) runs on the wide two-dofs-per-lane kernels."""
from .bipedal import BipedalRescueEnv, BipedalVectorEnv  # noqa: F401
from .construction import ConstructionVectorEnv, HumanoidConstructionEnv  # noqa: F401
from .dancing import DancingVectorEnv, HumanoidDancingEnv  # noqa: F401
from .parkour import ParkourVectorEnv, QuadrupedParkourEnv  # noqa: F401
from .soccer import HumanoidSoccerEnv, SoccerVectorEnv, register_envs  # noqa: F401
