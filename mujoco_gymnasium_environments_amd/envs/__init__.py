"""Task environments. humanoid_soccer is the headline task (BASELINE.json)."""
from .soccer import HumanoidSoccerEnv, SoccerVectorEnv, register_envs  # noqa: F401
