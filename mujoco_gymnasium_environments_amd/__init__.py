"""MI355X-native batched physics step for the MuJoCo Gymnasium tasks of
hasnainfarid/Mujoco_Gymnasium_Environments.

Public surface:
  mjcf.compile_xml           MJCF -> model tables (mujoco.MjModel.from_xml_string)
  batch.PhysicsBatch         N env states on one GPU + mgx_step (mujoco.mj_step)
  envs.SoccerVectorEnv       batched humanoid_soccer (device tensors)
  envs.HumanoidSoccerEnv     drop-in gymnasium-style single env
  envs.ParkourVectorEnv      batched quadruped_parkour (10 substeps per env step)
  envs.QuadrupedParkourEnv   drop-in gymnasium-style single env
  envs.BipedalVectorEnv      batched bipedal_rescue (RK4, rows in global scratch)
  envs.BipedalRescueEnv      drop-in gymnasium-style single env
  envs.DancingVectorEnv      batched humanoid_dancing (RK4)
  envs.HumanoidDancingEnv    drop-in gymnasium-style single env
The compute path is libmgx.so (HIP, gfx950); there is no CPU fallback.
"""
__version__ = "0.1.0"


def __getattr__(name):  # lazy: importing the package must not require a GPU
    if name in ("HumanoidSoccerEnv", "SoccerVectorEnv", "register_envs", "ParkourVectorEnv", "QuadrupedParkourEnv",
                "BipedalVectorEnv", "BipedalRescueEnv",
                "DancingVectorEnv", "HumanoidDancingEnv"):
        from . import envs
        return getattr(envs, name)
    raise AttributeError(name)
