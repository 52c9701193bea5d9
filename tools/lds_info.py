"""Print the per-env LDS footprint and capacities the library chose for a task model (GPU box).

usage: python tools/lds_info.py [assembly|bipedal|soccer|soccer_full|martial|dancing] [f32|f64]
       (MGX_MAX_NEFC / MGX_MAX_NCON override)
Monolithic kernels: envs per CU = floor(160 KiB / lds_bytes_per_env). Staged tasks also print
the row builder's and the finisher's per-wave LDS (lds_bytes_rows / lds_bytes_finish).
"""
import sys

sys.path.insert(0, ".")


def main(task: str, prec: str) -> None:
    if task == "bipedal":
        from mujoco_gymnasium_environments_amd.envs.bipedal import BipedalVectorEnv
        e = BipedalVectorEnv(2, precision=prec)
        nat = e.batch.native if hasattr(e, "batch") else e.native
    elif task.startswith("soccer"):
        from mujoco_gymnasium_environments_amd.envs.soccer import SoccerVectorEnv
        e = SoccerVectorEnv(2, precision=prec, full_capacity=task == "soccer_full")
        nat = e.native
    elif task == "martial":
        from mujoco_gymnasium_environments_amd.envs.martial import MartialArtsVectorEnv
        e = MartialArtsVectorEnv(2, precision=prec)
        nat = e.batch.native if hasattr(e, "batch") else e.native
    elif task == "dancing":
        from mujoco_gymnasium_environments_amd.envs.dancing import DancingVectorEnv
        e = DancingVectorEnv(2, precision=prec)
        nat = e.batch.native if hasattr(e, "batch") else e.native
    else:
        from mujoco_gymnasium_environments_amd.envs.assembly import AssemblyVectorEnv
        e = AssemblyVectorEnv(2, precision=prec)
        nat = e.batch.native
    i = nat.info
    print(task, prec, "lds_bytes_per_env", i.lds_bytes_per_env, "envs_per_cu", (160 * 1024) // max(1, i.lds_bytes_per_env),
          "lds_bytes_rows", i.lds_bytes_rows, "rows_waves_per_cu", (160 * 1024) // max(1, i.lds_bytes_rows),
          "lds_bytes_finish", i.lds_bytes_finish, "max_nefc", i.max_nefc, "max_ncon", i.max_ncon)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "assembly", sys.argv[2] if len(sys.argv) > 2 else "f64")
