"""Print the per-env LDS footprint and capacities the library chose for a task model (GPU box).

usage: python tools/lds_info.py [assembly|bipedal]   (MGX_MAX_NEFC / MGX_MAX_NCON override)
Envs per CU = floor(160 KiB / lds_bytes_per_env) for the one-wave-per-env kernels.
"""
import sys

sys.path.insert(0, ".")


def main(task: str) -> None:
    if task == "bipedal":
        from mujoco_gymnasium_environments_amd.envs.bipedal import BipedalVectorEnv
        e = BipedalVectorEnv(2, precision="f32")
    else:
        from mujoco_gymnasium_environments_amd.envs.assembly import AssemblyVectorEnv
        e = AssemblyVectorEnv(2, precision="f64")
    i = e.batch.native.info
    print(task, "lds_bytes_per_env", i.lds_bytes_per_env, "envs_per_cu", (160 * 1024) // max(1, i.lds_bytes_per_env),
          "max_nefc", i.max_nefc, "max_ncon", i.max_ncon)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "assembly")
