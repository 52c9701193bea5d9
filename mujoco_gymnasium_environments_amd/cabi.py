"""ctypes mirror of include/mgx.h (the library's C-ABI) and model packing.

``pack_model(model)`` turns a compiled :class:`~.mjcf.Model` into an ``mgx_model_desc``
whose pointers reference numpy arrays kept alive by the returned holder.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .mjcf import Model

P_I32 = C.POINTER(C.c_int32)
P_U32 = C.POINTER(C.c_uint32)
P_F64 = C.POINTER(C.c_double)

# (field, kind) in declaration order of mgx_model_desc
_INT_SIZES = ["nq", "nv", "nu", "nbody", "njnt", "ngeom", "npair", "nM", "nmaskword",
              "solver", "integrator", "cone", "iterations", "efc_capacity", "con_capacity", "layout_flags"]
_REAL_SCALARS = ["timestep", "tolerance", "impratio", "meaninertia"]
_ARRAYS = [
    ("body_parentid", "i"), ("body_rootid", "i"), ("body_weldid", "i"), ("body_jntnum", "i"),
    ("body_jntadr", "i"), ("body_dofnum", "i"), ("body_dofadr", "i"), ("body_geomnum", "i"),
    ("body_geomadr", "i"), ("body_subtree_end", "i"), ("body_dofmask", "u"),
    ("body_pos", "d"), ("body_quat", "d"), ("body_ipos", "d"), ("body_iquat", "d"),
    ("body_mass", "d"), ("body_inertia", "d"), ("body_invweight0", "d"),
    ("jnt_type", "i"), ("jnt_bodyid", "i"), ("jnt_qposadr", "i"), ("jnt_dofadr", "i"),
    ("jnt_limited", "i"),
    ("jnt_pos", "d"), ("jnt_axis", "d"), ("jnt_range", "d"), ("jnt_stiffness", "d"),
    ("jnt_margin", "d"), ("jnt_solref", "d"), ("jnt_solimp", "d"),
    ("dof_bodyid", "i"), ("dof_jntid", "i"), ("dof_parentid", "i"), ("dof_Madr", "i"),
    ("dof_armature", "d"), ("dof_damping", "d"), ("dof_frictionloss", "d"), ("dof_invweight0", "d"),
    ("geom_type", "i"), ("geom_bodyid", "i"),
    ("geom_size", "d"), ("geom_pos", "d"), ("geom_quat", "d"), ("geom_rbound", "d"),
    ("pair_geom", "i"), ("pair_condim", "i"),
    ("pair_friction", "d"), ("pair_margin", "d"), ("pair_gap", "d"),
    ("pair_solref", "d"), ("pair_solimp", "d"),
    ("actuator_trnid", "i"), ("actuator_ctrllimited", "i"), ("actuator_forcelimited", "i"),
    ("actuator_gear", "d"), ("actuator_ctrlrange", "d"), ("actuator_forcerange", "d"),
    ("actuator_gainprm", "d"), ("actuator_biasprm", "d"),
    ("qpos0", "d"), ("qpos_spring", "d"),
]
_PTR = {"i": P_I32, "u": P_U32, "d": P_F64}
_NP = {"i": np.int32, "u": np.uint32, "d": np.float64}


MGX_ABI_VERSION = 6  # include/mgx.h: the struct layouts below
MGX_E_ARG, MGX_E_CAPACITY, MGX_E_HIP, MGX_E_UNSUPPORTED = -1, -2, -3, -4  # include/mgx.h error codes
MGX_KEEP_CVEL = 1  # mgx_model_desc.layout_flags (include/mgx.h)
MGX_ROWS_IN_SCRATCH = 2  # layout_flags: constraint rows in per-env global scratch (include/mgx.h)


class MgxModelDesc(C.Structure):
    _fields_ = ([(n, C.c_int32) for n in _INT_SIZES] +
                [(n, C.c_double) for n in _REAL_SCALARS] +
                [("gravity", C.c_double * 3)] +
                [(n, _PTR[k]) for n, k in _ARRAYS])


class MgxModelInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in
                ["nq", "nv", "nu", "nbody", "njnt", "ngeom", "npair", "max_nv", "max_nbody",
                 "max_ncon", "max_nefc", "max_njnt", "precision", "lds_bytes_per_env", "lds_bytes_rows",
                 "lds_bytes_finish", "scratch_bytes_per_env"]]


class MgxState(C.Structure):
    _fields_ = [("qpos", C.c_void_p), ("qvel", C.c_void_p), ("qacc_warmstart", C.c_void_p),
                ("ctrl", C.c_void_p), ("qfrc_applied", C.c_void_p), ("xfrc_applied", C.c_void_p),
                ("time", C.c_void_p), ("warning", C.c_void_p), ("scratch", C.c_void_p),
                ("overflow", C.c_void_p)]


class MgxFrames(C.Structure):
    _fields_ = [("xpos", C.c_void_p), ("xquat", C.c_void_p), ("subtree_com", C.c_void_p),
                ("ncon", C.c_void_p), ("nefc", C.c_void_p), ("niter", C.c_void_p)]


class MgxSoccerEnv(C.Structure):
    _fields_ = [("prev_ball_pos", C.c_void_p), ("prev_robot_pos", C.c_void_p), ("wind", C.c_void_p),
                ("step", C.c_void_p), ("goal_scored", C.c_void_p), ("stats", C.c_void_p),
                ("episode", C.c_void_p), ("flags", C.c_void_p), ("rollout", C.c_void_p),
                ("workspace", C.c_void_p), ("workspace_bytes", C.c_uint64), ("banks", C.c_int32),
                ("action_f64", C.c_int32)]


class MgxSoccerLogicIO(C.Structure):
    _fields_ = [("qpos", C.c_void_p), ("qvel", C.c_void_p), ("xpos", C.c_void_p), ("xquat", C.c_void_p),
                ("subtree_com", C.c_void_p), ("ncon", C.c_void_p), ("con_geom", C.c_void_p),
                ("con_dist", C.c_void_p), ("con_mu", C.c_void_p), ("max_contacts", C.c_int32),
                ("pad0", C.c_int32), ("prev_ball_pos", C.c_void_p), ("prev_robot_pos", C.c_void_p),
                ("wind", C.c_void_p), ("stats", C.c_void_p), ("step", C.c_void_p), ("goal_scored", C.c_void_p),
                ("qfrc_applied", C.c_void_p), ("xfrc_applied", C.c_void_p), ("action", C.c_void_p),
                ("obs", C.c_void_p), ("reward", C.c_void_p), ("terminated", C.c_void_p),
                ("truncated", C.c_void_p), ("flags", C.c_void_p)]


class MgxParkourIds(C.Structure):
    _fields_ = [("torso", C.c_int32), ("feet", C.c_int32 * 4), ("platform_qpos", C.c_int32),
                ("pendulum_qpos", C.c_int32), ("platform_act", C.c_int32), ("pendulum_act", C.c_int32),
                ("n_leg", C.c_int32), ("max_episode_steps", C.c_int32), ("act_lim", C.c_float * 16)]


class MgxParkourEnv(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ["last_position", "max_progress", "episode_reward", "er_kind", "reached", "fall_count", "stuck",
                 "step", "episode", "rollout"]] + \
               [("workspace", C.c_void_p), ("workspace_bytes", C.c_uint64), ("banks", C.c_int32),
                ("action_f64", C.c_int32)]


class MgxParkourLogicIO(C.Structure):
    _fields_ = [("qpos", C.c_void_p), ("qvel", C.c_void_p), ("xpos", C.c_void_p), ("ncon", C.c_void_p),
                ("con_geom", C.c_void_p), ("max_contacts", C.c_int32), ("pad0", C.c_int32), ("ctrl", C.c_void_p),
                ("action", C.c_void_p), ("obs", C.c_void_p), ("reward", C.c_void_p), ("terminated", C.c_void_p),
                ("truncated", C.c_void_p)]


class MgxMartialIds(C.Structure):
    _fields_ = [("torso", C.c_int32), ("right_hand", C.c_int32), ("left_hand", C.c_int32), ("right_foot", C.c_int32),
                ("left_foot", C.c_int32), ("dummy1", C.c_int32), ("dummy2", C.c_int32), ("n_act", C.c_int32),
                ("max_episode_steps", C.c_int32), ("pad0", C.c_int32), ("ctrl_scale", C.c_double * 32)]


class MgxMartialEnv(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ["scal", "ints", "episode", "rollout"]] + \
               [("action_f64", C.c_int32), ("pad0", C.c_int32)]


class MgxMartialLogicIO(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ["qpos", "qvel", "xpos", "xquat", "cvel", "ctrl", "action", "obs", "reward",
                                          "terminated", "truncated"]]


ASSEMBLY_NCOMP = 9
ASSEMBLY_MAX_GEOM = 128


class MgxAssemblyIds(C.Structure):
    _fields_ = [("comp_body", C.c_int32 * ASSEMBLY_NCOMP), ("ee_body", C.c_int32), ("n_geom", C.c_int32),
                ("max_episode_steps", C.c_int32), ("substeps", C.c_int32), ("settle_steps", C.c_int32),
                ("geom_comp", C.c_int8 * ASSEMBLY_MAX_GEOM), ("geom_pad", C.c_uint8 * ASSEMBLY_MAX_GEOM),
                ("ee_pos", C.c_double * 3), ("targets", C.c_double * (3 * ASSEMBLY_NCOMP)),
                ("place_reward", C.c_double * ASSEMBLY_NCOMP), ("joint_low", C.c_double * 7),
                ("joint_high", C.c_double * 7), ("action_low", C.c_float * 9), ("action_high", C.c_float * 9)]


class MgxAssemblyEnv(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ["ints", "cumulative", "episode", "rollout", "reset_qpos"]] + \
               [("action_f64", C.c_int32), ("pad0", C.c_int32)]


class MgxAssemblyLogicIO(C.Structure):
    _fields_ = [("qpos", C.c_void_p), ("qvel", C.c_void_p), ("xpos", C.c_void_p), ("xquat", C.c_void_p),
                ("ncon", C.c_void_p), ("con_geom", C.c_void_p), ("con_dist", C.c_void_p),
                ("max_contacts", C.c_int32), ("pad0", C.c_int32), ("ctrl", C.c_void_p), ("action", C.c_void_p),
                ("obs", C.c_void_p), ("reward", C.c_void_p), ("terminated", C.c_void_p), ("truncated", C.c_void_p)]


class MgxBipedalIds(C.Structure):
    _fields_ = [("torso", C.c_int32), ("victims", C.c_int32 * 5), ("obs_qposadr", C.c_int32 * 26),
                ("obs_dofadr", C.c_int32 * 26), ("root_x", C.c_int32), ("root_y", C.c_int32), ("root_z", C.c_int32),
                ("root_dof", C.c_int32), ("victim_x", C.c_int32 * 5), ("victim_y", C.c_int32 * 5),
                ("n_act", C.c_int32), ("max_episode_steps", C.c_int32)]


class MgxBipedalEnv(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ["step", "energy", "energy_used", "rescued", "carried", "carrying", "closest", "prev_rescued",
                 "prev_carried", "prev_sz", "fall_timer", "victims_rescued", "distance", "ttfr", "falls", "collisions",
                 "prev_robot_pos", "episode", "rollout"]] + \
               [("workspace", C.c_void_p), ("workspace_bytes", C.c_uint64), ("banks", C.c_int32),
                ("action_f64", C.c_int32), ("energy_kind", C.c_void_p)]


class MgxBipedalLogicIO(C.Structure):
    _fields_ = [("qpos", C.c_void_p), ("qvel", C.c_void_p), ("xpos", C.c_void_p), ("xquat", C.c_void_p),
                ("ncon", C.c_void_p), ("con_dist", C.c_void_p), ("max_contacts", C.c_int32), ("pad0", C.c_int32),
                ("ctrl", C.c_void_p), ("action", C.c_void_p), ("obs", C.c_void_p), ("reward", C.c_void_p),
                ("terminated", C.c_void_p), ("truncated", C.c_void_p), ("upright", C.c_void_p)]


class MgxDancingIds(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ["torso", "right_foot", "left_foot", "floor", "stage", "n_act",
                                         "max_episode_steps", "n_range"]] + \
               [("jnt_lo", C.c_double * 32), ("jnt_hi", C.c_double * 32)]


class MgxDancingEnv(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ["scal", "ints", "hist", "moves", "durations", "prev_jvel", "episode", "rollout"]] + \
               [("action_f64", C.c_int32), ("pad0", C.c_int32)]


class MgxDancingLogicIO(C.Structure):
    _fields_ = [("qpos", C.c_void_p), ("qvel", C.c_void_p), ("xpos", C.c_void_p), ("xquat", C.c_void_p),
                ("subtree_com", C.c_void_p), ("ncon", C.c_void_p), ("con_geom", C.c_void_p),
                ("max_contacts", C.c_int32), ("pad0", C.c_int32), ("ctrl", C.c_void_p), ("action", C.c_void_p),
                ("obs", C.c_void_p), ("reward", C.c_void_p), ("terminated", C.c_void_p), ("truncated", C.c_void_p)]


class MgxConstructionIds(C.Structure):
    _fields_ = [("humanoid", C.c_int32), ("n_act", C.c_int32), ("max_episode_steps", C.c_int32),
                ("action_limit", C.c_float)]


class MgxConstructionEnv(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ["scal", "ints", "total_reward", "episode", "rollout"]] + \
               [("action_f64", C.c_int32), ("pad0", C.c_int32), ("total_kind", C.c_void_p)]


class MgxConstructionLogicIO(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ["qpos", "qvel", "xpos", "ctrl", "action", "obs", "reward", "terminated",
                                          "truncated"]]


class MgxSoccerIds(C.Structure):
    _fields_ = [(n, C.c_int32) for n in
                ["torso", "ball", "goalkeeper", "ball_geom", "right_foot", "left_foot", "field_geom",
                 "ball_qposadr", "ball_dofadr", "gk_qposadr", "gk_dofadr", "max_episode_steps"]] + \
               [("obs_jnt_qposadr", C.c_int32 * 25), ("obs_jnt_dofadr", C.c_int32 * 25),
                ("obs_jnt_range", C.c_double * 50),
                ("robot_geom_mask_lo", C.c_uint64), ("robot_geom_mask_hi", C.c_uint64)]


class PackedModel:
    """Holds an ``MgxModelDesc`` plus the contiguous numpy arrays it points to."""

    def __init__(self, model: Model):
        self.model = model
        # per-env capacities: task modules may set these hints on the model (0 = library default)
        efc_capacity = int(getattr(model, "efc_capacity", 0))
        con_capacity = int(getattr(model, "con_capacity", 0))
        self.arrays = {}
        d = MgxModelDesc()
        A = model.arrays
        nmask = A["body_dofmask"].shape[1] if A["body_dofmask"].ndim == 2 else 1
        sizes = dict(nq=model.nq, nv=model.nv, nu=model.nu, nbody=model.nbody, njnt=model.njnt,
                     ngeom=model.ngeom, npair=int(A["pair_geom"].shape[0]), nM=model.nM,
                     nmaskword=nmask, solver=model.solver, integrator=model.integrator,
                     cone=model.cone, iterations=model.iterations, efc_capacity=efc_capacity,
                     con_capacity=con_capacity, layout_flags=int(getattr(model, "layout_flags", 0)))
        for k, v in sizes.items():
            setattr(d, k, int(v))
        d.timestep, d.tolerance = model.timestep, model.tolerance
        d.impratio, d.meaninertia = model.impratio, model.meaninertia
        for i in range(3):
            d.gravity[i] = float(model.gravity[i])
        for name, kind in _ARRAYS:
            arr = np.ascontiguousarray(A[name], dtype=_NP[kind]).reshape(-1)
            if arr.size == 0:
                arr = np.zeros(1, dtype=_NP[kind])
            self.arrays[name] = arr
            setattr(d, name, arr.ctypes.data_as(_PTR[kind]))
        self.desc = d

    def ref(self):
        return C.byref(self.desc)


def pack_model(model: Model) -> PackedModel:
    return PackedModel(model)
