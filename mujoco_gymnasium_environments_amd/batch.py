"""Device-resident batch of MuJoCo-model states driven by libmgx (the MjData replacement).

One ``PhysicsBatch`` owns N envs' state as torch tensors on one GPU, env-major rows
(``qpos[N, nq]`` ...), and steps them with ``mgx_step`` (mujoco.mj_step, e.g.
humanoid_soccer_env/soccer_env.py:414). torch is used only for device memory and streams.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np
import torch

from . import cabi, mjcf
from .native import MGX_F32, MGX_F64, check, lib

DEBUG_FIELDS = ["xpos", "xquat", "xipos", "subtree_com", "cinert", "cdof", "qM", "qLD", "geom_xpos", "geom_xmat",
                "ncon", "con_dist", "con_pos", "con_frame", "con_geom", "nefc", "efc_type", "efc_id", "efc_pos",
                "efc_margin", "efc_R", "efc_aref", "Bmat", "cvel", "cdof_dot", "qfrc_smooth", "qacc_smooth",
                "efc_force", "qacc", "qfrc_constraint", "niter"]


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_handle(stream: Optional[torch.cuda.Stream] = None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


class NativeModel:
    """Device-resident model constants (mgx_model_create)."""

    def __init__(self, model: mjcf.Model, precision: str = "f64", device: int = 0):
        self.model = model
        self.packed = cabi.pack_model(model)
        self.precision = precision
        self.dtype = torch.float32 if precision == "f32" else torch.float64
        h = C.c_void_p()
        check(lib().mgx_model_create(C.byref(self.packed.desc), MGX_F32 if precision == "f32" else MGX_F64,
                                     device, C.byref(h)), "mgx_model_create")
        self.handle = h
        info = cabi.MgxModelInfo()
        check(lib().mgx_model_get_info(self.handle, C.byref(info)), "mgx_model_get_info")
        self.info = info

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                lib().mgx_model_destroy(h)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass
            self.handle = None


class PhysicsBatch:
    def __init__(self, model: mjcf.Model, n_env: int, precision: str = "f64", device: str = "cuda:0",
                 native: Optional[NativeModel] = None):
        self.model = model
        self.n = n_env
        self.device = torch.device(device)
        idx = self.device.index or 0
        self.native = native or NativeModel(model, precision, idx)
        dt = self.native.dtype
        self.dtype = dt
        m = model
        self.qpos = torch.tensor(m.qpos0, dtype=dt, device=self.device).repeat(n_env, 1).contiguous()
        self.qvel = torch.zeros(n_env, m.nv, dtype=dt, device=self.device)
        self.qacc_warmstart = torch.zeros(n_env, m.nv, dtype=dt, device=self.device)
        self.ctrl = torch.zeros(n_env, max(m.nu, 1), dtype=dt, device=self.device)
        self.qfrc_applied = torch.zeros(n_env, m.nv, dtype=dt, device=self.device)
        self.xfrc_applied = torch.zeros(n_env, m.nbody, 6, dtype=dt, device=self.device)
        self.time = torch.zeros(n_env, dtype=dt, device=self.device)
        self.warning = torch.zeros(n_env, dtype=torch.int32, device=self.device)
        self.overflow = torch.zeros(n_env, dtype=torch.int32, device=self.device)
        self.xpos = torch.zeros(n_env, m.nbody, 3, dtype=dt, device=self.device)
        self.xquat = torch.zeros(n_env, m.nbody, 4, dtype=dt, device=self.device)
        self.subtree_com = torch.zeros(n_env, m.nbody, 3, dtype=dt, device=self.device)
        self.ncon = torch.zeros(n_env, dtype=torch.int32, device=self.device)
        self.nefc = torch.zeros(n_env, dtype=torch.int32, device=self.device)
        self.niter = torch.zeros(n_env, dtype=torch.int32, device=self.device)
        # constraint-row scratch for models whose rows do not fit the per-env LDS budget
        sb = int(self.native.info.scratch_bytes_per_env)
        self.scratch = torch.empty(n_env * sb, dtype=torch.uint8, device=self.device) if sb > 0 else None
        self._state = cabi.MgxState(*[t.data_ptr() for t in (self.qpos, self.qvel, self.qacc_warmstart, self.ctrl,
                                                             self.qfrc_applied, self.xfrc_applied, self.time,
                                                             self.warning)],
                                    self.scratch.data_ptr() if self.scratch is not None else None,
                                    self.overflow.data_ptr())
        self._frames = cabi.MgxFrames(*[t.data_ptr() for t in (self.xpos, self.xquat, self.subtree_com, self.ncon,
                                                              self.nefc, self.niter)])

    @property
    def state(self) -> cabi.MgxState:
        return self._state

    def step(self, nsub: int = 1, mask: Optional[torch.Tensor] = None, frames: bool = True, stream=None) -> None:
        """mj_step x nsub for every (masked) env, asynchronously on the stream."""
        if mask is not None:
            assert mask.dtype == torch.uint8 and mask.numel() == self.n and mask.is_cuda
        check(lib().mgx_step(self.native.handle, C.byref(self._state), C.byref(self._frames) if frames else None,
                             self.n, nsub, _ptr(mask), stream_handle(stream)), "mgx_step")

    def reset(self, mask: Optional[torch.Tensor] = None, stream=None) -> None:
        """mj_resetData for every (masked) env."""
        check(lib().mgx_reset_data(self.native.handle, C.byref(self._state), self.n, _ptr(mask),
                                   stream_handle(stream)), "mgx_reset_data")

    def debug_forward(self, n_env: Optional[int] = None) -> Dict[str, np.ndarray]:
        """Stage outputs of one forward pass per env (test-only; synchronises)."""
        n = self.n if n_env is None else n_env
        offs = (C.c_int32 * 64)()
        cnt = lib().mgx_debug_layout(self.native.handle, offs, 64)
        total = offs[cnt - 1]
        buf = torch.zeros(n, total, dtype=self.dtype, device=self.device)
        check(lib().mgx_debug_forward(self.native.handle, C.byref(self._state), n, _ptr(buf),
                                      stream_handle()), "mgx_debug_forward")
        torch.cuda.synchronize(self.device)
        host = buf.cpu().numpy()
        out = {}
        for i, name in enumerate(DEBUG_FIELDS):
            out[name] = host[:, offs[i]:offs[i + 1]]
        return out
