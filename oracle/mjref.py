"""ctypes wrapper over oracle/_build/libmjref.so (TEST INFRASTRUCTURE ONLY).

The C library restates MuJoCo's mj_step stage by stage in fp64 (see mjref.h for what it
follows and its parity status). This wrapper exposes one env as numpy views.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MJREF_LIB selects another build of the same source (the sanitizer build, `make asan`)
LIB_PATH = os.environ.get("MJREF_LIB") or os.path.join(HERE, "_build", "libmjref.so")
_INT_FIELDS = {"warning", "ncon", "con_geom", "con_dim", "con_pair", "nefc", "efc_type", "efc_id",
               "solver_niter"}
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if os.path.exists(os.path.join(HERE, "Makefile")) and not os.environ.get("MJREF_LIB"):
            build()  # make: rebuilds when mjref.c / mjref.h / include/mgx.h changed
        elif not os.path.exists(LIB_PATH):
            raise FileNotFoundError(LIB_PATH)
        _lib = C.CDLL(LIB_PATH)
        _lib.ref_create.restype = C.c_void_p
        _lib.ref_create.argtypes = [C.c_void_p, C.c_int, C.c_int]
        _lib.ref_free.argtypes = [C.c_void_p]
        for f in ("ref_reset", "ref_forward", "ref_step"):
            getattr(_lib, f).argtypes = [C.c_void_p, C.c_void_p]
        _lib.ref_field.restype = C.c_void_p
        _lib.ref_field.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_int)]
        _lib.ref_collide_pair.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        _lib.ref_collide_pair.restype = C.c_int
        _lib.ref_narrowphase_stats.argtypes = [C.POINTER(C.c_long), C.c_int]
        _lib.ref_set_pgs_order.argtypes = [C.c_void_p, C.c_int]
    return _lib


NP_STATS = ("capsule_box_1", "capsule_box_2", "capsule_capsule", "capsule_capsule_parallel",
            "capsule_capsule_parallel_contacts") + tuple(f"box_box_{k}" for k in range(9))


def narrowphase_stats(reset: bool = False) -> dict:
    """Process-wide narrowphase branch counters of the oracle (mjref.c g_np_stats)."""
    buf = (C.c_long * 16)()
    lib().ref_narrowphase_stats(buf, 1 if reset else 0)
    return dict(zip(NP_STATS, list(buf)[:len(NP_STATS)]))


class RefSim:
    """One MjData-like env on the CPU oracle."""

    def __init__(self, packed, ncon_max: int = 256, nefc_max: int = 1024):
        self.packed = packed
        self.m = packed.model
        self.L = lib()
        self.d = self.L.ref_create(C.addressof(packed.desc), ncon_max, nefc_max)

    def __del__(self):
        if getattr(self, "d", None):
            self.L.ref_free(self.d)
            self.d = None

    def field(self, name: str) -> np.ndarray:
        n = C.c_int()
        p = self.L.ref_field(self.d, name.encode(), C.byref(n))
        if not p:
            raise KeyError(name)
        ct = C.c_int32 if name in _INT_FIELDS else C.c_double
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), shape=(n.value,))

    def __getattr__(self, name):
        if name in ("packed", "m", "L", "d"):
            raise AttributeError(name)
        return self.field(name)

    def set_pgs_reverse(self, reverse: bool = True):
        """Twin knob: sum each PGS residual in reverse column order (same algorithm, other
        fp64 rounding; mjref.c ref_set_pgs_order)."""
        self.L.ref_set_pgs_order(self.d, 1 if reverse else 0)

    def reset(self):
        self.L.ref_reset(C.addressof(self.packed.desc), self.d)

    def forward(self):
        self.L.ref_forward(C.addressof(self.packed.desc), self.d)

    def step(self, n: int = 1):
        for _ in range(n):
            self.L.ref_step(C.addressof(self.packed.desc), self.d)

    def contacts(self):
        n = int(self.field("ncon")[0])
        return dict(dist=self.field("con_dist")[:n].copy(), pos=self.field("con_pos")[:3 * n].reshape(n, 3).copy(),
                    frame=self.field("con_frame")[:9 * n].reshape(n, 9).copy(),
                    geom=self.field("con_geom")[:2 * n].reshape(n, 2).copy(),
                    pair=self.field("con_pair")[:n].copy())
