"""Loader for the in-tree HIP library ``libmgx.so`` (C-ABI in include/mgx.h).

The product path has no CPU fallback: if the library is missing or cannot be loaded this
module raises. ``build()`` compiles it for gfx950 with hipcc (cross-compiles without a GPU).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import subprocess

from . import cabi

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
# MGX_LIB: load another build of the same sources (A/B measurements of a kernel variant)
LIB_PATH = os.environ.get("MGX_LIB") or os.path.join(PKG, "libmgx.so")
CSRC = os.path.join(PKG, "csrc")
SOURCES = ["mgx_api.hip", "mgx_pgs.hip", "mgx_rk_staged.hip", "mgx_pk_staged.hip", "mgx_step.hip", "mgx_parkour.hip", "mgx_bipedal.hip",
           "mgx_dancing.hip",
           "mgx_martial.hip", "mgx_assembly.hip", "mgx_construction.hip"]
# per-translation-unit flags: the staged solver's FMA chains must not be SLP-packed (mgx_pgs.hip)
SOURCE_FLAGS = {"mgx_pgs.hip": ["-fno-slp-vectorize"], "mgx_rk_staged.hip": ["-fno-slp-vectorize"],
                "mgx_pk_staged.hip": ["-fno-slp-vectorize"]}
HEADERS = ["mgx_common.h", "mgx_collide.h", "mgx_physics.h", "mgx_soccer.h", "mgx_staged.h", "mgx_parkour.h",
           "mgx_bipedal.h", "mgx_dancing.h", "mgx_martial.h", "mgx_internal.h", "mgx_wide.h", "mgx_construction.h"]
# task headers included by one translation unit only (so editing one rebuilds one object)
TU_HEADERS = {"mgx_assembly.hip": ["mgx_assembly.h"]}

MGX_OK = 0
MGX_F32 = 0
MGX_F64 = 1


class NativeError(RuntimeError):
    pass


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile libmgx.so for gfx950 in-tree (hipcc). Returns the library path."""
    common = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "mgx.h")]

    def deps(src):
        return [os.path.join(CSRC, src)] + common + [os.path.join(CSRC, h) for h in TU_HEADERS.get(src, [])]

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC"]
    build_dir = os.path.join(PKG, "_build")

    def command(src, obj):
        return [hipcc, *flags, *SOURCE_FLAGS.get(src, []), "-c", "-o", obj, os.path.join(CSRC, src)]

    def deps_hash(src):
        h = hashlib.sha1()
        for d in deps(src):
            with open(d, "rb") as f:
                h.update(f.read())
        return h.hexdigest()

    def stamp_ok(src, obj):
        # an object is reused only when it was built by the same command (compiler, common and
        # per-source flags) from the same source and header contents, both recorded next to it
        # (contents, not mtimes: a header edited while a build runs must not leave objects of the
        # old and the new struct layouts side by side)
        try:
            with open(obj + ".cmd") as f:
                if f.read() != " ".join(command(src, obj)) + "\n" + deps_hash(src):
                    return False
        except OSError:
            return False
        return True

    objs = [os.path.join(build_dir, src.replace(".hip", ".o")) for src in SOURCES]
    if not force and os.path.exists(LIB_PATH):
        lib_t = os.path.getmtime(LIB_PATH)
        if all(os.path.exists(o) and stamp_ok(s, o) and os.path.getmtime(o) <= lib_t for s, o in zip(SOURCES, objs)):
            return LIB_PATH
    os.makedirs(build_dir, exist_ok=True)
    # one translation unit per task family, compiled in parallel, then linked
    procs = []
    for src, obj in zip(SOURCES, objs):
        if not force and os.path.exists(obj) and stamp_ok(src, obj):
            continue
        cmd = command(src, obj)
        dh = deps_hash(src)  # the contents this compile starts from
        procs.append((src, obj, cmd, dh, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                                          text=True)))
    for src, obj, cmd, dh, p in procs:
        _, err = p.communicate()
        if p.returncode != 0:
            raise NativeError(f"hipcc {src} failed ({p.returncode}):\n{err[-4000:]}")
        with open(obj + ".cmd", "w") as f:
            f.write(" ".join(cmd) + "\n" + dh)
    r = subprocess.run([hipcc, *flags, "-shared", "-o", LIB_PATH + ".tmp", *objs], capture_output=True, text=True)
    if r.returncode != 0:
        raise NativeError(f"hipcc link failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    if verbose:
        print(f"built {LIB_PATH}")
    return LIB_PATH


_lib = None

_VP = C.c_void_p
_SIGS = {
    "mgx_model_create": ([C.POINTER(cabi.MgxModelDesc), C.c_int, C.c_int, C.POINTER(_VP)], C.c_int),
    "mgx_model_destroy": ([_VP], C.c_int),
    "mgx_model_get_info": ([_VP, C.POINTER(cabi.MgxModelInfo)], C.c_int),
    "mgx_last_error": ([], C.c_char_p),
    "mgx_abi_version": ([], C.c_int),
    "mgx_step": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxFrames), C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_reset_data": ([_VP, C.POINTER(cabi.MgxState), C.c_int, _VP, _VP], C.c_int),
    "mgx_debug_forward": ([_VP, C.POINTER(cabi.MgxState), C.c_int, _VP, _VP], C.c_int),
    "mgx_debug_layout": ([_VP, C.POINTER(C.c_int32), C.c_int32], C.c_int),
    "mgx_soccer_configure": ([_VP, C.POINTER(cabi.MgxSoccerIds)], C.c_int),
    "mgx_soccer_configure_reset": ([_VP, C.c_int, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_double)], C.c_int),
    "mgx_soccer_step": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxSoccerEnv), _VP, _VP, _VP, _VP, _VP,
                         _VP, C.c_int, C.c_uint64, C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_soccer_reset": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxSoccerEnv), _VP, _VP, C.c_uint64,
                          C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_soccer_logic_test": ([_VP, C.POINTER(cabi.MgxSoccerLogicIO), C.c_int, _VP], C.c_int),
    "mgx_parkour_workspace_bytes": ([_VP, C.c_int, C.c_int], C.c_int64),
    "mgx_parkour_workspace_init": ([_VP, _VP, C.c_uint64, C.c_int, C.c_int, _VP], C.c_int),
    "mgx_bipedal_workspace_bytes": ([_VP, C.c_int, C.c_int], C.c_int64),
    "mgx_bipedal_workspace_init": ([_VP, _VP, C.c_uint64, C.c_int, C.c_int, _VP], C.c_int),
    "mgx_bipedal_workspace_layout": ([_VP, C.c_int, C.c_int, C.POINTER(C.c_int64), C.c_int], C.c_int),
    "mgx_soccer_workspace_bytes": ([_VP, C.c_int, C.c_int], C.c_int64),
    "mgx_soccer_workspace_init": ([_VP, _VP, C.c_uint64, C.c_int, C.c_int, _VP], C.c_int),
    "mgx_soccer_workspace_layout": ([_VP, C.c_int, C.c_int, C.POINTER(C.c_int64), C.c_int], C.c_int),
    "mgx_parkour_configure": ([_VP, C.POINTER(cabi.MgxParkourIds)], C.c_int),
    "mgx_parkour_step": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxParkourEnv), _VP, _VP, _VP, _VP, _VP,
                          _VP, C.c_int, C.c_uint64, C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_parkour_reset": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxParkourEnv), _VP, _VP, C.c_uint64,
                           C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_parkour_logic_test": ([_VP, C.POINTER(cabi.MgxParkourLogicIO), C.POINTER(cabi.MgxParkourEnv), C.c_int, _VP],
                               C.c_int),
    "mgx_bipedal_configure": ([_VP, C.POINTER(cabi.MgxBipedalIds)], C.c_int),
    "mgx_bipedal_step": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxBipedalEnv), _VP, _VP, _VP, _VP, _VP,
                          _VP, C.c_int, C.c_uint64, C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_bipedal_reset": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxBipedalEnv), _VP, _VP, C.c_uint64,
                           C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_bipedal_logic_test": ([_VP, C.POINTER(cabi.MgxBipedalLogicIO), C.POINTER(cabi.MgxBipedalEnv), C.c_int, _VP],
                               C.c_int),
    "mgx_dancing_configure": ([_VP, C.POINTER(cabi.MgxDancingIds)], C.c_int),
    "mgx_dancing_step": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxDancingEnv), _VP, _VP, _VP, _VP, _VP,
                          _VP, C.c_int, C.c_uint64, C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_dancing_reset": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxDancingEnv), _VP, _VP, C.c_uint64,
                           C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_dancing_logic_test": ([_VP, C.POINTER(cabi.MgxDancingLogicIO), C.POINTER(cabi.MgxDancingEnv), C.c_int, _VP],
                               C.c_int),
    "mgx_martial_configure": ([_VP, C.POINTER(cabi.MgxMartialIds)], C.c_int),
    "mgx_martial_step": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxMartialEnv), _VP, _VP, _VP, _VP, _VP,
                          _VP, C.c_int, C.c_uint64, C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_martial_reset": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxMartialEnv), _VP, _VP, C.c_uint64,
                           C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_martial_logic_test": ([_VP, C.POINTER(cabi.MgxMartialLogicIO), C.POINTER(cabi.MgxMartialEnv), C.c_int, _VP],
                               C.c_int),
    "mgx_construction_configure": ([_VP, C.POINTER(cabi.MgxConstructionIds)], C.c_int),
    "mgx_construction_step": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxConstructionEnv), _VP, _VP, _VP, _VP,
                               _VP, _VP, C.c_int, C.c_uint64, C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_construction_reset": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxConstructionEnv), _VP, _VP,
                                C.c_uint64, C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_construction_logic_test": ([_VP, C.POINTER(cabi.MgxConstructionLogicIO), C.POINTER(cabi.MgxConstructionEnv),
                                     C.c_int, _VP], C.c_int),
    "mgx_assembly_configure": ([_VP, C.POINTER(cabi.MgxAssemblyIds)], C.c_int),
    "mgx_assembly_step": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxAssemblyEnv), _VP, _VP, _VP, _VP, _VP,
                           _VP, C.c_int, C.c_int, _VP, _VP], C.c_int),
    "mgx_assembly_reset": ([_VP, C.POINTER(cabi.MgxState), C.POINTER(cabi.MgxAssemblyEnv), _VP, C.c_int, _VP, _VP],
                           C.c_int),
    "mgx_assembly_logic_test": ([_VP, C.POINTER(cabi.MgxAssemblyLogicIO), C.POINTER(cabi.MgxAssemblyEnv), C.c_int,
                                 _VP], C.c_int),
}
EXPORTS = tuple(_SIGS)


def lib() -> C.CDLL:
    """Load libmgx.so (raises NativeError if absent — there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} not found: run __graft_entry__.build() (hipcc, gfx950)")
        L = C.CDLL(LIB_PATH)
        for name, (argt, rest) in _SIGS.items():
            f = getattr(L, name)
            f.argtypes = argt
            f.restype = rest
        if L.mgx_abi_version() != cabi.MGX_ABI_VERSION:
            raise NativeError(f"{LIB_PATH}: ABI version {L.mgx_abi_version()}, the bindings expect "
                              f"{cabi.MGX_ABI_VERSION} (include/mgx.h): rebuild")
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc < 0:
        msg = lib().mgx_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed ({rc}): {msg}")
