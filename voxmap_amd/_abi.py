"""ctypes mirror of include/voxmap.h (the C ABI of libvoxmap_hip.so).

The shared library is the product; this module only declares its structs and
signatures.  Loading fails loudly when the library is missing: there is no
CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libvoxmap_hip.so")
if os.environ.get("VOXMAP_LIB"):          # experiment variants (voxmap_amd/build.py out=...)
    LIB_PATH = os.environ["VOXMAP_LIB"]

VX_OK = 0
VX_EINVAL, VX_EIO, VX_EFORMAT, VX_ECRYPTO, VX_ESIZE, VX_EDEVICE, VX_ENOMEM = -1, -2, -3, -4, -5, -6, -7
ERROR_NAMES = {
    VX_EINVAL: "VX_EINVAL", VX_EIO: "VX_EIO", VX_EFORMAT: "VX_EFORMAT", VX_ECRYPTO: "VX_ECRYPTO",
    VX_ESIZE: "VX_ESIZE", VX_EDEVICE: "VX_EDEVICE", VX_ENOMEM: "VX_ENOMEM",
}

FORMAT_AUTO, FORMAT_BIN, FORMAT_BIN_GZ, FORMAT_BLOB, FORMAT_GRID = 0, 1, 2, 3, 4
PIXEL_RGBA32F, PIXEL_RGBA8 = 0, 1
FLAG_NO_SHADOW, FLAG_NO_AO, FLAG_NO_CLOUDS, FLAG_PRIMARY_ONLY = 0x1, 0x2, 0x4, 0x8
FLAG_REFLECT, FLAG_ROUGH = 0x10, 0x20          # extensions
FLAG_FULL_QUALITY = FLAG_REFLECT | FLAG_ROUGH
FLAG_INT_INDEX = 0x40                           # diagnostics: integer primary index path
FLAG_SOFT_POOL = 0x80                           # soft shadows by the pooled wave march (same frames)
FLAG_SOFT_BRICK = 0x100                         # + LDS 8^3 brick staging (same frames)
FLAG_NO_EXIT = 0x200                            # diagnostics: march without the sun exit tables (same frames)
FLAG_NO_CONE = 0x400                            # diagnostics: orthant exit tables only (same frames)
FLAG_UNIT_GBUF = 0x800                          # diagnostics: the unit-cell G-buffer split (ABI <= 7)
FLAG_GLASS_ORDER = 0x1000                       # diagnostics: the whole frame through the general draw-order kernel
FLAG_GLASS_SINGLE = 0x8000                      # diagnostics: nearest pane only (ABI <= 8); default = draw order
FLAG_REFLECT_ALL = 0x2000                       # ext: every first surface mirrors the scene
FLAG_ROWS_BOTTOM_UP = 0x4000                    # diagnostics: blocks dispatched bottom row first (same frames)
FLAG_NO_DOOM = 0x20000                          # diagnostics: cone copy without the sun doom table (same frames)
MAX_SHADOW_SAMPLES = 16
DEFAULT_DIST_CAP = 64                           # vx_scene_desc.dist_cap = 0 (ABI 9; was 32)
FALLBACK_DIST_CAP = 32                          # dist_cap = 0 on a field the default cap does not fit (ABI 10)
ABI_VERSION = 10
PAL_SIZE, GLASS = 22, 21          # render.vert:21; air is B = PAL_SIZE in map.bin
MGPU_UID_BYTES = 128


class SceneDesc(C.Structure):
    _fields_ = [
        ("map_path", C.c_char_p), ("map_bytes", C.c_void_p), ("map_size", C.c_size_t),
        ("map_format", C.c_int), ("key_jwk_k", C.c_char_p),
        ("noise_path", C.c_char_p), ("noise_bytes", C.c_void_p), ("noise_size", C.c_size_t),
        ("noise_format", C.c_int), ("noise_w", C.c_int), ("noise_h", C.c_int),
        ("X", C.c_int), ("Y", C.c_int), ("Z", C.c_int),
        ("device", C.c_int), ("dist_cap", C.c_int), ("noise_seed", C.c_uint32), ("mesh_chunk", C.c_int),
    ]


class FrameParams(C.Structure):
    """vx_frame_params: the per-frame uniforms of drawScene (render.js:287-295)."""
    _fields_ = [
        ("quality", C.c_int), ("frame", C.c_int), ("time", C.c_float),
        ("cam_cell", C.c_int * 3), ("cam_fract", C.c_float * 3), ("sun_dir", C.c_float * 3),
        ("ray_fwd", C.c_float * 3), ("ray_right", C.c_float * 3), ("ray_up", C.c_float * 3),
        ("flags", C.c_uint32), ("max_shadow_steps", C.c_int),
        ("shadow_samples", C.c_int), ("sun_radius", C.c_float),
    ]

    def copy(self) -> "FrameParams":
        out = FrameParams()
        C.memmove(C.byref(out), C.byref(self), C.sizeof(FrameParams))
        return out


class MgpuXfer(C.Structure):
    """vx_mgpu_xfer: one band moved by the gather."""
    _fields_ = [("band", C.c_int), ("src", C.c_int), ("dst", C.c_int), ("rows", C.c_int),
                ("offset", C.c_uint64), ("bytes", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [
        ("pixels", C.c_uint64), ("sky_px", C.c_uint64), ("block_px", C.c_uint64), ("glass_px", C.c_uint64),
        ("primary_fetches", C.c_uint64), ("shadow_rays", C.c_uint64), ("shadow_fetches", C.c_uint64),
        ("ao_samples", C.c_uint64), ("noise_px", C.c_uint64), ("primary_cap_hits", C.c_uint64),
        ("reflect_rays", C.c_uint64), ("reflect_fetches", C.c_uint64), ("rough_px", C.c_uint64),
        ("primary_wave_iters", C.c_uint64), ("march_wave_iters", C.c_uint64), ("march_lane_slots", C.c_uint64),
        ("shadow_rays_resolved", C.c_uint64),
        ("alg_bytes", C.c_uint64), ("kernel_ms", C.c_double),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class ExitInfo(C.Structure):
    """vx_exit_info (ABI 7): which sun exit copy a frame's march reads."""
    _fields_ = [("kind", C.c_int), ("octant", C.c_int), ("kx", C.c_int), ("ky", C.c_int), ("build_ms", C.c_float)]


# (name, restype, argtypes) of every symbol include/voxmap.h declares
SIGNATURES = [
    ("vx_scene_create", C.c_int, [C.POINTER(SceneDesc), C.POINTER(C.c_void_p)]),
    ("vx_scene_destroy", None, [C.c_void_p]),
    ("vx_scene_read_field", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("vx_scene_read_field_copy", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    ("vx_scene_read_boxes", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    ("vx_scene_dims", C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    ("vx_scene_read_face_quads", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("vx_scene_vertex2d", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("vx_render", C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_int, C.c_int, C.c_int,
                            C.c_void_p, C.c_int, C.c_void_p, C.POINTER(Stats)]),
    ("vx_render_tiles", C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_int, C.c_int, C.c_int,
                                  C.POINTER(C.c_int), C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                  C.POINTER(Stats)]),
    ("vx_detile", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_int, C.c_int,
                            C.c_void_p, C.c_void_p, C.c_void_p]),
    ("vx_render_bands", C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_int, C.c_int, C.c_int,
                                  C.POINTER(C.c_int), C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                  C.POINTER(Stats)]),
    ("vx_prepare_sun", C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_void_p, C.POINTER(ExitInfo)]),
    ("vx_mgpu_unique_id", C.c_int, [C.c_void_p]),
    ("vx_mgpu_create", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    ("vx_mgpu_render", C.c_int, [C.c_void_p, C.POINTER(FrameParams), C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_void_p, C.c_void_p, C.POINTER(Stats)]),
    ("vx_mgpu_gather", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    ("vx_mgpu_rank", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("vx_mgpu_destroy", None, [C.c_void_p]),
    ("vx_mgpu_bands", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_int]),
    ("vx_mgpu_band_rows", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("vx_mgpu_transfers", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]),
    ("vx_frame_from_orbit", C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int, C.c_int,
                                      C.POINTER(FrameParams)]),
    ("vx_frame_from_matrix", C.c_int, [C.POINTER(C.c_float), C.POINTER(C.c_double), C.POINTER(FrameParams)]),
    ("vx_sun_from_hour", None, [C.c_double, C.POINTER(C.c_float)]),
    ("vx_sun_samples", C.c_int, [C.POINTER(C.c_float), C.c_float, C.c_int, C.POINTER(C.c_float)]),
    ("vx_decode", C.c_int, [C.c_void_p, C.c_size_t, C.c_int, C.c_char_p, C.c_void_p, C.c_size_t,
                            C.POINTER(C.c_size_t)]),
    ("vx_blob_encrypt", C.c_int, [C.c_void_p, C.c_size_t, C.c_char_p, C.c_void_p, C.c_size_t,
                                  C.POINTER(C.c_size_t)]),
    ("vx_field_build", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]),
    ("vx_vertex2d", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_size_t,
                              C.POINTER(C.c_size_t)]),
    ("vx_noise_synth", C.c_int, [C.c_uint32, C.c_int, C.c_int, C.c_void_p]),
    ("vx_field_build_gpu", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int]),
    ("vx_last_error", C.c_char_p, []),
    ("vx_abi_version", C.c_int, []),
]

_lib = None


def lib() -> C.CDLL:
    """Load libvoxmap_hip.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"voxmap_amd: HIP library not built ({LIB_PATH} missing); run "
                "`python -c 'import __graft_entry__ as g; g.build()'` — there is no CPU fallback")
        # One HIP runtime per process: torch (the device-memory / stream /
        # RCCL plumbing) bundles its own libamdhip64 under a different file
        # name; loading torch first makes libvoxmap_hip.so bind to that same
        # runtime (same SONAME) so device pointers and streams are shared.
        try:
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch-less hosts use /opt/rocm's runtime
            pass
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class VoxmapError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


def check(rc: int) -> None:
    if rc != VX_OK:
        raise VoxmapError(rc, lib().vx_last_error().decode(errors="replace"))
