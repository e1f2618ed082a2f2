"""CPU ORACLE bindings — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the timed CPU baseline.  The product
path (voxmap_amd, libvoxmap_hip.so) never touches it.

Parity status: "parity unpinned" against reference outputs (the reference is
browser GLSL with no tests or golden images); the oracle is
pinned by hand-derived known-answer tests (tests/test_oracle_kat.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libvxo.so")


class OScene(C.Structure):
    _fields_ = [("X", C.c_int), ("Y", C.c_int), ("Z", C.c_int), ("field", C.c_void_p), ("noise", C.c_void_p),
                ("noise_w", C.c_int), ("noise_h", C.c_int), ("oct_e", C.c_void_p * 8), ("fp2d", C.c_void_p),
                ("exit_mode", C.c_int), ("held", C.c_void_p), ("held_oct", C.c_int), ("held_kx", C.c_int),
                ("held_ky", C.c_int), ("qoff", C.c_void_p), ("chunk", C.c_int), ("unit_split", C.c_int),
                ("held_doom", C.c_void_p), ("held_dplan", C.c_int * 7)]


class OStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("pixels", "sky_px", "block_px", "glass_px", "primary_fetches",
                                          "shadow_rays", "shadow_fetches", "ao_samples", "noise_px",
                                          "primary_cap_hits", "reflect_rays", "reflect_fetches",
                                          "rough_px")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class OMarch(C.Structure):
    _fields_ = [("cell", C.c_int * 3), ("fract", C.c_float * 3), ("normal", C.c_float * 3), ("min_dist", C.c_float),
                ("step", C.c_int), ("fetches", C.c_int)]


class OGbuf(C.Structure):
    _fields_ = [("id", C.c_int), ("color", C.c_int), ("normal_idx", C.c_int), ("cell", C.c_int * 3),
                ("fract", C.c_float * 3), ("t", C.c_float), ("key", C.c_uint64)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.vxo_render.argtypes = [C.POINTER(OScene), C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                 C.POINTER(OStats), C.c_int]
        L.vxo_render.restype = None
        L.vxo_march.argtypes = [C.POINTER(OScene), C.POINTER(C.c_int), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                C.c_int, C.POINTER(OMarch)]
        L.vxo_primary.argtypes = [C.POINTER(OScene), C.c_void_p, C.POINTER(C.c_float), C.POINTER(OGbuf),
                                  C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.vxo_primary.restype = C.c_int
        L.vxo_shade.argtypes = [C.POINTER(OScene), C.c_void_p, C.POINTER(OGbuf), C.POINTER(C.c_float),
                                C.POINTER(C.c_float), C.c_void_p]
        L.vxo_pixel_dir.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
        L.vxo_glass_layers.argtypes = [C.POINTER(OScene), C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int]
        L.vxo_glass_layers.restype = None
        L.vxo_sun_samples.argtypes = [C.POINTER(C.c_float), C.c_float, C.c_int, C.POINTER(C.c_float)]
        L.vxo_sun_samples.restype = None
        L.vxo_palette.argtypes = [C.POINTER(C.c_float)]
        L.vxo_palette.restype = None
        L.vxo_exp2.argtypes = [C.c_float]
        L.vxo_exp2.restype = C.c_float
        L.vxo_field_build.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.vxo_field_octant.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.vxo_field_box.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.vxo_field_exit.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.vxo_field_exit.restype = None
        L.vxo_exit_plan.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    C.POINTER(C.c_int)]
        L.vxo_exit_plan.restype = C.c_int
        L.vxo_doom_plan.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int)]
        L.vxo_doom_plan.restype = None
        L.vxo_field_doom.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_void_p]
        L.vxo_field_doom.restype = None
        L.vxo_face_quads.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.vxo_face_quads.restype = None
        L.vxo_face_order.argtypes = [C.POINTER(C.c_int), C.c_int, C.c_uint16, C.c_int, C.c_int, C.c_int, C.c_int]
        L.vxo_face_order.restype = C.c_uint64
        L.vxo_render_terms.argtypes = [C.POINTER(OScene), C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                       C.c_void_p, C.c_int]
        L.vxo_render_terms.restype = None
        _lib = L
    return _lib


class Oracle:
    """Scalar restatement of render.frag over one field + noise texture."""

    def __init__(self, field_zyx4: np.ndarray, noise_hw4: np.ndarray, cap: int = 64, oct_e=None, exit=False,
                 quad=True, chunk: int = 0):
        """exit=False: the reference's literal march (every step of
        render.frag:92-136 counted).  exit=True: the build's sun exit tables
        (field_exit, chosen per frame by exit_plan) where the HIP kernel has
        them -- fields with Z <= 126 and every R, G <= Z (its padded int8 march
        copies) -- so the shadow fetch counters match the kernel's;
        exit="orthant": the orthant tables only (the kernel's VX_FLAG_NO_CONE).
        With a cone table a frame also reads the sun doom table
        (vxo_field_doom) unless its flags carry VX_FLAG_NO_DOOM or VX_FLAG_SOFT_BRICK.
        Frames are identical in every mode.

        quad=True (default, as the kernel): the quad-relative G-buffer
        (DESIGN.md §5): primary records carry the greedy quad's origin as
        v_cellPos and the hit minus it as v_fractPos, as the raster hands them
        to render.frag (render.vert:25-28; face_quads, the sdf.cpp:281-356
        mesher with CHUNK = chunk or Z).  quad may also be a precomputed
        face_quads() array; quad=False: the unit-cell split (the kernel's
        VX_FLAG_UNIT_GBUF)."""
        self.field = np.ascontiguousarray(field_zyx4, np.uint8)
        self.noise = np.ascontiguousarray(noise_hw4, np.uint8)
        Z, Y, X, _ = self.field.shape
        H, W, _ = self.noise.shape
        # the primary traversal's octant boxes (vxo_field_box), from the colours;
        # oct_e: precomputed (Z, Y, X, 3) arrays (e.g. device copies checked
        # elsewhere against field_box) for fields too large for the scalar pass
        if oct_e is None:
            self.oct_e = [field_box(self.field, o, cap) for o in range(8)]
        else:
            self.oct_e = [np.ascontiguousarray(e, np.uint8) for e in oct_e]
        for e in self.oct_e:
            assert e.shape == (Z, Y, X, 3)
        self.fp2d = footprint_2d(self.field)
        mode = 0
        if exit and Z <= 126 and int(self.field[..., :2].max(initial=0)) <= Z:
            mode = 2 if exit == "orthant" else 1
        self.sc = OScene(X, Y, Z, self.field.ctypes.data, self.noise.ctypes.data, W, H,
                         (C.c_void_p * 8)(*[e.ctypes.data for e in self.oct_e]), self.fp2d.ctypes.data, mode)
        # the quad table serves the split and the glass draw order (its face keys)
        self.qoff = (np.ascontiguousarray(quad, np.uint16) if isinstance(quad, np.ndarray)
                     else face_quads(self.field, chunk))
        assert self.qoff.shape == (Z, Y, X, 6)
        self.sc.qoff = self.qoff.ctypes.data
        self.sc.chunk = chunk
        self.sc.unit_split = 1 if quad is False or quad is None else 0

    def hold_exit_table(self, params):
        """Build the exit table the frame `params` reads (exit mode, every sample
        on one table) once and keep it, so renders of that sun skip the build."""
        if not self.sc.exit_mode:
            return None
        d = sun_samples(params.sun_dir[:], params.sun_radius, params.shadow_samples)
        cone, octs, kx, ky = exit_plan(d, allow_cone=self.sc.exit_mode == 1 and self.sc.Z >= 3)
        if len(set(octs)) != 1 or octs[0] < 0:
            return None
        self._held = field_exit(self.field, octs[0], kx, ky)
        self.sc.held = self._held.ctypes.data
        self.sc.held_oct, self.sc.held_kx, self.sc.held_ky = octs[0], kx, ky
        if cone and not (params.flags & (0x20000 | 0x100)):      # the cone plan's doom table
            Z = self.sc.Z
            plan = doom_plan(d, params.max_shadow_steps if params.max_shadow_steps > 0 else 2 * Z)
            if plan[6] >= 1:
                self._held_doom = field_doom(self.field, plan)
                self.sc.held_doom = self._held_doom.ctypes.data
                self.sc.held_dplan = (C.c_int * 7)(*plan)
        return octs[0], kx, ky

    def render(self, params, w: int, h: int, row0: int = 0, row_step: int = 1, threads: int = 0, out=None):
        """RGBA fp32 (h, w, 4); rows not in (row0::row_step) are NaN."""
        if out is None:
            out = np.full((h, w, 4), np.nan, np.float32)
        st = OStats()
        lib().vxo_render(C.byref(self.sc), C.addressof(params), w, h, row0, row_step, out.ctypes.data,
                         C.byref(st), threads)
        return out, st

    def terms(self, params, w: int, h: int, row0: int = 0, row_step: int = 1, threads: int = 0):
        """Per pixel (h, w, 2): lit samples of the sun march of the first surface
        (slot 0) and of what a glass pane blends over (slot 1), 255 = no march;
        and sdf() of the AO sample (render.frag:223), NaN = none."""
        lit = np.full((h, w, 2), 255, np.uint8)
        amb = np.full((h, w, 2), np.nan, np.float32)
        lib().vxo_render_terms(C.byref(self.sc), C.addressof(params), w, h, row0, row_step, lit.ctypes.data,
                               amb.ctypes.data, threads)
        return lit, amb

    def march(self, cell, fract, direction, max_steps=None):
        m = OMarch()
        lib().vxo_march(C.byref(self.sc), (C.c_int * 3)(*cell), (C.c_float * 3)(*fract),
                        (C.c_float * 3)(*direction), int(max_steps if max_steps else 2 * self.sc.Z), C.byref(m))
        return m

    def primary(self, params, direction):
        g = (OGbuf * 2)()
        fetches = C.c_int()
        cap = C.c_int()
        n = lib().vxo_primary(C.byref(self.sc), C.addressof(params), (C.c_float * 3)(*direction), g,
                              C.byref(fetches), C.byref(cap))
        return n, [g[0], g[1]], fetches.value, cap.value

    def shade(self, params, gbuf, prim_dir):
        out = (C.c_float * 4)()
        lib().vxo_shade(C.byref(self.sc), C.addressof(params), C.byref(gbuf), (C.c_float * 3)(*prim_dir), out, None)
        return tuple(out)

    def glass_layers(self, params, w: int, h: int, threads: int = 0) -> np.ndarray:
        """(h, w) uint8: front-facing glass faces in front of each pixel's opaque hit."""
        out = np.zeros((h, w), np.uint8)
        lib().vxo_glass_layers(C.byref(self.sc), C.addressof(params), w, h, out.ctypes.data, threads)
        return out

    def pixel_dir(self, params, w, h, px, py):
        d = (C.c_float * 3)()
        lib().vxo_pixel_dir(C.addressof(params), w, h, px, py, d)
        return tuple(d)


def footprint(field_zyx4: np.ndarray) -> np.ndarray:
    """(Y, X) uint8: each column's top block with z >= 1 (a block has R == 0,
    sdf.cpp:430; z2d starts at 0 and only z > z2d replaces it, sdf.cpp:201-204),
    its meshed colour (1..21), else 0."""
    f = np.asarray(field_zyx4)
    Z = f.shape[0]
    out = np.zeros(f.shape[1:3], np.uint8)
    done = np.zeros(f.shape[1:3], bool)
    for z in range(Z - 1, 0, -1):
        blk = (f[z, :, :, 0] == 0) & ~done
        b = f[z, :, :, 2]
        out[blk] = np.where((b[blk] >= 1) & (b[blk] <= 21), b[blk], 0)
        done |= blk
    return out


def footprint_2d(field_zyx4: np.ndarray) -> np.ndarray:
    """(Y, X, 2) uint32 for the oracle's 2D mode: colour, quad corner x0 | y0 << 16
    of the footprint's greedy quads (mesh_ref.mesh2d: sdf.cpp:362-401, pinned
    byte for byte against the reference's vertex2d.bin)."""
    from . import mesh_ref
    c = footprint(field_zyx4)
    Y, X = c.shape
    out = np.zeros((Y, X, 2), np.uint32)
    out[..., 0] = c
    c2d = np.where(c == 0, 22, c).T.copy()                 # [x][y], air = pal_size as sdf.cpp remaps it
    for (x, y, w, h, col, _id) in mesh_ref.mesh2d(c2d):
        out[y:y + h, x:x + w, 1] = x | (y << 16)
    return np.ascontiguousarray(out)


def face_quads(field_zyx4: np.ndarray, chunk: int = 0) -> np.ndarray:
    """(Z, Y, X, 6) uint16: per cell and normal index, du | dv << 8 = the face's
    offset from the origin of the greedy quad covering it (vxo_face_quads,
    sdf.cpp:281-356 with CHUNK = chunk or Z); 0xFFFF where no face is."""
    f = np.ascontiguousarray(field_zyx4, np.uint8)
    Z, Y, X, _ = f.shape
    out = np.empty((Z, Y, X, 6), np.uint16)
    lib().vxo_face_quads(f.ctypes.data, X, Y, Z, int(chunk), out.ctypes.data)
    return out


def field_build(color_zyx: np.ndarray) -> np.ndarray:
    col = np.ascontiguousarray(color_zyx, np.uint8)
    Z, Y, X = col.shape
    out = np.empty((Z, Y, X, 4), np.uint8)
    lib().vxo_field_build(col.ctypes.data, X, Y, Z, out.ctypes.data)
    return out


def field_octant(field_zyx4: np.ndarray, oct: int, cap: int = 64) -> np.ndarray:
    """(Z, Y, X) uint8: size of the all-air cube ahead of each cell for ray octant ``oct``."""
    f = np.ascontiguousarray(field_zyx4, np.uint8)
    Z, Y, X, _ = f.shape
    out = np.empty((Z, Y, X), np.uint8)
    lib().vxo_field_octant(f.ctypes.data, X, Y, Z, cap, oct, out.ctypes.data)
    return out


def field_box(field_zyx4: np.ndarray, oct: int, cap: int = 64, r_cube=None) -> np.ndarray:
    """(Z, Y, X, 3) uint8: extents (ex, ey, ez) of the all-air box ahead of each
    cell for ray octant ``oct`` (vxo_field_box, grown from field_octant)."""
    f = np.ascontiguousarray(field_zyx4, np.uint8)
    Z, Y, X, _ = f.shape
    r = np.ascontiguousarray(field_octant(f, oct, cap) if r_cube is None else r_cube, np.uint8)
    out = np.empty((Z, Y, X, 3), np.uint8)
    lib().vxo_field_box(f.ctypes.data, X, Y, Z, cap, oct, r.ctypes.data, out.ctypes.data)
    return out


def field_exit(field_zyx4: np.ndarray, oct: int, kx: int = -1, ky: int = -1) -> np.ndarray:
    """(Z, Y, X) uint8: the sun exit table (vxo_field_exit) for
    sun octant ``oct`` (bit i: r_i > 0) and window (kx, ky); -1 = unbounded,
    the orthant table.  1 marks a cell from which the march cannot end unlit."""
    f = np.ascontiguousarray(field_zyx4, np.uint8)
    Z, Y, X, _ = f.shape
    out = np.empty((Z, Y, X), np.uint8)
    lib().vxo_field_exit(f.ctypes.data, X, Y, Z, oct, kx, ky, out.ctypes.data)
    return out


def doom_plan(dirs, max_steps: int):
    """(sx, sy, xlo, xhi, ylo, yhi, hmax): the doom table's sub-cell window for
    a frame's sun samples (vxo_doom_plan; all fast, one octant, r_z > 0) and the
    largest h its stop rule can use at MAX = max_steps."""
    d = np.ascontiguousarray(np.asarray(dirs, np.float32).reshape(-1, 3))
    v = (C.c_int * 7)()
    lib().vxo_doom_plan(d.ctypes.data, d.shape[0], int(max_steps), v)
    return tuple(v)


def field_doom(field_zyx4: np.ndarray, plan) -> np.ndarray:
    """(Z, Y, X) uint8: the sun doom table (vxo_field_doom): the
    crossing bound C(h) where every ray of the window provably enters a solid
    cell h <= hmax layers up, else 0."""
    f = np.ascontiguousarray(field_zyx4, np.uint8)
    Z, Y, X, _ = f.shape
    out = np.empty((Z, Y, X), np.uint8)
    lib().vxo_field_doom(f.ctypes.data, X, Y, Z, (C.c_int * 7)(*plan), out.ctypes.data)
    return out


def exit_plan(dirs, allow_cone: bool = True):
    """(cone, [octant per sample or -1], kx, ky): the build's table choice for
    a frame's sun directions (vxo_exit_plan)."""
    d = np.ascontiguousarray(np.asarray(dirs, np.float32).reshape(-1, 3))
    n = d.shape[0]
    oct = (C.c_int * n)()
    kx, ky = C.c_int(), C.c_int()
    cone = lib().vxo_exit_plan(d.ctypes.data, n, int(allow_cone), oct, C.byref(kx), C.byref(ky))
    return bool(cone), list(oct), kx.value, ky.value


def sun_samples(sun, radius: float, n: int) -> np.ndarray:
    """(max(n,1), 3) float32 soft-shadow sun directions (vxo_sun_samples)."""
    m = max(1, min(int(n), 16))
    out = np.zeros((m, 3), np.float32)
    lib().vxo_sun_samples((C.c_float * 3)(*sun), float(radius), int(n),
                          out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def vxo_palette() -> np.ndarray:
    """(22, 3) float32 palette of render.vert:21."""
    out = np.zeros((22, 3), np.float32)
    lib().vxo_palette(out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def exp2(x: float) -> float:
    return lib().vxo_exp2(float(x))
