"""Host-side mirror of the reference's renderer interface (src/web/render.js).

The reference host is browser JavaScript: ``loadTextures`` /
``loadEncryptedTextures`` upload the noise and field textures
(render.js:134-245) and ``drawScene(projection_matrix, position, sun, frame,
time)`` sets the uniforms and draws (render.js:267-298).  ``Scene`` plays the
texture-owning role over the C ABI (``vx_scene_create``) and
``Scene.draw_scene`` keeps drawScene's argument meaning; ``Scene.render`` is
the lower-level call on prepared ``FrameParams``.  Every call goes through
libvoxmap_hip.so; errors raise ``VoxmapError`` with the library's message.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import numpy as np

from . import _abi
from ._abi import FrameParams, Stats, check, lib

DEFAULT_DIMS = (1024, 256, 32)  # render.h:14-16


def _f3(arr) -> tuple:
    return tuple(float(v) for v in arr)


def frame_from_orbit(sbj, rot, w: int, h: int) -> FrameParams:
    """Camera of map.js:373-391 (orbit around ``sbj`` at radius sbj.z)."""
    p = FrameParams()
    s = (C.c_double * 3)(*sbj)
    r = (C.c_double * 3)(*rot)
    check(lib().vx_frame_from_orbit(s, r, int(w), int(h), C.byref(p)))
    return p


def frame_from_matrix(u_matrix, cam_pos) -> FrameParams:
    """From a column-major u_matrix (render.js:288) and the camera position."""
    p = FrameParams()
    m = (C.c_float * 16)(*[float(v) for v in u_matrix])
    pos = (C.c_double * 3)(*cam_pos)
    check(lib().vx_frame_from_matrix(m, pos, C.byref(p)))
    return p


def sun_from_hour(hour: float) -> tuple:
    """map.js:399-402."""
    out = (C.c_float * 3)()
    lib().vx_sun_from_hour(float(hour), out)
    return tuple(out)


def hour_from_time_ms(time_ms: float) -> float:
    """map.js:399: hour = 4*t/1000/60/60/12*pi - 0.5 (t in local ms)."""
    return 4 * time_ms / 1000 / 60 / 60 / 12 * math.pi - 0.5


@dataclass
class Frame:
    """Everything drawScene needs besides the textures (render.js:267)."""
    params: FrameParams
    width: int
    height: int


def make_frame(sbj, rot, w, h, *, sun=None, hour=1.0, time=123.0, quality=1, frame=0,
               flags=0, max_shadow_steps=0, shadow_samples=0, sun_radius=0.0) -> Frame:
    p = frame_from_orbit(sbj, rot, w, h)
    sd = sun if sun is not None else sun_from_hour(hour)
    for i in range(3):
        p.sun_dir[i] = float(sd[i])
    p.time = float(time) % 1000.0          # render.js:293
    p.quality = int(quality)               # render.js:287 (3D mode -> 1)
    p.frame = int(frame)
    p.flags = int(flags)
    p.max_shadow_steps = int(max_shadow_steps)
    p.shadow_samples = int(shadow_samples)  # ext soft shadows (<= 1: hard, render.frag:232-235)
    p.sun_radius = float(sun_radius)
    return Frame(p, int(w), int(h))


def sun_samples(sun, radius: float, n: int):
    """The soft-shadow sun directions a frame with ``shadow_samples = n`` marches (vx_sun_samples)."""
    import numpy as _np
    m = max(1, min(int(n), _abi.MAX_SHADOW_SAMPLES))
    out = _np.zeros((m, 3), _np.float32)
    check(lib().vx_sun_samples((C.c_float * 3)(*sun), float(radius), int(n),
                               out.ctypes.data_as(C.POINTER(C.c_float))))
    return out


class Scene:
    """Device-resident field + noise textures on one GPU (render.js:134-206)."""

    def __init__(self, *, map_path=None, map_bytes=None, map_format=_abi.FORMAT_AUTO, key=None,
                 noise_path=None, noise_bytes=None, noise_format=_abi.FORMAT_AUTO, noise_size=(1024, 1024),
                 dims=DEFAULT_DIMS, device=0, dist_cap=0, noise_seed=0, mesh_chunk=0):
        L = lib()
        d = _abi.SceneDesc()
        self._keep = []
        if map_path is not None:
            d.map_path = str(map_path).encode()
        if map_bytes is not None:
            buf = np.ascontiguousarray(np.frombuffer(memoryview(map_bytes).cast("B"), dtype=np.uint8))
            self._keep.append(buf)
            d.map_bytes = buf.ctypes.data
            d.map_size = buf.nbytes
        d.map_format = map_format
        if key is not None:
            d.key_jwk_k = key.encode() if isinstance(key, str) else key
        if noise_path is not None:
            d.noise_path = str(noise_path).encode()
        if noise_bytes is not None:
            nb = np.ascontiguousarray(np.frombuffer(memoryview(noise_bytes).cast("B"), dtype=np.uint8))
            self._keep.append(nb)
            d.noise_bytes = nb.ctypes.data
            d.noise_size = nb.nbytes
        d.noise_format = noise_format
        d.noise_w, d.noise_h = int(noise_size[0]), int(noise_size[1])
        d.X, d.Y, d.Z = (int(v) for v in dims)
        d.device = int(device)
        d.dist_cap = int(dist_cap)
        d.noise_seed = int(noise_seed)
        d.mesh_chunk = int(mesh_chunk)
        h = C.c_void_p()
        check(L.vx_scene_create(C.byref(d), C.byref(h)))
        self._h = h
        self._keep = []
        self.dims = tuple(int(v) for v in dims)
        self.device = int(device)

    @property
    def handle(self) -> C.c_void_p:
        if self._h is None:
            raise ValueError("scene is closed")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None:
            lib().vx_scene_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def read_field(self, octant: int = 0) -> np.ndarray:
        """(Z, Y, X, 4) RGBA8 of the device field copy for ray octant ``octant``."""
        X, Y, Z = self.dims
        out = np.empty((Z, Y, X, 4), np.uint8)
        check(lib().vx_scene_read_field_copy(self.handle, octant, out.ctypes.data, out.nbytes))
        return out

    def vertex2d(self) -> bytes:
        """The 2D mode mesh as vertex2d.bin bytes (sdf.cpp:362-401, vx_scene_vertex2d)."""
        n = C.c_size_t()
        check(lib().vx_scene_vertex2d(self.handle, None, 0, C.byref(n)))
        out = np.empty(n.value, np.uint8)
        check(lib().vx_scene_vertex2d(self.handle, out.ctypes.data, out.size, C.byref(n)))
        return out.tobytes()

    def read_face_quads(self) -> np.ndarray:
        """(Z, Y, X, 6) uint16: per cell and normal index, the face's offset du | dv << 8
        from the origin of its greedy quad (vx_scene_read_face_quads); 0xFFFF = no face."""
        X, Y, Z = self.dims
        out = np.empty((Z, Y, X, 6), np.uint16)
        check(lib().vx_scene_read_face_quads(self.handle, out.ctypes.data, out.nbytes))
        return out

    def read_boxes(self, octant: int = 0) -> np.ndarray:
        """(Z, Y, X, 4) uint8: colour, ex, ey, ez of the octant's traversal boxes."""
        X, Y, Z = self.dims
        out = np.empty((Z, Y, X, 4), np.uint8)
        check(lib().vx_scene_read_boxes(self.handle, octant, out.ctypes.data, out.nbytes))
        return out

    def render(self, frame: Frame, *, pixel_format=_abi.PIXEL_RGBA32F, stats: bool = False):
        """Render to host memory; returns (image[h, w, 4], Stats or None)."""
        w, h = frame.width, frame.height
        if pixel_format == _abi.PIXEL_RGBA32F:
            out = np.empty((h, w, 4), np.float32)
        else:
            out = np.empty((h, w, 4), np.uint8)
        st = Stats() if stats else None
        check(lib().vx_render(self.handle, C.byref(frame.params), w, h, pixel_format, out.ctypes.data, 0,
                              None, C.byref(st) if st is not None else None))
        return out, st

    def render_device(self, frame: Frame, out_ptr: int, *, pixel_format=_abi.PIXEL_RGBA32F, stream=None,
                      stats: bool = False):
        """Render into a device buffer (e.g. a torch tensor's data_ptr()); stream-ordered."""
        st = Stats() if stats else None
        check(lib().vx_render(self.handle, C.byref(frame.params), frame.width, frame.height, pixel_format,
                              C.c_void_p(out_ptr), 1, C.c_void_p(stream) if stream else None,
                              C.byref(st) if st is not None else None))
        return st

    def render_tiles(self, frame: Frame, tile_size: int, tile_ids, out_ptr: int, *,
                     pixel_format=_abi.PIXEL_RGBA8, stream=None, stats: bool = False):
        ids = np.ascontiguousarray(np.asarray(tile_ids, dtype=np.int32))
        st = Stats() if stats else None
        check(lib().vx_render_tiles(self.handle, C.byref(frame.params), frame.width, frame.height,
                                    int(tile_size), ids.ctypes.data_as(C.POINTER(C.c_int)), int(ids.size),
                                    pixel_format, C.c_void_p(out_ptr), C.c_void_p(stream) if stream else None,
                                    C.byref(st) if st is not None else None))
        return st

    def prepare_sun(self, frame: Frame, *, stream=None) -> dict:
        """Build (or find) the sun exit copy frame's march reads (vx_prepare_sun,
        synchronises the stream): {"kind": 0 none / 1 orthant / 2 cone, "octant",
        "kx", "ky", "build_ms": GPU time of the copy built now (0: already built)}."""
        info = _abi.ExitInfo()
        check(lib().vx_prepare_sun(self.handle, C.byref(frame.params), C.c_void_p(stream) if stream else None,
                                   C.byref(info)))
        return {k: getattr(info, k) for k, _ in info._fields_}

    def render_bands(self, frame: Frame, band_rows: int, band_ids, out_ptr: int, *, inplace: bool = True,
                     pixel_format=_abi.PIXEL_RGBA8, stream=None, stats: bool = False):
        """Full-width bands of rows (vx_render_bands): in place in a w*h frame, or compact."""
        ids = np.ascontiguousarray(np.asarray(band_ids, dtype=np.int32))
        st = Stats() if stats else None
        check(lib().vx_render_bands(self.handle, C.byref(frame.params), frame.width, frame.height, int(band_rows),
                                    ids.ctypes.data_as(C.POINTER(C.c_int)), int(ids.size), pixel_format,
                                    C.c_void_p(out_ptr), 1 if inplace else 0,
                                    C.c_void_p(stream) if stream else None, C.byref(st) if st is not None else None))
        return st

    def detile(self, w, h, tile_size, tile_ids, tiles_ptr, frame_ptr, *, pixel_format=_abi.PIXEL_RGBA8,
               stream=None):
        ids = np.ascontiguousarray(np.asarray(tile_ids, dtype=np.int32))
        check(lib().vx_detile(self.handle, int(w), int(h), int(tile_size), ids.ctypes.data_as(C.POINTER(C.c_int)),
                              int(ids.size), pixel_format, C.c_void_p(tiles_ptr), C.c_void_p(frame_ptr),
                              C.c_void_p(stream) if stream else None))

    def draw_scene(self, projection_matrix, position, sun, frame, time, *, width, height, mode_3d=True,
                   pixel_format=_abi.PIXEL_RGBA8):
        """drawScene(projection_matrix, position, sun, frame, time) of render.js:267, returning the canvas."""
        p = frame_from_matrix(projection_matrix, position)
        for i in range(3):
            p.sun_dir[i] = float(sun[i])
        p.quality = 1 if mode_3d else 0
        p.frame = int(frame)
        p.time = float(time) % 1000.0
        img, _ = self.render(Frame(p, int(width), int(height)), pixel_format=pixel_format)
        return img


def mgpu_unique_id() -> bytes:
    """Rank 0: the RCCL unique id (VX_MGPU_UID_BYTES) every rank passes to MultiGPU."""
    buf = (C.c_char * _abi.MGPU_UID_BYTES)()
    check(lib().vx_mgpu_unique_id(buf))
    return bytes(buf)


def mgpu_bands(h: int, band_rows: int, nranks: int, rank: int) -> list:
    """The band deal of vx_mgpu_render (band b -> rank b % nranks)."""
    n = lib().vx_mgpu_bands(int(h), int(band_rows), int(nranks), int(rank), None, 0)
    if n < 0:
        check(n)
    ids = (C.c_int * max(n, 1))()
    lib().vx_mgpu_bands(int(h), int(band_rows), int(nranks), int(rank), ids, n)
    return list(ids[:n])


def mgpu_band_rows(h: int, nranks: int, max_rows: int = 64) -> int:
    """The deal's band height for an h-row frame over nranks ranks (vx_mgpu_band_rows)."""
    r = lib().vx_mgpu_band_rows(int(h), int(nranks), int(max_rows))
    check(r if r < 0 else 0)
    return r


def mgpu_transfers(w: int, h: int, band_rows: int, nranks: int, rank: int, pixel_format: int = 1) -> list:
    """The gather's transfer list as ``rank`` issues it (vx_mgpu_transfers, a pure
    host function): [(band, src, dst, rows, byte offset, bytes), ...] in band order."""
    args = (int(w), int(h), int(band_rows), int(pixel_format), int(nranks), int(rank))
    n = lib().vx_mgpu_transfers(*args, None, 0)
    if n < 0:
        check(n)
    xs = (_abi.MgpuXfer * max(n, 1))()
    check(0 if lib().vx_mgpu_transfers(*args, C.cast(xs, C.c_void_p), n) == n else -1)
    return [(x.band, x.src, x.dst, x.rows, x.offset, x.bytes) for x in xs[:n]]


class MultiGPU:
    """One rank of a frame shared by the GPUs of a node (vx_mgpu_*: bands
    rendered in place, gathered into rank 0's frame over RCCL)."""

    def __init__(self, scene: Scene, uid: bytes, nranks: int, rank: int):
        h = C.c_void_p()
        buf = (C.c_char * _abi.MGPU_UID_BYTES).from_buffer_copy(uid)
        check(lib().vx_mgpu_create(scene.handle, buf, int(nranks), int(rank), C.byref(h)))
        self._h = h
        self.scene = scene
        self.nranks, self.rank = int(nranks), int(rank)

    def render(self, frame: Frame, band_rows: int, frame_ptr: int, *, pixel_format=_abi.PIXEL_RGBA8, stream=None,
               stats: bool = False):
        st = Stats() if stats else None
        check(lib().vx_mgpu_render(self._h, C.byref(frame.params), frame.width, frame.height, int(band_rows),
                                   pixel_format, C.c_void_p(frame_ptr), C.c_void_p(stream) if stream else None,
                                   C.byref(st) if st is not None else None))
        return st

    def gather(self, width: int, height: int, band_rows: int, frame_ptr: int, *, pixel_format=_abi.PIXEL_RGBA8,
               stream=None):
        """The gather step of render() alone (collective): ranks 1..n-1's bands into rank 0's frame rows."""
        check(lib().vx_mgpu_gather(self._h, int(width), int(height), int(band_rows), pixel_format,
                                   C.c_void_p(frame_ptr), C.c_void_p(stream) if stream else None))

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().vx_mgpu_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


# ---- host helpers over the ABI ------------------------------------------------

def field_build(color_zyx: np.ndarray, n_threads: int = 0) -> np.ndarray:
    """map.bin texels (Z, Y, X, 4) from a palette-index grid (Z, Y, X) — sdf.cpp:405-470."""
    col = np.ascontiguousarray(color_zyx, dtype=np.uint8)
    Z, Y, X = col.shape
    out = np.empty((Z, Y, X, 4), np.uint8)
    check(lib().vx_field_build(col.ctypes.data, X, Y, Z, out.ctypes.data, int(n_threads)))
    return out


def field_build_gpu(color_zyx: np.ndarray, device: int = 0) -> np.ndarray:
    """vx_field_build on GPU ``device`` (same bytes, plane-parallel on the device)."""
    col = np.ascontiguousarray(color_zyx, dtype=np.uint8)
    Z, Y, X = col.shape
    out = np.empty((Z, Y, X, 4), np.uint8)
    check(lib().vx_field_build_gpu(col.ctypes.data, X, Y, Z, out.ctypes.data, int(device)))
    return out


def vertex2d(field_zyx4: np.ndarray) -> bytes:
    """vertex2d.bin bytes (sdf.cpp:362-401) of a map.bin field (vx_vertex2d, host C++)."""
    f = np.ascontiguousarray(field_zyx4, dtype=np.uint8)
    Z, Y, X, _ = f.shape
    n = C.c_size_t()
    check(lib().vx_vertex2d(f.ctypes.data, X, Y, Z, None, 0, C.byref(n)))
    out = np.empty(n.value, np.uint8)
    check(lib().vx_vertex2d(f.ctypes.data, X, Y, Z, out.ctypes.data, out.size, C.byref(n)))
    return out.tobytes()


def noise_synth(seed: int = 0, w: int = 1024, h: int = 1024) -> np.ndarray:
    out = np.empty((h, w, 4), np.uint8)
    check(lib().vx_noise_synth(int(seed), w, h, out.ctypes.data))
    return out


def decode(data: bytes, fmt: int, key: str | None = None) -> bytes:
    L = lib()
    buf = np.frombuffer(data, np.uint8)
    n = C.c_size_t()
    k = key.encode() if key else None
    check(L.vx_decode(buf.ctypes.data, buf.size, fmt, k, None, 0, C.byref(n)))
    out = np.empty(n.value, np.uint8)
    check(L.vx_decode(buf.ctypes.data, buf.size, fmt, k, out.ctypes.data, out.size, C.byref(n)))
    return out.tobytes()


def blob_encrypt(data: bytes, key: str) -> bytes:
    L = lib()
    buf = np.frombuffer(data, np.uint8)
    n = C.c_size_t()
    check(L.vx_blob_encrypt(buf.ctypes.data, buf.size, key.encode(), None, 0, C.byref(n)))
    out = np.empty(n.value, np.uint8)
    check(L.vx_blob_encrypt(buf.ctypes.data, buf.size, key.encode(), out.ctypes.data, out.size, C.byref(n)))
    return out.tobytes()


def params_to_dict(p: FrameParams) -> dict:
    return {
        "quality": p.quality, "frame": p.frame, "time": p.time,
        "cam_cell": list(p.cam_cell), "cam_fract": _f3(p.cam_fract), "sun_dir": _f3(p.sun_dir),
        "ray_fwd": _f3(p.ray_fwd), "ray_right": _f3(p.ray_right), "ray_up": _f3(p.ray_up),
        "flags": p.flags, "max_shadow_steps": p.max_shadow_steps,
        "shadow_samples": p.shadow_samples, "sun_radius": p.sun_radius,
    }
