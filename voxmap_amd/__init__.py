"""voxmap_amd — MI355X-native Voxmap shading path (primary visibility + render.frag).

The product is libvoxmap_hip.so (HIP kernels for gfx950 behind the C ABI of
include/voxmap.h).  This package is the host-side mirror of the reference's
renderer interface (src/web/render.js) over that ABI; it never computes pixels
itself and raises if the library is missing.
"""
from ._abi import (FLAG_GLASS_ORDER, FLAG_GLASS_SINGLE, FLAG_REFLECT_ALL, FLAG_UNIT_GBUF, FLAG_FULL_QUALITY, FLAG_INT_INDEX, FLAG_SOFT_POOL, FLAG_SOFT_BRICK, FLAG_NO_EXIT, FLAG_NO_CONE, FLAG_NO_DOOM, FLAG_NO_AO, FLAG_NO_CLOUDS, FLAG_NO_SHADOW, FLAG_PRIMARY_ONLY, FLAG_REFLECT,
                   FLAG_ROUGH, FORMAT_AUTO, FORMAT_BIN, FORMAT_BIN_GZ, FORMAT_BLOB, FORMAT_GRID, PIXEL_RGBA8, PIXEL_RGBA32F,
                   FrameParams, Stats, VoxmapError, lib)
from .renderer import (Frame, MultiGPU, Scene, blob_encrypt, decode, field_build, frame_from_matrix, frame_from_orbit,
                       hour_from_time_ms, make_frame, mgpu_band_rows, mgpu_bands, mgpu_transfers, mgpu_unique_id, noise_synth, field_build_gpu,
                       params_to_dict, sun_from_hour, sun_samples, vertex2d)

__all__ = [
    "Scene", "Frame", "FrameParams", "Stats", "VoxmapError", "lib", "make_frame", "frame_from_orbit",
    "frame_from_matrix", "sun_from_hour", "hour_from_time_ms", "field_build", "noise_synth", "decode",
    "blob_encrypt", "params_to_dict", "PIXEL_RGBA32F", "PIXEL_RGBA8", "FORMAT_AUTO", "FORMAT_BIN",
    "FORMAT_BIN_GZ", "FORMAT_BLOB", "FLAG_NO_SHADOW", "FLAG_NO_AO", "FLAG_NO_CLOUDS", "FLAG_PRIMARY_ONLY",
    "FLAG_REFLECT", "FLAG_ROUGH", "FLAG_FULL_QUALITY", "FLAG_INT_INDEX", "FLAG_SOFT_POOL", "FLAG_SOFT_BRICK", "FLAG_NO_EXIT", "FLAG_NO_CONE", "FLAG_NO_DOOM",
    "FLAG_UNIT_GBUF", "FLAG_GLASS_ORDER", "FLAG_GLASS_SINGLE", "FLAG_REFLECT_ALL", "sun_samples", "field_build_gpu", "FORMAT_GRID",
    "MultiGPU", "mgpu_unique_id", "mgpu_band_rows", "mgpu_bands", "mgpu_transfers", "vertex2d",
]
