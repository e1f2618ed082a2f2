"""Per-scene host state under concurrent use:
band / tile-id lists of one scene rendered by two host threads on their own
streams, each changing its list every frame (a list is uploaded once per
distinct list and never rewritten while cached: vx_api.cpp list_acquire), and
the sun's cone copies recycled after a stream that read them was destroyed (the
scene keeps no stream handle of the caller's: cone_copy).  Every frame is
compared with the same pixels rendered by vx_render alone."""
import ctypes as C
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(built):
    try:
        import torch
        ok = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        ok = False
    if not ok:
        pytest.skip("no GPU visible")


@pytest.fixture(scope="module")
def scene(noise):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (192, 96, 24)
    field = vx.field_build(scenes.small_proc(41, dims=dims, n_boxes=24, n_glass=6))
    sc = vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=dims, device=0)
    yield sc
    sc.close()


def _hip():
    """The HIP runtime this process already runs (torch's libamdhip64, which
    libvoxmap_hip.so resolves to as well): raw streams that are really destroyed
    (torch.cuda.Stream comes from a pool and is never destroyed)."""
    import torch
    L = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    L.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
    L.hipStreamDestroy.argtypes = [C.c_void_p]
    L.hipStreamSynchronize.argtypes = [C.c_void_p]
    return L


def _stream(L):
    s = C.c_void_p()
    assert L.hipStreamCreateWithFlags(C.byref(s), 1) == 0     # hipStreamNonBlocking
    return s.value


def _rgba8(img):
    return np.ascontiguousarray(img[0] if isinstance(img, tuple) else img).view(np.uint8).reshape(-1)


def test_two_threads_render_different_band_lists(scene):
    """Two host threads, each on its own stream, render bands of one scene in
    place, switching between two different band lists every frame (so every
    frame asks for a list the other thread is not using): each frame's bands
    equal the full frame's rows and the other rows stay untouched."""
    import threading

    import torch

    import voxmap_amd as vx
    W, H, BR = 512, 320, 16
    fr = vx.make_frame((96.0, 48.0, 30.0), (1.1, 0.0, 0.6), W, H, flags=vx.FLAG_FULL_QUALITY)
    ref = _rgba8(scene.render(fr, pixel_format=vx.PIXEL_RGBA8)).reshape(H, W * 4)
    nb = H // BR
    lists = {0: [list(range(0, nb, 2)), list(range(0, nb // 2))],
             1: [list(range(1, nb, 2)), list(range(nb // 2, nb))]}
    errors = []

    def worker(tid):
        try:
            st = torch.cuda.Stream()
            buf = torch.zeros(H * W * 4, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()     # the fill on torch's stream before st uses the buffer
            for rep in range(16):
                ids = lists[tid][rep % 2]
                with torch.cuda.stream(st):
                    buf.zero_()
                scene.render_bands(fr, BR, ids, buf.data_ptr(), inplace=True, pixel_format=vx.PIXEL_RGBA8,
                                   stream=st.cuda_stream)
                st.synchronize()
                got = buf.cpu().numpy().reshape(H, W * 4)
                mask = np.zeros(H, bool)
                for b in ids:
                    mask[b * BR:(b + 1) * BR] = True
                if not (np.array_equal(got[mask], ref[mask]) and not got[~mask].any()):
                    errors.append((tid, rep))
        except Exception as e:  # pragma: no cover - reported below
            errors.append((tid, repr(e)))

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:5]


def test_tile_lists_from_two_threads(scene):
    """The same with compact tile lists + vx_detile: two threads, different and
    changing tile lists, each de-tiled into its own frame on its own stream."""
    import threading

    import torch

    import voxmap_amd as vx
    W, H, TS = 448, 256, 64
    fr = vx.make_frame((96.0, 48.0, 30.0), (1.0, 0.0, -0.5), W, H, flags=vx.FLAG_FULL_QUALITY)
    ref = _rgba8(scene.render(fr, pixel_format=vx.PIXEL_RGBA8)).reshape(H, W, 4)
    tx, ty = (W + TS - 1) // TS, (H + TS - 1) // TS
    n = tx * ty
    lists = {0: [list(range(0, n, 3)), list(range(0, n, 2))], 1: [list(range(1, n, 3)), list(range(n - 1, -1, -2))]}
    errors = []

    def worker(tid):
        try:
            st = torch.cuda.Stream()
            tiles = torch.empty(n * TS * TS * 4, dtype=torch.uint8, device="cuda")
            frame = torch.zeros(H * W * 4, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()     # the fill on torch's stream before st uses the buffer
            for rep in range(12):
                ids = lists[tid][rep % 2]
                with torch.cuda.stream(st):
                    frame.zero_()
                scene.render_tiles(fr, TS, ids, tiles.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=st.cuda_stream)
                scene.detile(W, H, TS, ids, tiles.data_ptr(), frame.data_ptr(), pixel_format=vx.PIXEL_RGBA8,
                             stream=st.cuda_stream)
                st.synchronize()
                got = frame.cpu().numpy().reshape(H, W, 4)
                mask = np.zeros((H, W), bool)
                for t in ids:
                    x0, y0 = (t % tx) * TS, (t // tx) * TS
                    mask[y0:y0 + TS, x0:x0 + TS] = True
                if not (np.array_equal(got[mask], ref[mask]) and not got[~mask].any()):
                    errors.append((tid, rep))
        except Exception as e:  # pragma: no cover - reported below
            errors.append((tid, repr(e)))

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:5]


def _sun(el_deg, az_deg):
    el, az = math.radians(el_deg), math.radians(az_deg)
    return (math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el))


def test_cone_recycle_after_reader_stream_destroyed(scene):
    """render with a sun on a stream and destroy that stream at once
    (its work maybe still in flight), then force that sun's cone copy out of the
    scene's two slots from new streams (which may reuse the dead handle), and
    back again.  No dead handle is touched (the scene keeps none) and every
    frame equals the frame rendered alone."""
    import torch

    import voxmap_amd as vx
    L = _hip()
    W, H = 256, 160
    suns = [(33, 30), (40, 120), (60, 210)]          # three cone windows, two slots
    frames = {k: vx.make_frame((96.0, 48.0, 34.0), (1.0, 0.0, -0.4), W, H, sun=_sun(*k),
                               flags=vx.FLAG_FULL_QUALITY) for k in suns}
    refs = {k: _rgba8(scene.render(f, pixel_format=vx.PIXEL_RGBA8)) for k, f in frames.items()}
    outs = []
    for rep in range(3):
        for k in suns:
            st = _stream(L)
            buf = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
            scene.render_device(frames[k], buf.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=st)
            assert L.hipStreamDestroy(C.c_void_p(st)) == 0      # destroyed with its frame maybe in flight
            outs.append((k, buf))
    torch.cuda.synchronize()
    for k, buf in outs:
        assert np.array_equal(buf.cpu().numpy(), refs[k]), k
