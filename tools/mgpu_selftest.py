"""vx_mgpu_* with N ranks (processes) on the GPUs this box has: each rank
renders its bands, rank 0 gathers; rank 0's frame must equal a single-GPU
vx_render of the whole frame.  With fewer GPUs than ranks every rank uses
device rank % n_devices (RCCL may refuse two ranks on one GPU: then the
script says so and exits 3).  usage: python tools/mgpu_selftest.py [N]"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, q):
    import numpy as np
    import torch
    import torch.distributed as dist
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = rank % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    grid = presets.scene_grid("s_proc")
    Z, Y, X = grid.shape
    sc = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                  dims=(X, Y, Z), device=dev)
    w, h = 1920, 1080
    fr = presets.camera_frame("K1", w, h, flags=vx.FLAG_FULL_QUALITY)
    uid = [vx.mgpu_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    try:
        mg = vx.MultiGPU(sc, uid[0], world, rank)
    except Exception as e:  # RCCL refusing duplicate devices
        q.put(("init", rank, str(e)))
        dist.destroy_process_group()
        return
    frame = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        st = mg.render(fr, 64, frame.data_ptr(), stats=True)
    torch.cuda.synchronize()
    dist.barrier()
    if rank == 0:
        want, _ = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
        got = frame.cpu().numpy()
        q.put(("ok" if np.array_equal(got, want) else "mismatch", rank,
               int(np.count_nonzero(np.any(got != want, axis=2)))))
    mg.close()
    sc.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = []
    while not q.empty():
        res.append(q.get())
    print("results", res, "exitcodes", [p.exitcode for p in procs], flush=True)
    if any(r[0] == "init" for r in res):
        sys.exit(3)
    sys.exit(0 if res and all(r[0] == "ok" for r in res) else 1)
