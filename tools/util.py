"""Lane utilisation of the traversal / march loops (STATS counters) for a bench config."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401
import voxmap_amd as vx
from voxmap_amd import presets

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
flags = int(sys.argv[2]) if len(sys.argv) > 2 else 48
samples = int(sys.argv[3]) if len(sys.argv) > 3 else presets.CONFIGS[cfg].get("samples", 1)
c = presets.CONFIGS[cfg]
grid = presets.scene_grid(c["scene"])
Z, Y, X = grid.shape
sc = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, dims=(X, Y, Z), device=0)
up = 3.0 if c["scene"] == "s_up3" else 1.0
fr = presets.camera_frame(c["camera"], c["w"], c["h"], scale=up, flags=flags, shadow_samples=samples,
                          sun_radius=0.03 if samples > 1 else 0.0)
import torch
out = torch.empty(c["w"] * c["h"] * 4, dtype=torch.uint8, device="cuda")
st = sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stats=True)
d = st.as_dict()
loop_fetch = d["primary_fetches"] - d["pixels"]
print(cfg, "flags", flags, "samples", samples, {k: d[k] for k in ("pixels", "sky_px", "block_px", "glass_px",
      "primary_fetches", "shadow_rays", "shadow_fetches", "primary_wave_iters", "march_wave_iters")})
print("primary loop lane utilisation %.3f (per-pixel loop steps %.2f)" %
      (loop_fetch / (64.0 * d["primary_wave_iters"]), loop_fetch / d["pixels"]))
print("march lane utilisation %.3f (steps per shadow ray %.2f)" %
      (d["shadow_fetches"] / (64.0 * max(1, d["march_wave_iters"])), d["shadow_fetches"] / max(1, d["shadow_rays"])))
