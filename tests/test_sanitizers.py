"""The host half of the C ABI (voxmap_amd/csrc/vx_host.cpp + the codec, field
builder and frame-constant sources) under AddressSanitizer and
UndefinedBehaviorSanitizer: tests/sanitize/vx_host_san.cpp drives the
untrusted-input paths -- every truncation and random corruptions of .bin.gz and
.blob containers (the reference's D.fetch chain, utils.js:10-30), hostile scene
descriptions and frame parameters, the field builder and 2D mesher on random and
edge-size grids -- with -fno-sanitize-recover=all, so any finding fails the run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "voxmap_amd", "csrc")
SOURCES = [os.path.join(CSRC, s) for s in ("vx_host.cpp", "vx_codec.cpp", "vx_field.cpp", "vx_frame.cpp")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_abi_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "vx_host_san")
    cmd = ["g++", "-std=c++20", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-ffp-contract=off", "-I" + os.path.join(ROOT, "include"), "-o", exe,
           *SOURCES, os.path.join(ROOT, "tests", "sanitize", "vx_host_san.cpp"), "-lz", "-lcrypto", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, ROOT], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "SAN_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-6000:])


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sanitizer_build_catches_an_overflow(tmp_path):
    """Negative control: the same flags do stop a one-past-the-end read, so the
    clean run above is a real finding-free run, not a build without the runtime."""
    src = tmp_path / "oob.cpp"
    src.write_text("#include <vector>\nint main(int c, char **) { std::vector<unsigned char> v(16); "
                   "return v.data()[16 + c - 1]; }\n")
    exe = str(tmp_path / "oob")
    r = subprocess.run(["g++", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-o", exe,
                        str(src)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr
