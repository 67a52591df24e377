"""The t <= 4 RS emission schedules (paritypartyfs_amd/csrc/rs_sched.hpp) on the host: every piece of
a tile emitted once, interior pieces only in rounds 0-2, a round-3 piece in every wave, the interior
pieces' 4-shift windows equal to the codeword / payload bytes, and no more window-read bank
conflicts than the natural piece order (tests/cpp/test_sched.cpp).  CPU only: g++ builds it."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rs_emission_schedules(tmp_path):
    exe = str(tmp_path / "test_sched")
    src = os.path.join(ROOT, "tests", "cpp", "test_sched.cpp")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", src, "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
