"""The C++ mirror of kodr's API (include/kodr/kodr.hpp) builds against the
C ABI on CPU; its kodr-style test program runs on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "api_test.cpp")
BIN = os.path.join(ROOT, "tests", "cpp", "api_test")


def build():
    libdir = os.path.join(ROOT, "kodr_amd")
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), SRC, "-o", BIN,
           "-L", libdir, "-lkodr_rlnc", f"-Wl,-rpath,{libdir}", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_cpp_api_builds_and_links():
    build()
    assert os.path.exists(BIN)


@pytest.mark.gpu
def test_cpp_api_runs_kodr_flows():
    build()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok (0 failures)" in r.stdout


def test_host_pool_runs_every_task_once():
    """kodr_amd/csrc/host_pool.hpp (the grouped entry points' per-decoder host
    work): every task once per call, calls from two threads kept apart, and
    with KODR_HOST_THREADS=1 (no workers) the same results."""
    src = os.path.join(ROOT, "tests", "cpp", "host_pool_test.cpp")
    exe = os.path.join(ROOT, "tests", "cpp", "host_pool_test")
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", "-Wall", src, "-o", exe], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr
    for threads in ("8", "1"):
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120,
                           env={**os.environ, "KODR_HOST_THREADS": threads})
        assert r.returncode == 0 and "ok (0 failures)" in r.stdout, r.stdout + r.stderr


def test_decoder_core_continued_state():
    """DecoderCore::load_continued (the continued decoders of the batched GPU
    AddPiece and of the grouped flush) against kodr's route row by row, on the
    CPU: k = 2..256, r = 1..k-1 held rows (dense, a systematic prefix, and a
    dependent row that must be refused), M^-1 given alone or as whole state
    rows at a padded pitch."""
    src = os.path.join(ROOT, "tests", "cpp", "core_continued_test.cpp")
    core = os.path.join(ROOT, "kodr_amd", "csrc", "decoder_core.cpp")
    exe = os.path.join(ROOT, "tests", "cpp", "core_continued_test")
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", src, core, "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok (0 failures)" in r.stdout, r.stdout + r.stderr[-3000:]
