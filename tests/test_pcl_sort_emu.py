"""The device's PCL-order sort (csrc/pcl_sort.hpp) compiled for the host and run under a lane-per-thread
emulation of one workgroup (tests/ps_emu.cpp): its wave-level partitions, work queue and workgroup
phase leave exactly libstdc++'s std::sort order. CPU test (the GPU tests check the kernels themselves)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    exe = tmp_path_factory.mktemp("psemu") / "ps_emu"
    subprocess.check_call(["g++", "-std=c++20", "-O1", "-pthread", "-w", "-o", str(exe), os.path.join(HERE, "ps_emu.cpp")])
    return str(exe)


def test_device_sort_matches_libstdcxx_under_emulation(emu):
    # 2 waves of 64 lanes; sizes up to 4096 (one wave segment) and 4000-8000 (workgroup phase first)
    r = subprocess.run([emu, "5", "11"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


@pytest.mark.parametrize("tail", [None, 4096], ids=["default_tail", "waves_early"])
def test_ls_sort_matches_libstdcxx_under_emulation(tmp_path, tail):
    # csrc/ls_sort.hpp on 2 emulated waves (n <= 128 * 16): every introsort level of every segment at once,
    # the sparse tail per wave (LS_TAIL 4096: the waves take over as soon as <= 2 segments are active)
    exe = tmp_path / "ls_emu"
    defs = [f"-DLS_TAIL_DEF={tail}"] if tail else []
    subprocess.check_call(["g++", "-std=c++20", "-O1", "-pthread", "-w", *defs, "-o", str(exe), os.path.join(HERE, "ps_emu.cpp")])
    r = subprocess.run([str(exe), "40", "13", "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_ls_sort_global_matches_libstdcxx_under_emulation(emu):
    # csrc/ls_sort.hpp's global sort (n 4000-8000, split to segments <= cap, each sorted in the LDS buffer)
    r = subprocess.run([emu, "16", "17", "2"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
