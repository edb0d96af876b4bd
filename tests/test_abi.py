"""The C-ABI boundary: header <-> shared library <-> ctypes mirror (CPU-only checks)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from lvo_amd_loader import abi, lvo

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "aloam_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(aloam_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_python_symbol_list():
    assert declared_functions() == sorted(lvo.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    assert os.path.exists(lvo.LIB_PATH), "run __graft_entry__.build() first"
    out = subprocess.check_output(["nm", "-D", "--defined-only", lvo.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in declared_functions() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_abi_version():
    L = lvo.lib()
    assert L.aloam_abi_version() == 7


def test_struct_layouts_match_header():
    # compile a tiny C program against the header and compare sizeof / offsetof with ctypes
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "aloam_hip.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(aloam_params), sizeof(aloam_cloud), sizeof(aloam_features),
        sizeof(aloam_lm_summary), sizeof(aloam_odom_result), sizeof(aloam_map_result), sizeof(aloam_factor), sizeof(aloam_timing));
 printf("%zu %zu %zu\n", offsetof(aloam_odom_result, lm), offsetof(aloam_map_result, lm), offsetof(aloam_factor, b));
 return 0;}
'''
    tmp = os.path.join(REPO, "tests", "_layout_check.c")
    exe = tmp[:-2]
    with open(tmp, "w") as f:
        f.write(prog)
    try:
        subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), tmp, "-o", exe])
        line1, line2 = subprocess.check_output([exe], text=True).split("\n")[:2]
    finally:
        for p in (tmp, exe):
            if os.path.exists(p):
                os.remove(p)
    sizes = [int(v) for v in line1.split()]
    assert sizes == [C.sizeof(t) for t in (abi.Params, abi.Cloud, abi.Features, abi.LMSummary, abi.OdomResult,
                                            abi.MapResult, abi.Factor, abi.Timing)]
    offs = [int(v) for v in line2.split()]
    assert offs == [abi.OdomResult.lm.offset, abi.MapResult.lm.offset, abi.Factor.b.offset]


def test_default_params_match_python_mirror():
    L = lvo.lib()
    for lines in (16, 32, 64, 128):
        p = abi.Params()
        L.aloam_default_params(C.byref(p), lines)
        q = abi.default_params(lines)
        for name, _ in abi.Params._fields_:
            assert getattr(p, name) == pytest.approx(getattr(q, name)), (lines, name)


def test_no_cpu_fallback_without_gpu():
    """Without a HIP device the product path must refuse to run (no silent CPU fallback)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(lvo.ALOAMError):
        lvo.Context(abi.default_params(64))
    L = lvo.lib()
    assert L.aloam_create(C.byref(abi.default_params(64)), 0) is None
    assert b"device" in L.aloam_last_error(None)


def test_null_context_is_an_argument_error():
    L = lvo.lib()
    assert L.aloam_odometry(None, None) == abi.ALOAM_E_ARG
    assert L.aloam_scan_registration(None, None, 0, 0) == abi.ALOAM_E_ARG


def test_cpp_host_tool_links_against_the_abi():
    """tools/aloam_kitti (C++ host over include/aloam_hip.h only) is built and resolves the library;
    without arguments it prints its usage before touching any device."""
    exe = os.path.join(REPO, "lidar-visual-odometry_amd", "tools", "aloam_kitti")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr
    assert "libaloam_hip.so" in subprocess.check_output(["ldd", exe], text=True)


def test_lazy_result_matches_eager_conversion():
    """Pipeline.push returns LazyResult mappings: the same keys and values as odom_to_dict /
    map_to_dict, the pose keys readable before (and after) the full conversion."""
    import numpy as np
    od = abi.OdomResult()
    od.rounds = 3
    od.t_w_curr[0], od.q_w_curr[3] = 1.25, 1.0
    for i in range(3):
        od.corner_correspondence[i] = 10 + i
        od.lm[i].iterations = 4
    lz = abi.LazyResult(od, abi.odom_to_dict)
    assert np.array_equal(lz["t_w_curr"], [1.25, 0.0, 0.0])     # pose key straight from the struct
    eager = abi.odom_to_dict(od)
    assert set(lz) == set(eager) and len(lz) == len(eager)
    for k, v in eager.items():
        assert np.array_equal(np.asarray(lz[k], dtype=object), np.asarray(v, dtype=object)), k
    assert lz.get("missing") is None and "rounds" in lz
    mp = abi.MapResult()
    mp.map_total_points = 7
    lm = abi.LazyResult(mp, abi.map_to_dict)
    assert lm["map_total_points"] == 7 and np.array_equal(lm["q_w_curr"], abi.map_to_dict(mp)["q_w_curr"])
