"""The device's PCL-order sort (csrc/ls_sort.hpp + pcl_sort.hpp) compiled for the host and run under a
lane-per-fiber emulation of workgroups (tests/ps_emu.cpp): its level-synchronous partitions, per-wave
tail, global split and segment lists leave exactly libstdc++'s std::sort order. CPU test (the GPU tests
check the kernels themselves)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    exe = tmp_path_factory.mktemp("psemu") / "ps_emu"
    subprocess.check_call(["g++", "-std=c++20", "-O1", "-w", "-o", str(exe), os.path.join(HERE, "ps_emu.cpp")])
    return str(exe)


@pytest.mark.parametrize("tail", [None, 4096], ids=["default_tail", "waves_early"])
def test_ls_sort_matches_libstdcxx_under_emulation(tmp_path, tail):
    # csrc/ls_sort.hpp on 2 emulated waves (n <= 128 * 16): every introsort level of every segment at once,
    # the sparse tail per wave (LS_TAIL 4096: the waves take over as soon as <= 2 segments are active)
    exe = tmp_path / "ls_emu"
    defs = [f"-DLS_TAIL_DEF={tail}"] if tail else []
    subprocess.check_call(["g++", "-std=c++20", "-O1", "-w", *defs, "-o", str(exe), os.path.join(HERE, "ps_emu.cpp")])
    r = subprocess.run([str(exe), "120", "13", "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_ls_sort_global_matches_libstdcxx_under_emulation(emu):
    # csrc/ls_sort.hpp's global sort (n 4000-8000, split to segments <= cap, each sorted in the LDS buffer)
    r = subprocess.run([emu, "48", "17", "2"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_ls_split_list_sort_matches_libstdcxx_under_emulation(emu):
    # split into segments of <= limit (one workgroup), segments sorted by 2 workgroups: the > 64-element ones
    # staged through LDS (ls_sort), the short ones one per wave in registers
    r = subprocess.run([emu, "48", "19", "3"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


@pytest.mark.parametrize("mode", [1, 2, 3], ids=["lds", "global", "split_list"])
def test_heap_sort_fallbacks_match_libstdcxx_under_emulation(emu, mode):
    # sorted prefix + short tail (a map cube's old points + the appended stack points): median-of-3 introsort
    # exhausts its depth on much of such an array, so the heap sorts (std::__partial_sort) of the LDS levels,
    # the wave tail and the global split carry the result (a flipped tie rule in them fails these trials)
    r = subprocess.run([emu, "20", str(20 + mode), str(mode), "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


@pytest.mark.parametrize("mode,cube", [(1, 0), (3, 0), (1, 1), (3, 1)], ids=["lds", "split_list", "lds_cube", "split_list_cube"])
def test_relevance_gated_sort_orders_relevant_leaves_like_libstdcxx(emu, mode, cube):
    # csrc/rvg.hpp relevance mode: rel marks the points of >= 3-point keys; depth-exhausted segments with
    # fewer than two of them are left unsorted, the others heap-sorted by a whole wave (ws_heap_sort: make_heap
    # by depth levels, six-level pops, stop once the smallest relevant key is out). Every >= 3-point key's
    # points must still come out in std::sort's order.
    r = subprocess.run([emu, "32" if cube else "96", str(40 + 2 * mode + cube), str(mode), str(cube), "1"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_wave_heap_sort_orders_relevant_keys_like_libstdcxx(emu):
    # csrc/pcl_sort.hpp ws_heap_sort on one emulated wave vs libstdc++'s heap sort (std::partial_sort(f, l, l)):
    # random / mostly ascending / distinct-but-one-group inputs up to 1016 points; the post-order closed form
    # (no relevant point in its danger zone) and the six-level pops with the early stop must both leave every
    # >= 3-point key's points in libstdc++'s order
    r = subprocess.run([emu, "300", "53", "4"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
    assert "postorder segments 0" not in r.stdout


def test_flag_heap_pops_match_libstdcxx(emu):
    # csrc/pcl_sort.hpp fh_sort_heap_lds (the pops walked on per-node child flags: top six levels from a scalar
    # copy, deeper ones six at a time by a ballot, path values moved by their lanes) on one emulated wave, up
    # to FH_MAX = 4095 points: with every pop the whole array must equal libstdc++'s heap sort; with the
    # relevance early stop every >= 3-point key's points must be in its order
    r = subprocess.run([emu, "100", "71", "6"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


def test_batched_leaf_sums_match_the_leaf_loop(emu):
    # csrc/rvg.hpp rvg_reduce_batched (the map filter's leaf sums: chunk entries and points loaded in batches,
    # leaves summed from registers, relevant leaves in fpos order) against the leaf-at-a-time loop on one
    # emulated 128-thread workgroup: the same centroids bit for bit and the same leaf count, across chunk
    # boundaries, leaves running past a chunk, all-relevant and no-relevant inputs
    r = subprocess.run([emu, "300", "29", "5"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout


@pytest.mark.parametrize("seed", [101, 303])
def test_heap_postorder_fuzz_edges(emu, seed):
    """Fuzz aimed at ws_heap_postorder's edges (advisor item): lengths close to 1024, many duplicates, up to five
    relevant groups per segment with the largest / smallest / existing keys, members placed at the input's end
    (the danger zone after make_heap); the closed form or the pops (child flags) must leave every >= 3-point
    key's points in libstdc++'s heap-sort order, and the closed form must be taken in some trials."""
    r = subprocess.run([emu, "200", str(seed), "7"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
    assert "postorder segments 0" not in r.stdout
