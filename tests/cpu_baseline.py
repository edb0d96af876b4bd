#!/usr/bin/env python3
"""CPU baseline of bench.py: the oracle restatement of the reference path
(oracle/liboracle.so, g++ -O3 -ffp-contract=off, the reference's Release flags CMakeLists.txt:5-6)
timed on this host's cores, single-threaded per process like the reference's nodes.

Test infrastructure: run only by bench.py's cpu_baseline leg (as a child process, so nothing of the
parent's GPU state is inherited) or by hand. Forms:
  serial     one process pinned to one core runs scanRegistration -> laserOdometry -> laserMapping per
             scan: scans/s = 1 / (sum of the stages)
  pipelined  the reference's deployment: three processes, one per node (scanRegistration.cpp:461,
             laserOdometry.cpp:236, laserMapping.cpp:895), each pinned to a core of its own and connected
             by pipes carrying what the ROS topics carry (the four feature clouds; corner / surf last +
             /laser_odom_to_init); scans/s in steady state at the mapping node's output
  box        P independent sequences, one serial process per core (P = the cores this process may use,
             at most --box-max): the host's aggregate scans/s
Prints one JSON object (stdout).

  late       (--late-start S --late-frames F) one serial sequence through frames 0 .. S+F-1 (the map grows as
             in the GPU run), only the last F frames timed: the steady-state rate at a grown map, its TicToc
             stages, the 3-node rate estimated as 1 / the slowest node's mean stage time, and the whole
             trajectory (for the ATE over S+F frames)

usage: python tests/cpu_baseline.py [--frames N] [--start K] [--box-frames M] [--box-max P] [--late-start S --late-frames F]
"""
import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _pin(core):
    try:
        os.sched_setaffinity(0, {core})
    except (AttributeError, OSError):
        pass


def _frames(start, n):
    from lvo_amd_loader import synth
    return [synth.scan("hdl64", start + k) for k in range(n)]


def _oracle():
    import oracle_binding as ob
    from lvo_amd_loader import abi
    return ob.Oracle(abi.default_params(64))


def _serial(core, start, n, q):
    """One sequence through process_scan on one pinned core; frame 0 (system init) untimed."""
    _pin(core)
    import numpy as np
    fr = _frames(start, n)
    o = _oracle()
    traj, t, tt, nt = [], 0.0, None, 0
    for k, f in enumerate(fr):
        t1 = time.perf_counter()
        _, m = o.process_scan(f)
        dt = time.perf_counter() - t1
        traj.append([float(v) for v in m["t_w_curr"]])
        if k >= 1:
            t += dt
            d = o.tictoc()
            tt = {key: (tt[key] if tt else 0.0) + v for key, v in d.items()}
            nt += 1
    q.put({"core": core, "frames": n - 1, "seconds": t, "traj": traj,
           "tictoc_ms": {k: round(v / max(nt, 1), 3) for k, v in (tt or {}).items()}})
    del np


def _late(core, start, s0, nl, q):
    """Frames start .. start+s0+nl-1 serially on one pinned core; the last nl timed (steady state)."""
    _pin(core)
    o = _oracle()
    traj, t, tt, nt = [], 0.0, None, 0
    st = [0.0, 0.0, 0.0]
    for k in range(s0 + nl):
        f = _frames(start + k, 1)[0]
        t1 = time.perf_counter()
        _, m = o.process_scan(f)
        dt = time.perf_counter() - t1
        traj.append([float(v) for v in m["t_w_curr"]])
        if k >= s0:
            t += dt
            d = o.tictoc()
            tt = {key: (tt[key] if tt else 0.0) + v for key, v in d.items()}
            sm = o.stage_times()
            st = [a + b for a, b in zip(st, sm)]
            nt += 1
    q.put({"frames": [s0, s0 + nl - 1], "seconds": t, "traj": traj, "stage_ms": [v / max(nt, 1) for v in st],
           "tictoc_ms": {k: round(v / max(nt, 1), 3) for k, v in (tt or {}).items()}})


def _node_scan(core, start, n, out):
    _pin(core)
    fr = _frames(start, n)
    o = _oracle()
    for k, f in enumerate(fr):
        o.scan_registration(f)
        ft = o.features()
        out.send((k, ft["sharp"], ft["less_sharp"], ft["flat"], ft["less_flat"]))
    out.send(None)


def _node_odom(core, inp, out):
    _pin(core)
    o = _oracle()
    while True:
        msg = inp.recv()
        if msg is None:
            break
        k, sharp, less_sharp, flat, less_flat = msg
        o.set_features(sharp, less_sharp, flat, less_flat)
        od = o.odometry()
        if od["publish_to_mapping"]:
            out.send((k, less_sharp, less_flat, od["q_w_curr"], od["t_w_curr"]))
    out.send(None)


def _node_map(core, inp, q):
    _pin(core)
    o = _oracle()
    done = []
    while True:
        msg = inp.recv()
        if msg is None:
            break
        k, corner, surf, qw, tw = msg
        o.set_mapping_input(corner, surf, qw, tw)
        o.mapping()
        done.append(time.perf_counter())
    q.put(done)


def pipelined(cores, start, n, warm=3):
    ctx = mp.get_context("spawn")
    a_out, b_in = ctx.Pipe()
    b_out, c_in = ctx.Pipe()
    q = ctx.Queue()
    ps = [ctx.Process(target=_node_scan, args=(cores[0], start, n, a_out)),
          ctx.Process(target=_node_odom, args=(cores[1 % len(cores)], b_in, b_out)),
          ctx.Process(target=_node_map, args=(cores[2 % len(cores)], c_in, q))]
    for p in ps:
        p.start()
    done = q.get(timeout=600)
    for p in ps:
        p.join(timeout=60)
    w = min(warm, len(done) - 2)
    return (len(done) - 1 - w) / (done[-1] - done[w]) if len(done) > w + 1 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--start", type=int, default=0)
    ap.add_argument("--box-frames", type=int, default=6)
    ap.add_argument("--box-max", type=int, default=16, help="cores of the box form (the GPU box's CPU share is 16)")
    ap.add_argument("--late-start", type=int, default=0, help="steady-state window: first timed frame (0 = skip)")
    ap.add_argument("--late-frames", type=int, default=20)
    args = ap.parse_args()
    cores = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    late = None
    p = ctx.Process(target=_serial, args=(cores[0], args.start, args.frames, q))
    p.start()
    ser = q.get(timeout=900)
    p.join()
    pipe = pipelined(cores[:3], args.start, args.frames)
    P = max(1, min(len(cores), args.box_max))
    t0 = time.perf_counter()
    ps = [ctx.Process(target=_serial, args=(cores[i], args.start + 1000 * (i + 1), args.box_frames, q)) for i in range(P)]
    for b in ps:
        b.start()
    box = [q.get(timeout=900) for _ in range(P)]
    for b in ps:
        b.join()
    wall = time.perf_counter() - t0
    if args.late_start > 0:                       # after the other forms: no core shared with them
        ql = ctx.Queue()
        pl = ctx.Process(target=_late, args=(cores[0], args.start, args.late_start, args.late_frames, ql))
        pl.start()
        late = ql.get(timeout=1800)
        pl.join()
    box_rate = sum(r["frames"] for r in box) / max(max(r["seconds"] for r in box), 1e-9)
    out = {
        "host": {"cpu_model": model, "nproc": os.cpu_count(), "cores_usable": len(cores), "cores_used": cores[:max(3, P)]},
        "build": "oracle/liboracle.so: g++ -O3 -ffp-contract=off -std=c++17, no -march (reference CMakeLists.txt:5-6)",
        "serial": {"scans_per_s": ser["frames"] / ser["seconds"], "cores": 1, "frames": ser["frames"],
                   "tictoc_ms": ser["tictoc_ms"]},
        "pipelined": {"scans_per_s": pipe, "cores": 3, "frames": args.frames},
        "box": {"scans_per_s": box_rate, "cores": P, "frames_per_sequence": args.box_frames - 1, "wall_s": round(wall, 2)},
        "traj": ser["traj"],
    }
    if late is not None:
        sm = late["stage_ms"]
        out["late"] = {"frames": late["frames"], "serial_scans_per_s": (late["frames"][1] - late["frames"][0] + 1) / late["seconds"],
                       "stage_ms": {"scan_registration": sm[0], "odometry": sm[1], "mapping": sm[2]},
                       "pipelined_est_scans_per_s": 1000.0 / max(sm) if max(sm) > 0 else None,
                       "tictoc_ms": late["tictoc_ms"], "traj": late["traj"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
