"""Benchmark of the stereo hot path (BASELINE.json metric) on 1..N MI355X GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one pass of the hot path over one batch of synthetic rectified pairs already resident
in HBM: StereoSGBM::compute (prefilter, BT cost, block sum, path aggregation, WTA/uniqueness/
subpixel, LR check, median 3x3, speckle filter) + convertTo(1/16) + reprojectImageTo3D.
Frames shard across ranks (rank r owns its own frame stream); with N > 1 each step's int16
disparity is gathered to rank 0 over RCCL (the north star's frame-shard + gather).  Rank 0
prints one JSON line.  value = all ranks' pixels / max-over-ranks wall time.

`--gpus N` with N > 1 and no launcher environment (WORLD_SIZE unset) starts the N ranks itself:
this process never touches HIP, runs `torch.distributed.run --nproc-per-node N` on this same
script as a child, relays rank 0's JSON line and exits with the child's status.  Under a
launcher, WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "stereo Mpix/s (disparity+reproject) at 1280×720 d=128, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
CLOCK_GHZ = 2.4  # MI355X_MICROARCH.md chip table: max clock (the latency floors' cycles -> time)

# name -> (description, W, H, SGBM args (create order), batch, reproject handleMissing, kind)
#   kind "sgbm":  rectified gray pairs -> compute + /16 + reprojectImageTo3D (pcd_write.cpp:111-116)
#   kind "live":  ZED2 side-by-side BGR -> rectify -> StereoDisparity::computeDisparity (gray,
#                 INTER_AREA 0.5x, left + right 3WAY, WLS, /16) -> computeDepth
#                 (stereo_displayer.cpp:155-162, the reference app's per-frame loop)
#   kind "cloud": side-by-side BGR -> gray -> compute -> reproject(handleMissing) ->
#                 convertCVMatToPCL(left) -> VoxelGrid(5 mm)   (pcd_write.cpp:81-130)
# frames in flight a config defaults to (--streams), from round-5 sweeps on one MI355X
# (profiles/r5_streams_sweep.md): C2 is flat from 2 to 6 (1737-1772 fps); the class path's frame
# (C4: ~30 short launches, the sequential FGS passes a few hundred workgroups each) fills the chip
# only with more frames beside it, 2367 fps at 3 and 3592-3651 at 6
# frames in flight per config: C4's short launches fill the chip only with several frames beside
# each other (profiles/r5_streams_sweep.md); C2 is flat from 2 to 6 in flight, and with RCCL's own
# stream beside them 3 streams lost ~4.6 % of the rate against 1.4-1.8 % at 2
# (profiles/r6_streams_c2/: the RCCL world-1 line against the plain one, two rounds on one box)
STREAMS_DEFAULT = {"c4": 6, "c2": 2}

CONFIGS = {
    "c2": ("C2 (BASELINE configs[1]): 1280x720 d=128 MODE_SGBM 5-path + reprojectImageTo3D(Q, "
           "handleMissing), batch 1", 1280, 720, (0, 128, 5, 600, 2400, 1, 63, 12, 200, 2, 0), 1, True, "sgbm"),
    "c3": ("C3 (configs[2]): 1280x720 d=256 MODE_HH 8-path + reproject, batch 32", 1280, 720,
           (0, 256, 5, 600, 2400, 1, 63, 12, 200, 2, 1), 32, True, "sgbm"),
    "c4": ("C4 (configs[3]): ZED2 2560x720 side-by-side BGR stream -> rectify (config/stereo.yaml maps, "
           "remap INTER_LINEAR) -> StereoDisparity::computeDisparity (BGR2GRAY, INTER_AREA 0.5x, 3WAY d=80 "
           "left + right matcher, WLS lambda 8000 sigma 1.1, /16) -> computeDepth; frame shard per GPU + "
           "RCCL gather of the filtered disparity", 1280, 720, (0, 80, 5, 600, 2400, 1, 63, 12, 200, 2, 2), 1,
           False, "live"),
    "c5": ("C5 (configs[4]): 3840x1080 side-by-side BGR (2x1920x1080) -> BGR2GRAY -> MODE_HH 8-path d=256 -> "
           "reprojectImageTo3D(handleMissing) -> convertCVMatToPCL(left) -> VoxelGrid(5 mm); 8 frames per GPU "
           "per step (64 across 8 GPUs)", 1920, 1080, (0, 256, 5, 600, 2400, 1, 63, 12, 200, 2, 1), 8, True,
           "cloud"),
    "c0": ("C0 reference-exact matcher: 640x360 d=80 MODE_SGBM_3WAY (stereo_disparity.cpp:5-9) + reproject",
           640, 360, (0, 80, 5, 600, 2400, 1, 63, 12, 200, 2, 2), 1, False, "sgbm"),
    "pcd": ("pcd_write.cpp:102-116: 1280x720 d=80 MODE_SGBM_3WAY + reproject(handleMissing)", 1280, 720,
            (0, 80, 5, 600, 2400, 1, 63, 12, 200, 2, 2), 1, True, "sgbm"),
}
MODE_NAMES = {0: "MODE_SGBM", 1: "MODE_HH", 2: "MODE_SGBM_3WAY"}
NPATHS = {0: 5, 1: 8, 2: 3}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu():
    """(lscpu-style model name, logical CPUs this process may run on)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return model, n


def cpu_baseline(cfg, seconds_target=15.0):
    """The oracle (C restatement of the reference's OpenCV/ximgproc/PCL path) timed on host cores
    on a bounded sample of the same workload, two ways:
      throughput -- one frame per thread, `threads` frames at a time (ctypes releases the GIL);
      latency    -- one thread, one frame at a time (OpenCV's SGBM/HH run single-threaded).
    threads = this GPU's share of the host: nproc / 8 (one of the node's 8 GPUs; nproc shows the
    whole machine on the GPU box), capped by OMP_NUM_THREADS when the driver's policy sets it
    lower (the box sets 16 against nproc / 8 = 32); `host.policy` says which applies."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    from stereo_depth_ruler_amd import synthetic as S

    # the restatement built -O3 -march=native, compiled here on the host that times it
    try:
        build_flags = O.select_build("native")
        O.lib()
    except Exception as e:  # no compiler on this host: the shipped portable build
        build_flags = O.select_build("portable") + f" (native build failed: {type(e).__name__})"
    _, W, H, args, _, hm, kind = cfg
    model, ncpu = host_cpu()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    gpu_share = max(1, ncpu // 8)
    if omp > 0 and omp < gpu_share:
        threads, policy = omp, f"OMP_NUM_THREADS={omp} (driver policy) is below nproc/8={gpu_share}: {omp} threads"
    else:
        threads, policy = gpu_share, f"nproc/8 = {gpu_share} threads (one of the node's 8 GPUs' share of the host)"
    p = O.make_params(*args)
    if kind == "sgbm":
        L, R, _ = S.make_pair(H, W, args[1], seed=12345)

        def one(_):
            d = O.sgbm_compute(L, R, p)
            O.reproject(O.disp_to_float(d), S.REFERENCE_Q, hm)
            return 1
        what = (f"{MODE_NAMES[args[10]]} d={args[1]} full compute (median+speckle) + reproject on {W}x{H} "
                f"rectified gray pairs")
    elif kind == "live":
        from stereo_depth_ruler_amd.config import StereoConfiguration

        cfgf = StereoConfiguration()
        cfgf.loadFromFile(os.path.join(ROOT, "tests", "golden", "stereo.yaml"))
        maps = [O.init_undistort_rectify_map(K, Dd, Rr, P, W, H) for K, Dd, Rr, P in (
            (cfgf.cameraMatrixLeft, cfgf.distCoeffsLeft, cfgf.R1, cfgf.P1),
            (cfgf.cameraMatrixRight, cfgf.distCoeffsRight, cfgf.R2, cfgf.P2))]
        frame = S.sbs_bgr_color_frame(H, W, 80, seed=12345)
        pl = O.make_params(0, 80, 5, 600, 2400, 1000000, 63, 0, 0, 2, 2)
        pr = O.make_params(-79, 80, 5, 600, 2400, 1000000, 63, 0, 0, 2, 2)
        q = O.wls_params_for_sgbm(0, 80, 5, W // 2, H // 2, 8000.0, 1.1)

        def one(_):
            gl = O.resize_area_half(O.bgr2gray(O.remap_bilinear(frame[:, :W], *maps[0])))
            gr = O.resize_area_half(O.bgr2gray(O.remap_bilinear(frame[:, W:], *maps[1])))
            dl, dr = O.sgbm_compute(gl, gr, pl), O.sgbm_compute(gr, gl, pr)
            f = O.disp_to_float(O.wls_filter(dl, dr, gl, q))
            O.reproject(f, cfgf.Q, False)
            return 1
        what = ("live-loop frames (remap x2, gray, INTER_AREA, 3WAY d=80 left + right, WLS, /16, reproject) "
                f"from {2 * W}x{H} side-by-side BGR")
    else:
        frame = S.sbs_bgr_color_frame(H, W, args[1], seed=12345)

        def one(_):
            gl, gr = O.bgr2gray(frame[:, :W]), O.bgr2gray(frame[:, W:])
            d = O.sgbm_compute(gl, gr, p)
            xyz = O.reproject(O.disp_to_float(d), S.REFERENCE_Q, hm)
            O.voxel_grid(O.xyz_to_cloud(xyz, frame[:, :W]), 0.005)
            return 1
        what = (f"pcd_write frames (gray, {MODE_NAMES[args[10]]} d={args[1]}, reproject, cloud, VoxelGrid) from "
                f"{2 * W}x{H} side-by-side BGR")
    lat = []
    for _ in range(3):  # latency: one thread, one frame
        t = time.perf_counter()
        one(0)
        lat.append(time.perf_counter() - t)
    lat_s = float(np.median(lat))
    frames = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t0 < seconds_target:
            frames += sum(ex.map(one, range(threads)))
    el = time.perf_counter() - t0
    return {
        "value": round(frames * W * H / el / 1e6, 4),
        "unit": "Mpix/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{frames} {what}, {threads} threads x 1 frame each, {el:.1f} s wall; oracle/*.c "
                  f"(a scalar C restatement of OpenCV 4.6 / ximgproc / PCL, not OpenCV itself, which is "
                  f"absent on this image)",
        "latency": {"ms_per_frame": round(lat_s * 1e3, 2), "value": round(W * H / lat_s / 1e6, 4),
                    "unit": "Mpix/s", "threads": 1, "frames": len(lat)},
        "host": {"cpu_model": model, "nproc": ncpu, "threads_used": threads,
                 "omp_num_threads": omp or None, "policy": policy},
        "build": build_flags,
    }


def load_traffic(kernel_tag):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel_tag, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def stream_probe(dev, mib=2048, iters=20):
    """This box's streaming rates (sdr_stream_probe_ex over 2 GiB buffers, far beyond the 256 MiB
    Infinity Cache): the fastest copy (read + write bytes), read-only and write-only.  A path kernel
    reads and writes in about equal parts, so `gbs` (the copy) is its yardstick; box-to-box spread
    shows up here and in `achieved` alike (profiles/r6_copy_rate.txt: 85 copy shapes on one box,
    5.0-5.8 TB/s; reads 6.3-6.4)."""
    import ctypes

    from stereo_depth_ruler_amd._lib import check, lib

    g = (ctypes.c_double * 3)()
    check(lib().sdr_stream_probe_ex(dev.index, mib << 20, iters, g))
    return {"gbs": round(g[0], 1), "read_gbs": round(g[1], 1), "write_gbs": round(g[2], 1),
            "what": f"sdr_stream_probe_ex: the fastest of 16 copy shapes (4 or 8 16-B loads in flight per "
                    f"thread, plain or non-temporal stores, 2/4/8/16 workgroups a CU), {iters} copies of "
                    f"{mib} MiB each, read + write bytes; read-only and write-only beside"}


def free_port() -> int:
    """A free TCP port on 127.0.0.1 for the ranks' rendezvous."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(nproc: int, port: int, argv) -> list:
    """torch.distributed.run over this script with the same arguments (one rank per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def relay(cmd, nproc: int, env=None) -> int:
    """Runs the launcher as a child, passes its output through (stdout line by line, so the
    driver's progress watch sees it), checks that exactly one JSON line came back and that it
    reports nproc GPUs, and returns the exit status (the child's, or 3 for a bad line)."""
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1, env=env)
    lines = []
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
        s = line.strip()
        if s.startswith("{") and s.endswith("}"):
            try:
                lines.append(json.loads(s))
            except ValueError:
                pass
    rc = p.wait()
    if rc != 0:
        log(f"bench: launcher exited with status {rc}")
        return rc
    if len(lines) != 1 or lines[0].get("n_gpus") != nproc:
        log(f"bench: expected one JSON line with n_gpus={nproc}, got {[ln.get('n_gpus') for ln in lines]}")
        return 3
    return 0


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=8, help="distinct resident frames per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-kernel HIP-event segment after the timed region (no roofline)")
    ap.add_argument("--in-flight-timing", action="store_true",
                    help="also put HIP events around matcher 0's launches inside the timed region "
                         "(roofline.in_flight; the events cost ~2 %% of the frame rate)")
    ap.add_argument("--streams", type=int, default=None,
                    help="frames in flight (one matcher + stream each); default per config (STREAMS_DEFAULT)")
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per step instead of the config's (experiments; the workload string says so)")
    ap.add_argument("--iso-steps", type=int, default=30, help="single-stream steps for roofline.isolated")
    ap.add_argument("--stream-probe", action=argparse.BooleanOptionalAction, default=True,
                    help="time a 2 GiB device copy after the run (roofline.stream_probe: this box's "
                         "streaming rate beside the dominant kernel's)")
    ap.add_argument("--hbm-only", action=argparse.BooleanOptionalAction, default=True,
                    help="C2: also time k_paths over a 4-frame batch whose cost volume exceeds the "
                         "Infinity Cache (roofline.hbm_only)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL over xGMI) for real runs; gloo rehearses the N>1 path with every "
                         "rank on the one GPU of a 1-GPU box (gather staged through host memory)")
    ap.add_argument("--dist-world1", action="store_true",
                    help="run the distributed path (process group, gathers, gather_check) at world size 1 "
                         "under torch.distributed.run --nproc-per-node 1 (RCCL on a one-GPU box)")
    ap.add_argument("--status-every", type=int, default=16,
                    help="N>1: ranks exchange their step status (host-side, gloo) every this many steps "
                         "and after the last; a failed rank keeps joining the gathers with zeros until "
                         "then, and every rank exits non-zero (RankFailure) instead of blocking")
    ap.add_argument("--gather-every", type=int, default=8,
                    help="N>1 (and --dist-world1): the gather to rank 0 collects this many steps' "
                         "disparities in one collective (every frame is gathered)")
    ap.add_argument("--inject-failure", default=None, metavar="RANK:STEP",
                    help="test hook: rank RANK's step STEP raises SDR_ERR_ARG (failure-path tests)")
    a = ap.parse_args(argv)
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    return a


def main():
    a = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        # no launcher: start the N ranks from here, before anything initialises HIP (this process
        # imports no torch; the ranks are fresh child processes)
        sys.exit(relay(launcher_cmd(a.gpus, free_port(), sys.argv[1:]), a.gpus,
                       env=dict(os.environ, SDR_BENCH_SELF_LAUNCHED="1")))
    world = int(env_world or "1")
    # --dist-world1: the distributed data path (RCCL process group, status exchanges, the gather to
    # rank 0 and its check) at world size 1, under torch.distributed.run --nproc-per-node 1, so the
    # path the 8-GPU run takes executes on a one-GPU box too
    dist_on = world > 1 or a.dist_world1
    if a.dist_world1 and env_world is None:
        raise SystemExit("bench: --dist-world1 runs under a launcher (torch.distributed.run --nproc-per-node 1)")
    if world != a.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {a.gpus}: the launcher and the "
                         f"arguments disagree on the number of ranks")

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gloo = a.dist_backend == "gloo"
    from stereo_depth_ruler_amd.distributed import check_ranks, error_code, init_process_group

    if dist_on:
        # every collective bounded by SDR_DIST_TIMEOUT (default 120 s): a rank that dies outright
        # cannot leave the others blocked (stereo_depth_ruler_amd/distributed.py)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        ndev = torch.cuda.device_count()
        if gloo:
            local = local % ndev
            torch.cuda.set_device(local)
            init_process_group("gloo")
        else:
            if ndev < world:
                raise SystemExit(f"bench: {world} ranks over RCCL need {world} GPUs, this node shows {ndev} "
                                 f"(--dist-backend gloo rehearses the N>1 path on fewer)")
            torch.cuda.set_device(local)
            init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != a.gpus:
            raise SystemExit(f"bench: the process group has {dist.get_world_size()} ranks, --gpus {a.gpus}")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    if os.environ.get("SDR_BENCH_LIB"):
        # experiment A/B only: time another build of the engine (scripts/; never the driver's run)
        from stereo_depth_ruler_amd import _lib as _l
        _l.use_library(os.environ["SDR_BENCH_LIB"])
    import stereo_depth_ruler_amd as sdr
    from stereo_depth_ruler_amd import synthetic as S
    from stereo_depth_ruler_amd.distributed import as_bytes
    from stereo_depth_ruler_amd import sgbm as _sg
    KERNEL_KINDS = {"prefilter": _sg.KERNEL_PREFILTER, "k_cost": _sg.KERNEL_COST, "k_paths": _sg.KERNEL_PATHS,
                    "k_south_wta": _sg.KERNEL_WTA_LR, "k_lr_check": _sg.KERNEL_LR_CHECK,
                    "median": _sg.KERNEL_MEDIAN, "speckle": _sg.KERNEL_SPECKLE,
                    "reproject": _sg.KERNEL_REPROJECT, "k_sweep": _sg.KERNEL_SWEEP,
                    "k_sweep_down": _sg.KERNEL_SWEEP_DOWN,
                    "k_wls_prep": _sg.KERNEL_WLS_PREP, "fgs_coef": _sg.KERNEL_FGS_COEF,
                    "fgs_pass": _sg.KERNEL_FGS, "k_wls_final": _sg.KERNEL_WLS_FINAL}

    desc, W, H, args, batch, hm, kind = CONFIGS[a.config]
    if a.batch is not None:
        # (an experiment knob: the BASELINE configs' lines use their own batch)
        if a.batch < 1:
            raise SystemExit("bench: --batch must be >= 1")
        batch = a.batch
        desc = f"{desc} [--batch {batch}: not the config's own batch]"
    D, mode = args[1], args[10]
    nf = max(a.frames, batch)
    ns = max(1, a.streams if a.streams is not None else STREAMS_DEFAULT.get(a.config, 3))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(ns - 1)]
    gather_bytes = batch * H * W * 2  # int16 disparity per step
    if kind == "sgbm":
        Ls, Rs = S.make_batch(nf, H, W, D, seed0=1000 * rank)
        Ld = torch.from_numpy(Ls).to(dev)
        Rd = torch.from_numpy(Rs).to(dev)
        # S in-flight frames: one matcher (own scratch) and one HIP stream per slot, frames issued
        # round-robin, so one frame's compute-bound stages (cost volume, speckle CCL) overlap the
        # next frame's bandwidth-bound ones (path aggregation, WTA) and the E/W chain tail
        ms = [sdr.StereoSGBM.create(*args, device=dev.index) for _ in range(ns)]
        disp = [torch.empty((batch, H, W), dtype=torch.int16, device=dev) for _ in range(2 * ns)]
        xyz = [torch.empty((batch, H, W, 3), dtype=torch.float32, device=dev) for _ in range(ns)]
        closers = ms

        def run(j, k, slot, out=None):
            d = disp[slot] if out is None else out
            ms[k].compute_reproject(Ld[j:j + batch], Rd[j:j + batch], S.REFERENCE_Q, hm, disp=d, xyz=xyz[k])
            return d
    else:
        from stereo_depth_ruler_amd.config import StereoConfiguration
        from stereo_depth_ruler_amd.pipeline import CloudEmit, LiveLoop
        from stereo_depth_ruler_amd.rectify import StereoRectifier

        sbs = torch.empty((nf, H, 2 * W, 3), dtype=torch.uint8, device=dev)
        for i in range(nf):
            sbs[i].copy_(torch.from_numpy(S.sbs_bgr_color_frame(H, W, D if kind == "cloud" else 80,
                                                                seed=1000 * rank + i)))
        if kind == "live":
            cfg = StereoConfiguration()
            assert cfg.loadFromFile(os.path.join(ROOT, "tests", "golden", "stereo.yaml"))
            rect = StereoRectifier(cfg, device=dev.index)
            pipes = [LiveLoop(rect, cfg.Q, batch, device=dev.index, args=args) for _ in range(ns)]
            gather_bytes = batch * (H // 2) * (W // 2) * 2
        else:
            pipes = [CloudEmit(W, H, args, batch, S.REFERENCE_Q, device=dev.index) for _ in range(ns)]
        ms = [p.matcher() for p in pipes]
        closers = pipes

        def run(j, k, slot, ingest_events=None):
            if kind == "live":
                return pipes[k].enqueue(sbs[j:j + batch], streams[k], ingest_events=ingest_events)
            if ns == 1:
                return pipes[k].enqueue(sbs[j:j + batch], streams[k])
            d = pipes[k].enqueue(sbs[j:j + batch], streams[k], voxel=False)
            flush_voxel()
            pending["k"] = k
            return d
    m = ms[0]
    # the cloud pipeline's voxel grids synchronise their stream (the counts are host values): with
    # several streams, a step's voxel stage runs after the NEXT step's frames are enqueued on the
    # next stream, so the GPU has that work while the host waits (every frame's voxel grid still
    # runs, inside the timed region: flush_voxel after the loop)
    pending = {"k": None}

    def flush_voxel():
        if pending["k"] is not None:
            pipes[pending["k"]].voxel(streams[pending["k"]])
            pending["k"] = None

    # the gather to rank 0, batched per stream: the frames a stream computes land
    # in a set of G slots (the compute writes MODE_SGBM's disparity straight into its slot), and one
    # collective per G of that stream's steps gathers the set from every rank, issued on that same
    # stream (no cross-stream events: every event record is a barrier packet in the queue); two sets
    # per stream alternate, a set written again only after the stream has waited for its gather.
    # A gather per step (and its event records) cost ~45 us of every 0.56 ms C2 step at world size 1
    # (VERDICT r5 item 5).  Every frame is gathered.
    G = max(1, a.gather_every)
    gset = gbufs = None
    if dist_on:
        gset = [[torch.empty((G, gather_bytes), dtype=torch.uint8, device=dev) for _ in range(2)] for _ in range(ns)]
        if rank == 0:  # RCCL has no int16: the disparity bytes
            gbufs = [[[torch.empty(G * gather_bytes, dtype=torch.uint8, device="cpu" if gloo else dev)
                       for _ in range(world)] for _ in range(2)] for _ in range(ns)]
    works = [[None, None] for _ in range(ns)]
    failure = {"code": 0, "err": None}  # this rank's first failed step (reported at the next check)
    inject = tuple(int(v) for v in a.inject_failure.split(":")) if a.inject_failure else None
    from stereo_depth_ruler_amd._lib import SDRError

    def slot_of(i):
        """(stream, set, slot) of step i: stream i mod ns; the stream's m-th step, m = i // ns."""
        m = i // ns
        return i % ns, (m // G) % 2, m % G

    def step(i, last=False):
        j = (i * batch) % (nf - batch + 1) if nf > batch else 0
        k, sidx, q = slot_of(i)
        slot = i % (2 * ns)
        with torch.cuda.stream(streams[k]):
            if dist_on and q == 0 and works[k][sidx] is not None:
                works[k][sidx].wait()  # this stream waits until the set's last gather has read it
                works[k][sidx] = None
            out = gset[k][sidx][q].view(torch.int16).view(batch, H, W) if dist_on and kind == "sgbm" else None
            try:
                if inject is not None and inject == (rank, i):
                    raise SDRError(-1, f"injected failure at rank {rank} step {i}")
                res = run(j, k, slot) if out is None else run(j, k, slot, out=out)
            except Exception as e:  # noqa: BLE001 -- any failed step is reported to every rank
                if not dist_on:
                    raise
                if failure["err"] is None:
                    failure["code"], failure["err"] = error_code(e), e
                    log(f"rank {rank}: step {i} failed ({e!r}); reporting at the next status check")
                gset[k][sidx][q].zero_()
                res = None
            if dist_on and ((i + 1) % max(1, a.status_every) == 0):
                check_ranks(failure["code"])  # RankFailure on every rank if any step failed
            if dist_on:
                if res is not None and out is None:
                    b = as_bytes(res) if res.dtype != torch.uint8 else res
                    gset[k][sidx][q].copy_(b.reshape(-1))
                if q == G - 1 or last:
                    src = gset[k][sidx].reshape(-1)
                    if gloo:
                        src = src.cpu()  # gloo gathers host tensors (synchronises this stream)
                    works[k][sidx] = dist.gather(src, gbufs[k][sidx] if rank == 0 else None, dst=0,
                                                 async_op=True)

    def drain():
        for k in range(ns):
            for sidx in range(2):
                if works[k][sidx] is not None:
                    works[k][sidx].wait()
                works[k][sidx] = None

    def last_of(i, end):
        """Step i is its stream's last before `end`: its set is gathered even if not full."""
        return i + ns >= end

    for i in range(a.warmup):
        step(i, last=last_of(i, a.warmup))
    flush_voxel()
    drain()
    if dist_on:
        check_ranks(failure["code"])
    torch.cuda.synchronize()
    if not a.no_kernel_timing and a.in_flight_timing:
        m.enable_timing(2)
        m.kernel_time(-1, reset=True)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(a.warmup + i, last=last_of(a.warmup + i, a.warmup + a.steps))
    flush_voxel()  # the last step's voxel grids, inside the timed region
    host_el = time.perf_counter() - t0  # the host's enqueue time (the GPU may still be running)
    drain()
    torch.cuda.synchronize()
    # a batched MODE_HH step whose row sweep gave up waiting wrote INVALID frames and reports it
    # here (sdr_sgbm_last_status): such a run has no valid number.  Every rank checks its own
    # matchers before the last status exchange, so a rank that finds one fails every rank there
    # instead of leaving the others in the collectives below
    for mm in ms:
        try:
            mm.check_status()
        except SDRError as e:
            if not dist_on:
                raise
            if failure["err"] is None:
                failure["code"], failure["err"] = error_code(e), e
                log(f"rank {rank}: {e!r}")
    if dist_on:
        check_ranks(failure["code"])
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ranks = None
    if dist_on:
        # every rank's own wall time (host-side exchange), then the max over ranks
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"rank": rank, "device": dev.index, "host": socket.gethostname(),
                                          "ms_per_step": round(el / a.steps * 1e3, 4), "_s": el})
        el = max(r.pop("_s") for r in per_rank)
        ranks = {"backend": "gloo" if gloo else "nccl (RCCL)", "world_size_seen": dist.get_world_size(),
                 "launcher": ("bench.py --gpus (torch.distributed.run child)"
                              if os.environ.get("SDR_BENCH_SELF_LAUNCHED") else "external"),
                 "per_rank": per_rank}
    gather_check = None
    if dist_on:
        # end-to-end check of the data path (after the timed region): rank 0's copy of every rank's
        # bytes from the last timed step equals what that rank sent (position-weighted checksums)
        def cks(b):
            b = b.reshape(-1).to(torch.int64)
            return int((b * (torch.arange(b.numel(), device=b.device) % 251 + 1)).sum())

        li = a.warmup + a.steps - 1
        lk, ls, lq = slot_of(li)
        sums = [None] * world
        dist.all_gather_object(sums, cks(gset[lk][ls][lq]))
        if rank == 0:
            got = [gbufs[lk][ls][r][lq * gather_bytes:(lq + 1) * gather_bytes] for r in range(world)]
            gather_check = {"step": li, "ranks": world, "gather_every": G,
                            "ok": all(cks(got[r]) == sums[r] for r in range(world))}

    Wm, Hm = (W // 2, H // 2) if kind == "live" else (W, H)  # the left matcher's frame
    w1 = Wm - max(args[0] + D, 0) + min(args[0], 0)
    # the class path (live) runs the left and the right matcher as one paired batch through the
    # same launches (stereo_disparity.cpp:27-28); the right one (minD = -(minD + D) + 1) matches
    # the same W1 columns
    nmatch = 2 if kind == "live" else 1
    cells = nmatch * batch * Hm * w1 * D
    P = NPATHS[mode]

    def kernel_report(mm, extra=None, step_us=None, steps=1):
        """Per-kernel HIP-event times of matcher mm since its last reset -> (kernels, roofline).
        extra: {name: (total_ms, launches)} of launches timed outside the handle (the ingest).
        step_us: the single-stream step time of the same launches with no events (None: no
        correction).  An event pair around a launch also spans its dispatch (~2 us a launch on
        MI355X), so the events' sum exceeds the step; the excess per launch is subtracted from
        every kernel's average (`avg_us`; the raw figure is `avg_us_events`), which puts the
        per-kernel table in line with rocprofv3's kernel durations and its sum at or below the
        step.  steps: the steps the events cover (per-step times)."""
        per_kind = {name: mm.kernel_time(kind, reset=False) for name, kind in KERNEL_KINDS.items()}
        all_ms, _ = mm.kernel_time(-1, reset=True)
        for name, v in (extra or {}).items():
            per_kind[name] = v
            all_ms += v[0]
        launches = sum(c for _, c in per_kind.values())
        ovh_us = 0.0
        if step_us is not None and launches:
            ovh_us = max(0.0, (all_ms * 1e3 - step_us * steps) / launches)
        corr = {name: (ms - c * ovh_us / 1e3, c) for name, (ms, c) in per_kind.items()}
        all_corr = sum(ms for ms, c in corr.values() if c)
        kern = {name: {"avg_us": round(ms / c * 1e3, 2), "avg_us_events": round(per_kind[name][0] / c * 1e3, 2),
                       "launches": c, "share": round(ms / all_corr, 4) if all_corr else None}
                for name, (ms, c) in corr.items() if c}
        if not per_kind["k_paths"][1]:
            return kern, None
        fgs = fgs_model(per_kind, corr, all_corr, steps) if kind == "live" else None
        # algorithmic bytes per launch of the path kernels (2 B per int16 cell):
        #   k_paths: each of its directions reads C and writes its own record;
        #   k_sweep (batched MODE_HH, up: N, NE, NW) and k_sweep_down (SE, SW): one pass reads C
        #     once and writes one record for its directions, so k_paths keeps E and W only;
        #   k_south_wta: reads C and the other directions' records (top-to-bottom fused)
        sweep = per_kind["k_sweep"][1] > 0
        kp_dirs = 2 if sweep else P - 1
        nrec = 3 if sweep else P - 1
        models = {
            "k_paths": (cells * 4 * kp_dirs, f"4*{kp_dirs}*cells: {kp_dirs} directions "
                        f"({'E, W; the others in k_sweep16' if sweep else 'all but top-to-bottom'}), "
                        f"C read + record write each"),
            "k_sweep": (cells * 4, "4*cells: one C read + one record write (up pass: N, NE, NW; halo re-reads "
                        "excluded)"),
            "k_sweep_down": (cells * 8, "8*cells: C + the E, W, up records read (down pass: S, SE, SW and the "
                             "WTA; halo re-reads excluded)"),
            "k_south_wta": (cells * 2 * (1 + nrec), f"2*(1+{nrec})*cells: C + {nrec} records read"),
        }
        # the dominant kernel: the largest per-step time of ONE kernel (each kind is one kernel)
        name = max((n for n in models if per_kind[n][1]), key=lambda n: corr[n][0])
        tot_ms, cnt = corr[name]
        bytes_per_launch, model = models[name]
        # the primary figure is the raw event-timed duration (the per-launch event
        # overhead is not uniform across kernels, so the corrected time is kept as an estimate)
        avg_s = per_kind[name][0] / cnt / 1e3
        achieved = bytes_per_launch / avg_s / 1e9
        avg_s_corr = tot_ms / cnt / 1e3
        label = {
            "k_paths": f"k_paths<DPL={2 if D <= 128 else 4}> or k_paths_tc (two chains per wave, the engine's pick "
                       f"for latency-bound launches) ({kp_dirs} of the {P} path directions of a batch in "
                       f"one launch; the top-to-bottom one is fused into k_south_wta)",
            "k_sweep": "k_sweep16 up pass (row-synchronous N, NE, NW of batched MODE_HH)",
            "k_sweep_down": "k_sweep16 down pass (row-synchronous S, SE, SW of batched MODE_HH + the WTA)",
            "k_south_wta": f"k_south_wta (top-to-bottom path fused with the WTA, reading {nrec} records)",
        }[name]
        roof = {
            "bound": "hbm",
            "kernel": label,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": load_traffic(f"{a.config}:{name}") or load_traffic(f"{a.config}:{name}_tc"),
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "bytes_model": f"{model}; cells={'2 matchers*' if nmatch == 2 else ''}batch*H*W1*D={cells}",
            "avg_launch_us": round(avg_s * 1e6, 2),
            "avg_launch_us_overhead_corrected": round(avg_s_corr * 1e6, 2),
            "achieved_overhead_corrected": round(bytes_per_launch / avg_s_corr / 1e9, 1),
            "event_overhead_us_per_launch": round(ovh_us, 2),
            "launches_timed": cnt,
            "kernel_share_of_gpu_time": round(tot_ms / all_corr, 4) if all_corr else None,
        }
        # the other path kernels at their own rates (each against its own byte model)
        roof["path_kernels"] = {
            n: {"avg_us": round(corr[n][0] / corr[n][1] * 1e3, 2),
                "achieved": round(models[n][0] / (corr[n][0] / corr[n][1] / 1e3) / 1e9, 1),
                "frac": round(models[n][0] / (corr[n][0] / corr[n][1] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
            for n in models if per_kind[n][1]}
        # whole pipeline: cost write + the path kernels' data flow above, over the summed kernel
        # time of one step
        # (batched MODE_HH: cost 2 + E/W 8 + up 4 + down with the WTA 8 = 22 B a cell)
        pipe_bytes = cells * (2 + 4 * kp_dirs + (4 + 8 if sweep else 2 * (1 + nrec)))
        gpu_s = all_corr / 1e3 / max(1, steps)
        roof["pipeline"] = {
            "algorithmic_bytes_per_step": pipe_bytes,
            "kernel_time_per_step_us": round(gpu_s * 1e6, 1),
            "single_stream_step_us": round(step_us, 1) if step_us is not None else None,
            "achieved": round(pipe_bytes / gpu_s / 1e9, 1),
            "frac": round(pipe_bytes / gpu_s / 1e9 / HBM_PEAK_GBS, 4),
        }
        if fgs is not None and fgs["share_of_gpu_time"] > roof["kernel_share_of_gpu_time"]:
            # the class path's frame: the sequential FGS passes, not a path kernel, take the most
            # time; the line names them with their latency model, the HBM-bound path kernel beside
            fgs["hbm_path_kernel"] = roof
            roof = fgs
        return kern, roof

    def fgs_model(per_kind, corr, all_corr, steps):
        """The class path's sequential FGS passes (SDR_FGS_THOMAS: ximgproc's order) as a
        latency-bound kernel: k_fgs_lr (round 6, lines resident in LDS, one solver wave per
        right-hand side) or k_fgs_th.  A pass solves every line of the WLS ROI (rows: rh lines of
        rw samples, columns: rw lines of rh): each line is a chain of rw (or rh) forward steps then
        as many back steps, each step a dependent sequence of f32 ops -- 5 forward (a*p, x - a*p,
        q0 = x/den by the reciprocal, the Markstein remainder fma, the correction fma), 2 back
        (t*q, x - t*q) -- at 4.9 cycles a dependent op on one wave (profiles/r5_probe_fgs_step.txt,
        v_fma_f32 chain).  floor = the chain's dependent-op cycles at the peak clock; frac = floor /
        measured pass time."""
        tot, cnt = per_kind["fgs_pass"]
        if not cnt:
            return None
        roi = pipes[0].wls.getROI(Wm, Hm)
        rw, rh = roi[2], roi[3]
        # the passes alternate rows and columns (3 iterations: 3 + 3 per frame)
        chain = (rw + rh) / 2.0
        cyc_op, fwd_ops, back_ops = 4.9, 5, 2
        floor_us = chain * (fwd_ops + back_ops) * cyc_op / (CLOCK_GHZ * 1e3)
        avg_us = tot / cnt * 1e3
        samples = nmatch // 2 * batch * rw * rh  # line-samples one pass solves (both images together)
        coef = per_kind["fgs_coef"]
        avg_us_corr = corr["fgs_pass"][0] / cnt * 1e3
        # HBM bytes a pass moves by its data flow: per line-sample the two right-hand sides and the
        # four coefficients read (8 + 16 B, the LDS images' chunk layout), the two results written
        fgs_bytes = samples * (8 + 16 + 8)
        return {
            "bound": "latency",
            "kernel": "k_fgs_lr (sequential FGS pass, SDR_FGS_THOMAS: the lines resident in LDS, one solver "
                      "wave per right-hand side, 4 samples x up to 8 lines a lane-instruction (SDR_FGS_LR_MAXL), two "
                      "DMA loader / writer waves beside them)",
            "achieved": round(samples / (avg_us * 1e-6) / 1e9, 3),
            "peak": round(samples / (floor_us * 1e-6) / 1e9, 3),
            "unit": "G line-samples/s",
            "frac": round(floor_us / avg_us, 4),
            "traffic": load_traffic(f"{a.config}:k_fgs_lr"),
            "traffic_unit": "HBM bytes a launch (PMC, profiles/pmc_traffic.json); the pass is latency-bound",
            "algorithmic_bytes_per_launch": fgs_bytes,
            "bytes_model": "32 B a line-sample: 8 (two right-hand sides) + 16 (coefficients) read, 8 written",
            "model": (f"a pass = lines of a {rw}x{rh} ROI, mean chain {chain:.0f} samples (rows {rw}, columns "
                      f"{rh}); floor = chain x ({fwd_ops} fwd + {back_ops} back dependent ops) x {cyc_op} "
                      f"cycles at {CLOCK_GHZ} GHz = {floor_us:.2f} us a pass"),
            "avg_launch_us": round(avg_us, 2),
            "avg_launch_us_overhead_corrected": round(avg_us_corr, 2),
            "frac_overhead_corrected": round(floor_us / avg_us_corr, 4) if avg_us_corr > 0 else None,
            "floor_us": round(floor_us, 2),
            "measured_cycles_per_sample": round(avg_us * CLOCK_GHZ * 1e3 / chain, 1),
            "floor_cycles_per_sample": round((fwd_ops + back_ops) * cyc_op, 1),
            "launches_timed": cnt,
            "passes_per_frame": cnt / max(1, steps) / max(1, batch),
            "coef_jobs_us_per_launch": round(coef[0] / coef[1] * 1e3, 2) if coef[1] else None,
            "share_of_gpu_time": round((corr["fgs_pass"][0] + corr["fgs_coef"][0]) / all_corr, 4) if all_corr else 0,
        }

    roofline = None
    kernels = None
    if not a.no_kernel_timing:
        inflight = None
        if a.in_flight_timing:
            _, inflight = kernel_report(m, steps=a.steps)
            if inflight is not None:
                inflight["measured"] = (f"HIP events around each launch of matcher 0 over the timed region "
                                        f"({ns} frames in flight: an event pair also spans the wait for CUs "
                                        f"held by the other streams' kernels, so it overstates the duration)")
        # the dominant kernel's roofline: the same launches with nothing beside them, a
        # single-stream segment timed right after the timed region (no events inside the timed
        # region; rocprofv3's per-dispatch durations of these launches agree:
        # profiles/r2_segments_c2.md)
        iso = max(1, a.iso_steps)

        def iso_run(timed):
            ingest = []
            with torch.cuda.stream(streams[0]):
                for i in range(iso):
                    j = (i * batch) % (nf - batch + 1) if nf > batch else 0
                    if kind == "live" and timed:  # k_sbs_ingest runs on the rectifier's handle: torch events
                        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                        ingest.append(ev)
                        run(j, 0, 0, ingest_events=ev)
                    else:
                        run(j, 0, 0)
            return ingest

        def hbm_only_paths(frames=4, reps=5):
            """k_paths with a cost volume the 256 MiB Infinity Cache cannot hold:
            the same C2 launch shape over `frames` frames in one batch (C = frames x 212 MB), so its
            four re-reads of C come from HBM, not the cache; one matcher, single stream, event-timed
            (raw durations, no overhead correction)."""
            mm = sdr.StereoSGBM.create(*args, device=dev.index)
            f = min(frames, nf)
            dd = torch.empty((f, H, W), dtype=torch.int16, device=dev)
            xx = torch.empty((f, H, W, 3), dtype=torch.float32, device=dev)
            with torch.cuda.stream(streams[0]):
                mm.compute_reproject(Ld[:f], Rd[:f], S.REFERENCE_Q, hm, disp=dd, xyz=xx)  # warm, allocate
                torch.cuda.synchronize()
                mm.enable_timing(2)
                mm.kernel_time(-1, reset=True)
                for _ in range(reps):
                    mm.compute_reproject(Ld[:f], Rd[:f], S.REFERENCE_Q, hm, disp=dd, xyz=xx)
            torch.cuda.synchronize()
            ms_, c = mm.kernel_time(_sg.KERNEL_PATHS, reset=True)
            mm.close()
            cells_f = f * H * w1 * D
            b = cells_f * 4 * (P - 1)
            us = ms_ / c * 1e3
            return {"kernel": "k_paths (the C2 launch shape)", "frames_per_launch": f,
                    "cost_volume_MB": round(cells_f * 2 / 1e6, 1), "algorithmic_bytes_per_launch": b,
                    "avg_launch_us": round(us, 2), "launches": c, "achieved": round(b / us / 1e3, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(b / us / 1e3 / HBM_PEAK_GBS, 4),
                    "note": "C beyond the Infinity Cache: the fraction of HBM itself; the main roofline's "
                            "batch-1 C (212 MB) is partly re-read from the 256 MiB cache"}

        # the same single-stream steps without events first: the step time the per-kernel table
        # is reconciled with (kernel_report's step_us)
        torch.cuda.synchronize()
        iso_run(False)  # warm
        torch.cuda.synchronize()
        t_iso = time.perf_counter()
        iso_run(False)
        torch.cuda.synchronize()
        step_us = (time.perf_counter() - t_iso) / iso * 1e6
        m.enable_timing(2)
        m.kernel_time(-1, reset=True)
        ingest = iso_run(True)
        torch.cuda.synchronize()
        extra = {"k_sbs_ingest": (sum(e0.elapsed_time(e1) for e0, e1 in ingest), len(ingest))} if ingest else None
        kernels, roofline = kernel_report(m, extra, step_us=step_us, steps=iso)
        if roofline is not None:
            roofline["measured"] = (f"HIP events around each launch, {iso} single-stream steps after the timed "
                                    f"region, less the events' own overhead per launch (the events' sum over "
                                    f"the same {iso} steps run without events)")
            roofline["kernels"] = kernels
            if inflight is not None:
                roofline["in_flight"] = inflight
            if a.stream_probe:
                probe = stream_probe(dev)
                hb = roofline.get("hbm_path_kernel", roofline)
                hb["stream_probe"] = probe
                hb["frac_of_probe"] = round(hb["achieved"] / probe["gbs"], 4)
            if a.hbm_only and kind == "sgbm" and mode == 0:
                roofline["hbm_only"] = hbm_only_paths()
                if a.stream_probe:
                    roofline["hbm_only"]["frac_of_probe"] = round(roofline["hbm_only"]["achieved"] /
                                                                  probe["gbs"], 4)
        m.enable_timing(0)
    pix = world * a.steps * batch * W * H
    value = pix / el / 1e6
    if roofline is not None:
        # B_frame = cells*(2+6P) + 16 B/px, times the whole job's frame rate
        b_frame = cells * (2 + 6 * P) + 16 * Hm * Wm * batch * nmatch
        job = b_frame * world * a.steps / el / 1e9
        roofline["job"] = {"model_bytes_per_step": b_frame, "achieved": round(job, 1),
                           "frac": round(job / HBM_PEAK_GBS / world, 4),
                           "note": "canonical unfused data-flow bytes x steps/s (per GPU); the fused "
                                   "kernels move fewer real bytes"}
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(el / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": ("synthetic seeded rectified pairs (SURVEY.md 8d recipe); reference assets absent" if kind == "sgbm"
                 else "synthetic seeded side-by-side BGR frames (SURVEY.md 8d recipe); reference assets absent"),
        "config": {
            "workload": desc,
            "width": W, "height": H, "numDisparities": D, "mode": MODE_NAMES[mode],
            "paths": NPATHS[mode], "batch": batch, "pipeline": kind,
            "params": dict(zip(["minDisparity", "numDisparities", "blockSize", "P1", "P2",
                                "disp12MaxDiff", "preFilterCap", "uniquenessRatio",
                                "speckleWindowSize", "speckleRange", "mode"], args)),
            "parallelism": f"frame shard x{world}" + ((" + gloo gather to rank 0 (rehearsal)" if gloo else
                                                      " + RCCL gather to rank 0") if dist_on else ""),
            "streams_per_gpu": ns,
        },
        "fps": round(world * a.steps * batch / el, 2),
        # rank 0's enqueue loop alone: near ms_per_step means the host's launch rate bounds the line
        "host_enqueue_ms_per_step": round(host_el / a.steps * 1e3, 4),
        "ranks": ranks,
        "gather_check": gather_check,
        "roofline": roofline,
        "kernels": kernels,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(CONFIGS[a.config])
        except Exception as e:  # the baseline never hides the GPU number
            log("cpu baseline failed:", repr(e))
    if rank == 0:
        print(json.dumps(out), flush=True)
    for mm in closers:
        mm.close()
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
