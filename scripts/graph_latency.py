"""Per-frame latency of the C4 live-loop frame (rectify + class path + computeDepth, bench.py's
"live" pipeline) enqueued directly vs. captured once into a hipGraph and replayed, one frame at a
time with a synchronize after each (the reference's blocking loop, stereo_displayer.cpp:145-198),
and back-to-back on one stream.  Prints one JSON line; the replayed outputs are compared with the
direct ones bit for bit.

    python scripts/graph_latency.py [--frames 300]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stereo_depth_ruler_amd import synthetic as S  # noqa: E402
from stereo_depth_ruler_amd.config import StereoConfiguration  # noqa: E402
from stereo_depth_ruler_amd.pipeline import LiveLoop  # noqa: E402
from stereo_depth_ruler_amd.rectify import StereoRectifier  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    W, H = 1280, 720
    cfg = StereoConfiguration()
    assert cfg.loadFromFile(os.path.join(ROOT, "tests", "golden", "stereo.yaml"))
    rect = StereoRectifier(cfg, device=0)
    sbs = torch.empty((4, H, 2 * W, 3), dtype=torch.uint8, device=dev)
    for i in range(4):
        sbs[i].copy_(torch.from_numpy(S.sbs_bgr_color_frame(H, W, 80, seed=i)))
    src = torch.empty((1, H, 2 * W, 3), dtype=torch.uint8, device=dev)
    pipe = LiveLoop(rect, cfg.Q, 1, device=0)

    def direct(i):
        src.copy_(sbs[i % 4:i % 4 + 1])
        return pipe.enqueue(src, torch.cuda.current_stream(dev))

    for i in range(20):
        direct(i)
    torch.cuda.synchronize()
    ref = []
    for i in range(4):
        ref.append((direct(i).clone(), pipe.depth.clone()))
    torch.cuda.synchronize()

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = pipe.enqueue(src, torch.cuda.current_stream())

    def replay(i):
        src.copy_(sbs[i % 4:i % 4 + 1])
        g.replay()
        return out

    exact = True
    for i in range(4):
        replay(i)
        torch.cuda.synchronize()
        exact &= bool(torch.equal(out, ref[i][0])) and bool(torch.equal(pipe.depth, ref[i][1]))

    res = {"workload": "C4 live-loop frame (2560x720 SBS -> 640x360 3WAY L+R + WLS + computeDepth), batch 1",
           "frames": a.frames, "graph_bit_exact": exact}
    for name, fn in (("direct", direct), ("graph", replay)):
        for i in range(10):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.frames):
            fn(i)
            torch.cuda.synchronize()
        blocking = (time.perf_counter() - t0) / a.frames * 1e3
        t0 = time.perf_counter()
        for i in range(a.frames):
            fn(i)
        torch.cuda.synchronize()
        stream = (time.perf_counter() - t0) / a.frames * 1e3
        res[name] = {"blocking_ms_per_frame": round(blocking, 4), "stream_ms_per_frame": round(stream, 4)}
    print(json.dumps(res))
    pipe.close()


if __name__ == "__main__":
    main()
