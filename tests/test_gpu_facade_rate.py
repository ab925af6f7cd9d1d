"""The reference's host-memory call patterns through the C++ facade (tests/cpp/facade_rate.cpp):
pcd_write.cpp's compute -> convertTo(1/16) -> reprojectImageTo3D(handleMissing) with
facade-allocated (page-locked) Mats, and the live loop's StereoDisparity::computeDisparity ->
computeDepth on host BGR frames.  Outputs bit-exact against the oracle; the frame rates are
printed (and recorded by scripts/pcie_rate.py's --facade run in profiles/)."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from stereo_depth_ruler_amd import synthetic as S  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_facade_rate(out):
    libdir = os.path.join(ROOT, "stereo_depth_ruler_amd", "lib")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "facade_rate.cpp"), "-L", libdir, "-lsdr",
                           f"-Wl,-rpath,{libdir}", "-o", str(out)])


def write_inputs(d, seed=5):
    H, W = 720, 1280
    L, R, _ = S.make_pair(H, W, 128, seed=seed)
    frame = S.sbs_bgr_color_frame(H, W, 80, seed=seed)
    L.tofile(os.path.join(d, "l.bin"))
    R.tofile(os.path.join(d, "r.bin"))
    np.ascontiguousarray(frame[:, :W]).tofile(os.path.join(d, "bl.bin"))
    np.ascontiguousarray(frame[:, W:]).tofile(os.path.join(d, "br.bin"))
    np.asarray(S.REFERENCE_Q, np.float64).tofile(os.path.join(d, "q.bin"))
    return L, R, np.ascontiguousarray(frame[:, :W]), np.ascontiguousarray(frame[:, W:])


def test_facade_host_patterns_bit_exact(oracle, tmp_path):
    from test_gpu_parity import class_path_ref

    exe = tmp_path / "facade_rate"
    build_facade_rate(exe)
    L, R, bl, br = write_inputs(str(tmp_path))
    res = subprocess.run([str(exe), str(tmp_path), "3"], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    print(res.stdout.strip())
    rates = json.loads(res.stdout)
    assert rates["pcd_separate"]["fps"] > 0 and rates["class_computeDisparity_computeDepth"]["fps"] > 0
    H, W = 720, 1280
    ref = oracle.sgbm_compute(L, R, oracle.make_params(0, 128, 5, 600, 2400, 1, 63, 12, 200, 2, 0))
    assert np.array_equal(np.fromfile(tmp_path / "pcd_disp.bin", np.int16).reshape(H, W), ref)
    ref_xyz = oracle.reproject(oracle.disp_to_float(ref), S.REFERENCE_Q, True)
    assert np.array_equal(np.fromfile(tmp_path / "pcd_xyz.bin", np.uint32).reshape(H, W, 3), ref_xyz.view(np.uint32))
    _, _, _, _, ref_cls = class_path_ref(oracle, bl, br)
    got = np.fromfile(tmp_path / "cls_disp.bin", np.float32).reshape(H // 2, W // 2)
    assert np.array_equal(got.view(np.uint32), ref_cls.view(np.uint32))
    ref_depth = oracle.reproject(ref_cls, S.REFERENCE_Q, False)
    got_depth = np.fromfile(tmp_path / "cls_depth.bin", np.uint32).reshape(H // 2, W // 2, 3)
    assert np.array_equal(got_depth, ref_depth.view(np.uint32))
