"""bench.py's rank launcher on CPU: `--gpus N` without a launcher environment starts N ranks
through torch.distributed.run itself (the driver's N-GPU SCALE runs must not silently
report N=1), WORLD_SIZE must agree with --gpus, and the parent relays exactly one JSON line.
The launch on a GPU box is tests/test_gpu_distributed.py::test_bench_gpus2_self_launch."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launcher_cmd_runs_this_script_with_the_same_args():
    cmd = bench.launcher_cmd(4, 29511, ["--gpus", "4", "--steps", "5"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "5"]


def test_free_port_is_bindable():
    import socket

    p = bench.free_port()
    with socket.socket() as s:
        s.bind(("127.0.0.1", p))


def _py(code):
    return [sys.executable, "-c", code]


def test_relay_passes_one_line_through(capsys):
    line = json.dumps({"metric": "m", "n_gpus": 2, "value": 1.0})
    assert bench.relay(_py(f"print('warmup noise'); print({line!r})"), 2) == 0
    out = capsys.readouterr().out
    assert line in out and "warmup noise" in out


@pytest.mark.parametrize("code,rc", [
    ("import sys; sys.exit(7)", 7),                                           # a rank failed
    ("print('{\"n_gpus\": 1}')", 3),                                          # N=1 line for --gpus 2
    ("print('{\"n_gpus\": 2}'); print('{\"n_gpus\": 2}')", 3),                # two lines
    ("print('no json')", 3),
])
def test_relay_rejects_bad_children(code, rc):
    assert bench.relay(_py(code), 2) == rc


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "WORLD_SIZE=3 but --gpus 2" in r.stderr


def test_gpus_must_be_positive():
    with pytest.raises(SystemExit):
        bench.parse_args(["--gpus", "0"])


def test_frames_in_flight_default_per_config():
    # --streams unset: the config's measured default (profiles/r5_streams_sweep.md), 3 otherwise
    assert bench.parse_args([]).streams is None
    assert bench.STREAMS_DEFAULT.get("c4") == 6
    assert all(c in bench.CONFIGS for c in bench.STREAMS_DEFAULT)
    assert bench.parse_args(["--config", "c4", "--streams", "2"]).streams == 2


def test_batch_override_is_opt_in():
    assert bench.parse_args([]).batch is None
    assert bench.parse_args(["--config", "c4", "--batch", "4"]).batch == 4
