"""bench.py --gpus N starts and proves N ranks itself (CPU only).

The driver runs ``python bench.py --gpus N`` on an N-GPU node; without a launcher around it the
script must start the N ranks itself, never run fewer, and report the rank count the
communicator saw.  ``--launcher-selftest`` makes the ranks run only the gloo control plane (one
all-reduce, no GPU); MD2_BENCH_FAKE_DEVICES stands in for the visible-device count here."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                          timeout=240)


def test_launcher_starts_two_ranks_and_prints_one_line():
    r = _run(["--gpus", "2", "--launcher-selftest"], {"MD2_BENCH_FAKE_DEVICES": "2"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["comm"]["nranks"] == 2 and out["comm"]["allreduce_ranks_seen"] == 2
    pids = out["comm"]["rank_pids"]
    assert len(set(pids)) == 2 and os.getpid() not in pids
    assert "started 2 ranks" in r.stderr


def test_launcher_four_ranks():
    r = _run(["--gpus", "4", "--launcher-selftest"], {"MD2_BENCH_FAKE_DEVICES": "8"})
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip())
    assert out["n_gpus"] == 4 and out["comm"]["allreduce_ranks_seen"] == 4


def test_too_few_devices_exits_nonzero():
    r = _run(["--gpus", "2", "--launcher-selftest"], {"MD2_BENCH_FAKE_DEVICES": "1"})
    assert r.returncode != 0
    assert "needs 2 visible GPUs, found 1" in r.stderr
    assert r.stdout.strip() == ""


def test_real_device_count_is_checked():
    # no fake count: this container has no GPU (and no KFD topology), so --gpus 2 must refuse --
    # either for too few devices (a 1-GPU box) or because they cannot be counted without HIP
    r = _run(["--gpus", "2"])
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr or "cannot count GPUs without initialising HIP" in r.stderr


def test_kfd_count_and_visible_device_cap(tmp_path, monkeypatch):
    """The launcher counts GPU agents in the KFD sysfs topology (CPU nodes report no SIMDs) and
    caps the count by the *_VISIBLE_DEVICES lists -- no HIP call in the parent."""
    import bench
    for i, simds in enumerate([0, 1024, 1024, 1024]):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count {0 if simds else 64}\nsimd_count {simds}\n")
    monkeypatch.setattr(bench, "KFD_NODES", str(tmp_path))
    assert bench._kfd_gpus(str(tmp_path)) == 3
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setattr(bench, "_kfd_gpus", lambda root=None: 3)
    assert bench._visible_devices(False) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert bench._visible_devices(False) == 2
    monkeypatch.setattr(bench, "_kfd_gpus", lambda root=None: -1)
    assert bench._visible_devices(False) == -1
    assert bench._kfd_gpus(str(tmp_path / "missing")) == -1


def test_launcher_refuses_under_profiler():
    r = _run(["--gpus", "2"], {"ROCPROF_OUTPUT_PATH": "/tmp/x", "MD2_BENCH_FAKE_DEVICES": "2"})
    assert r.returncode == 2 and "under a profiler" in r.stderr


def test_under_a_launcher_does_not_spawn_again():
    # WORLD_SIZE set (torchrun around us): this process IS a rank; world 1 here, one JSON line
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
           "MASTER_PORT": str(_port())}
    r = _run(["--gpus", "1", "--launcher-selftest"], env, drop=())
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip())
    assert out["n_gpus"] == 1 and out["comm"]["rank_pids"] == [out["comm"]["rank_pids"][0]]
    assert "started" not in r.stderr


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "8", "--launcher-selftest"], {"WORLD_SIZE": "2", "RANK": "0"}, drop=())
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 8" in r.stderr


def _port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n", [0, -1])
def test_bad_gpu_count(n):
    assert _run(["--gpus", str(n), "--launcher-selftest"]).returncode != 0
