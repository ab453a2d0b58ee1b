"""bench.py's N>1 entry points (CPU): ``python bench.py --gpus N`` with no torch.distributed.run
around it starts the launcher as a child process (the driver's form: --nnodes=1, one rank per GPU,
127.0.0.1 rendezvous), relays what the ranks print and exits with the launcher's code; under an
outside launcher (WORLD_SIZE set) it never re-launches."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_self_launch_argv_dry_run():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--steps", "7", "--warmup", "2", "--launch-dry-run"],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert p.returncode == 0, p.stderr
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    cmd = rec["self_launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(BENCH)
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "7", "--warmup", "2"]  # the flag itself is dropped
    assert rec["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_self_launch_relays_output_and_exit_code(monkeypatch, capfd):
    """The child's stdout reaches this process's stdout and its exit code is returned (a stand-in
    child: no GPU here)."""
    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("TONY_BENCH_DEVICE", "0")  # rehearsal form: skips the device-count check
    child = [sys.executable, "-c", "import json, sys; print(json.dumps({'metric': 'x', 'value': 1.0})); sys.exit(3)"]
    monkeypatch.setattr(bench, "self_launch_cmd", lambda argv, n, port: (child, dict(os.environ)))
    rc = bench.main(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    out = capfd.readouterr().out
    assert rc == 3
    assert json.loads(out.strip().splitlines()[-1]) == {"metric": "x", "value": 1.0}


def test_self_launch_refuses_more_ranks_than_gpus(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("TONY_BENCH_DEVICE", raising=False)
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    assert bench.main(["--gpus", "4"]) == 2


@pytest.mark.parametrize("world", ["1", "2"])
def test_no_relaunch_under_an_outside_launcher(world):
    """WORLD_SIZE set: bench.py is a rank; a --gpus / WORLD_SIZE mismatch is an error, not a launch."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE=world, RANK="0"))
    assert p.returncode == 2
    assert "self_launch" not in p.stdout
    assert "WORLD_SIZE" in p.stderr
