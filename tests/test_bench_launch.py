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


# -- the other BASELINE configs (bench.py --config, tony_amd/bench_configs.py) -----------------------------
def _last_json(stdout: str) -> dict:
    return json.loads([ln for ln in stdout.splitlines() if ln.startswith("{")][-1])


def test_config_ddp_mnist_two_ranks_gloo():
    """ddp-mnist through the self-launch (2 ranks, gloo, CPU): one JSON line with the whole-job rate."""
    p = subprocess.run([sys.executable, BENCH, "--config", "ddp-mnist", "--gpus", "2", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300,
                       env=_env(TONY_BENCH_DEVICE="0", TONY_BENCH_BACKEND="gloo", CUDA_VISIBLE_DEVICES=""))
    assert p.returncode == 0, p.stderr[-3000:]
    rec = _last_json(p.stdout)
    assert rec["metric"].startswith("samples/sec") and rec["n_gpus"] == 2 and rec["steps"] == 3
    assert rec["config"]["global_batch"] == 256 and rec["value"] > 0 and rec["higher_is_better"]


def test_config_mxnet_kv_dist_sync_launch():
    """mxnet-kv: scheduler + 1 server + 2 workers as processes with the DMLC_* contract, dist_sync."""
    p = subprocess.run([sys.executable, BENCH, "--config", "mxnet-kv", "--gpus", "2", "--steps", "4", "--warmup", "1",
                        "--kv-device", "cpu"], capture_output=True, text=True, timeout=300, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    rec = _last_json(p.stdout)
    assert rec["config"]["kvstore"] == "dist_sync" and rec["n_gpus"] == 2
    assert rec["config"]["global_batch"] == 2048 and rec["value"] > 0


def test_config_dry_runs():
    p = subprocess.run([sys.executable, BENCH, "--config", "hvd-resnet50", "--gpus", "8", "--launch-dry-run"],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert p.returncode == 0, p.stderr
    cmd = json.loads(p.stdout.strip().splitlines()[-1])["self_launch"]
    assert "--nproc-per-node=8" in cmd and cmd[cmd.index(BENCH) + 1:] == ["--config", "hvd-resnet50", "--gpus", "8"]
    p = subprocess.run([sys.executable, BENCH, "--config", "mxnet-kv", "--gpus", "8", "--launch-dry-run"],
                       capture_output=True, text=True, timeout=120, env=_env())
    roles = json.loads(p.stdout.strip().splitlines()[-1])["mxnet_kv_launch"]
    assert [r[0] for r in roles] == ["scheduler", "server"] + ["worker"] * 8
    assert all(r[2]["DMLC_NUM_WORKER"] == "8" and r[2]["DMLC_NUM_SERVER"] == "1" for r in roles)


def test_rank_cpu_affinity_choice():
    """Verdict r5 #5: each rank of an N-GPU bench runs on its GPU's NUMA node, the node's CPUs split among
    the ranks that share it (fake inventory: 8 GPUs, 2 nodes of 64 CPUs)."""
    from tony_amd.gpu.inventory import rank_cpus
    from tony_amd.native import GpuDevice

    devs = [GpuDevice(i, bdf=f"fake:{i:02x}", numa_node=i // 4, fake=True) for i in range(8)]
    node = {0: list(range(0, 64)), 1: list(range(64, 128))}
    got = [rank_cpus(o, list(range(8)), devs, cpus_of_node=node.get, allowed=list(range(128))) for o in range(8)]
    assert got[0] == list(range(0, 16)) and got[3] == list(range(48, 64)) and got[4] == list(range(64, 80))
    assert sorted(c for g in got for c in g) == list(range(128))  # disjoint, every CPU used once
    # 2 ranks on GPUs 0 and 5: each gets its whole node; a restricted allowed set is respected
    assert rank_cpus(5, [0, 5], devs, cpus_of_node=node.get, allowed=list(range(128))) == list(range(64, 128))
    assert rank_cpus(0, [0, 1], devs, cpus_of_node=node.get, allowed=list(range(8))) == [0, 1, 2, 3]
    # nothing known: leave affinity alone
    unk = [GpuDevice(0, bdf="fake:00", numa_node=-1, fake=True)]
    assert rank_cpus(0, [0], unk, cpus_of_node=node.get, allowed=list(range(8))) == []
    assert rank_cpus(0, [0], devs, cpus_of_node=node.get, allowed=[100]) == []


def test_ps_async_needs_dedicated_mode():
    """--ps-async is the paper topology's asynchronous PS (dedicated ps rank): refused with colocated shards,
    before any GPU call; passed through to the ranks of a self-launch."""
    p = subprocess.run([sys.executable, BENCH, "--ps-async"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "--ps-mode dedicated" in p.stderr, p.stderr[-500:]
    p = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--ps-mode", "dedicated", "--ps-async",
                        "--launch-dry-run"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-500:]
    assert "--ps-async" in json.loads(p.stdout.strip().splitlines()[-1])["self_launch"]
