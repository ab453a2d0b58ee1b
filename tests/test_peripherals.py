"""Peripheral modules: Azkaban job type (TestTonyJob), version info (VersionInfo), docker task
runtime (TestHadoopCompatibleAdapter docker env), checkpoint manager."""
import os
import sys

import pytest
import torch

from tony_amd.conf import Configuration
from tony_amd.conf import keys as K

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "fixtures")


def test_azkaban_job_args_tags_and_conf(tmp_path):
    from tony_amd.azkaban import TonyJob, load_properties

    p = tmp_path / "job.properties"
    p.write_text("type=tony\n# comment\ntony.worker.instances=2\ntony.application.name=az\n"
                 "executes=train.py\ntask_params=--lr 0.1 \\\n  --epochs 2\npython_binary_path=bin/python\n"
                 "python_venv=venv.zip\nworker_env.A=1\nworker_env.B=two\nazkaban.flow.execid=123\n"
                 "azkaban.flow.flowid=flow\nazkaban.flow.projectname=proj\nazkaban.input.dataset=a,b\n"
                 "hdfs_classpath=/libs\n")
    props = load_properties(str(p))
    assert props["task_params"] == "--lr 0.1 --epochs 2"
    job = TonyJob("j1", {}, props, str(tmp_path))
    args = job.main_args()
    assert args[:2] == ["--src_dir", "src"]
    assert ["--shell_env", "A=1"] == args[args.index("A=1") - 1:args.index("A=1") + 1]
    assert "--executes" in args and args[args.index("--executes") + 1] == "train.py"
    assert args[args.index("--task_params") + 1] == "--lr 0.1 --epochs 2"
    assert "AZKABAN_INPUT_DATASET=a;b" in args
    assert args[args.index("--hdfs_classpath") + 1] == "/libs"
    tags = job.tony_conf.get("tony.application.tags")
    assert "azkaban.flow.execid:123" in tags and "azkaban.flow.projectname:proj" in tags
    path = job.setup_job_configuration_file()
    c = Configuration.from_xml(path)
    assert c.get("tony.worker.instances") == "2" and c.get("type") is None


def test_version_info_injected(tmp_path):
    from tony_amd import version

    info = version.version_info()
    assert set(info) == set(version.KEYS) and info["version"]
    assert len(version.source_checksum()) == 32
    c = Configuration()
    version.inject(c)
    assert c.get(K.VERSION_INFO_PREFIX + "checksum") == info["checksum"]


def test_docker_command_construction():
    from tony_amd.utils.docker import docker_command, parse_mounts

    assert parse_mounts("/a:/b,/c:/d:ro") == ["/a:/b:rw", "/c:/d:ro"]
    with pytest.raises(ValueError):
        parse_mounts("/a")
    cmd = docker_command("python train.py", "rocm/pytorch:latest", {"HIP_VISIBLE_DEVICES": "3", "PATH": "/x"},
                         "/work", "/data:/data:ro")
    assert "--device=/dev/kfd" in cmd and "--device=/dev/dri" in cmd and "--ipc=host" in cmd
    assert "--env=HIP_VISIBLE_DEVICES=3" in cmd and "PATH=/x" not in cmd
    assert "--volume=/data:/data:ro" in cmd and cmd.endswith("rocm/pytorch:latest bash -c 'python train.py'")
    with pytest.raises(ValueError):
        docker_command("x", "", {}, "/w")


def test_docker_enabled_job_runs_through_runtime(tmp_path):
    """tony.docker.enabled -> the agent wraps the user command (a fake docker binary runs it here)."""
    from tony_amd.client.tony_client import TonyClient

    log = tmp_path / "docker.log"
    c = Configuration()
    c.set(K.SECURITY_ENABLED, "false")
    c.set(K.AMD_STAGING_DIR, str(tmp_path / "staging"))
    c.set(K.AMD_FAKE_GPUS, "8")
    c.set(K.AMD_VISIBLE_DEVICES_MODE, "none")
    c.set(K.DOCKER_ENABLED, "true")
    c.set(K.DOCKER_CONTAINERS_IMAGE, "rocm/pytorch:test")
    c.set(K.DOCKER_CONTAINERS_MOUNT, "/tmp:/tmp:ro")
    c.set(K.AM_WAIT_CLIENT_STOP_TIMEOUT, "5")
    client = TonyClient(c)
    assert client.init(["--src_dir", os.path.join(FIX, "scripts"), "--executes", "exit_0_check_env.py",
                        "--python_binary_path", sys.executable, "--shell_env", "ENV_CHECK=ENV_CHECK",
                        "--shell_env", f"TONY_DOCKER_BIN={os.path.join(FIX, 'bin', 'fake_docker')}",
                        "--shell_env", f"FAKE_DOCKER_LOG={log}",
                        "--conf", "tony.worker.instances=1", "--conf", "tony.ps.instances=0"])
    assert client.start() == 0
    text = log.read_text()
    assert "run --rm" in text and "rocm/pytorch:test" in text and "/tmp:/tmp:ro" in text


def test_checkpoint_manager_rotation_and_restore(tmp_path):
    from tony_amd.utils.checkpoint import CheckpointManager, resume_step, training_state

    m = torch.nn.Linear(3, 2)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    m(torch.randn(4, 3)).sum().backward()
    opt.step()
    ck = CheckpointManager(str(tmp_path / "ck"), keep_max=2, save_steps=10, rank=0)
    for s in range(1, 41):
        ck.save(s, training_state(m, opt, note="x"))
    ck.wait()
    assert [s for s, _ in ck.checkpoints()] == [30, 40]
    st = ck.restore()
    assert resume_step(st) == 40 and st["note"] == "x"
    m2 = torch.nn.Linear(3, 2)
    m2.load_state_dict(st["model"])
    torch.testing.assert_close(m2.weight, m.weight)
    assert CheckpointManager(str(tmp_path / "ck"), rank=1).save(50, {}, force=True) is None  # non-chief
    assert not any(f.endswith(".tmp") for f in os.listdir(tmp_path / "ck"))


def test_tracing_ranges_and_hang_watchdog(tmp_path):
    import subprocess

    from tony_amd.utils import tracing

    with tracing.trace_range("noop"):  # disabled by default: a no-op
        pass
    tracing.set_enabled(True)
    with tracing.trace_range("cpu-only"):  # no GPU here: must not raise
        pass
    tracing.set_enabled(False)
    # a "hung" rank: the watchdog dumps every thread's stack to stderr
    code = ("import time; from tony_amd.utils import tracing; tracing.hang_watchdog(0.3); "
            "time.sleep(1.0)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=30,
                       cwd=os.path.dirname(HERE))
    assert "Thread" in r.stderr and "time.sleep" not in r.stdout


def test_monitor_reports_new_uncorrectable_ecc(monkeypatch):
    from tony_amd import constants as C
    from tony_amd import native
    from tony_amd.agent.monitor import TaskMonitor

    counts = iter([5, 5, 7])
    monkeypatch.setattr(native, "smi_sample", lambda g: native.GpuSample(10, 5, 100, 1000, 300.0, 60.0, 0,
                                                                         next(counts)))
    m = TaskMonitor(lambda: os.getpid(), [0], 1000, lambda _: None, gpu_metrics=True)
    for _ in range(3):
        m.refresh()
    assert m.metrics()[C.GPU_ECC_UNCORRECTABLE] == 2.0


def test_node_example_tony_sh_writes_loadable_conf(tmp_path):
    """examples/mi355x-node/tony.sh (counterpart of tony-in-gcp/scripts/tony.sh) -> tony.xml that the
    configuration loader layers over tony-default.xml."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "tony.xml"
    env = dict(os.environ, TONY_WORKERS="4", TONY_WORKER_GPUS="1", TONY_PS="1", TONY_FRAMEWORK="pytorch")
    subprocess.run(["bash", os.path.join(root, "examples", "mi355x-node", "tony.sh"), str(out)], check=True, env=env,
                   capture_output=True)
    c = Configuration().add_resource(str(out))
    assert c.get("tony.worker.instances") == "4" and c.get("tony.worker.gpus") == "1"
    assert c.get("tony.ps.instances") == "1" and c.get(K.FRAMEWORK_NAME if hasattr(K, "FRAMEWORK_NAME")
                                                       else "tony.application.framework") == "pytorch"
