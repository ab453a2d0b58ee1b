"""The reference jobs end to end through TonyClient -> coordinator -> task agents -> runtime env ->
user process, in local mode on CPU (gloo).  One test per runtime/parallelism pairing of
SURVEY.md §2.6 (the "end-to-end 1-step smoke for every runtime" of the test strategy).
"""
import json
import os
import sys

import pytest
import torch

from tony_amd.client.tony_client import TonyClient
from tony_amd.conf import Configuration
from tony_amd.conf import keys as K

JOBS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tony_amd", "jobs")
PY = sys.executable

pytestmark = pytest.mark.timeout(300)


@pytest.fixture
def conf(tmp_path):
    c = Configuration()
    c.set(K.SECURITY_ENABLED, "false")
    c.set(K.AMD_STAGING_DIR, str(tmp_path / "staging"))
    c.set(K.AMD_FAKE_GPUS, "8")
    c.set(K.AMD_VISIBLE_DEVICES_MODE, "none")
    c.set(K.TASK_HEARTBEAT_INTERVAL_MS, "500")
    c.set("tony.amd.stop-grace-sec", "3")
    c.set(K.AM_WAIT_CLIENT_STOP_TIMEOUT, "5")
    return c


class Infos:
    def __init__(self):
        self.infos = set()

    def on_application_id_received(self, app_id):
        pass

    def on_task_infos_updated(self, infos):
        self.infos = infos


def run_job(conf, script, confs, params=None, env=None):
    client = TonyClient(conf)
    h = Infos()
    client.add_listener(h)
    args = ["--src_dir", JOBS, "--executes", script, "--python_binary_path", PY,
            "--shell_env", "OMP_NUM_THREADS=1", "--shell_env", "TONY_DIST_BACKEND=gloo"]
    for k, v in (env or {}).items():
        args += ["--shell_env", f"{k}={v}"]
    for kv in confs:
        args += ["--conf", kv]
    if params:
        args += ["--task_params", params]
    assert client.init(args)
    rc = client.start()
    return rc, client, h


def _metrics(client):
    out = []
    logs = os.path.join(client.job_dir, "logs")
    for root, _, files in os.walk(logs):
        for f in files:
            if f == "stdout":
                with open(os.path.join(root, f), errors="replace") as fh:
                    for line in fh:
                        if line.startswith("TONY_METRIC "):
                            out.append(json.loads(line[len("TONY_METRIC "):]))
    return out


def _diag(client):
    logs = os.path.join(client.job_dir, "logs")
    tail = []
    for root, _, files in os.walk(logs):
        for f in files:
            with open(os.path.join(root, f), errors="replace") as fh:
                tail.append(f"--- {root}/{f}\n" + "".join(fh.readlines()[-15:]))
    return "\n".join(tail)


def test_pytorch_ddp_mnist(conf):
    rc, client, _ = run_job(conf, "mnist_pytorch_ddp.py",
                            ["tony.application.framework=pytorch", "tony.worker.instances=2", "tony.ps.instances=0"],
                            "--steps-per-epoch 10 --checkpoint-steps 5")
    assert rc == 0, _diag(client)
    ms = _metrics(client)
    assert len(ms) == 2 and all(m["loss"] < 2.3 for m in ms)
    assert os.listdir(os.path.join(client.job_dir, "model", "mnist_ddp"))  # rank-0 checkpoint


@pytest.mark.parametrize("sync", [False, True])
def test_tf_ps_mnist(conf, sync):
    rc, client, h = run_job(conf, "mnist_tf_ps.py", ["tony.ps.instances=1", "tony.worker.instances=2"],
                            "--steps 8" + (" --sync" if sync else ""))
    assert rc == 0, _diag(client)
    assert len(_metrics(client)) == 2


def test_tf_allreduce_mnist(conf):
    rc, client, _ = run_job(conf, "mnist_tf_allreduce.py", ["tony.ps.instances=0", "tony.worker.instances=3"],
                            "--steps 5")
    assert rc == 0, _diag(client)
    ms = _metrics(client)
    assert {m["global_batch"] for m in ms} == {192}


def test_estimator_chief_worker_ps_evaluator(conf):
    rc, client, _ = run_job(conf, "mnist_estimator.py",
                            ["tony.chief.instances=1", "tony.worker.instances=1", "tony.ps.instances=1",
                             "tony.evaluator.instances=1"], "--steps 10 --save-steps 3 --eval-timeout 120")
    assert rc == 0, _diag(client)
    evals = [m for m in _metrics(client) if "eval_step" in m]
    assert evals and max(m["eval_step"] for m in evals) == 10


def test_horovod_mnist(conf):
    rc, client, _ = run_job(conf, "hvd_mnist.py", ["tony.application.framework=horovod",
                                                   "tony.worker.instances=2"], "--steps 6")
    assert rc == 0, _diag(client)
    ms = _metrics(client)
    assert len(ms) == 1 and ms[0]["size"] == 2


@pytest.mark.parametrize("kvstore", ["dist_sync", "dist_async"])
def test_mxnet_kvstore_linreg(conf, kvstore):
    rc, client, _ = run_job(conf, "mxnet_linreg.py",
                            ["tony.application.framework=mxnet", "tony.scheduler.instances=1",
                             "tony.server.instances=1", "tony.worker.instances=2", "tony.ps.instances=0"],
                            f"--kvstore {kvstore} --rows 8192 --epochs 3 --lr 0.5")
    assert rc == 0, _diag(client)
    ms = _metrics(client)
    assert ms and all(m["mse"] < 0.05 for m in ms if m["epoch"] == 2)


def test_inception_ps_colocated_tiny(conf):
    rc, client, h = run_job(conf, "inception_ps.py", ["tony.ps.instances=1", "tony.worker.instances=2"],
                            "--ps-mode colocated --batch-size 2 --image-size 299 --steps 1 --warmup 1")
    assert rc == 0, _diag(client)
    ms = _metrics(client)
    assert len(ms) == 1 and ms[0]["workers"] == 2 and ms[0]["ps_mode"] == "colocated"
    assert ms[0]["dtype"] == "fp32" and ms[0]["sync"] is True  # CPU ranks compute in fp32


def test_inception_ps_dedicated_tiny(conf):
    """The paper topology (1 ps + 2 workers, the ps owning the variables) through the launcher.  The ps
    task and the workers must issue matching collective sequences (per-step bucket reduce / broadcast,
    the timing barrier, the rate all-reduce): a mismatch hangs or corrupts the gloo group."""
    rc, client, h = run_job(conf, "inception_ps.py", ["tony.ps.instances=1", "tony.worker.instances=2"],
                            "--ps-mode dedicated --batch-size 2 --image-size 299 --steps 2 --warmup 1")
    assert rc == 0, _diag(client)
    ms = _metrics(client)
    assert len(ms) == 1 and ms[0]["workers"] == 2 and ms[0]["ps_mode"] == "dedicated"
    assert ms[0]["images_per_sec"] > 0


def test_cluster_discovery(conf):
    rc, client, _ = run_job(conf, "cluster_discovery.py", ["tony.head.instances=1", "tony.worker.instances=1",
                                                           "tony.ps.instances=0"])
    assert rc == 0, _diag(client)


def test_resnet50_ddp_minimum_slice(conf):
    """SURVEY.md §7.3's minimum slice: PyTorch runtime env -> init_process_group -> ResNet-50 under
    tony_amd's bucketed DDP (tiny images on the CPU here; bf16 fused kernels on a GPU node)."""
    rc, client, _ = run_job(conf, "resnet50_ddp.py", ["tony.application.framework=pytorch", "tony.worker.instances=2",
                                                      "tony.ps.instances=0"],
                            "--batch-size 2 --image-size 32 --steps 1 --warmup 1")
    assert rc == 0, _diag(client)
    ms = _metrics(client)
    assert len(ms) == 1 and ms[0]["world"] == 2 and ms[0]["images_per_sec"] > 0


def _final_shards(d):
    out = {}
    for n in sorted(os.listdir(d)):
        if n.startswith("ckpt-4-shard"):
            out[n] = torch.load(os.path.join(d, n), weights_only=True)
    return out


def test_inception_ps_sharded_checkpoint_resume_after_gang_retry(conf, tmp_path):
    """A worker dies mid-training (session 0); the coordinator's retry relaunches the gang, which
    restores every rank's PS shard from the newest complete step and finishes with variables, fp32
    masters and momentum BIT-identical to an uninterrupted run (3 workers = 3 shards over gloo)."""
    confs = ["tony.ps.instances=1", "tony.worker.instances=3"]
    args = "--ps-mode colocated --batch-size 2 --image-size 299 --steps 4 --warmup 0 --save-steps 2"
    ref_dir, dir_ = tmp_path / "ref", tmp_path / "retry"
    rc, client, _ = run_job(conf, "inception_ps.py", confs, f"{args} --checkpoint-dir {ref_dir}")
    assert rc == 0, _diag(client)
    rc, client, _ = run_job(conf, "inception_ps.py", confs + ["tony.am.retry-count=1"],
                            f"{args} --checkpoint-dir {dir_} --fail-at-step 3")
    assert rc == 0, _diag(client)
    ms = _metrics(client)
    assert ms and ms[-1]["start_step"] == 2 and ms[-1]["steps"] == 4   # resumed at the step-2 checkpoint
    ref, got = _final_shards(ref_dir), _final_shards(dir_)
    assert sorted(ref) == sorted(got) and len(ref) == 3
    for name in ref:
        a, b = ref[name]["ps"], got[name]["ps"]
        assert torch.equal(a["flat"], b["flat"]), name
        assert a["shards"].keys() == b["shards"].keys() and len(a["shards"]) == 1
        for r in a["shards"]:
            assert torch.equal(a["shards"][r]["master"], b["shards"][r]["master"])
            assert torch.equal(a["shards"][r]["opt"]["momentum_buffer"], b["shards"][r]["opt"]["momentum_buffer"])
