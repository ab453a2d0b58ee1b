"""Unit specs of the control plane (TonY's TT/util/TestUtils, TestTaskScheduler, TestTonySession,
TestHorovodRuntime, TestLocalizableResource, TestTonyConfigurationFields, TestTaskStatus,
TestEventHandler, TestParserUtils, TestHistoryFileUtils, TestTonyClient, TestPortAllocation,
TestTaskMonitor equivalents)."""
import io
import json
import os
import socket
import time
import zipfile

import pytest

from tony_amd import constants as C
from tony_amd.conf import DEFAULT_XML, Configuration
from tony_amd.conf import keys as K
from tony_amd.utils import core as U

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")


# -- configuration ----------------------------------------------------------------------
def test_default_xml_parity_with_keys():
    """TestTonyConfigurationFields: every key constant with a default is in tony-default.xml."""
    c = Configuration()
    must = [K.APPLICATION_NAME, K.FRAMEWORK_NAME, K.APPLICATION_DISTRIBUTED_MODE, K.TASK_HEARTBEAT_INTERVAL_MS,
            K.TASK_MAX_MISSED_HEARTBEATS, K.TASK_METRICS_UPDATE_INTERVAL_MS, K.AM_RETRY_COUNT, K.UNTRACKED_JOBTYPES,
            K.SIDECAR_JOBTYPES, K.STOP_ON_FAILURE_JOBTYPES, K.FAIL_ON_WORKER_FAILURE_ENABLED,
            K.CONTAINER_ALLOCATION_TIMEOUT, K.HISTORY_LOCATION, K.HTTPS_PORT, K.SECURITY_ENABLED,
            K.HOROVOD_TEST_MODE, K.AMD_VISIBLE_DEVICES_MODE, K.AMD_REGISTRATION_POLL_MS]
    for k in must:
        assert c.get(k) is not None, k
    assert c.get(K.FRAMEWORK_NAME) == "tensorflow"
    assert c.get_int(K.TASK_MAX_MISSED_HEARTBEATS) == 25
    assert c.get(K.UNTRACKED_JOBTYPES) == "ps"
    assert c.get(K.CONTAINER_ALLOCATION_TIMEOUT) == "-1"


def test_conf_layering_final_and_programmatic(tmp_path):
    a = tmp_path / "a.xml"
    b = tmp_path / "b.xml"
    a.write_text("<configuration><property><name>x</name><value>1</value><final>true</final></property>"
                 "<property><name>y</name><value>1</value></property></configuration>")
    b.write_text("<configuration><property><name>x</name><value>2</value></property>"
                 "<property><name>y</name><value>2</value></property>"
                 "<property><name>z</name><value>${y}-${env.HOME}</value></property></configuration>")
    c = Configuration(load_defaults=False)
    c.set("y", "cli")
    c.add_resource(str(a))
    c.add_resource(str(b))
    assert c.get("x") == "1"          # final wins over a later resource
    assert c.get("y") == "cli"        # programmatic set beats every resource, even ones added later
    assert c.get("z") == f"cli-{os.environ['HOME']}"
    out = tmp_path / "final.xml"
    c.write_xml(str(out))
    c2 = Configuration.from_xml(str(out))
    assert c2.get("y") == "cli" and c2.is_final("x")


def test_multi_value_conf_appends():
    from tony_amd.client.tony_client import TonyClient

    c = Configuration()
    c.set(K.CONTAINERS_RESOURCES, "a.zip")
    cl = TonyClient(c)
    cl.init_tony_conf(c, {"conf": [f"{K.CONTAINERS_RESOURCES}=b.zip", "tony.worker.instances=3"]})
    assert c.get(K.CONTAINERS_RESOURCES) == "a.zip,b.zip"
    assert c.get_int("tony.worker.instances") == 3


# -- utils (TestUtils) ------------------------------------------------------------------------
def test_parse_memory_string():
    assert U.parse_memory_string("2g") == 2048
    assert U.parse_memory_string("512m") == 512
    assert U.parse_memory_string("1024") == 1024
    assert U.parse_memory_string("4G") == 4096


def test_poll_and_poll_till_non_null():
    assert U.poll(lambda: True, 0, 1)
    assert not U.poll(lambda: False, 0.01, 0.05)
    n = {"i": 0}

    def f():
        n["i"] += 1
        return "x" if n["i"] > 2 else None

    assert U.poll_till_non_null(f, 0.001, 1) == "x"
    assert U.poll_till_non_null(lambda: None, 0.01, 0.05) is None
    with pytest.raises(ValueError):
        U.poll(lambda: True, -1, 1)


def test_parse_key_value():
    assert U.parse_key_value(["A=1", "B", "C=x=y", " D=2 "]) == {"A": "1", "B": "", "C": "x=y", "D": "2"}


def test_is_archive(tmp_path):
    assert U.is_archive(os.path.join(FIX, "test.zip"))
    p = tmp_path / "t.txt"
    p.write_text("hello world")
    assert not U.is_archive(str(p))
    import tarfile

    tgz = tmp_path / "t.tar.gz"
    with tarfile.open(tgz, "w:gz") as t:
        t.add(str(p), arcname="t.txt")
    assert U.is_archive(str(tgz))


def test_unzip_archive(tmp_path):
    assert U.unzip_archive(os.path.join(FIX, "test.zip"), str(tmp_path / "out"))
    assert (tmp_path / "out" / "123.xml").exists()
    assert not U.unzip_archive(str(tmp_path / "missing.zip"), str(tmp_path / "o2"))


def test_container_requests_and_stages():
    c = Configuration()
    for k, v in {"tony.worker.instances": "3", "tony.worker.gpus": "1", "tony.worker.memory": "4g",
                 "tony.ps.instances": "1", "tony.db.instances": "1", "tony.dbloader.instances": "1",
                 K.APPLICATION_PREPARE_STAGE: "dbloader,db", K.APPLICATION_TRAINING_STAGE: "ps,worker"}.items():
        c.set(k, v)
    reqs = U.parse_container_requests(c)
    assert set(reqs) == {"worker", "ps", "db", "dbloader"}
    assert reqs["worker"].num_instances == 3 and reqs["worker"].memory_mb == 4096 and reqs["worker"].gpus == 1
    assert sorted(reqs["worker"].depends_on) == ["db", "dbloader"]
    assert reqs["db"].depends_on == []
    assert len({r.priority for r in reqs.values()}) == 4


def test_stage_auto_fill_and_integrity():
    prep, train = [], ["worker"]
    U.ensure_staged_tasks_integrity(prep, train, ["worker", "ps"])
    assert prep == ["ps"]
    with pytest.raises(ValueError):
        U.ensure_staged_tasks_integrity(["a"], ["b"], ["a", "b", "c"])


def test_construct_tf_config_evaluator_filtering():
    spec = json.dumps({"chief": ["h:1"], "worker": ["h:2"], "evaluator": ["h:3"], "tensorboard": ["h:4"]})
    w = json.loads(U.construct_tf_config(spec, "worker", 0))
    assert "evaluator" not in w["cluster"] and "tensorboard" not in w["cluster"]
    assert w["task"] == {"type": "worker", "index": 0}
    e = json.loads(U.construct_tf_config(spec, "evaluator", 0))
    assert "evaluator" in e["cluster"] and "tensorboard" not in e["cluster"]


def test_execute_shell_exit_codes():
    assert U.execute_shell("exit 3") == 3
    assert U.execute_shell("definitely_not_a_command_xyz") == 127
    t0 = time.time()
    U.execute_shell("sleep 5", timeout_ms=200)
    assert time.time() - t0 < 3


def test_job_type_helpers():
    c = Configuration()
    c.set(K.UNTRACKED_JOBTYPES, "ps,driver")
    assert U.is_untracked_job_type("driver", c)
    assert U.is_sidecar_job_type("tensorboard", c)
    assert not U.is_job_type_monitored("ps", c)
    assert U.is_job_type_monitored("worker", c)


# -- resources (TestLocalizableResource) ----------------------------------------------------------
def test_localizable_resource_parsing(tmp_path):
    from tony_amd.utils.resources import LocalizableResource, ResourceParseError, localize_all

    z = os.path.join(FIX, "test.zip")
    r = LocalizableResource.parse(f"{z}::test20.zip")
    assert r.localized_name == "test20.zip" and not r.is_archive
    r = LocalizableResource.parse(f"{z}#archive")
    assert r.is_archive and r.localized_name == "test.zip"
    r = LocalizableResource.parse(f"{z}::alias#archive")
    assert r.is_archive and r.localized_name == "alias"
    with pytest.raises(ResourceParseError):
        LocalizableResource.parse(f"{z}::a::b")
    out = localize_all([f"{z}::x.zip", f"{z}#archive", os.path.join(FIX, "libdir")], str(tmp_path))
    assert (tmp_path / "x.zip").is_file() and (tmp_path / "test.zip" / "123.xml").is_file()
    assert (tmp_path / "a.jar").is_file() and len(out) == 4


# -- session / scheduler / monitor ------------------------------------------------------------------
def _session(conf_kv):
    from tony_amd.cluster.session import TonySession

    c = Configuration()
    for k, v in conf_kv.items():
        c.set(k, v)
    return TonySession(c)


def test_session_tracked_accounting_and_chief():
    s = _session({"tony.worker.instances": "2", "tony.ps.instances": "1", "tony.tensorboard.instances": "1"})
    assert s.total_tasks() == 4 and s.total_tracked_tasks() == 2
    assert s.is_chief("worker", "0") and not s.is_chief("worker", "1")
    s2 = _session({"tony.chief.instances": "1", "tony.worker.instances": "1"})
    assert s2.is_chief("chief", "0") and not s2.is_chief("worker", "0")


def test_session_final_status_policies():
    from tony_amd.cluster.session import KILLED_BY_AM, FinalStatus, TaskStatus

    s = _session({"tony.worker.instances": "3", "tony.ps.instances": "1"})
    tasks = [s.init_task("worker") for _ in range(3)] + [s.init_task("ps")]
    s.on_task_completed("worker", "1", 1)          # non-chief failure: keep training
    assert not s.training_finished
    s.on_task_completed("worker", "0", 0)
    s.on_task_completed("worker", "2", 0)
    s.on_task_completed("ps", "0", KILLED_BY_AM)
    assert tasks[3].info.status == TaskStatus.FINISHED
    s.update_session_status()
    assert s.final_status == FinalStatus.SUCCEEDED    # some non-chief worker failures still succeed
    s = _session({"tony.worker.instances": "2"})
    [s.init_task("worker") for _ in range(2)]
    s.on_task_completed("worker", "0", 2)          # chief failure short-circuits
    assert s.training_finished and s.final_status == FinalStatus.FAILED
    s = _session({"tony.worker.instances": "2", K.FAIL_ON_WORKER_FAILURE_ENABLED: "true"})
    [s.init_task("worker") for _ in range(2)]
    s.on_task_completed("worker", "1", 1)
    assert s.training_finished
    s = _session({"tony.worker.instances": "2", "tony.ps.instances": "1"})
    [s.init_task("worker") for _ in range(2)] + [s.init_task("ps")]
    s.on_task_completed("ps", "0", 1)              # stop-on-failure job type (default: ps)
    assert s.training_finished


def test_session_all_workers_failed_fails():
    from tony_amd.cluster.session import FinalStatus

    s = _session({"tony.worker.instances": "2", "tony.chief.instances": "1"})
    s.init_task("chief")
    [s.init_task("worker") for _ in range(2)]
    s.on_task_completed("chief", "0", 0)
    s.on_task_completed("worker", "0", 1)
    s.on_task_completed("worker", "1", 1)
    s.update_session_status()
    assert s.final_status == FinalStatus.SUCCEEDED    # 2 of 3 tracked failed, chief ok
    s = _session({"tony.worker.instances": "2"})
    [s.init_task("worker") for _ in range(2)]
    s.on_task_completed("worker", "1", 1)
    s.on_task_completed("worker", "0", 1)
    s.update_session_status()
    assert s.final_status == FinalStatus.FAILED


def test_task_status_first_verdict_wins():
    s = _session({"tony.worker.instances": "1"})
    t = s.init_task("worker")
    t.set_exit_status(0)
    t.set_exit_status(1)
    assert t.exit_status == 0


def test_scheduler_dag_detection_and_countdown():
    from tony_amd.cluster.scheduler import TaskScheduler, is_dag

    a = U.JobContainerRequest("a", 1, 1, 1, 0, 0, None, ["b"])
    b = U.JobContainerRequest("b", 1, 1, 1, 0, 1, None, ["a"])
    assert not is_dag([a, b])
    s = _session({"tony.worker.instances": "2", "tony.ps.instances": "1", "tony.db.instances": "2",
                  K.APPLICATION_PREPARE_STAGE: "db", K.APPLICATION_TRAINING_STAGE: "ps,worker"})
    launched = []
    sch = TaskScheduler(s, lambda r: launched.append(r.job_name))
    sch.schedule_tasks()
    assert launched == ["db"] and s.num_expected_tasks == 2
    sch.register_dependency_completed("db")
    assert launched == ["db"]
    sch.register_dependency_completed("db")
    assert sorted(launched) == ["db", "ps", "worker"] and s.num_expected_tasks == 5


def test_heartbeat_monitor_expiry_and_unregister():
    from tony_amd.cluster.liveliness import HeartbeatMonitor

    dead = []
    m = HeartbeatMonitor(20, 3, dead.append)
    m.start()
    m.register("worker:0")
    m.register("worker:1")
    m.unregister("worker:1")
    for _ in range(10):
        time.sleep(0.01)
    time.sleep(0.2)
    m.stop()
    assert dead == ["worker:0"]


def test_task_monitor_running_stats():
    from tony_amd.agent.monitor import RunningStat, TaskMonitor

    r = RunningStat()
    for v in (1, 5, 3):
        r.add(v)
    assert r.max == 5 and r.avg == 3
    pushed = []
    m = TaskMonitor(lambda: os.getpid(), [], 10, pushed.append, gpu_metrics=False)
    m.refresh()
    assert m.metrics()[C.MAX_MEMORY_BYTES] > 0


# -- ports (TestPortAllocation) ---------------------------------------------------------------
def test_port_reservation_reuse_semantics():
    from tony_amd import native

    a = native.PortReservation(0, reuse_port=True)
    b = native.PortReservation(a.port, reuse_port=True)    # SO_REUSEPORT lets the user process bind too
    assert a.port == b.port
    c = native.PortReservation(0, reuse_port=False)
    with pytest.raises(OSError):
        native.PortReservation(c.port, reuse_port=False)
    c.release()
    d = native.PortReservation(c.port, reuse_port=False)   # released -> free again
    for r in (a, b, d):
        r.release()


def test_native_spawn_new_session(tmp_path):
    from tony_amd import native

    out = tmp_path / "o"
    pid = native.spawn(["bash", "-c", "echo $PWD; exit 7"], dict(os.environ), cwd=str(tmp_path), stdout=str(out))
    assert os.getpgid(pid) == pid
    _, st = os.waitpid(pid, 0)
    assert os.WEXITSTATUS(st) == 7 and out.read_text().strip() == str(tmp_path)


# -- horovod (TestHorovodRuntime / TestHorovodDriver) ----------------------------------------------
def test_horovod_slot_plan_and_worker_list():
    from tony_amd.horovod import HorovodClusterSpec, host_assignments, parse_hosts
    from tony_amd.runtime.horovod import HorovodAM

    slots = host_assignments(parse_hosts("h1:2,h2:1"))
    assert [(s.hostname, s.rank, s.localRank, s.crossRank, s.crossSize) for s in slots] == \
        [("h1", 0, 0, 0, 2), ("h1", 1, 1, 0, 1), ("h2", 2, 0, 1, 2)]
    s = _session({"tony.worker.instances": "3", "tony.driver.instances": "1"})
    for i, host in enumerate(["h1", "h1", "h2"]):
        t = s.init_task("worker")
        t.set_host_port(f"{host}:{100 + i}")
    d = s.init_task("driver")
    d.set_host_port("h1:99")
    am = HorovodAM()
    am.set_session(s)
    same = []
    wl = am.build_worker_list("h1", same)
    assert sorted(wl.split(",")) == ["h1:2", "h2:1"] and sorted(same) == [0, 1]
    spec = HorovodClusterSpec([], "9999", "h1", [0, 1]).to_json()
    assert HorovodClusterSpec.from_json(spec).sameHostTaskIndexList == [0, 1]


def test_horovod_validate_conf_injects_driver():
    from tony_amd.runtime.horovod import HorovodAM

    c = Configuration()
    am = HorovodAM()
    assert am.validate_and_update_config(c)
    assert c.get("tony.driver.instances") == "1" and c.get(K.UNTRACKED_JOBTYPES) == "driver"
    c2 = Configuration()
    c2.set("tony.driver.memory", "4g")
    assert not HorovodAM().validate_and_update_config(c2)    # user driver keys are illegal
    c3 = Configuration()
    c3.set(K.HOROVOD_DRIVER_DEBUG_MODE, "true")
    assert not HorovodAM().validate_and_update_config(c3)    # debug mode needs tony.driver.command


def test_horovod_driver_test_mode_port_file():
    from tony_amd.horovod.driver import HorovodDriver

    d = HorovodDriver.create("localhost:2", {}, "localhost", test_mode=True)
    try:
        assert d.port == "9999" and len(d.slot_infos) == 2
        info = json.loads(d.callback_info())
        assert info["port"] == "9999" and info["host"] == "localhost"
    finally:
        d.close()
        d.wait_for(5)


def test_rendezvous_kv_server():
    from tony_amd.horovod.rendezvous import RendezvousServer, kv_get, kv_put

    srv = RendezvousServer("127.0.0.1")
    port = srv.start()
    kv_put("127.0.0.1", port, "scope/k", b"v1")
    assert kv_get("127.0.0.1", port, "scope/k", 2) == b"v1"
    with pytest.raises(TimeoutError):
        kv_get("127.0.0.1", port, "scope/missing", 0.2)
    srv.stop()


# -- client helpers (TestTonyClient) -----------------------------------------------------------
def test_client_option_parsing_styles():
    from tony_amd.client.tony_client import ClientOptionError, build_task_command, parse_args

    o = parse_args(["-executes", "a.py", "--conf", "x=1", "--conf=y=2", "--shell_env", "A=B"])
    assert o["executes"] == "a.py" and o["conf"] == ["x=1", "y=2"] and o["shell_env"] == ["A=B"]
    with pytest.raises(ClientOptionError):
        parse_args(["--bogus", "1"])
    assert build_task_command("v.zip", "bin/python", "a.py", "--lr 1") == "venv/bin/python a.py --lr 1"
    assert build_task_command(None, "/usr/bin/python", "a.py", None) == "/usr/bin/python a.py"


def test_client_instance_and_gpu_limits():
    from tony_amd.client.tony_client import TonyClient

    c = Configuration()
    c.set(K.AMD_FAKE_GPUS, "8")
    cl = TonyClient(c)
    assert not cl.init(["--executes", "x", "--conf", "tony.worker.instances=3", "--conf",
                        "tony.worker.max-instances=2"])
    c = Configuration()
    c.set(K.AMD_FAKE_GPUS, "8")
    assert not TonyClient(c).init(["--executes", "x", "--conf", "tony.worker.instances=3", "--conf",
                                   "tony.task.max-total-instances=2"])
    c = Configuration()
    c.set(K.AMD_FAKE_GPUS, "8")
    assert not TonyClient(c).init(["--executes", "x", "--conf", "tony.worker.instances=4", "--conf",
                                   "tony.worker.gpus=2", "--conf", "tony.task.max-total-gpus=4"])
    c = Configuration()
    c.set(K.AMD_FAKE_GPUS, "8")
    assert TonyClient(c).init(["--executes", "x", "--conf", "tony.worker.instances=4", "--conf",
                               "tony.worker.gpus=2"])


def test_merge_tasks_and_sort_by_attention():
    from tony_amd.client.tony_client import merge_tasks
    from tony_amd.cluster.session import TaskInfo, TaskStatus

    ts = [TaskInfo("ps", "0"), TaskInfo("ps", "1"), TaskInfo("worker", "0"), TaskInfo("worker", "1")]
    assert merge_tasks(ts) == "ps [0, 1] worker [0, 1] "
    infos = [TaskInfo("w", "0", status=TaskStatus.RUNNING), TaskInfo("w", "1", status=TaskStatus.FAILED),
             TaskInfo("w", "2", status=TaskStatus.SUCCEEDED)]
    assert [t.status for t in sorted(infos, key=TaskInfo.sort_key)] == \
        [TaskStatus.FAILED, TaskStatus.SUCCEEDED, TaskStatus.RUNNING]


# -- events / history (TestEventHandler, TestParserUtils, TestHistoryFileUtils) ----------------------
def test_avro_roundtrip_all_types():
    from tony_amd.events.avro import DataFileReader, DataFileWriter, Schema

    sch = Schema({"type": "record", "name": "R", "fields": [
        {"name": "b", "type": "boolean"}, {"name": "i", "type": "int"}, {"name": "l", "type": "long"},
        {"name": "f", "type": "float"}, {"name": "d", "type": "double"}, {"name": "s", "type": "string"},
        {"name": "by", "type": "bytes"}, {"name": "u", "type": ["null", "string"]},
        {"name": "e", "type": {"type": "enum", "name": "E", "symbols": ["A", "B"]}},
        {"name": "a", "type": {"type": "array", "items": "long"}},
        {"name": "m", "type": {"type": "map", "values": "string"}}]})
    recs = [{"b": True, "i": -5, "l": 2 ** 40, "f": 1.5, "d": -2.25, "s": "héllo", "by": b"\x00\x01", "u": None,
             "e": "B", "a": [1, -2, 3], "m": {"k": "v"}},
            {"b": False, "i": 0, "l": -1, "f": 0.0, "d": 0.0, "s": "", "by": b"", "u": "x", "e": "A", "a": [],
             "m": {}}]
    for codec in ("null", "deflate"):
        buf = io.BytesIO()
        w = DataFileWriter(buf, sch, codec=codec)
        for r in recs:
            w.append(r)
        w.flush()
        buf.seek(0)
        assert list(DataFileReader(buf)) == recs


def test_reads_tony_written_jhist_fixture():
    """A .jhist written by TonY's Java Avro writer (tony-portal example history) parses."""
    from tony_amd.events.avro import read_all

    p = ("/root/reference/tony-portal/example/tony-history/finished/2019/01/08/application_123456_0001/"
         "application_123456_0001-1546910478024-1546910517303-testuser-SUCCEEDED.jhist")
    if not os.path.exists(p):
        pytest.skip("reference tree not mounted")
    ev = read_all(p)
    assert ev[0]["type"] == "APPLICATION_INITED" and ev[-1]["type"] == "APPLICATION_FINISHED"


def test_event_handler_roundtrip(tmp_path):
    from tony_amd.events import schema as S
    from tony_amd.events.handler import EventHandler
    from tony_amd.events.history import (JobMetadata, is_valid_hist_file_name, map_event_to_job_log,
                                         parse_config, parse_events, parse_metadata)

    d = tmp_path / "application_1_0001"
    h = EventHandler()
    md = JobMetadata("application_1_0001", 1000, user="u")
    assert h.set_up(str(d), md)
    h.start()
    assert h.in_progress_file.endswith(".jhist.inprogress")
    h.emit(S.application_inited("application_1_0001", 2, "host", "c0"))
    h.emit(S.task_started("worker", 0, "host", "c1"))
    h.emit(S.task_finished("worker", 0, "SUCCEEDED", [{"name": "m", "value": 1.0}]))
    md.completed, md.status = 2000, "SUCCEEDED"
    f = h.stop(str(d), md)
    assert os.path.basename(f) == "application_1_0001-1000-2000-u-SUCCEEDED.jhist"
    assert is_valid_hist_file_name(os.path.basename(f))
    assert parse_metadata(str(d)).status == "SUCCEEDED"
    evs = parse_events(str(d))
    assert [e.type for e in evs] == ["APPLICATION_INITED", "TASK_STARTED", "TASK_FINISHED"]
    assert map_event_to_job_log(evs[1]).container_id == "c1"
    (d / "tony-final.xml").write_text(Configuration(load_defaults=False).to_xml())
    assert parse_config(str(d)) == []


def test_hist_file_name_validation():
    from tony_amd.events.history import is_valid_hist_file_name

    assert is_valid_hist_file_name("application_1_2-123-user.jhist.inprogress")
    assert is_valid_hist_file_name("application_1_2-123-456-user-FAILED.jhist")
    assert not is_valid_hist_file_name("application_1_2-123-456-USER-FAILED.jhist")
    assert not is_valid_hist_file_name("job-1-2.jhist")


def test_tony_final_xml_fixture_with_missing_subelements():
    """TTR/application_123_456/tony-final.xml has properties missing name/value."""
    from tony_amd.events.history import parse_config

    d = "/root/reference/tony-core/src/test/resources/application_123_456"
    if not os.path.exists(d):
        pytest.skip("reference tree not mounted")
    cfgs = parse_config(d)
    assert all(c.name and c.value is not None for c in cfgs)


# -- rpc ---------------------------------------------------------------------------------------
def test_rpc_token_auth_and_roundtrip():
    import grpc

    from tony_amd.rpc import protocol as P
    from tony_amd.rpc.client import RpcClient
    from tony_amd.rpc.server import RpcServer

    calls = []
    handlers = {m: (lambda r, m=m: calls.append(m) or P.MESSAGES[P.METHODS[m][1]]()) for m in P.METHODS}
    handlers["registerWorkerSpec"] = lambda r: P.RegisterWorkerSpecResponseProto(spec=r.spec + "!")
    srv = RpcServer(handlers, token="s3cret").start()
    try:
        ok = RpcClient("127.0.0.1", srv.port, "s3cret", retries=0)
        assert ok.register_worker_spec("worker:0", "h:1") == "h:1!"
        ok.task_executor_heartbeat("worker:0")
        bad = RpcClient("127.0.0.1", srv.port, "wrong", retries=0)
        with pytest.raises(grpc.RpcError) as e:
            bad.get_cluster_spec()
        assert e.value.code() == grpc.StatusCode.UNAUTHENTICATED
    finally:
        srv.stop(0)


# -- GPU ordinal mapping and CPU slicing (amd-smi index != HIP ordinal) -------------------
def test_hip_ordinals_follow_kfd_order_by_bdf():
    from tony_amd.gpu.inventory import hip_ordinals
    from tony_amd.native import GpuDevice

    # amd-smi lists the GPUs in one order, KFD (= HIP) in another: map by BDF
    smi = [GpuDevice(i, bdf=b, numa_node=i // 4) for i, b in
           enumerate(["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0",
                      "0000:85:00.0", "0000:95:00.0", "0000:e5:00.0", "0000:f5:00.0"])]
    kfd = ["0000:15:00.0", "0000:05:00.0", "0000:75:00.0", "0000:65:00.0",
           "0000:95:00.0", "0000:85:00.0", "0000:f5:00.0", "0000:e5:00.0"]
    m = hip_ordinals(smi, kfd)
    assert m == {0: 1, 1: 0, 2: 3, 3: 2, 4: 5, 5: 4, 6: 7, 7: 6}
    # amd-smi may print the BDF without the domain / function
    assert hip_ordinals([GpuDevice(0, bdf="15:00.0")], kfd) == {0: 0}
    with pytest.raises(RuntimeError, match="not among the HIP-visible"):
        hip_ordinals([GpuDevice(0, bdf="0000:aa:00.0")], kfd)
    with pytest.raises(RuntimeError, match="no PCI BDF"):
        hip_ordinals([GpuDevice(0)], kfd)
    fake = [GpuDevice(i, bdf=f"fake:{i:02x}", fake=True) for i in range(3)]
    assert hip_ordinals(fake, kfd) == {0: 0, 1: 1, 2: 2}


def test_kfd_bdfs_read_in_node_order(tmp_path):
    from tony_amd.gpu.inventory import kfd_gpu_bdfs

    for node, (simd, loc) in {"0": (0, 0), "2": (304, 0x7500), "10": (304, 0x0500), "1": (304, 0x1508)}.items():
        d = tmp_path / node
        d.mkdir()
        (d / "properties").write_text(f"simd_count {simd}\nlocation_id {loc}\ndomain 0\nnuma_node 0\n")
    # node ids sort numerically (1, 2, 10); the CPU node (simd 0) is skipped
    assert kfd_gpu_bdfs(str(tmp_path)) == ["0000:15:01.0", "0000:75:00.0", "0000:05:00.0"]


def test_verify_visible_device_detects_mispinning(monkeypatch):
    from types import SimpleNamespace

    import torch

    from tony_amd.gpu.inventory import verify_visible_device

    props = SimpleNamespace(pci_domain_id=0, pci_bus_id=0x75, pci_device_id=0)
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")
    monkeypatch.setenv("TONY_GPU_BDFS", "0000:75:00.0")
    assert verify_visible_device(0) == "0000:75:00.0"
    monkeypatch.setenv("TONY_GPU_BDFS", "0000:65:00.0")
    with pytest.raises(RuntimeError, match="does not select the allocated GPU"):
        verify_visible_device(0)


def test_allocator_slices_numa_cpus_by_vcores():
    from tony_amd.gpu.inventory import GpuAllocator
    from tony_amd.native import GpuDevice

    devs = [GpuDevice(i, bdf=f"fake:{i}", numa_node=i // 4, fake=True) for i in range(8)]
    cpus = {0: list(range(0, 16)), 1: list(range(16, 32))}
    a = GpuAllocator(devs, cpus_of_node=lambda n: cpus[n])
    s1 = a.allocate("w0", 1, vcores=4)
    s2 = a.allocate("w1", 1, vcores=4)
    assert s1.numa_node == s2.numa_node == 0
    assert len(s1.cpus) == 4 and len(s2.cpus) == 4 and not set(s1.cpus) & set(s2.cpus)
    whole = a.allocate("w2", 1, vcores=0)
    assert whole.cpus == cpus[0]
    a.release("w0")
    s3 = a.allocate("w3", 1, vcores=4)
    assert s3.cpus == s1.cpus                        # released CPUs are handed out again
    big = a.allocate("w4", 1, vcores=12)             # only 4 unowned left on node 0: oversubscribe
    assert len(big.cpus) == 12


def test_task_monitor_gpu_fault_and_xgmi_rates(monkeypatch):
    """New uncorrectable ECC errors on a pinned GPU call the agent's fault handler once (it stops the
    task); xGMI GB/s come from amd-smi's accumulated per-link KB counters."""
    from tony_amd import constants as C
    from tony_amd import native
    from tony_amd.agent import monitor as M

    state = {"ecc": 0, "rd": 0, "t": 100.0}

    def sample(_gpu):
        return native.GpuSample(50, 10, 1000, 2000, 500.0, 60.0, 0, state["ecc"], state["rd"], state["rd"] // 2, 64)

    monkeypatch.setattr(native, "smi_sample", sample)
    monkeypatch.setattr(M.time, "monotonic", lambda: state["t"])
    faults = []
    mon = M.TaskMonitor(lambda: None, [0], 1000, lambda m: None, True, on_fault=faults.append)
    mon.refresh()
    state["rd"], state["t"] = 2_000_000, 101.0   # 2 GB read over 1 s
    mon.refresh()
    assert faults == [] and mon.fault is None
    state["ecc"], state["t"] = 3, 102.0
    mon.refresh()
    mon.refresh()
    assert len(faults) == 1 and "uncorrectable ECC" in faults[0] and mon.fault_code == C.EXIT_GPU_FAULT
    m = mon.metrics()
    assert m[C.GPU_ECC_UNCORRECTABLE] == 3.0
    assert m[C.MAX_XGMI_READ_GBPS] == pytest.approx(2.0) and m[C.MAX_XGMI_WRITE_GBPS] == pytest.approx(1.0)


def test_task_monitor_memory_limit(monkeypatch):
    from tony_amd import constants as C
    from tony_amd.agent import monitor as M

    monkeypatch.setattr(M, "tree_rss_bytes", lambda pid: 300 << 20)
    faults = []
    mon = M.TaskMonitor(lambda: 1234, [], 1000, lambda m: None, False, on_fault=faults.append,
                        memory_limit_bytes=256 << 20)
    mon.refresh()
    assert len(faults) == 1 and "memory limit" in faults[0] and mon.fault_code == C.EXIT_MEMORY_LIMIT


def test_flat_sgd_resync_reseeds_master_from_changed_compute_copy():
    """FlatSGD(resync=True): elements of the bf16 compute copy changed outside the optimizer re-seed the
    fp32 master before the update (the CPU form of csrc/optim.hip's resync); untouched ones keep it."""
    import torch

    from tony_amd.ops.optim import FlatSGD

    master = torch.linspace(-1, 1, 16)
    opt = FlatSGD(master.clone(), lr=0.5, momentum=0.0, resync=True)
    cur = opt.w.to(torch.bfloat16)
    cur[3] = 7.0  # e.g. load_state_dict into the module
    g = torch.ones(16)
    before = opt.w.clone()
    opt.step(g, out_bf16=cur)
    assert opt.w[3].item() == 7.0 - 0.5
    keep = [i for i in range(16) if i != 3]
    assert torch.allclose(opt.w[keep], before[keep] - 0.5)


def test_gpu_pinning_env_modes():
    """what each visible-devices mode exports.  none keeps every GPU visible for RCCL P2P /
    peer-memory mapping and names the task's GPUs by HIP ordinal; hip / rocr hide the rest (auto, the
    default, resolves to one of them per job: resolve_visible_mode)."""
    from tony_amd.cluster.coordinator import gpu_pinning_env
    from tony_amd.conf import Configuration
    from tony_amd.conf import keys as K
    from tony_amd.native import GpuDevice

    assert Configuration().get(K.AMD_VISIBLE_DEVICES_MODE) == "auto"
    devs = [GpuDevice(i, bdf=f"0000:{0x10 * (i + 1):02x}:00.0", numa_node=0, fake=True) for i in range(8)]
    hip_ord = {0: 3, 1: 2, 2: 1, 3: 0, 4: 4, 5: 5, 6: 6, 7: 7}  # amd-smi order != HIP order
    e = gpu_pinning_env("none", [1], hip_ord, devs)
    assert e["TONY_HIP_ORDINALS"] == "2" and e["TONY_GPU_BDFS"] == "0000:20:00.0" and e["TONY_VISIBLE_MODE"] == "none"
    assert "HIP_VISIBLE_DEVICES" not in e and "ROCR_VISIBLE_DEVICES" not in e
    e = gpu_pinning_env("hip", [0, 5], hip_ord, devs)
    assert e["HIP_VISIBLE_DEVICES"] == "3,5" and "ROCR_VISIBLE_DEVICES" not in e
    e = gpu_pinning_env("rocr", [2], hip_ord, devs)
    assert e["ROCR_VISIBLE_DEVICES"] == "1" and "HIP_VISIBLE_DEVICES" not in e
    with pytest.raises(ValueError):
        gpu_pinning_env("cuda", [0], hip_ord, devs)


def test_visible_mode_auto_isolates_unless_a_peer_plane_is_configured():
    """the default (auto) keeps per-task HIP_VISIBLE_DEVICES isolation for arbitrary user
    programs and leaves every GPU visible only for jobs on a peer-mapping tony_amd data plane."""
    from tony_amd.cluster.coordinator import resolve_visible_mode
    from tony_amd.conf import Configuration

    def conf(**kv):
        c = Configuration()
        for k, v in kv.items():
            c.set(k.replace("__", "."), str(v))
        return c

    assert resolve_visible_mode(conf()) == "hip"  # a plain job
    assert resolve_visible_mode(conf(tony__application__framework="pytorch", tony__worker__instances=4)) == "hip"
    assert resolve_visible_mode(conf(tony__amd__collective="hip")) == "none"
    # an ordinary user TF PS job keeps its isolation (the ps-plane key's xgmi default alone
    # does not count); tony_amd's own PS program, or an explicit xgmi plane, maps peer GPUs
    assert resolve_visible_mode(conf(tony__ps__instances=1, tony__worker__instances=4)) == "hip"
    # only tony_amd's exact entry points count -- a user script named inception_ps.py, or one under a
    # path containing "tony_amd", keeps its isolation; the same name shipped from tony_amd/jobs (the client
    # marks that --src_dir) or named as a module / an installed path maps peer GPUs
    assert resolve_visible_mode(conf(tony__ps__instances=1, tony__worker__instances=4,
                                     tony__containers__command="python3 inception_ps.py --batch-size 32")) == "hip"
    assert resolve_visible_mode(conf(tony__ps__instances=1, tony__worker__instances=4,
                                     tony__containers__command="python3 /home/u/tony_amd_fork/train.py")) == "hip"
    assert resolve_visible_mode(conf(tony__ps__instances=1, tony__worker__instances=4,
                                     tony__containers__command="python3 inception_ps.py --batch-size 32",
                                     **{"tony__amd__src-is-tony-jobs": "true"})) == "none"
    assert resolve_visible_mode(conf(tony__ps__instances=1, tony__worker__instances=4,
                                     tony__containers__command="python3 -m tony_amd.jobs.inception_ps")) == "none"
    import tony_amd.jobs.inception_ps as ips
    assert resolve_visible_mode(conf(tony__ps__instances=1, tony__worker__instances=4,
                                     tony__containers__command=f"python3 {ips.__file__} --steps 3")) == "none"
    assert resolve_visible_mode(conf(tony__ps__instances=1, **{"tony__amd__ps-plane": "xgmi"})) == "none"
    assert resolve_visible_mode(conf(tony__ps__instances=1, **{"tony__amd__ps-plane": "rccl"})) == "hip"
    # the decision survives the round trip through tony-final.xml (sources are written and re-read)
    import tempfile

    from tony_amd.conf import keys as K

    with tempfile.TemporaryDirectory() as d:
        for c, want in ((conf(tony__ps__instances=1), "hip"),
                        (conf(tony__ps__instances=1, **{"tony__amd__ps-plane": "xgmi"}), "none")):
            path = os.path.join(d, "tony-final.xml")
            c.write_xml(path)
            back = Configuration.from_xml(path)
            assert back.get_source(K.AMD_PS_PLANE) == c.get_source(K.AMD_PS_PLANE)
            assert resolve_visible_mode(back) == want
    assert resolve_visible_mode(conf(tony__application__framework="pytorch", tony__ps__instances=1)) == "hip"
    # MXNet kvstore servers with GPU workers: the payload plane maps peer windows
    mx = dict(tony__application__framework="mxnet", tony__server__instances=1, tony__worker__gpus=1)
    assert resolve_visible_mode(conf(**mx)) == "none"
    assert resolve_visible_mode(conf(**mx, **{"tony__amd__kv-plane": "gloo"})) == "hip"
    assert resolve_visible_mode(conf(tony__application__framework="mxnet", tony__server__instances=1)) == "hip"
    for m in ("none", "hip", "rocr"):
        assert resolve_visible_mode(conf(**{"tony__amd__visible-devices-mode": m, "tony__amd__collective": "hip"})) == m
    assert Configuration().get("tony.amd.visible-devices-mode") == "auto"


def test_verify_visible_device_in_all_visible_mode(monkeypatch):
    """visible-devices-mode none: the task's device is TONY_HIP_ORDINALS[0]; picking any other ordinal, or
    an ordinal whose BDF is not the allocated GPU's, raises."""
    from types import SimpleNamespace

    import torch

    from tony_amd.gpu.inventory import verify_visible_device

    props = {2: SimpleNamespace(pci_domain_id=0, pci_bus_id=0x20, pci_device_id=0),
             5: SimpleNamespace(pci_domain_id=0, pci_bus_id=0x60, pci_device_id=0)}
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props[i])
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.setenv("TONY_VISIBLE_MODE", "none")
    monkeypatch.setenv("TONY_HIP_ORDINALS", "2")
    monkeypatch.setenv("TONY_GPU_BDFS", "0000:20:00.0")
    assert verify_visible_device(2) == "0000:20:00.0"
    with pytest.raises(RuntimeError, match="not among this task's GPUs"):
        verify_visible_device(5)
    monkeypatch.setenv("TONY_GPU_BDFS", "0000:21:00.0")
    with pytest.raises(RuntimeError, match="does not select the allocated GPU"):
        verify_visible_device(2)


def test_gpu_task_memory_sized_when_left_at_default():
    """a GPU jobtype whose memory is the 2g default gets 32g per GPU (a PyTorch-ROCm rank alone
    exceeds 2 GB RSS and the agent enforces the limit); explicit values and CPU jobtypes are untouched."""
    from tony_amd.conf import Configuration
    from tony_amd.utils import core as U

    c = Configuration()
    c.set("tony.worker.instances", "2")
    c.set("tony.worker.gpus", "2")
    c.set("tony.ps.instances", "1")
    c.set("tony.evaluator.instances", "1")
    c.set("tony.evaluator.gpus", "1")
    c.set("tony.evaluator.memory", "8g")
    changed = U.size_gpu_task_memory(c)
    # the 0-GPU ps sits on a worker's GPU (tony.amd.ps-share-gpu): a GPU process, sized as one GPU
    assert changed == {"worker": 65536, "ps": 32768}
    reqs = U.parse_container_requests(c)
    assert reqs["worker"].memory_mb == 65536 and reqs["ps"].memory_mb == 32768 and reqs["evaluator"].memory_mb == 8192
    c.set("tony.amd.ps-share-gpu", "false")
    c.set("tony.ps.memory", "2g", source="tony-default.xml")
    assert "ps" not in U.size_gpu_task_memory(c)
    assert "<name>tony.worker.memory</name>" in c.to_xml()


def test_ps_checkpoint_without_layout_is_refused():
    """a PS shard checkpoint without its 'layout' record (older format, shard order
    unverifiable) must be refused, not loaded into a possibly different bucket order."""
    import torch

    from tony_amd.parallel.ps import ParameterServer

    net = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 4))
    ps = ParameterServer(net, optimizer="sgd", lr=0.1, dtype=torch.float32, device="cpu")
    sd = ps.state_dict()
    ps.load_state_dict(sd)  # round trip with the layout record works
    del sd["layout"]
    with pytest.raises(ValueError, match="no 'layout' record"):
        ps.load_state_dict(sd)
    sd["layout"] = dict(ps.layout(), world=2)
    with pytest.raises(ValueError, match="does not match"):
        ps.load_state_dict(sd)


def test_ps_shares_a_worker_gpu_policy_and_allocator():
    """TonY's default 0-GPU ps of a GPU TensorFlow job is placed on a worker's GPU, shared
    (the GPU stays owned by the worker; the ps is recorded as a sharer and released with its task)."""
    from tony_amd.conf import Configuration
    from tony_amd.gpu.inventory import GpuAllocator, discover
    from tony_amd.utils import core as U

    c = Configuration()
    c.set("tony.ps.instances", "1")
    c.set("tony.worker.instances", "4")
    c.set("tony.worker.gpus", "1")
    assert U.ps_shares_worker_gpu(c)
    for k, v in (("tony.amd.ps-share-gpu", "false"), ("tony.ps.gpus", "1"), ("tony.application.framework", "pytorch"),
                 ("tony.worker.gpus", "0")):
        d = Configuration()
        for kk, vv in (("tony.ps.instances", "1"), ("tony.worker.instances", "4"), ("tony.worker.gpus", "1")):
            d.set(kk, vv)
        d.set(k, v)
        assert not U.ps_shares_worker_gpu(d), k
    a = GpuAllocator(discover(4))
    w0 = a.allocate("worker:0", 1)
    assert w0.gpus == [0]
    s = a.share("ps:0", w0.gpus[0])
    assert s.gpus == [0] and a.owners() == {0: "worker:0"} and a.sharers() == {0: ["ps:0"]}
    assert a.free_count() == 3  # sharing takes no GPU from the free list
    a.release("ps:0")
    assert a.sharers() == {} and a.owners() == {0: "worker:0"}


def test_shared_gpu_stays_allocated_until_its_last_sharer_leaves():
    """a worker that owns a GPU exits while the ps sharing it still runs -- the GPU must not
    go back to the free list (the next allocation would land on a busy GPU) until the ps releases it."""
    from tony_amd.gpu.inventory import GpuAllocator, discover

    a = GpuAllocator(discover(2))
    w0 = a.allocate("worker:0", 1)
    a.share("ps:0", w0.gpus[0])
    a.release("worker:0")
    assert a.owners() == {} and a.sharers() == {0: ["ps:0"]}
    assert a.free_count() == 1
    nxt = a.allocate("worker:1", 1)
    assert nxt.gpus == [1]          # not the GPU the ps is still on
    assert a.allocate("worker:2", 1) is None
    a.release("ps:0")
    assert a.free_count() == 1 and a.allocate("worker:2", 1).gpus == [0]
    # owner leaving after its sharer: freed at once
    b = GpuAllocator(discover(1))
    g = b.allocate("worker:0", 1).gpus[0]
    b.share("ps:0", g)
    b.release("ps:0")
    b.release("worker:0")
    assert b.free_count() == 1
