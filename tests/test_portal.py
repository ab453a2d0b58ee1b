"""Portal + history maintenance (tony-portal TestHistoryFileMover / TestHistoryFilePurger /
controllers), and the notebook proxy."""
import datetime as dt
import json
import os
import shutil
import socket
import subprocess
import sys
import threading
import urllib.request

import pytest

from tony_amd.events import schema as S
from tony_amd.events.handler import EventHandler
from tony_amd.events.history import JobMetadata
from tony_amd.portal import (CacheWrapper, HistoryFileMover, HistoryFilePurger, PortalServer, purge_finished_dir,
                             purge_intermediate_dir)
from tony_amd.portal.history import killed_file_name, owner_alive, write_owner

REF_HIST = "/root/reference/tony-portal/example/tony-history"


def _job(inter, app_id, started, completed=None, status=None, user="alice"):
    d = os.path.join(inter, app_id)
    h = EventHandler()
    md = JobMetadata(app_id, started, user=user)
    h.set_up(d, md)
    h.start()
    h.emit(S.application_inited(app_id, 1, "host1", "c0"))
    h.emit(S.task_started("worker", 0, "host1", "c1"))
    if completed is None:
        h._stopped.set()
        h._thread.join()
        h._writer.close()
        return d
    md.completed, md.status = completed, status
    h.stop(d, md)
    return d


def test_killed_file_name():
    assert os.path.basename(killed_file_name("/x/application_1_1-100-bob.jhist.inprogress", 5)) == \
        "application_1_1-100-5-bob-KILLED.jhist"


def test_mover_moves_finished_and_marks_dead_owner_killed(tmp_path):
    inter, fin = str(tmp_path / "intermediate"), str(tmp_path / "finished")
    ts = int(dt.datetime(2024, 3, 5, 12, tzinfo=dt.timezone.utc).timestamp() * 1000)
    _job(inter, "application_1_0001", ts - 1000, ts, "SUCCEEDED")
    dead = _job(inter, "application_1_0002", ts)
    live = _job(inter, "application_1_0003", ts)
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    p.wait()
    with open(os.path.join(dead, "coordinator.owner"), "w") as f:
        json.dump({"host": socket.gethostname(), "pid": p.pid, "start": 0}, f)
    write_owner(live)
    assert owner_alive(live) is True and owner_alive(dead) is False
    moved = HistoryFileMover(inter, fin).run_once()
    assert os.path.isdir(os.path.join(fin, "2024", "03", "05", "application_1_0001"))
    assert len(moved) == 2                                           # finished + the killed one
    killed = [m for m in moved if m.endswith("application_1_0002")][0]
    assert any(f.endswith("-alice-KILLED.jhist") for f in os.listdir(killed))
    assert os.listdir(inter) == ["application_1_0003"]              # still running: untouched


def test_purger_finished_and_intermediate(tmp_path):
    fin, inter = tmp_path / "finished", tmp_path / "intermediate"
    for p in ("2018/05/01/a", "2019/01/07/b", "2019/01/08/c", "2019/02/01/d", "2020/01/01/e"):
        (fin / p).mkdir(parents=True)
    old, new = inter / "application_1_1", inter / "application_1_2"
    old.mkdir(parents=True)
    new.mkdir()
    t = dt.datetime(2019, 1, 1).timestamp()
    os.utime(old, (t, t))
    cutoff = dt.date(2019, 1, 8)
    gone = purge_finished_dir(str(fin), cutoff)
    assert not (fin / "2018").exists() and not (fin / "2019/01/07").exists()
    assert (fin / "2019/01/08/c").exists() and (fin / "2019/02/01/d").exists() and (fin / "2020").exists()
    assert len(gone) == 2
    assert purge_intermediate_dir(str(inter), cutoff) == [str(old)]
    assert new.exists()
    assert HistoryFilePurger(str(inter), str(fin), 10 ** 10).run_once() == []   # cutoff centuries ago
    assert len(HistoryFilePurger(str(inter), str(fin), 0).run_once()) == 2      # cutoff today: years 2019, 2020
    assert new.exists()


@pytest.fixture
def portal(tmp_path):
    inter, fin = str(tmp_path / "intermediate"), str(tmp_path / "finished")
    os.makedirs(inter)
    if os.path.isdir(REF_HIST):
        shutil.copytree(os.path.join(REF_HIST, "finished"), fin)
    d = _job(inter, "application_7_0001", 1000, 5000, "FAILED", user="bob")
    write_owner(d, str(tmp_path / "staging" / "application_7_0001"))
    (tmp_path / "x.xml").write_text("")
    shutil.copy(os.path.join(os.path.dirname(__file__), "..", "tony_amd", "conf", "tony-default.xml"),
                os.path.join(d, "tony-final.xml"))
    srv = PortalServer(CacheWrapper(inter, fin, 10))
    srv.start()
    yield f"http://127.0.0.1:{srv.port}", tmp_path
    srv.stop()


def _get(url):
    return json.loads(urllib.request.urlopen(url, timeout=10).read())


def test_portal_pages(portal):
    base, tmp = portal
    jobs = _get(base + "/?format=json")
    ids = [j["id"] for j in jobs]
    assert "application_7_0001" in ids
    if os.path.isdir(REF_HIST):  # the TonY-written example history renders too
        assert ids[0] == "application_123456_0001"   # completed desc
        ev = _get(base + "/jobs/application_123456_0001?format=json")
        assert ev[0]["type"] == "APPLICATION_INITED"
        assert any(c["name"] == "tony.worker.instances" for c in _get(base + "/config/application_123456_0001"
                                                                        "?format=json"))
    cfg = _get(base + "/config/application_7_0001?format=json")
    assert any(c["name"] == "tony.application.framework" for c in cfg)
    logs = _get(base + "/logs/application_7_0001?format=json")
    assert {lg["container_id"] for lg in logs} == {"c0", "c1"}
    assert logs[0]["log_link"].startswith(str(tmp / "staging" / "application_7_0001" / "logs"))
    page = urllib.request.urlopen(base + "/", timeout=10).read().decode()
    assert "application_7_0001" in page and "<table>" in page
    with pytest.raises(urllib.error.HTTPError):
        urllib.request.urlopen(base + "/jobs/application_9_9", timeout=10)


def test_proxy_server_relays_bytes():
    from tony_amd.proxy import ProxyServer

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)

    def echo():
        c, _ = srv.accept()
        while True:
            b = c.recv(65536)
            if not b:
                break
            c.sendall(b.upper())
        c.close()

    threading.Thread(target=echo, daemon=True).start()
    px = ProxyServer("127.0.0.1", srv.getsockname()[1])
    port = px.start_background()
    s = socket.create_connection(("127.0.0.1", port), timeout=5)
    payload = b"abc" * 100000
    s.sendall(payload)
    s.shutdown(socket.SHUT_WR)
    got = b""
    while True:
        b = s.recv(65536)
        if not b:
            break
        got += b
    assert got == payload.upper()
    px.stop()
    srv.close()
