"""Job history: jhist naming, models and parsers.

Parity: T/util/HistoryFileUtils.java:11-35 (file names), T/models/JobMetadata.java,
JobConfig.java, JobEvent.java, JobLog.java (models), T/util/ParserUtils.java:49-318
(validation / latest-file selection / metadata, config and event parsing),
T/util/HdfsUtils.java:31-165 (job-dir discovery), on the local filesystem.

File names: ``<appId>-<started>-<user>.jhist.inprogress`` while running, then
``<appId>-<started>-<completed>-<user>-<STATUS>.jhist``.  Layout:
``<history>/intermediate/<appId>/`` -> ``<history>/finished/yyyy/MM/dd/<appId>/``.
"""
from __future__ import annotations

import datetime as _dt
import logging
import os
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import List, Optional

from .. import constants as C
from .avro import read_all

LOG = logging.getLogger(__name__)
DEFAULT_JOB_ID_REGEX = r"^application_\d+_\d+$"


@dataclass
class JobMetadata:
    id: str
    started: int = -1
    completed: int = -1
    status: str = ""
    user: str = ""

    @property
    def job_link(self) -> str:
        return f"/{C.JOBS_SUFFIX}/{self.id}"

    @property
    def config_link(self) -> str:
        return f"/{C.CONFIG_SUFFIX}/{self.id}"

    @classmethod
    def from_hist_file_name(cls, name: str) -> "JobMetadata":
        base = os.path.basename(name)
        parts = base[:base.index(".")].split("-")
        md = cls(parts[0], int(parts[1]))
        if base.endswith(C.INPROGRESS):
            md.user = parts[2]
            md.status = C.RUNNING
        else:
            md.completed = int(parts[2])
            md.user = parts[3]
            md.status = parts[4]
        return md


def generate_file_name(md: JobMetadata) -> str:
    s = f"{md.id}-{md.started}-"
    if md.completed != -1:
        s += f"{md.completed}-"
    s += md.user
    if md.status:
        return f"{s}-{md.status}.{C.HISTFILE_SUFFIX}"
    return f"{s}.{C.HISTFILE_SUFFIX}.{C.INPROGRESS}"


def is_valid_hist_file_name(name: str, job_id_regex: str = DEFAULT_JOB_ID_REGEX) -> bool:
    if not name:
        return False
    base = name[:name.index(".")] if "." in name else name
    parts = base.split("-")
    if len(parts) < 3:
        return False
    if name.endswith(C.INPROGRESS):
        return bool(re.match(job_id_regex, parts[0]) and parts[1].isdigit() and parts[2] == parts[2].lower())
    if len(parts) != 5:
        return False
    return bool(re.match(job_id_regex, parts[0]) and parts[1].isdigit() and parts[2].isdigit()
                and parts[3] == parts[3].lower() and parts[4] == parts[4].upper())


def get_jhist_file_path(job_dir: str) -> Optional[str]:
    """Latest (by start time) history file of a job dir (covers coordinator retries)."""
    try:
        files = [f for f in os.listdir(job_dir) if C.HISTFILE_SUFFIX in f]
    except OSError:
        return None
    if not files:
        return None

    def started(f):
        try:
            return int(f.split("-")[1])
        except (IndexError, ValueError):
            return -1

    return os.path.join(job_dir, max(files, key=started))


def completed_time_from_file_name(name: str) -> int:
    return int(os.path.basename(name).split("-")[2])


def parse_metadata(job_dir: str, job_id_regex: str = DEFAULT_JOB_ID_REGEX) -> Optional[JobMetadata]:
    path = get_jhist_file_path(job_dir)
    if path is None:
        return None
    name = os.path.basename(path)
    if not is_valid_hist_file_name(name, job_id_regex):
        LOG.warning("Invalid history file name %s", name)
        return None
    return JobMetadata.from_hist_file_name(name)


@dataclass
class JobConfig:
    name: str
    value: str
    final: bool = False
    source: Optional[str] = None


def parse_config(job_dir: str) -> List[JobConfig]:
    path = os.path.join(job_dir, C.TONY_FINAL_XML)
    if not os.path.exists(path):
        path = os.path.join(job_dir, "config.xml")
    try:
        root = ET.parse(path).getroot()
    except (OSError, ET.ParseError):
        return []
    out = []
    for p in root.iter("property"):
        name, value = p.findtext("name"), p.findtext("value")
        if name is None or value is None:
            continue
        out.append(JobConfig(name, value, (p.findtext("final") or "").lower() == "true", p.findtext("source")))
    return out


@dataclass
class JobEvent:
    type: str
    event: dict
    timestamp: int

    @property
    def date(self) -> str:
        return _dt.datetime.fromtimestamp(self.timestamp / 1000, tz=_dt.timezone.utc).strftime(
            "%d %b %Y %H:%M:%S:%f")[:-3] + " +0000"


def parse_events(job_dir: str) -> List[JobEvent]:
    path = get_jhist_file_path(job_dir)
    if path is None:
        return []
    try:
        recs = read_all(path)
    except Exception:  # noqa: BLE001
        LOG.exception("failed to read %s", path)
        return []
    return [JobEvent(r["type"], r["event"], r["timestamp"]) for r in recs]


@dataclass
class JobLog:
    host: str
    container_id: str
    log_link: str


def map_event_to_job_log(ev: JobEvent, logs_root: Optional[str] = None) -> Optional[JobLog]:
    """APPLICATION_INITED / TASK_STARTED events carry the host + container (task log dir)."""
    if ev.type not in ("APPLICATION_INITED", "TASK_STARTED"):
        return None
    host = ev.event.get("host")
    cid = ev.event.get("containerID")
    if not host or not cid:
        return None
    link = os.path.join(logs_root, cid) if logs_root else cid
    return JobLog(host, cid, link)


def year_month_day_dir(root: str, ts_ms: int, tz: str = "UTC") -> str:
    d = _dt.datetime.fromtimestamp(ts_ms / 1000, tz=_dt.timezone.utc)
    if tz and tz.upper() != "UTC":
        try:
            from zoneinfo import ZoneInfo

            d = d.astimezone(ZoneInfo(tz))
        except Exception:  # noqa: BLE001
            pass
    return os.path.join(root, f"{d.year:04d}", f"{d.month:02d}", f"{d.day:02d}")


def find_job_dirs(root: str, job_id_regex: str = DEFAULT_JOB_ID_REGEX) -> List[str]:
    """Recursively find job folders (named like an app id) under ``root`` (HdfsUtils.getJobDirs)."""
    out = []
    if not os.path.isdir(root):
        return out
    for dirpath, dirnames, _ in os.walk(root):
        for d in list(dirnames):
            if re.match(job_id_regex, d):
                out.append(os.path.join(dirpath, d))
                dirnames.remove(d)
    return sorted(out)


@dataclass
class HistoryLayout:
    location: str
    intermediate: str = ""
    finished: str = ""
    timezone: str = "UTC"
    extras: dict = field(default_factory=dict)

    @classmethod
    def from_conf(cls, conf) -> "HistoryLayout":
        from ..conf import keys as K

        loc = conf.get(K.HISTORY_LOCATION, "/path/to/tony-history")
        inter = conf.get(K.HISTORY_INTERMEDIATE) or os.path.join(loc, C.TONY_HISTORY_INTERMEDIATE)
        fin = conf.get(K.HISTORY_FINISHED) or os.path.join(loc, C.TONY_HISTORY_FINISHED)
        return cls(loc, inter, fin, conf.get(K.HISTORY_FINISHED_DIR_TIMEZONE, "UTC"))
