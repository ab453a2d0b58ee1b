"""Azkaban job type for TonY jobs (tony-azkaban TonyJob.java:27-194, TonyJobArg.java:8-24).

An Azkaban job of type ``tony`` carries its settings as job properties; ``TonyJob`` turns them
into what the TonY client takes:

* every ``tony.*`` property goes into a generated ``tony.xml`` (passed as ``--conf_file``);
* the flow identity (``azkaban.flow.execid``, ``azkaban.flow.flowid``,
  ``azkaban.flow.projectname``, ``azkaban.webserverhost``) becomes ``tony.application.tags``
  as ``key:value`` pairs;
* ``src_dir`` (default ``src``), ``hdfs_classpath``, ``task_params``, ``python_binary_path``,
  ``python_venv`` and ``executes`` map to the client options of the same names;
* ``worker_env.K=V`` properties become ``--shell_env K=V``;
* ``azkaban.input.dataset`` / ``azkaban.output.dataset`` are exported to the tasks as
  ``AZKABAN_INPUT_DATASET`` / ``AZKABAN_OUTPUT_DATASET`` with ``,`` replaced by ``;``.

``python -m tony_amd.azkaban job.properties`` runs a job from a Java-style properties file.
"""
from __future__ import annotations

import os
import sys
import uuid
from typing import Dict, List, Optional

from ..conf import Configuration

TONY_CONF_PREFIX = "tony."
TONY_APPLICATION_TAGS = "tony.application.tags"
WORKER_ENV_PREFIX = "worker_env."
AZKABAN_INPUT_DATASET_JOB_PROP = "azkaban.input.dataset"
AZKABAN_INPUT_DATASET_ENV_VAR_KEY = "AZKABAN_INPUT_DATASET"
AZKABAN_OUTPUT_DATASET_JOB_PROP = "azkaban.output.dataset"
AZKABAN_OUTPUT_DATASET_ENV_VAR_KEY = "AZKABAN_OUTPUT_DATASET"
TAG_KEYS = ("azkaban.flow.execid", "azkaban.flow.flowid", "azkaban.flow.projectname", "azkaban.webserverhost")
# job property -> TonyClient option (TonyJobArg)
ARG_PROPS = ("hdfs_classpath", "task_params", "python_binary_path", "python_venv", "executes")


def load_properties(path: str) -> Dict[str, str]:
    """Minimal Java .properties reader (``k=v`` / ``k: v``, ``#``/``!`` comments, ``\\`` continuations)."""
    props: Dict[str, str] = {}
    with open(path) as f:
        lines = f.read().splitlines()
    buf = ""
    for raw in lines:
        line = raw.strip()
        if not buf and (not line or line[0] in "#!"):
            continue
        if line.endswith("\\") and not line.endswith("\\\\"):
            buf += line[:-1]
            continue
        line, buf = buf + line, ""
        for i, ch in enumerate(line):
            if ch in "=:":
                props[line[:i].strip()] = line[i + 1:].strip()
                break
        else:
            props[line] = ""
    return props


class TonyJob:
    def __init__(self, job_id: str, sys_props: Dict[str, str], job_props: Dict[str, str],
                 working_dir: Optional[str] = None):
        self.job_id = job_id
        self.sys_props = dict(sys_props)
        self.job_props = dict(job_props)
        self.working_dir = working_dir or os.getcwd()
        self.tony_xml = os.path.join(self.working_dir, f"_tony-conf-{job_id}-{uuid.uuid4()}", "tony.xml")
        self.tony_conf = self._job_configuration()

    def _job_configuration(self) -> Configuration:
        c = Configuration(load_defaults=False)
        for k, v in self.job_props.items():
            if k.startswith(TONY_CONF_PREFIX):
                c.set(k, v, "azkaban job props")
        c.set(TONY_APPLICATION_TAGS, self.application_tags(), "azkaban flow")
        return c

    def application_tags(self) -> str:
        tags = []
        for k in TAG_KEYS:
            v = self.job_props.get(k)
            if v is not None:
                tags.append(f"{k}:{v}"[:100])
        return ",".join(tags)

    def main_args(self) -> List[str]:
        p = self.job_props
        args = ["--src_dir", p.get("src_dir", "src")]
        if p.get("hdfs_classpath") is not None:
            args += ["--hdfs_classpath", p["hdfs_classpath"]]
        for k in sorted(p):
            if k.startswith(WORKER_ENV_PREFIX):
                args += ["--shell_env", f"{k[len(WORKER_ENV_PREFIX):]}={p[k]}"]
        for name in ("task_params", "python_binary_path", "python_venv", "executes"):
            if p.get(name) is not None:
                args += [f"--{name}", p[name]]
        for prop, env in ((AZKABAN_INPUT_DATASET_JOB_PROP, AZKABAN_INPUT_DATASET_ENV_VAR_KEY),
                          (AZKABAN_OUTPUT_DATASET_JOB_PROP, AZKABAN_OUTPUT_DATASET_ENV_VAR_KEY)):
            if p.get(prop) is not None:
                args += ["--shell_env", f"{env}={p[prop].replace(',', ';')}"]
        return args

    def setup_job_configuration_file(self) -> str:
        os.makedirs(os.path.dirname(self.tony_xml), exist_ok=True)
        self.tony_conf.write_xml(self.tony_xml)
        return self.tony_xml

    def run(self) -> int:
        from ..cli.cluster_submitter import ClusterSubmitter

        path = self.setup_job_configuration_file()
        return ClusterSubmitter().submit(self.main_args() + ["--conf_file", path])


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print("usage: python -m tony_amd.azkaban <job.properties> [sys.properties]", file=sys.stderr)
        return 2
    job_props = load_properties(argv[0])
    sys_props = load_properties(argv[1]) if len(argv) > 1 else {}
    job = TonyJob(os.path.splitext(os.path.basename(argv[0]))[0], sys_props, job_props,
                  os.path.dirname(os.path.abspath(argv[0])))
    return job.run()
