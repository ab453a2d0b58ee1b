"""Run a task's user process inside a container (tony.docker.*; T/HadoopCompatibleAdapter.java:95-142).

On YARN, TonY only exported ``YARN_CONTAINER_RUNTIME_TYPE=docker`` / ``..._DOCKER_IMAGE`` /
``..._DOCKER_CONTAINER_MOUNTS`` and the NodeManager started the container.  Here the task agent
does it: the user command becomes ``docker run`` with the ROCm device nodes (``/dev/kfd`` and
``/dev/dri``; the task's HIP_VISIBLE_DEVICES still selects its GPU inside), host networking and
IPC (RCCL / torch.distributed rendezvous and dmabuf IPC need both), the task's working directory
bind-mounted at the same path, the configured mounts (``src:dst[:ro|rw]`` comma-separated, the
YARN mount syntax), and the task's environment passed through.
"""
from __future__ import annotations

import shlex
from typing import Dict, List, Optional

# environment that belongs to the host side / the agent and must not leak into the container
_SKIP_ENV = {"PATH", "HOME", "HOSTNAME", "PWD", "OLDPWD", "SHLVL", "_", "LD_PRELOAD", "TERM"}


def parse_mounts(spec: Optional[str]) -> List[str]:
    out = []
    for m in (spec or "").split(","):
        m = m.strip()
        if not m:
            continue
        parts = m.split(":")
        if len(parts) == 2:
            parts.append("rw")
        if len(parts) != 3 or parts[2] not in ("ro", "rw"):
            raise ValueError(f"bad docker mount {m!r}: expected src:dst[:ro|rw]")
        out.append(":".join(parts))
    return out


def docker_command(user_cmd: str, image: str, env: Dict[str, str], cwd: str, mounts: Optional[str] = None,
                   docker_bin: str = "docker", extra_args: Optional[List[str]] = None) -> str:
    if not image:
        raise ValueError("docker is enabled but no image is configured (tony.docker.containers.image)")
    args = [docker_bin, "run", "--rm", "--network=host", "--ipc=host", "--device=/dev/kfd", "--device=/dev/dri",
            "--group-add=video", "--security-opt=seccomp=unconfined", f"--volume={cwd}:{cwd}:rw", f"--workdir={cwd}"]
    for m in parse_mounts(mounts):
        args.append(f"--volume={m}")
    for k in sorted(env):
        if k in _SKIP_ENV or k.startswith("YARN_CONTAINER_RUNTIME_"):
            continue
        args.append(f"--env={k}={env[k]}")
    args += list(extra_args or [])
    args += [image, "bash", "-c", user_cmd]
    return " ".join(shlex.quote(a) for a in args)


def wrap_if_enabled(user_cmd: str, env: Dict[str, str], cwd: str) -> str:
    if env.get("YARN_CONTAINER_RUNTIME_TYPE") != "docker":
        return user_cmd
    return docker_command(user_cmd, env.get("YARN_CONTAINER_RUNTIME_DOCKER_IMAGE", ""), env, cwd,
                          env.get("YARN_CONTAINER_RUNTIME_DOCKER_CONTAINER_MOUNTS"),
                          env.get("TONY_DOCKER_BIN", "docker"))
