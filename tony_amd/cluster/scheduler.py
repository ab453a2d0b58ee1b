"""DAG stage scheduler (behavioural parity with T/TaskScheduler.java:30-179).

Job types form a dependency graph through ``tony.application.prepare-stage`` /
``training-stage`` (every training-stage job type depends on every tracked
prepare-stage job type).  The scheduler refuses a cyclic graph, launches every
job type with no pending dependencies, and counts completions of the job types
others wait on; when a waiter's counts reach zero it is launched.  "Launch"
here is the coordinator's ``request(job_request)`` callback, which reserves GPU
slots and spawns the task agents -- the single-node stand-in for YARN's
``addContainerRequest``.
"""
from __future__ import annotations

import threading
from typing import Callable, Dict, List

from ..utils.core import JobContainerRequest


def is_dag(requests: List[JobContainerRequest]) -> bool:
    by_name = {r.job_name: r for r in requests}
    visited: set = set()

    def sub(node: JobContainerRequest, trace: List[str]) -> bool:
        if node.job_name in trace:
            return False
        if node.job_name in visited:
            return True
        trace.append(node.job_name)
        visited.add(node.job_name)
        for dep in node.depends_on:
            if dep in by_name and not sub(by_name[dep], trace):
                return False
        trace.remove(node.job_name)
        return True

    return all(r.job_name in visited or sub(r, []) for r in requests)


class TaskScheduler:
    def __init__(self, session, request: Callable[[JobContainerRequest], None]):
        self.session = session
        self.request = request
        self.dependency_check_passed = True
        self.waiting: Dict[str, Dict[str, int]] = {}
        self._lock = threading.Lock()
        self.scheduled: List[str] = []

    def schedule_tasks(self) -> None:
        requests = list(self.session.container_requests.values())
        if not is_dag(requests):
            self.session.set_final_status("FAILED", "App failed due to it not being a DAG.")
            self.dependency_check_passed = False
            return
        for r in requests:
            deps = {d: self.session.container_requests[d].num_instances for d in r.depends_on
                    if d and d in self.session.container_requests}
            if deps:
                self.waiting[r.job_name] = deps
        for r in requests:
            if not self.waiting.get(r.job_name):
                self._schedule(r)

    def _schedule(self, r: JobContainerRequest) -> None:
        self.scheduled.append(r.job_name)
        self.session.add_num_expected(r.num_instances)
        self.request(r)

    def check_dependency_satisfied(self, job: str) -> bool:
        return not self.waiting.get(job)

    def register_dependency_completed(self, job: str) -> None:
        ready = []
        with self._lock:
            for waiter, deps in self.waiting.items():
                if job in deps:
                    deps[job] -= 1
                    if deps[job] <= 0:
                        del deps[job]
            for waiter in list(self.waiting):
                if not self.waiting[waiter]:
                    del self.waiting[waiter]
                    ready.append(waiter)
        for waiter in ready:
            self._schedule(self.session.container_requests[waiter])
