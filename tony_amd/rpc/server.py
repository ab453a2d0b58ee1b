"""Coordinator RPC server (T/rpc/ApplicationRpcServer.java:26-162 + MetricsRpcServer).

gRPC on a loopback port (single node), one generic handler per method of
``protocol.METHODS``.  With ``tony.application.security.enabled`` a per-job
random token (file mode 0600 in the job dir) must be sent as the
``tony-token`` metadata entry; TonY uses Hadoop SASL/ClientToAMToken here.
"""
from __future__ import annotations

import logging
from concurrent import futures
from typing import Callable, Dict, Optional

import grpc

from . import protocol as P

LOG = logging.getLogger(__name__)
TOKEN_KEY = "tony-token"


class RpcServer:
    def __init__(self, handlers: Dict[str, Callable], host: str = "127.0.0.1", port: int = 0,
                 token: Optional[str] = None, max_workers: int = 32):
        """``handlers[method](request) -> response`` for each name in protocol.METHODS."""
        missing = set(P.METHODS) - set(handlers)
        if missing:
            raise ValueError(f"missing RPC handlers: {sorted(missing)}")
        self.token = token
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix="tony-rpc"),
                                   options=[("grpc.so_reuseport", 0)])
        rpc_handlers = {}
        for name, (req, resp) in P.METHODS.items():
            rpc_handlers[name] = grpc.unary_unary_rpc_method_handler(
                self._wrap(name, handlers[name]),
                request_deserializer=P.MESSAGES[req].FromString,
                response_serializer=P.MESSAGES[resp].SerializeToString)
        self._server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(P.FULL_SERVICE, rpc_handlers),))
        self.host = host
        self.port = self._server.add_insecure_port(f"{host}:{port}")
        if self.port == 0:
            raise OSError(f"cannot bind RPC server on {host}:{port}")

    def _wrap(self, name, fn):
        def handler(request, context):
            if self.token is not None:
                md = dict(context.invocation_metadata())
                if md.get(TOKEN_KEY) != self.token:
                    context.abort(grpc.StatusCode.UNAUTHENTICATED, "bad or missing job token")
            try:
                return fn(request)
            except Exception as e:  # noqa: BLE001
                LOG.exception("RPC %s failed", name)
                context.abort(grpc.StatusCode.INTERNAL, f"{type(e).__name__}: {e}")
        return handler

    def start(self) -> "RpcServer":
        self._server.start()
        return self

    def stop(self, grace: float = 0.5) -> None:
        self._server.stop(grace)
