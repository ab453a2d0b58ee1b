"""Local TCP port forwarder (tony-proxy ProxyServer.java:21-91).

TonY copies bytes with two threads per connection.  Here one asyncio loop
(on its own thread) serves every connection: each accepted client is paired
with a fresh connection to ``remote_host:remote_port`` and two stream pumps
copy bytes until either side closes.
"""
from __future__ import annotations

import asyncio
import logging
import threading
from typing import Optional

LOG = logging.getLogger("tony.proxy")
_CHUNK = 64 * 1024


async def _pump(reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
    try:
        while True:
            data = await reader.read(_CHUNK)
            if not data:
                break
            writer.write(data)
            await writer.drain()
        if writer.can_write_eof():
            writer.write_eof()  # half-close: the other direction keeps flowing
    except (ConnectionError, OSError, asyncio.CancelledError):
        pass


class ProxyServer:
    """Forward ``local_port`` on this host to ``remote_host:remote_port``."""

    def __init__(self, remote_host: str, remote_port: int, local_port: int = 0, bind: str = "127.0.0.1"):
        self.remote_host = remote_host
        self.remote_port = int(remote_port)
        self.local_port = int(local_port)
        self.bind = bind
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._server: Optional[asyncio.AbstractServer] = None
        self._thread: Optional[threading.Thread] = None
        self._ready = threading.Event()
        self.connections = 0

    async def _handle(self, creader: asyncio.StreamReader, cwriter: asyncio.StreamWriter) -> None:
        self.connections += 1
        try:
            rreader, rwriter = await asyncio.open_connection(self.remote_host, self.remote_port)
        except OSError as e:
            LOG.warning("proxy: cannot reach %s:%d: %s", self.remote_host, self.remote_port, e)
            cwriter.close()
            return
        try:
            await asyncio.gather(_pump(creader, rwriter), _pump(rreader, cwriter))
        finally:
            for w in (rwriter, cwriter):
                try:
                    w.close()
                except Exception:  # noqa: BLE001
                    pass

    async def _serve(self) -> None:
        self._server = await asyncio.start_server(self._handle, self.bind, self.local_port, reuse_address=True)
        self.local_port = self._server.sockets[0].getsockname()[1]
        LOG.info("proxy %s:%d -> %s:%d", self.bind, self.local_port, self.remote_host, self.remote_port)
        self._ready.set()
        async with self._server:
            await self._server.serve_forever()

    def _run(self) -> None:
        self._loop = asyncio.new_event_loop()
        try:
            self._loop.run_until_complete(self._serve())
        except asyncio.CancelledError:
            pass
        finally:
            self._ready.set()
            self._loop.close()

    def start_background(self) -> int:
        """Start serving on a daemon thread; returns the bound local port."""
        self._thread = threading.Thread(target=self._run, name="tony-proxy", daemon=True)
        self._thread.start()
        self._ready.wait(10)
        return self.local_port

    def start(self) -> None:
        """Serve in the calling thread until :meth:`stop` (ProxyServer.start of TonY blocks too)."""
        self._run()

    def stop(self) -> None:
        if self._loop is not None and self._server is not None:
            def _close():
                self._server.close()
                for t in asyncio.all_tasks(self._loop):
                    t.cancel()
            try:
                self._loop.call_soon_threadsafe(_close)
            except RuntimeError:
                pass
        if self._thread is not None:
            self._thread.join(5)


def main(argv=None) -> int:
    import argparse

    p = argparse.ArgumentParser(description="TCP port forwarder")
    p.add_argument("remote_host")
    p.add_argument("remote_port", type=int)
    p.add_argument("local_port", type=int, nargs="?", default=0)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    ProxyServer(a.remote_host, a.remote_port, a.local_port).start()
    return 0
