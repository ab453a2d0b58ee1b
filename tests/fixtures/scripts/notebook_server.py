"""Stand-in for a notebook server: serve one HTTP GET on $TB_PORT, then exit 0."""
import http.server
import os


class H(http.server.BaseHTTPRequestHandler):
    def do_GET(self):  # noqa: N802
        body = b"notebook-ok"
        self.send_response(200)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


srv = http.server.HTTPServer(("0.0.0.0", int(os.environ["TB_PORT"])), H)
srv.handle_request()
