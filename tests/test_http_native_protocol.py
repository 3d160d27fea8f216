"""HTTP/1.1 protocol edge cases of the native front end (localai_amd/native/http_server.cpp):
body limits for Content-Length and chunked bodies, incremental chunk decoding, and half-closed
clients. The reference's fiber server enforces one body limit for every transfer coding
(core/http/app.go:64-70, BodyLimit)."""
import socket
import threading
import time

import pytest

from localai_amd.native import http


@pytest.fixture()
def echo():
    """A raw native Server whose handler answers every request with its body length."""
    srv = http().Server("127.0.0.1", 0)
    srv.max_body = 1 << 20
    srv.start()
    stop = threading.Event()
    served = []

    def pump():
        while not stop.is_set():
            for conn, method, target, ver, hs, body, peer in srv.take_requests():
                served.append((method, target, len(body)))
                srv.respond(conn, 200, [("content-type", "text/plain")], str(len(body)))
            time.sleep(0.002)

    th = threading.Thread(target=pump, daemon=True)
    th.start()
    yield srv, served
    stop.set()
    th.join(5)
    srv.stop()


def _connect(srv):
    s = socket.create_connection(("127.0.0.1", srv.port), timeout=10)
    return s


def _read_all(s):
    out = b""
    while True:
        try:
            d = s.recv(65536)
        except socket.timeout:
            break
        if not d:
            break
        out += d
    return out


def test_chunked_body_decoded(echo):
    srv, served = echo
    s = _connect(srv)
    body = b"x" * 5000
    req = b"POST /e HTTP/1.1\r\nhost: a\r\ntransfer-encoding: chunked\r\nconnection: close\r\n\r\n"
    # many small chunks, split over several sends so the decoder resumes mid-body
    chunks = [body[i:i + 100] for i in range(0, len(body), 100)]
    wire = b"".join(b"%x\r\n%s\r\n" % (len(c), c) for c in chunks) + b"0\r\n\r\n"
    s.sendall(req)
    for i in range(0, len(wire), 777):
        s.sendall(wire[i:i + 777])
        time.sleep(0.001)
    resp = _read_all(s)
    assert resp.startswith(b"HTTP/1.1 200") and resp.endswith(b"5000")
    assert served[-1] == ("POST", b"/e", 5000)


def test_chunked_body_over_limit_is_413(echo):
    srv, served = echo
    s = _connect(srv)
    s.sendall(b"POST /e HTTP/1.1\r\nhost: a\r\ntransfer-encoding: chunked\r\n\r\n")
    piece = b"%x\r\n%s\r\n" % (64 * 1024, b"y" * 64 * 1024)
    got = b""
    try:
        for _ in range(40):  # 2.5 MiB against a 1 MiB limit
            s.sendall(piece)
    except (BrokenPipeError, ConnectionResetError):
        pass
    try:
        got = _read_all(s)
    except ConnectionResetError:
        pass
    assert got.startswith(b"HTTP/1.1 413")
    assert not served


def test_chunk_size_overflow_rejected(echo):
    srv, _ = echo
    s = _connect(srv)
    s.sendall(b"POST /e HTTP/1.1\r\nhost: a\r\ntransfer-encoding: chunked\r\n\r\n"
              b"ffffffffffffffffffff\r\nabc\r\n")
    assert _read_all(s).split(b"\r\n")[0] in (b"HTTP/1.1 400 Bad Request", b"HTTP/1.1 413 Payload Too Large")


def test_content_length_over_limit_is_413(echo):
    srv, _ = echo
    s = _connect(srv)
    s.sendall(b"POST /e HTTP/1.1\r\nhost: a\r\ncontent-length: %d\r\n\r\n" % (2 << 20))
    assert _read_all(s).startswith(b"HTTP/1.1 413")


def test_half_close_after_request_is_answered(echo):
    srv, served = echo
    s = _connect(srv)
    s.sendall(b"GET /v1/models HTTP/1.1\r\nhost: a\r\n\r\n")
    s.shutdown(socket.SHUT_WR)
    resp = _read_all(s)   # returns at the server's close
    # "connection: close" is announced when the FIN is seen before the response is built; when
    # the request is answered first, the FIN then ends the idle connection -- both are correct
    assert resp.startswith(b"HTTP/1.1 200") and resp.endswith(b"\r\n\r\n0")
    assert served and served[-1][1] == b"/v1/models"


def test_half_close_with_partial_request_closes(echo):
    srv, served = echo
    s = _connect(srv)
    s.sendall(b"GET /v1/mod")
    s.shutdown(socket.SHUT_WR)
    assert _read_all(s) == b""
    assert not served
