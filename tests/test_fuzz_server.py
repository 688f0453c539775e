"""Network-level fuzzing of the running server: random and mutated byte streams, split at
random points, over many connections. The server must never crash or hang, and must keep
answering well-formed requests afterwards."""
import random
import socket

from hypothesis import given, settings, strategies as st, HealthCheck

VALID = [
    b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n",
    b"HEAD /api/health HTTP/1.1\r\nHost: x\r\nAccept: text/*\r\n\r\n",
    b"GET /api/hola-chaining HTTP/1.1\r\nX-B3-TraceId: 1\r\nX-B3-SpanId: 2\r\nX-B3-Sampled: 1\r\n\r\n",
    b"POST /api/hola HTTP/1.1\r\nContent-Length: 3\r\n\r\nabc",
    b"GET /api/hola HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n1\r\na\r\n0\r\n\r\n",
    b"OPTIONS /api/hola HTTP/1.0\r\nConnection: keep-alive\r\n\r\n",
]


def mutate(rng: random.Random, data: bytes) -> bytes:
    b = bytearray(data)
    for _ in range(rng.randint(1, 6)):
        op = rng.randrange(4)
        if op == 0 and b:
            b[rng.randrange(len(b))] = rng.randrange(256)
        elif op == 1:
            b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        elif op == 2 and b:
            del b[rng.randrange(len(b))]
        else:
            i = rng.randrange(len(b) + 1)
            b[i:i] = rng.choice([b"\r\n", b":", b" ", b"\x00", b"%", b"\r\n\r\n", b"9" * 20])
    return bytes(b)


def send_stream(port: int, data: bytes, rng: random.Random) -> None:
    try:
        with socket.create_connection(("127.0.0.1", port), timeout=2) as c:
            i = 0
            while i < len(data):
                j = min(len(data), i + rng.randint(1, 64))
                c.sendall(data[i:j])
                i = j
            c.shutdown(socket.SHUT_WR)
            c.settimeout(0.5)
            try:
                while c.recv(65536):
                    pass
            except (socket.timeout, ConnectionResetError):
                pass
    except OSError:  # reset / not connected: the server closed after an error response
        pass


def test_mutation_fuzz(hola):
    s = hola(args=["--aloha-url", "http://127.0.0.1:1/", "--feign-log", "none", "--idle-timeout-ms", "1000"])
    rng = random.Random(1234)
    for _ in range(300):
        stream = b"".join(mutate(rng, rng.choice(VALID)) if rng.random() < 0.7 else rng.choice(VALID)
                          for _ in range(rng.randint(1, 5)))
        send_stream(s.port, stream, rng)
    assert s.proc.poll() is None
    assert s.get("/api/hola")[0] == 200


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.binary(max_size=2048))
def test_random_bytes(hola_server, data):
    send_stream(hola_server.port, data, random.Random(len(data)))
    assert hola_server.proc.poll() is None


import pytest  # noqa: E402


@pytest.fixture(scope="module")
def hola_server(hola_bin):
    from hola_amd.server import HolaProcess

    p = HolaProcess(args=["--feign-log", "none", "--idle-timeout-ms", "1000"], threads=2).start()
    yield p
    assert p.get("/api/health")[0] == 200
    p.stop()
