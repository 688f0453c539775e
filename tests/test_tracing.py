"""Zipkin tracing parity (ZipkinResource.java, ZipKinFilter.java, HolaResource.java:97-108)
against a fake collector, plus the B3 codec."""
import json
import time

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from hola_amd.testing.fakes import FakeAloha, FakeZipkin


@pytest.fixture
def zipkin():
    z = FakeZipkin().start()
    yield z
    z.stop()


def _annotations(span):
    return {a["value"] for a in span.get("annotations", [])}


def test_server_span_for_hola(hola, zipkin):
    s = hola(args=["--zipkin-url", zipkin.url.rstrip("/")])
    assert s.get("/api/hola")[0] == 200
    spans = zipkin.wait_for(lambda sp: len(sp) >= 1)
    assert len(spans) == 1
    sp = spans[0]
    assert zipkin.posts[0]["path"] == "/api/v1/spans"
    assert zipkin.posts[0]["content_type"] == "application/json"
    assert sp["name"] == "get"
    assert _annotations(sp) == {"sr", "ss"}
    assert all(a["endpoint"]["serviceName"] == "hola" for a in sp["annotations"])
    assert sp["traceId"] == sp["id"] and "parentId" not in sp  # new root trace
    assert "timestamp" in sp and sp["duration"] >= 1
    urls = [b["value"] for b in sp["binaryAnnotations"] if b["key"] == "http.url"]
    assert urls and urls[0].endswith("/api/hola")


def test_health_is_not_traced(hola, zipkin):
    s = hola(args=["--zipkin-url", zipkin.url])
    for _ in range(3):
        s.get("/api/health")
    s.get("/api/hola")
    spans = zipkin.wait_for(lambda sp: len(sp) >= 1)
    time.sleep(1.2)
    spans = zipkin.spans()
    assert len(spans) == 1 and spans[0]["binaryAnnotations"][0]["value"].endswith("/api/hola")


def test_joins_incoming_b3_trace(hola, zipkin):
    s = hola(args=["--zipkin-url", zipkin.url])
    s.get("/api/hola", headers={"X-B3-TraceId": "463ac35c9f6413ad", "X-B3-SpanId": "a2fb4a1d1a96d312",
                                "X-B3-ParentSpanId": "0020000000000001", "X-B3-Sampled": "1"})
    sp = zipkin.wait_for(lambda sp: len(sp) >= 1)[0]
    assert sp["traceId"] == "463ac35c9f6413ad"
    assert sp["id"] == "a2fb4a1d1a96d312"
    assert sp["parentId"] == "0020000000000001"
    assert "timestamp" not in sp  # shared span: the caller owns timestamp/duration


def test_ids_without_sampled_header_start_new_trace(hola, zipkin):
    # Brave 3.9's HttpServerRequestAdapter only honours incoming ids with X-B3-Sampled.
    s = hola(args=["--zipkin-url", zipkin.url])
    s.get("/api/hola", headers={"X-B3-TraceId": "463ac35c9f6413ad", "X-B3-SpanId": "a2fb4a1d1a96d312"})
    sp = zipkin.wait_for(lambda sp: len(sp) >= 1)[0]
    assert sp["traceId"] != "463ac35c9f6413ad"


def test_not_sampled_is_not_reported(hola, zipkin):
    s = hola(args=["--zipkin-url", zipkin.url])
    s.get("/api/hola", headers={"X-B3-Sampled": "0"})
    s.get("/api/hola", headers={"b3": "0"})
    time.sleep(1.5)
    assert zipkin.spans() == []


def test_chaining_client_span_and_b3_propagation(hola, zipkin):
    with FakeAloha() as aloha:
        s = hola(args=["--zipkin-url", zipkin.url, "--aloha-url", aloha.url])
        st, _, body = s.get("/api/hola-chaining")
        assert st == 200 and json.loads(body)[1] == "Aloha mai aloha-1"
        spans = zipkin.wait_for(lambda sp: len(sp) >= 2)
        server = next(x for x in spans if "sr" in _annotations(x))
        client = next(x for x in spans if "cs" in _annotations(x))
        assert _annotations(client) == {"cs", "cr"}
        assert client["traceId"] == server["traceId"]
        assert client["parentId"] == server["id"]
        hdr = aloha.requests[-1]["headers"]
        assert hdr["x-b3-traceid"] == server["traceId"]
        assert hdr["x-b3-spanid"] == client["id"]
        assert hdr["x-b3-parentspanid"] == server["id"]
        assert hdr["x-b3-sampled"] == "1"
        url = [b["value"] for b in client["binaryAnnotations"] if b["key"] == "http.url"][0]
        assert url.endswith("/api/aloha-chaining")


def test_v2_format(hola, zipkin):
    s = hola(args=["--zipkin-url", zipkin.url, "--zipkin-v2"])
    s.get("/api/hola")
    sp = zipkin.wait_for(lambda sp: len(sp) >= 1)[0]
    assert zipkin.posts[0]["path"] == "/api/v2/spans"
    assert sp["kind"] == "SERVER" and sp["localEndpoint"]["serviceName"] == "hola"
    assert sp["tags"]["http.url"].endswith("/api/hola")


def test_collector_down_never_blocks(hola):
    s = hola(args=["--zipkin-url", "http://127.0.0.1:1"])
    t0 = time.monotonic()
    for _ in range(200):
        assert s.get("/api/hola")[0] == 200
    assert time.monotonic() - t0 < 5
    time.sleep(1.3)
    st, _, body = s.get("/metrics")
    assert b"hola_span_post_failures_total" in body


def _self_signed(tmp_path, name: str, san: str) -> tuple[str, str]:
    import shutil
    import subprocess

    if not shutil.which("openssl"):
        pytest.skip("openssl CLI not installed")
    cert, key = tmp_path / f"{name}.pem", tmp_path / f"{name}.key"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-keyout", str(key),
                    "-out", str(cert), "-subj", f"/CN={name}", "-addext", f"subjectAltName={san}"],
                   check=True, capture_output=True)
    return str(cert), str(key)


def _post_failures(s) -> int:
    body = s.get("/metrics")[2].decode()
    return int(next(l.split()[1] for l in body.splitlines() if l.startswith("hola_span_post_failures_total ")))


def test_https_collector_verified_against_the_trust_store(hola, tmp_path):
    """ZIPKIN_SERVER_URL=https://...: spans go over TLS once the collector's certificate
    chains to a trusted CA ($SSL_CERT_FILE here) and names the host; otherwise nothing is
    sent and the failed POSTs are counted."""
    cert, key = _self_signed(tmp_path, "collector", "DNS:localhost,IP:127.0.0.1")
    with FakeZipkin(tls=(cert, key)) as z:
        assert z.url.startswith("https://")
        s = hola(env={"ZIPKIN_SERVER_URL": z.url.rstrip("/"), "SSL_CERT_FILE": cert})
        assert s.get("/api/hola")[0] == 200
        spans = z.wait_for(lambda sp: len(sp) >= 1)
        assert len(spans) == 1 and spans[0]["name"] == "get"
        # not trusted: the self-signed certificate is not in the store
        s2 = hola(env={"ZIPKIN_SERVER_URL": z.url.rstrip("/"), "SSL_CERT_FILE": str(tmp_path / "none.pem")})
        assert s2.get("/api/hola")[0] == 200
        time.sleep(1.5)
        assert len(z.spans()) == 1 and _post_failures(s2) >= 1
    # trusted, but issued for another name
    other_cert, other_key = _self_signed(tmp_path, "other", "DNS:other.example")
    with FakeZipkin(tls=(other_cert, other_key)) as z:
        s3 = hola(env={"ZIPKIN_SERVER_URL": z.url.rstrip("/"), "SSL_CERT_FILE": other_cert})
        assert s3.get("/api/hola")[0] == 200
        time.sleep(1.5)
        assert z.spans() == [] and _post_failures(s3) >= 1


def test_https_urls_parse(native):
    assert native.parse_url("https://zipkin:9411") == ("zipkin", 9411, "/", True)
    assert native.parse_url("https://zipkin/") == ("zipkin", 443, "/", True)
    assert native.parse_url("http://zipkin-query:9411") == ("zipkin-query", 9411, "/", False)
    assert native.parse_url("ftp://x") is None


def test_collector_interim_and_bare_204_answers(hola):
    """A collector (or a front) that answers each POST with an unasked-for 100 Continue and
    then a 204 without Content-Length: the reporter reads past the 1xx, takes the 204 as
    bodiless instead of reading to the connection's close (its 2 s timeout), and keeps the
    connection for the next flush."""
    with FakeZipkin(status=204, interim=True) as z:
        s = hola(args=["--zipkin-url", z.url.rstrip("/")])
        t0 = time.monotonic()
        for k in range(1, 4):
            assert s.get("/api/hola")[0] == 200
            z.wait_for(lambda sp, k=k: len(sp) >= k, timeout=5)
        elapsed = time.monotonic() - t0
        assert len(z.spans()) == 3, z.posts
        assert elapsed < 4.5, elapsed  # one ~1 s flush each, no 2 s read timeouts
        assert _post_failures(s) == 0
        assert len({p["peer_port"] for p in z.posts}) == 1  # one kept-alive connection throughout


def test_spans_flushed_on_shutdown(hola_bin, zipkin):
    from hola_amd.server import HolaProcess

    s = HolaProcess(args=["--zipkin-url", zipkin.url], env={"HOSTNAME": "h"}).start()
    s.get("/api/hola")
    s.stop()  # SIGTERM well before the 1 s flush interval
    assert len(zipkin.spans()) == 1


# ---- codec ----

def test_b3_extract_multi(native):
    d = native.b3_extract(trace_id="463ac35c9f6413ad48485a3953bb6124", span_id="a2fb4a1d1a96d312",
                          sampled="true")
    assert d["trace_id"] == "463ac35c9f6413ad48485a3953bb6124" and d["span_id"] == "a2fb4a1d1a96d312"
    assert d["parent_id"] is None and d["sampled"]
    assert native.b3_extract(sampled="0") == "not_sampled"
    assert native.b3_extract(sampled="false", trace_id="1", span_id="2") == "not_sampled"
    assert native.b3_extract(trace_id="1", span_id="2") == "none"
    assert native.b3_extract(trace_id="zz", span_id="2", sampled="1") == "none"
    d = native.b3_extract(trace_id="1", span_id="2", flags="1")
    assert d["debug"] and d["trace_id"] == "0000000000000001"


def test_b3_extract_single(native):
    d = native.b3_extract(single="80f198ee56343ba864fe8b2a57d3eff7-e457b5a2e4d86bd1-1-05e3ac9a4f6e3b90")
    assert d["trace_id"] == "80f198ee56343ba864fe8b2a57d3eff7"
    assert d["span_id"] == "e457b5a2e4d86bd1" and d["parent_id"] == "05e3ac9a4f6e3b90"
    assert native.b3_extract(single="0") == "not_sampled"
    assert native.b3_extract(single="a-b-0") == "not_sampled"
    assert native.b3_extract(single="d") == "none"  # a sampling flag alone carries no ids
    assert native.b3_extract(single="1-2-d")["debug"]


def test_b3_inject(native):
    h = native.b3_inject("463ac35c9f6413ad", "a2fb4a1d1a96d312", parent="0020000000000001")
    assert h == ("X-B3-TraceId: 463ac35c9f6413ad\r\nX-B3-SpanId: a2fb4a1d1a96d312\r\n"
                 "X-B3-ParentSpanId: 0020000000000001\r\nX-B3-Sampled: 1\r\n")


def test_span_json_v1(native):
    sp = json.loads(native.encode_span(False, "1", "2", parent="3", kind="client", start_us=10, end_us=25,
                                       url="http://aloha:8080/api/aloha-chaining", status=500))[0]
    assert sp["traceId"] == "0000000000000001" and sp["parentId"] == "0000000000000003"
    assert sp["timestamp"] == 10 and sp["duration"] == 15
    assert [a["value"] for a in sp["annotations"]] == ["cs", "cr"]
    keys = {b["key"]: b["value"] for b in sp["binaryAnnotations"]}
    assert keys["http.status_code"] == "500"
    assert sp["annotations"][0]["endpoint"] == {"serviceName": "hola", "ipv4": "127.0.0.1", "port": 8080}


def test_sample_rate_zero_reports_nothing(hola, zipkin):
    s = hola(args=["--zipkin-url", zipkin.url, "--trace-sample-rate", "0"])
    for _ in range(20):
        s.get("/api/hola")
    time.sleep(1.3)
    assert zipkin.spans() == []


def test_sample_rate_half(hola, zipkin):
    s = hola(args=["--zipkin-url", zipkin.url, "--trace-sample-rate", "0.5"], threads=1)
    for _ in range(400):
        s.get("/api/hola")
    spans = zipkin.wait_for(lambda sp: len(sp) >= 120, timeout=5)
    assert 120 <= len(spans) <= 280


def test_export_budget_drops_beyond_the_queue(hola, zipkin):
    """At most --trace-queue spans are exported per flush interval (Brave 3's collector
    queue holds 1000); the rest are counted as dropped with reason queue_full."""
    s = hola(args=["--zipkin-url", zipkin.url, "--trace-queue", "5"], threads=1)
    for _ in range(20):
        assert s.get("/api/hola")[0] == 200
    spans = zipkin.wait_for(lambda sp: len(sp) >= 5)
    time.sleep(1.3)  # one more flush: nothing beyond the budget arrives
    assert len(zipkin.spans()) == 5
    st, _, body = s.get("/metrics")
    assert b'hola_spans_dropped_total{reason="queue_full"} 15' in body
    assert b"hola_spans_reported_total 5" in body
    for _ in range(3):  # the next interval has a fresh budget
        s.get("/api/hola")
    assert len(zipkin.wait_for(lambda sp: len(sp) >= 8)) == 8


def test_native_discard_sink_counts_spans(hola_bin):
    """bench/zipkin_sink.cc (the bench's collector) answers 202 and counts every span of
    v1 and v2 batches."""
    import subprocess
    import tempfile
    from pathlib import Path

    from hola_amd.native import binary
    from hola_amd.server import HolaProcess
    from hola_amd.utils.net import http_get

    pf = Path(tempfile.mkdtemp()) / "port"
    sink = subprocess.Popen([str(binary("hola_zipkin_sink")), "--port", "0", "--port-file", str(pf)])
    try:
        deadline = time.monotonic() + 10
        while not pf.exists() and time.monotonic() < deadline:
            time.sleep(0.01)
        port = int(pf.read_text())
        for extra in ([], ["--zipkin-v2"]):
            s = HolaProcess(args=["--zipkin-url", f"http://127.0.0.1:{port}/", *extra]).start()
            for _ in range(10):
                s.get("/api/hola")
            s.get("/api/health")  # not traced
            s.stop()  # flushes
        st, _, body = http_get("127.0.0.1", port, "/stats")
        stats = json.loads(body)
        assert st == 200 and stats["spans"] == 20 and stats["bad"] == 0 and stats["posts"] >= 2
        assert http_get("127.0.0.1", port, "/api/v1/spans", method="POST", body=b"[]")[0] == 202
    finally:
        sink.terminate()
        sink.wait(timeout=10)


def test_filter_pattern_traces_every_method_on_exact_paths(hola, zipkin):
    """BraveServletFilter is mapped to exactly /api/hola and /api/hola-chaining for all
    methods (ZipKinFilter.java:43): OPTIONS, 405 and 406 answers there get a server span;
    /api/hola/ is served (JAX-RS tolerates the slash) but does not match the pattern."""
    s = hola(args=["--zipkin-url", zipkin.url], threads=1)
    assert s.get("/api/hola", method="OPTIONS")[0] == 200
    assert s.get("/api/hola", method="POST")[0] == 405
    assert s.get("/api/hola", headers={"Accept": "application/json"})[0] == 406
    assert s.get("/api/hola-chaining", method="DELETE")[0] == 405
    assert s.get("/api/hola/")[0] == 200
    assert s.get("/api/hola-chaining/", method="OPTIONS")[0] == 200
    spans = zipkin.wait_for(lambda sp: len(sp) >= 4)
    time.sleep(1.2)
    spans = zipkin.spans()
    assert len(spans) == 4
    names = sorted(sp["name"] for sp in spans)
    assert names == ["delete", "get", "options", "post"]
    codes = sorted(b["value"] for sp in spans for b in sp["binaryAnnotations"] if b["key"] == "http.status_code")
    assert codes == ["405", "405", "406"]
    urls = [b["value"] for sp in spans for b in sp["binaryAnnotations"] if b["key"] == "http.url"]
    assert not any(u.endswith("/") for u in urls)


def test_one_client_span_per_feign_attempt(hola, zipkin):
    """Brave's HttpClient interceptors run once per executed request: a call Feign retries
    5 times (503 + Retry-After: 0) records 5 client spans, children of the server span."""
    with FakeAloha() as aloha:
        aloha.set_mode("unavailable")
        s = hola(args=["--zipkin-url", zipkin.url, "--aloha-url", aloha.url, "--feign-log", "none"])
        st, _, body = s.get("/api/hola-chaining")
        assert st == 200 and json.loads(body)[1:] == ["Aloha response (fallback)"]
        spans = zipkin.wait_for(lambda sp: len(sp) >= 6)
    server = [sp for sp in spans if _annotations(sp) == {"sr", "ss"}]
    client = [sp for sp in spans if _annotations(sp) == {"cs", "cr"}]
    assert len(server) == 1 and len(client) == 5
    assert {sp["traceId"] for sp in spans} == {server[0]["traceId"]}
    assert all(sp["parentId"] == server[0]["id"] for sp in client)
    assert len({sp["id"] for sp in client}) == 5
    for sp in client:
        codes = [b["value"] for b in sp["binaryAnnotations"] if b["key"] == "http.status_code"]
        assert codes == ["503"]
    # each attempt carried its own B3 span id downstream
    sent = [r["headers"].get("x-b3-spanid") for r in aloha.requests]
    assert sorted(sent) == sorted(sp["id"] for sp in client)


@settings(max_examples=500, deadline=None)
@given(st.integers(min_value=1, max_value=2**64 - 1), st.integers(min_value=1, max_value=2**64 - 1),
       st.integers(min_value=0, max_value=2**64 - 1))
def test_b3_inject_hex_matches_python(native, trace, span, parent):
    """The shuffle-table hex encoder (src/tracing/b3.cc hex64) against Python's formatting."""
    h = native.b3_inject(f"{trace:016x}", f"{span:016x}", parent=f"{parent:016x}")
    assert f"X-B3-TraceId: {trace:016x}\r\n" in h and f"X-B3-SpanId: {span:016x}\r\n" in h
    assert f"X-B3-ParentSpanId: {parent:016x}\r\n" in h
