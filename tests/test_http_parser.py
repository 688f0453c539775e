"""HTTP/1.1 request parser, Accept negotiation and JSON codec (native), incl. fuzzing."""
import json

import pytest
from hypothesis import given, settings, strategies as st


def test_simple_request(native):
    r = native.parse_request(b"GET /api/hola?x=1 HTTP/1.1\r\nHost: a:1\r\nAccept: text/plain\r\n\r\n")
    assert r["method"] == "GET" and r["path"] == "/api/hola" and r["query"] == "x=1"
    assert r["host"] == "a:1" and r["accept"] == "text/plain" and r["keep_alive"]
    assert r["head_bytes"] == len(b"GET /api/hola?x=1 HTTP/1.1\r\nHost: a:1\r\nAccept: text/plain\r\n\r\n")


@pytest.mark.parametrize("raw", [b"", b"GET /api/hola HTTP/1.1\r\n", b"GET /api/hola HTTP/1.1\r\nHost: x\r\n",
                                 b"GET /api/ho"])
def test_incomplete(native, raw):
    assert native.parse_request(raw) == "incomplete"


@pytest.mark.parametrize("raw,status", [
    (b"GET\r\n\r\n", 400),
    (b"GET /x HTTP/1.1 extra\r\n\r\n", 400),
    (b"G@T /x HTTP/1.1\r\n\r\n", 400),
    (b"GET /x HTTP/3.0\r\n\r\n", 505),
    (b"GET /x HTTX/1.1\r\n\r\n", 400),
    (b"GET /x HTTP/1.1\r\n folded\r\n\r\n", 400),
    (b"GET /x HTTP/1.1\r\nName : v\r\n\r\n", 400),
    (b"GET /x HTTP/1.1\r\nContent-Length: abc\r\n\r\n", 400),
    (b"GET /x HTTP/1.1\r\nContent-Length: 1\r\nContent-Length: 2\r\n\r\n", 400),
    (b"GET /x HTTP/1.1\r\nTransfer-Encoding: gzip\r\n\r\n", 501),
    (b"GET /" + b"a" * 9000 + b" HTTP/1.1\r\n\r\n", 414),
    (b"GET /x HTTP/1.1\r\n" + b"X-Pad: " + b"a" * 17000 + b"\r\n\r\n", 431),
    (b"\r\n" * 9000, 400),  # endless blank lines before a request line are bounded too
])
def test_errors(native, raw, status):
    assert native.parse_request(raw) == status


def test_connection_semantics(native):
    assert not native.parse_request(b"GET / HTTP/1.1\r\nConnection: close\r\n\r\n")["keep_alive"]
    assert not native.parse_request(b"GET / HTTP/1.0\r\n\r\n")["keep_alive"]
    assert native.parse_request(b"GET / HTTP/1.0\r\nConnection: Keep-Alive\r\n\r\n")["keep_alive"]
    assert not native.parse_request(b"GET / HTTP/1.1\r\nConnection: upgrade, close\r\n\r\n")["keep_alive"]


def test_lf_only_and_leading_crlf(native):
    r = native.parse_request(b"\r\nGET /a HTTP/1.1\nHost: x\n\n")
    assert r["path"] == "/a" and r["host"] == "x"


def test_b3_header_extraction(native):
    r = native.parse_request(b"GET / HTTP/1.1\r\nX-B3-TraceId: ab\r\nx-b3-spanid: cd\r\nX-B3-ParentSpanId: ef\r\n"
                             b"X-B3-Sampled: 1\r\nX-B3-Flags: 1\r\nb3: 1-2-1\r\n\r\n")
    assert (r["b3_trace_id"], r["b3_span_id"], r["b3_parent_id"], r["b3_sampled"], r["b3_flags"], r["b3_single"]) == \
        ("ab", "cd", "ef", "1", "1", "1-2-1")


def test_absolute_form_target(native):
    r = native.parse_request(b"GET http://host:8080/api/hola?q HTTP/1.1\r\n\r\n")
    assert r["path"] == "/api/hola"


def test_chunked_body(native):
    assert native.skip_chunked_body(b"3\r\nabc\r\n0\r\n\r\n") == 13
    assert native.skip_chunked_body(b"3;ext=1\r\nabc\r\n0\r\nTrailer: x\r\n\r\nNEXT") == 31
    assert native.skip_chunked_body(b"3\r\nab") == "incomplete"
    assert native.skip_chunked_body(b"zz\r\n") == "error"


def test_decode_chunked_body(native):
    assert native.decode_chunked_body(b"3\r\nabc\r\n2;x=y\r\nde\r\n0\r\n\r\n") == (24, b"abcde")
    # bare-LF chunk lines (accepted by the framing) must decode, not overrun the buffer
    assert native.decode_chunked_body(b"3\nabc\n2\nde\n0\n\n") == (14, b"abcde")
    assert native.decode_chunked_body(b"3\r\nabc\r\n") == "incomplete"


@settings(max_examples=200, deadline=None)
@given(st.lists(st.binary(min_size=1, max_size=40), max_size=6), st.booleans())
def test_chunked_roundtrip(native, parts, crlf):
    eol = b"\r\n" if crlf else b"\n"
    raw = b"".join(b"%x" % len(p) + eol + p + eol for p in parts) + b"0" + eol + eol
    assert native.decode_chunked_body(raw) == (len(raw), b"".join(parts))
    assert native.skip_chunked_body(raw) == len(raw)
    for cut in range(len(raw)):
        assert native.decode_chunked_body(raw[:cut]) in ("incomplete", "error")


@settings(max_examples=300, deadline=None)
@given(st.binary(max_size=200))
def test_fuzz_chunked_total(native, data):
    r = native.decode_chunked_body(data)
    assert r in ("incomplete", "error") or (isinstance(r, tuple) and r[0] <= len(data))


_token = st.text(alphabet="abcdefghijklmnopqrstuvwxyz-", min_size=1, max_size=10)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.tuples(_token, st.text(alphabet=st.characters(min_codepoint=0x21, max_codepoint=0x7e),
                                          max_size=20)), max_size=6),
       st.integers(min_value=1, max_value=40))
def test_incremental_equals_whole(native, headers, cut):
    raw = b"GET /p HTTP/1.1\r\n" + b"".join(f"{k}: {v}\r\n".encode() for k, v in headers) + b"\r\n"
    whole = native.parse_request(raw)
    if isinstance(whole, int):
        return
    for i in range(0, len(raw), cut):
        part = native.parse_request(raw[:i])
        assert part == "incomplete" or (isinstance(part, int) and part == whole)
    assert whole["head_bytes"] == len(raw)


@settings(max_examples=500, deadline=None)
@given(st.binary(max_size=400))
def test_fuzz_parser_total(native, data):
    r = native.parse_request(data)
    assert r == "incomplete" or isinstance(r, (int, dict))


_target_bytes = st.lists(st.sampled_from([b"a", b"Z", b"/", b"?", b"%", b".", b" ", b"\t", b"\x01", b"\x7f", b"\x1f",
                                          b"=", b"\x80", b"~"]), min_size=0, max_size=45).map(b"".join)


def _without_head_bytes(r):
    return {k: v for k, v in r.items() if k != "head_bytes"} if isinstance(r, dict) else r


@settings(max_examples=600, deadline=None)
@given(_target_bytes, st.sampled_from([b"HTTP/1.1", b"HTTP/1.0", b"HTTP/2.0", b"HTTP/1.x"]))
def test_vector_and_byte_target_scans_agree(native, target, version):
    """The request target is scanned 32 bytes at a time when the buffer holds 32 more bytes,
    byte by byte otherwise. A padding header makes the same request line take the vector path:
    every outcome (fields, '?' split, 400 for control bytes or a missing SP, 505) must match."""
    def parse(raw):
        try:
            return native.parse_request(raw)
        except UnicodeDecodeError:  # parsed, but the binding cannot hand a 0x80 target to Python
            return "parsed, not UTF-8"

    line = b"GET " + target + b" " + version + b"\r\n"
    short = parse(line + b"\r\n")
    padded = parse(line + b"X-Pad: " + b"p" * 40 + b"\r\n\r\n")
    assert _without_head_bytes(short) == _without_head_bytes(padded), (target, version)


_known = ["Host", "Accept", "Expect", "Connection", "Content-Length", "Transfer-Encoding", "b3", "X-B3-TraceId",
          "X-B3-SpanId", "X-B3-ParentSpanId", "X-B3-Sampled", "X-B3-Flags"]


@settings(max_examples=300, deadline=None)
@given(st.sampled_from(_known), st.data())
def test_header_names_match_case_insensitively_and_nothing_else(native, name, data):
    """Header names are compared eight bytes at a time with a case fold: any mix of case
    matches, a name one token character off does not."""
    mixed = "".join(c.upper() if data.draw(st.booleans()) else c.lower() for c in name)
    assert native.parse_request(f"GET / HTTP/1.1\r\n{mixed}: 7\r\n\r\n".encode()) == \
        native.parse_request(f"GET / HTTP/1.1\r\n{name.lower()}: 7\r\n\r\n".encode())
    pos = data.draw(st.integers(min_value=0, max_value=len(name) - 1))
    other = data.draw(st.sampled_from([c for c in "abcxyz0189-^~_!" if c.lower() != name[pos].lower()]))
    off = name[:pos] + other + name[pos + 1:]
    r = native.parse_request(f"GET / HTTP/1.1\r\n{off}: 7\r\n\r\n".encode())
    plain = native.parse_request(b"GET / HTTP/1.1\r\n\r\n")
    assert _without_head_bytes(r) == _without_head_bytes(plain), off  # an unknown header changes nothing


# ---- negotiation ----

@pytest.mark.parametrize("accept,ok", [
    ("text/plain", True), ("TEXT/PLAIN", True), ("text/*", True), ("*/*", True), ("*", True),
    ("application/json", False), ("text/html", False), ("text/plain;q=0", False),
    ("*/*;q=0.5, text/plain;q=0", False), ("text/*;q=0, text/plain;q=0.1", True),
    ("text/plain; charset=utf-8", True), ("", True), ("garbage", True), ("text/plain;q=2", True),
    ("application/json, text/plain;q=0.001", True),
])
def test_accepts_text_plain(native, accept, ok):
    assert native.accepts(accept, "text", "plain") is ok


# ---- JSON ----

def test_json_string_array(native):
    assert native.string_array(["a", None, 'q"\\\n\x01é']) == '["a",null,"q\\"\\\\\\n\\u0001é"]'.encode()
    assert native.string_array([]) == b"[]"


def test_decode_string_list(native):
    assert native.decode_string_list(b'["a","b"]') == [b"a", b"b"]
    assert native.decode_string_list(b' [ "\\u00e9\\ud83d\\ude00", 1.5, true, null ] ') == \
        ["é😀".encode(), b"1.5", b"true", None]
    for bad in (b'{"a":1}', b'["a",', b'[["x"]]', b'["a"] x', b'', b'[01]'):
        r = native.decode_string_list(bad)
        assert isinstance(r, tuple) and r[0] == "error"


@settings(max_examples=300, deadline=None)
@given(st.lists(st.lists(st.one_of(st.none(), st.text(max_size=40)), max_size=6), min_size=1, max_size=4))
def test_decode_into_a_reused_vector(native, docs):
    """The chainer decodes every aloha answer into the same per-worker vector: each decode
    must give exactly its own document's list, whatever the previous ones held."""
    encoded = [native.string_array(d) for d in docs]
    got = native.decode_string_list_reusing(encoded)
    assert [None if x is None else x.decode() for x in got] == docs[-1]


@settings(max_examples=300, deadline=None)
@given(st.lists(st.one_of(st.none(), st.text(max_size=20)), max_size=8))
def test_json_roundtrip(native, items):
    enc = native.string_array(items)
    assert json.loads(enc) == items
    dec = native.decode_string_list(enc)
    assert [None if x is None else x.decode() for x in dec] == items


@pytest.mark.parametrize("path,want", [
    ("/api/hola", "/api/hola"), ("/api/../api/hola", "/api/hola"), ("/api/./hola", "/api/hola"),
    ("/../api/hola", "/api/hola"), ("/api/hola/.", "/api/hola/"), ("/api/hola/..", "/api/"),
    ("/.", "/"), ("/..", "/"), ("/a/b/../../c", "/c"), ("/api/.hidden", "/api/.hidden"),
    ("/api/..x/../hola", "/api/hola"), ("//a/../b", "//b"), ("rel/path", None),
])
def test_remove_dot_segments(native, path, want):
    assert native.remove_dot_segments(path) == want


def _rfc3986_remove_dot_segments(p: str) -> str:
    """RFC 3986 §5.2.4, step by step, as the oracle."""
    out = []
    while p:
        if p.startswith("../"):
            p = p[3:]
        elif p.startswith("./"):
            p = p[2:]
        elif p.startswith("/./"):
            p = p[2:]
        elif p == "/.":
            p = "/"
        elif p.startswith("/../"):
            p = p[3:]
            if out:
                out.pop()
        elif p == "/..":
            p = "/"
            if out:
                out.pop()
        elif p in (".", ".."):
            p = ""
        else:
            j = p.find("/", 1)
            j = len(p) if j < 0 else j
            out.append(p[:j])
            p = p[j:]
    return "".join(out) or "/"


@settings(max_examples=400, deadline=None)
@given(st.lists(st.sampled_from(["a", "bc", ".", "..", "", "..x", ".y"]), min_size=1, max_size=8))
def test_remove_dot_segments_matches_rfc_oracle(native, segs):
    path = "/" + "/".join(segs)
    assert native.remove_dot_segments(path) == _rfc3986_remove_dot_segments(path)


_seg = st.text(alphabet="abc/;=%3B.", max_size=12)


@given(st.lists(_seg, max_size=6))
@settings(max_examples=300, deadline=None)
def test_strip_path_parameters_properties(native, parts):
    """Against a Python oracle: every ';...' run up to the next '/' goes, '/' never does,
    and stripping is idempotent."""
    p = "/" + "/".join(parts)
    out = native.strip_path_parameters(p)
    oracle = "/".join(seg.split(";", 1)[0] for seg in p.split("/"))
    assert out == oracle
    assert ";" not in out and out.count("/") == p.count("/")
    assert native.strip_path_parameters(out) == out


@given(st.integers(min_value=0, max_value=10**6), st.integers(min_value=-10**6, max_value=10**6))
@settings(max_examples=200, deadline=None)
def test_retry_after_seconds_and_dates(native, secs, skew_s):
    import email.utils

    assert native.parse_retry_after(str(secs), 12345) == secs * 1000
    now_ms = 1_700_000_000_000
    date = email.utils.formatdate(now_ms / 1000 + skew_s, usegmt=True)
    assert native.parse_retry_after(date, now_ms) == skew_s * 1000


# ---- the aloha client's response parser (src/client/http_client.cc) ----

@settings(max_examples=800, deadline=None)
@given(st.one_of(st.binary(max_size=300),
                 st.lists(st.sampled_from([b"HTTP/1.1 ", b"200", b"100", b"204", b" OK", b"\r\n", b"\n", b":",
                                           b"Content-Length", b"content-length", b"Transfer-Encoding", b"chunked",
                                           b"Connection", b"close", b" 5", b"-1", b"+3", b"0\r\n\r\n", b"abc",
                                           b"\x00", b"\r"]), max_size=30).map(b"".join)),
       st.booleans())
def test_fuzz_client_response_parser_total(native, data, eof):
    rc, status, body, close, consumed, head_ok = native.client_parse_response(data, eof)
    assert rc in (-1, 0, 1)
    if rc == 1:
        assert 0 < consumed <= len(data) and status >= 100 and head_ok
        assert len(body) <= consumed


_resp_body = st.binary(max_size=60)


@settings(max_examples=300, deadline=None)
@given(_resp_body, st.sampled_from(["length", "chunked", "close"]), st.integers(min_value=0, max_value=2),
       st.lists(st.tuples(st.sampled_from(["X-A", "Retry-After", "Vary", "Content-Type"]),
                          st.text(alphabet="abc 123;=,", max_size=12)), max_size=3),
       st.integers(min_value=1, max_value=23))
def test_client_response_parser_prefixes_and_whole(native, body, framing, interims, headers, cut):
    """A well-formed response after 0-2 interim ones: every proper prefix needs more, the whole
    parses to the body with every byte consumed, and bytes after it are left alone."""
    head = b"".join(b"HTTP/1.1 100 Continue\r\n\r\n" if i % 2 == 0 else b"HTTP/1.1 103 Early Hints\r\nLink: </x>\r\n\r\n"
                    for i in range(interims))
    head += b"HTTP/1.1 200 OK\r\n" + b"".join(f"{k}: {v.strip()}\r\n".encode() for k, v in headers)
    if framing == "length":
        raw = head + b"Content-Length: %d\r\n\r\n" % len(body) + body
    elif framing == "chunked":
        chunks = [body[i:i + 7] for i in range(0, len(body), 7)]
        raw = head + b"Transfer-Encoding: chunked\r\n\r\n" + b"".join(b"%x\r\n%s\r\n" % (len(c), c) for c in chunks) + b"0\r\n\r\n"
    else:
        raw = head + b"Connection: close\r\n\r\n" + body
    for i in range(0, len(raw), cut):
        rc = native.client_parse_response(raw[:i], False)[0]
        assert rc == 0, (i, raw[:i])
    rc, status, got, close, consumed, head_ok = native.client_parse_response(raw, framing == "close")
    assert (rc, status, got, consumed) == (1, 200, body, len(raw))
    assert close == (framing == "close")
    if framing != "close":  # a pipelined next response is not part of this one
        rc2, _, got2, _, consumed2, _ = native.client_parse_response(raw + b"HTTP/1.1 200 OK\r\n", False)
        assert (rc2, got2, consumed2) == (1, body, len(raw))


@pytest.mark.parametrize("raw,body", [
    (b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\nContent-Length: 12abc\r\n\r\n[]", b"[]"),  # last parseable wins
    (b"HTTP/1.1 200 OK\r\nContent-Length: 9\r\nContent-Length: 2\r\n\r\n[]", b"[]"),
    (b"HTTP/1.1 200 OK\r\nContent-Length:  +2 \r\n\r\n[]", b"[]"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: gzip, chunked\r\n\r\n2\r\n[]\r\n0\r\n\r\n", b"[]"),
    (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked, identity\r\nContent-Length: 1\r\n\r\n[]", b"[]"),  # to the close
    (b"HTTP/1.1 200 OK\r\nContent-Length: -1\r\n\r\n[]", b"[]"),  # negative: to the close
])
def test_client_response_framing_cases(native, raw, body):
    rc, status, got, close, consumed, _ = native.client_parse_response(raw, True)
    assert (rc, status, got, consumed) == (1, 200, body, len(raw))


@settings(max_examples=2000, deadline=None)
@given(st.binary(max_size=80) | st.lists(st.sampled_from([b"a", b'"', b"\\", b"\x01", b"\x1f", b" ", b"\x7f",
                                                          b"\xc3\xa9", b"\x80", b"Hola de "]), max_size=30).map(b"".join))
def test_json_plain_prefix_matches_a_byte_loop(native, data):
    """The SSE2 / word-at-a-time scan (src/core/scan.h) against the byte loop it replaced, at
    every length around its 16- and 8-byte steps; and the encoder's size against its output."""
    want = next((i for i, c in enumerate(data) if c < 0x20 or c in (0x22, 0x5C)), len(data))
    assert native.json_plain_prefix(data) == want
    assert native.json_quoted_size(data) == len(native.json_quote(data))


_ITEM = st.lists(st.sampled_from([b"a", b'"', b"\\", b"\x01", b" ", b"\x7f", b"\xc3\xa9", b"/", b"Hola de ", b",", b"]"]),
                 max_size=6).map(b"".join)


@settings(max_examples=2000, deadline=None)
@given(st.lists(_ITEM, max_size=5), st.sampled_from(["compact", "spaced", "escaped"]))
def test_plain_string_list_is_exactly_what_reencodes_unchanged(native, items, style):
    """json::plain_string_list (aloha's list passed on as text) holds exactly when decoding the
    body and re-encoding its elements gives the same bytes: a compact list of strings with
    nothing to escape. Everything else goes through the decoder."""
    def enc(b):
        return native.json_quote(b)
    if style == "compact":
        body = b"[" + b",".join(enc(i) for i in items) + b"]"
    elif style == "spaced":
        body = b"[ " + b", ".join(enc(i) for i in items) + b" ]"
    else:  # '/' written escaped, as some encoders do
        body = b"[" + b",".join(enc(i).replace(b"/", b"\\/") for i in items) + b"]"
    got = native.json_plain_string_list(body)
    plain = all(native.json_plain_prefix(i) == len(i) for i in items)
    if style == "compact" and plain:
        assert got == len(items), body
    elif style == "spaced" or (style == "escaped" and any(b"/" in i for i in items)) or not plain:
        assert got is None, body
    else:
        assert got == len(items), body


@pytest.mark.parametrize("body", [b"", b"[", b"]", b"[,]", b'["a",]', b'[,"a"]', b'["a""b"]', b'["a]', b'["a"',
                                  b'[null]', b'["a",null]', b'[1]', b'[true]', b'["a\u0041"]', b'{"a":"b"}',
                                  b'["a"] ', b' ["a"]', b'["\x01"]'])
def test_plain_string_list_rejects_what_it_cannot_pass_on(native, body):
    assert native.json_plain_string_list(body) is None
