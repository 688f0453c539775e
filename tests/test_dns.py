"""aloha's and the Zipkin collector's names are resolved off the request path and off the
span reporter (client/http_client.cc AddressCache): a DNS server that never answers must
neither delay start-up by its timeouts, nor stall span export, nor hold up SIGTERM.

The reference resolves inside each Hystrix thread (HttpClient -> InetAddress), so a hung DNS
costs it one 600 ms timeout per chaining call and nothing else; these tests pin the same.
They run the server in a private network namespace (`unshare -rn`) whose 127.0.0.1:53 (the
container's resolv.conf nameserver) is a UDP socket that swallows every query, so no other
test's lookups are affected."""
import json
import os
import shutil
import subprocess
import sys

import pytest

INNER = r'''
import fcntl, json, os, signal, socket, struct, subprocess, sys, time, http.client

def lo_up():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    ifr = struct.pack("16sH14s", b"lo", 0, b"\0" * 14)
    flags = struct.unpack("16sH14s", fcntl.ioctl(s, 0x8913, ifr))[1]  # SIOCGIFFLAGS
    fcntl.ioctl(s, 0x8914, struct.pack("16sH14s", b"lo", flags | 1, b"\0" * 14))  # SIOCSIFFLAGS |= IFF_UP

try:
    lo_up()
    sink = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sink.bind(("127.0.0.1", 53))  # resolv.conf's nameserver: queries arrive and are never answered
except OSError as e:
    print("cannot set up the namespace:", e)
    sys.exit(77)
with open("/etc/resolv.conf") as f:
    if "nameserver 127.0.0.1" not in f.read():
        print("resolv.conf does not point at 127.0.0.1")
        sys.exit(77)

hola, pf = sys.argv[1], sys.argv[2]
if not os.access(hola, os.X_OK):
    print("the server binary is not reachable from the namespace")
    sys.exit(77)
t0 = time.monotonic()
p = subprocess.Popen([hola, "--host", "127.0.0.1", "--port", "0", "--port-file", pf, "--threads", "1",
                      "--log-level", "warn", "--aloha-url", "http://aloha-unanswered:8080/"],
                     env={**os.environ, "HOSTNAME": "h", "ZIPKIN_SERVER_URL": "http://zipkin-unanswered:9411"},
                     stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
while not (os.path.exists(pf) and open(pf).read().strip()):
    if p.poll() is not None or time.monotonic() - t0 > 20:
        p.kill()
        print(p.stderr.read().decode())
        sys.exit(1)
    time.sleep(0.01)
out = {"startup_s": time.monotonic() - t0}
port = int(open(pf).read())

def get(path):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    t = time.monotonic()
    c.request("GET", path)
    r = c.getresponse()
    return r.status, r.read().decode(), time.monotonic() - t

out["hola"] = get("/api/hola")[:2]
out["chaining"] = get("/api/hola-chaining")
time.sleep(1.2)  # a span flush falls due: the reporter must not be stuck resolving the collector
metrics = get("/metrics")[1]
out["dropped"] = sum(float(l.split()[-1]) for l in metrics.splitlines()
                     if l.startswith("hola_spans_dropped_total") and 'reason="collector"' in l)
t = time.monotonic()
p.send_signal(signal.SIGTERM)
out["rc"] = p.wait(timeout=30)
out["stop_s"] = time.monotonic() - t
out["stderr"] = p.stderr.read().decode(errors="replace")[-4000:]
# the query really was swallowed: the resolver was still waiting when the server left
sink.setblocking(False)
try:
    out["queries"] = len(sink.recv(512)) > 0
except BlockingIOError:
    out["queries"] = False
print(json.dumps(out))
'''


def test_unanswered_dns_neither_delays_startup_nor_shutdown(hola_bin, tmp_path):
    if not shutil.which("unshare"):
        pytest.skip("unshare is not installed")
    script = tmp_path / "inner.py"
    script.write_text(INNER)
    # root (this container) unshares the network alone; anyone else needs a user namespace
    unshare = ["unshare", "-n"] if os.geteuid() == 0 else ["unshare", "-rn"]
    r = subprocess.run([*unshare, sys.executable, str(script), str(hola_bin), str(tmp_path / "port")],
                       capture_output=True, text=True, timeout=90)
    if r.returncode == 77 or (r.returncode != 0 and "unshare" in r.stderr):
        pytest.skip(f"no private network namespace here: {r.stdout or r.stderr}")
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["queries"], res  # the server did ask the silent nameserver
    # start-up waits at most ~1 s for the first answer instead of the resolver's timeouts
    assert res["startup_s"] < 3.0, res
    assert res["hola"] == [200, "Hola de h"]
    status, body, secs = res["chaining"]
    assert status == 200 and json.loads(body) == ["Hola de h", "Aloha response (fallback)"]
    assert 0.5 <= secs < 2.0, res  # the Hystrix timeout, not a DNS timeout
    # the spans recorded so far went to the unresolvable collector and were counted as dropped
    assert res["dropped"] >= 2, res
    # SIGTERM waits for neither stuck getaddrinfo() (aloha's, the collector's)
    assert res["rc"] == 0 and res["stop_s"] < 3.0, res
    # leaving the resolver thread behind is clean under the sanitizer builds too
    assert "Sanitizer" not in res["stderr"] and "runtime error" not in res["stderr"], res["stderr"]
