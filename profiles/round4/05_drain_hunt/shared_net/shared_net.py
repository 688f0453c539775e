"""Two executor clusters handing out the SAME pod network (as before round 3's per-cluster
flock), both rolling their 8 pods without the shutdown delay under load, with the server of
the hang's era (HOLA_SERVER_BIN). Counts pods that outlive their grace period."""
import json, subprocess, sys, threading, time
from pathlib import Path
sys.path.insert(0, "/root/repo")
from hola_amd import native
from hola_amd.kube import Cluster
from hola_amd.kube import cluster as cl

OS = Path("/root/repo/deploy/openshift")
out = Path(sys.argv[1]); minutes = float(sys.argv[2])
out.mkdir(parents=True, exist_ok=True)
shared = {}
orig = cl.Cluster._claim_network
def claim(self):
    if "net" in shared:
        self.net = shared["net"]
        return open("/dev/null")
    f = orig(self)
    shared["net"] = self.net
    return f
cl.Cluster._claim_network = claim
clusters = [Cluster([OS / "hola-dc.yaml"], state_dir=out / f"c{i}", replicas=8, node_cpus=64,
                    service_port=0, zipkin=(i == 0)).start() for i in range(2)]
for c in clusters:
    c.wait_ready(8, timeout=300)
patch = {"spec": {"template": {"spec": {"containers": [{"name": "hola", "args": ["--shutdown-delay-ms", "0"]}]}}}}
for c in clusters:
    rev = c.rollout_status()["revision"]
    c.patch(patch)
    c.wait(lambda: c.rollout_status()["revision"] > rev and c.rollout_status()["complete"], 600, "patch")
lgs = [subprocess.Popen([str(native.binary("hola_loadgen")), "-t", "2", "-c", "256", "-d", "86400s", "--json",
                         c.service_url() + "/api/hola"], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
       for c in clusters]
stop = time.monotonic() + minutes * 60
def roll(c, k=[0]):
    i = 0
    while time.monotonic() < stop:
        i += 1
        rev = c.rollout_status()["revision"]
        c.set_env({"JAVA_OPTIONS": f"-Xmx512m -Dshared={i}"})
        try:
            c.wait(lambda: c.rollout_status()["revision"] > rev and c.rollout_status()["complete"], 300, "rollout")
            c.wait(lambda: all(p["status"] != "Terminating" for p in c.get_pods()), 120, "old gone")
        except TimeoutError as e:
            print("timeout", c.state, str(e)[:300], flush=True)
ts = [threading.Thread(target=roll, args=(c,)) for c in clusters]
[t.start() for t in ts]; [t.join() for t in ts]
for lg in lgs:
    lg.kill()
res = {}
for c in clusters:
    ev = list(c.events)
    res[str(c.state)] = {"killing": sum(e[2] == "Killing" for e in ev), "killed": [e[3][:600] for e in ev if e[2] == "Killed"],
                         "died": sum(e[2] in ("Died", "BackOff") for e in ev)}
for c in clusters:
    c.close(grace_s=5)
print(json.dumps(res, indent=1), flush=True)
