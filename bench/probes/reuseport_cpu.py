#!/usr/bin/env python3
"""Does the kernel honour SO_INCOMING_CPU inside an SO_REUSEPORT group? (diagnostic)

Two (or more) listeners on one port, each with SO_INCOMING_CPU set to a client CPU; clients
pinned to those CPUs connect; prints which listener accepted each client's connections.
Linux 6.1+ picks the listener whose incoming CPU matches the CPU the SYN is processed on
(commit "soreuseport: Fix socket selection for SO_INCOMING_CPU"); older kernels hash.

    python bench/probes/reuseport_cpu.py --cpus 128,144 [--per-client 16]
"""
import argparse
import json
import os
import select
import socket

SO_INCOMING_CPU = 49


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--cpus", default="128,144")
    ap.add_argument("--per-client", type=int, default=16)
    a = ap.parse_args()
    cpus = [int(x) for x in a.cpus.split(",")]
    lss = []
    port = 0
    for c in cpus:
        s = socket.socket()
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
        s.setsockopt(socket.SOL_SOCKET, SO_INCOMING_CPU, c)
        s.bind(("127.0.0.1", port))
        port = s.getsockname()[1]
        s.listen(256)
        s.setblocking(False)
        lss.append(s)
    counts = {c: {c2: 0 for c2 in cpus} for c in cpus}  # client cpu -> listener cpu -> n
    old = os.sched_getaffinity(0)
    for c in cpus:
        os.sched_setaffinity(0, {c})
        conns = [socket.create_connection(("127.0.0.1", port)) for _ in range(a.per_client)]
        os.sched_setaffinity(0, old)
        got = 0
        while got < a.per_client:
            r, _, _ = select.select(lss, [], [], 2)
            if not r:
                break
            for i, s in enumerate(lss):
                if s in r:
                    try:
                        while True:
                            x, _ = s.accept()
                            x.close()
                            counts[c][cpus[i]] += 1
                            got += 1
                    except BlockingIOError:
                        pass
        for x in conns:
            x.close()
    print(json.dumps({"kernel": os.uname().release, "accepted_by": {str(k): v for k, v in counts.items()}}))


if __name__ == "__main__":
    main()
