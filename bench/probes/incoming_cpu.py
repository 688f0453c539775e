#!/usr/bin/env python3
"""SO_INCOMING_CPU of loopback connections (diagnostic for the accept-locality counters).

For each (client CPU, server CPU) pair: a listener in a thread pinned to the server CPU, a
client pinned to the client CPU that connects and sends one byte; prints the accepted
socket's SO_INCOMING_CPU before and after that byte, i.e. which CPU the kernel processed the
handshake's last packet and the first data packet on.

    python bench/probes/incoming_cpu.py --clients 128,144 --servers 0,16
"""
import argparse
import json
import os
import socket
import threading

SO_INCOMING_CPU = 49


def one(client_cpu: int, server_cpu: int) -> dict:
    ls = socket.socket()
    ls.bind(("127.0.0.1", 0))
    ls.listen(8)
    port = ls.getsockname()[1]
    out = {}

    def serve():
        os.sched_setaffinity(0, {server_cpu})
        c, _ = ls.accept()
        out["at_accept"] = c.getsockopt(socket.SOL_SOCKET, SO_INCOMING_CPU)
        c.recv(1)
        out["after_data"] = c.getsockopt(socket.SOL_SOCKET, SO_INCOMING_CPU)
        c.close()

    t = threading.Thread(target=serve)
    t.start()
    done = threading.Event()

    def client():
        os.sched_setaffinity(0, {client_cpu})
        s = socket.create_connection(("127.0.0.1", port))
        s.sendall(b"x")
        t.join()
        s.close()
        done.set()

    c = threading.Thread(target=client)
    c.start()
    c.join()
    ls.close()
    return {"client": client_cpu, "server": server_cpu, **out}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--clients", default="128,136,144,152")
    ap.add_argument("--servers", default="0,8,16,24")
    a = ap.parse_args()
    for cc in map(int, a.clients.split(",")):
        for sc in map(int, a.servers.split(",")):
            print(json.dumps(one(cc, sc)), flush=True)


if __name__ == "__main__":
    main()
