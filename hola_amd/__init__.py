"""hola_amd — a native C++20 re-design of the `hola` greeting microservice (objectiser/hola)
for a single 8×MI355X node.

The service itself is the ``hola`` executable (epoll event loops pinned to the EPYC host
cores). This Python package is the tooling around it:

* :mod:`hola_amd.native`   — build / locate / load the native artefacts
* :mod:`hola_amd.server`   — run a ``hola`` process (tests, smoke, bench)
* :mod:`hola_amd.parallel` — replica scale-out: pinned replica sets, round-robin proxy,
  the 1/2/4/8 scaling harness (the service's analogue of data parallelism)
* :mod:`hola_amd.utils`    — host CPU topology / cgroup quota / port helpers
* :mod:`hola_amd.testing`  — fake aloha and fake Zipkin collector for integration tests
* :mod:`hola_amd.deploy`   — systemd units for a bare-metal node (replicas + proxy)

The GPUs stay idle by design: the reference has no tensor compute.
"""

__version__ = "0.1.0"

from hola_amd.native import binary, build, ensure_built, load_native  # noqa: E402,F401
