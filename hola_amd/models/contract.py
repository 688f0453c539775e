"""hola's HTTP contract (reference: HolaResource.java, JaxRsActivator.java, CorsFilter.java,
ZipKinFilter.java, HystrixServlet.java, SwaggerListener.java)."""
from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path

FALLBACK_GREETING = "Aloha response (fallback)"  # HolaResource.java:111-112
DEFAULT_GREETING = "Hola de %s"                  # HolaResource.java:60
HEALTH_BODY = "I'm ok"                           # HolaResource.java:85


@dataclass(frozen=True)
class Route:
    path: str
    produces: str | None      # @Produces media type (None: not negotiated)
    cors: bool                # Access-Control-Allow-Origin: * (JAX-RS responses only)
    traced: bool              # Brave servlet filter mapping (ZipKinFilter.java:43)
    methods: tuple[str, ...]
    reference: str


ROUTES: tuple[Route, ...] = (
    Route("/api/hola", "text/plain", True, True, ("GET", "HEAD", "OPTIONS"), "HolaResource.java:52-67"),
    Route("/api/hola-chaining", "application/json", True, True, ("GET", "HEAD", "OPTIONS"),
          "HolaResource.java:69-78"),
    Route("/api/health", "text/plain", True, False, ("GET", "HEAD", "OPTIONS"), "HolaResource.java:80-86"),
    Route("/api/swagger.json", "application/json", True, False, ("GET", "HEAD", "OPTIONS"),
          "SwaggerListener.java:29-42"),
    Route("/api/swagger.yaml", "application/yaml", True, False, ("GET", "HEAD", "OPTIONS"),
          "SwaggerListener.java:29-42"),
    Route("/hystrix.stream", "text/event-stream", False, False, ("GET",), "HystrixServlet.java:13-17"),
    Route("/", "text/html", False, False, ("GET", "HEAD", "OPTIONS"), "src/main/webapp/index.html"),
)


def swagger_spec() -> dict:
    """The Swagger 2.0 document the server embeds (assets/swagger.json)."""
    return json.loads((Path(__file__).resolve().parents[2] / "assets" / "swagger.json").read_text())
