"""The service model: the public HTTP contract of hola as data, shared by
the tests, the docs and anything that needs to know what the service promises.
"""
from hola_amd.models.contract import FALLBACK_GREETING, ROUTES, Route, swagger_spec  # noqa: F401
