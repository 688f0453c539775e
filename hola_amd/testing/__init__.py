"""Fakes for integration tests: a configurable aloha service and a Zipkin collector."""
