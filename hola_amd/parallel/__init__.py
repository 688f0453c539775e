"""Replica scale-out: the service-level analogue of data parallelism.

Stateless replicas pinned to disjoint host cores, fronted by client-side round-robin
(load generator) or the native L4 round-robin proxy (the k8s LoadBalancer role).
"""
