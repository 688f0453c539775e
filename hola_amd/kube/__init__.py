"""Local executor for the OpenShift/Kubernetes manifests in `deploy/openshift/` (BASELINE
config 5: "manifests applied to local cluster, 8 pods, health probes").

`Cluster` (cluster.py) runs the Service, the DeploymentConfig or Deployment and the
ConfigMaps on this node as host processes: pods from the image's ENTRYPOINT (image.py reads
`deploy/Dockerfile`), readiness-gated endpoints behind `hola_rrproxy`, scaling, ConfigMap
projection and rolling updates (kubelet.py for the per-pod parts). `python -m hola_amd
apply` / `python -m hola_amd oc` (cli.py) are its command line.
"""
from hola_amd.kube.cluster import Cluster, ClusterError

__all__ = ["Cluster", "ClusterError"]
