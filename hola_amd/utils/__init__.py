from hola_amd.utils.cpu import (  # noqa: F401
    allowed_cpus,
    cgroup_cpu_quota,
    cpu_budget,
    format_cpu_list,
    parse_cpu_list,
    physical_cores,
    plan_cores,
)
from hola_amd.utils.net import free_port, wait_http, http_get  # noqa: F401
