"""Deploy-descriptor parity with the reference's fabric8/docker configuration
(pom.xml:65-94, 242-280; Dockerfile:1-10). Structural checks only: there is no cluster or
docker daemon here to apply/build them."""
from pathlib import Path

import pytest
import yaml

ROOT = Path(__file__).resolve().parent.parent
OS = ROOT / "deploy" / "openshift"


def items(name: str = "hola.yaml"):
    doc = yaml.safe_load((OS / name).read_text())
    return {i["kind"]: i for i in doc["items"]}


def test_service_matches_fabric8_properties():
    svc = items()["Service"]
    assert svc["metadata"]["name"] == "hola"                       # fabric8.service.name
    assert svc["spec"]["type"] == "LoadBalancer"                   # fabric8.service.type
    (port,) = svc["spec"]["ports"]
    assert port["port"] == 8080 and port["targetPort"] == 8080     # service.port / containerPort
    labels = svc["metadata"]["labels"]
    assert labels["group"] == "msa" and labels["hystrix.enabled"] == "true"  # Turbine discovery


def test_deployment_env_ports_probe():
    dep = items()["Deployment"]
    tpl = dep["spec"]["template"]
    assert set(dep["spec"]["selector"]["matchLabels"].items()) <= set(tpl["metadata"]["labels"].items())
    svc_sel = items()["Service"]["spec"]["selector"]
    assert set(svc_sel.items()) <= set(tpl["metadata"]["labels"].items())
    (c,) = tpl["spec"]["containers"]
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["AB_OFF"] == "true" and env["JAVA_OPTIONS"] == "-Xmx512m"
    assert env["ZIPKIN_SERVER_URL"] == "http://zipkin-query:9411"
    ports = {p["name"]: p["containerPort"] for p in c["ports"]}
    assert ports == {"http": 8080, "jolokia": 8778}
    rp = c["readinessProbe"]
    assert rp["httpGet"] == {"path": "/api/health", "port": 8080}
    assert rp["initialDelaySeconds"] == 5 and rp["timeoutSeconds"] == 30
    assert "livenessProbe" not in c  # the reference declares none


def test_configmap_payload_matches_translation_properties(native):
    cm = yaml.safe_load((OS / "translation-configmap.yaml").read_text())
    payload = cm["data"]["translation.properties"].encode()
    parsed = native.parse_properties(payload)["map"]
    from_file = native.parse_properties((ROOT / "translation.properties").read_bytes())["map"]
    assert parsed == from_file
    patch = yaml.safe_load((OS / "translation-patch.yaml").read_text())
    c = patch["spec"]["template"]["spec"]["containers"][0]
    opts = next(e["value"] for e in c["env"] if e["name"] == "JAVA_OPTIONS")
    conf = native.parse_java_options(opts)["conf"]
    mount = c["volumeMounts"][0]["mountPath"]
    assert conf == f"{mount}/translation.properties"


def test_dockerfile_contract():
    df = (ROOT / "deploy" / "Dockerfile").read_text()
    assert "EXPOSE 8080" in df
    for k in ("AB_OFF=true", "JAVA_OPTIONS=-Xmx512m", "ZIPKIN_SERVER_URL=http://zipkin-query:9411"):
        assert k in df
    for path in ("CMakeLists.txt", "src", "assets", "conf/config.properties", "translation.properties"):
        assert (ROOT / path).exists()


def test_systemd_units_render(tmp_path):
    from hola_amd.deploy import write_units
    from hola_amd.utils.cpu import parse_cpu_list

    paths = write_units(tmp_path, replicas=2)
    names = sorted(p.name for p in paths)
    assert names == ["hola-replica0.service", "hola-replica1.service", "hola-rrproxy.service", "hola.target"]
    r0 = (tmp_path / "hola-replica0.service").read_text()
    r1 = (tmp_path / "hola-replica1.service").read_text()
    cpus0 = r0.split("--cpu-list ")[1].split()[0]
    cpus1 = r1.split("--cpu-list ")[1].split()[0]
    assert not set(parse_cpu_list(cpus0)) & set(parse_cpu_list(cpus1))  # disjoint pinning
    assert f"CPUAffinity={cpus0.replace(',', ' ')}" in r0
    assert "Restart=always" in r0 and "--port 18080" in r0 and "--port 18081" in r1
    px = (tmp_path / "hola-rrproxy.service").read_text()
    assert "--port 8080" in px and "--backends 127.0.0.1:18080,127.0.0.1:18081" in px
    assert "hola-replica1.service" in (tmp_path / "hola.target").read_text()


def test_systemd_units_reuseport(tmp_path):
    from hola_amd.deploy import render_units

    units = render_units(replicas=3, lb="reuseport", public_port=80)
    assert sorted(units) == ["hola-replica0.service", "hola-replica1.service", "hola-replica2.service", "hola.target"]
    for i in range(3):
        u = units[f"hola-replica{i}.service"]
        assert "--port 80 --accept reuseport" in u and "--host 127.0.0.1" not in u
        assert "AmbientCapabilities=CAP_NET_BIND_SERVICE" in u  # binds :80 itself
    assert "SO_REUSEPORT" in units["hola.target"]
    with pytest.raises(ValueError):
        render_units(replicas=1, lb="dns")


def test_license_matches_swagger_document():
    """C24: the project license is Apache-2.0, the one `SwaggerListener` advertises."""
    import json
    text = (ROOT / "LICENSE").read_text()
    assert "Apache-2.0" in text and "http://www.apache.org/licenses/LICENSE-2.0" in text
    lic = json.loads((ROOT / "assets" / "swagger.json").read_text())["info"]["license"]
    assert lic["url"] == "http://www.apache.org/licenses/LICENSE-2.0.html"


def test_deploymentconfig_flavour_for_oc_env_dc():
    """`oc env dc/hola JAVA_OPTIONS=...` (Readme.md:18-24) needs a DeploymentConfig named
    hola: hola-dc.yaml ships one, with the same Service and the same container spec as the
    apps/v1 Deployment in hola.yaml."""
    dc_items = items("hola-dc.yaml")
    assert set(dc_items) == {"Service", "DeploymentConfig"}
    assert dc_items["Service"] == items()["Service"]
    dc = dc_items["DeploymentConfig"]
    assert dc["apiVersion"] == "apps.openshift.io/v1" and dc["metadata"]["name"] == "hola"
    assert dc["metadata"]["labels"]["group"] == "msa" and dc["metadata"]["labels"]["hystrix.enabled"] == "true"
    tpl = dc["spec"]["template"]
    # DC selectors are plain label maps (no matchLabels), matching the pod template and Service
    assert set(dc["spec"]["selector"].items()) <= set(tpl["metadata"]["labels"].items())
    assert set(dc_items["Service"]["spec"]["selector"].items()) <= set(tpl["metadata"]["labels"].items())
    assert {"type": "ConfigChange"} in dc["spec"]["triggers"]
    assert tpl == items()["Deployment"]["spec"]["template"]  # the two flavours never drift
    (c,) = tpl["spec"]["containers"]
    assert c["image"] == "redhatmsa/hola:0.0.1-SNAPSHOT"  # pom.xml:71-72
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["JAVA_OPTIONS"] == "-Xmx512m" and env["AB_OFF"] == "true"
    rp = c["readinessProbe"]
    assert rp["httpGet"] == {"path": "/api/health", "port": 8080}
    assert rp["initialDelaySeconds"] == 5 and rp["timeoutSeconds"] == 30


def test_configmap_patch_applies_to_the_deploymentconfig(native):
    """`oc patch dc/hola -p "$(cat translation-patch.yaml)"`: a strategic merge by container
    name that mounts the ConfigMap and points -Dconf at it."""
    dc = items("hola-dc.yaml")["DeploymentConfig"]
    patch = yaml.safe_load((OS / "translation-patch.yaml").read_text())
    (pc,) = patch["spec"]["template"]["spec"]["containers"]
    (c,) = dc["spec"]["template"]["spec"]["containers"]
    assert pc["name"] == c["name"]
    merged_env = {e["name"]: e.get("value") for e in c["env"]}
    merged_env.update({e["name"]: e["value"] for e in pc["env"]})
    conf = native.parse_java_options(merged_env["JAVA_OPTIONS"])["conf"]
    (vol,) = patch["spec"]["template"]["spec"]["volumes"]
    cm = yaml.safe_load((OS / "translation-configmap.yaml").read_text())
    assert vol["configMap"]["name"] == cm["metadata"]["name"]
    assert conf == pc["volumeMounts"][0]["mountPath"] + "/translation.properties"
    assert "-Xmx512m" in merged_env["JAVA_OPTIONS"]


def test_dockerfile_offers_the_reference_image_name():
    df = (ROOT / "deploy" / "Dockerfile").read_text()
    assert "-t redhatmsa/hola:0.0.1-SNAPSHOT" in df


def test_dockerfile_build_stage_compiles_from_its_copy_set(tmp_path):
    """No docker daemon here, so replay the image's build stage: copy exactly what the
    Dockerfile COPYs into an empty tree and run its cmake commands. Catches a source the
    image would miss (e.g. a new directory that is not COPY'd)."""
    import shutil
    import subprocess

    df = (ROOT / "deploy" / "Dockerfile").read_text().split("\nFROM ", 2)[1]  # build stage only
    copies = [l.split()[1:] for l in df.splitlines() if l.startswith("COPY ") and "--from" not in l]
    assert copies
    for srcs in copies:
        *items, dest = srcs
        for item in items:
            src = ROOT / item
            dst = tmp_path / (item if dest.endswith("/") or dest == "./" else dest)
            if src.is_dir():
                shutil.copytree(src, dst, ignore=shutil.ignore_patterns("__pycache__"))
            else:
                dst.parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(src, dst)
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    bdir = tmp_path / "build"
    r = subprocess.run(["cmake", "-S", str(tmp_path), "-B", str(bdir), *gen, "-DCMAKE_BUILD_TYPE=Release",
                        "-DHOLA_BUILD_PYTHON=OFF"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run(["cmake", "--build", str(bdir), "--target", "hola", "-j", "8"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (bdir / "hola").exists()
