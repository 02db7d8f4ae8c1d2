"""Static checks of the deployment layer (L9) without a cluster: every K8s manifest parses, has
apiVersion/kind/metadata.name, GPU pods request amd.com/gpu, probes hit /health and /status
(reference k8s/api-deployment.yaml), KEDA scales the XAI worker on the task-queue depth, and the
Helm chart's templates reference only values that exist (a helm-free substitute for `helm lint`;
CI runs the real helm lint/template + kubeconform)."""
import glob
import os
import re

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _docs(path):
    with open(path) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def test_k8s_manifests_are_valid_objects():
    kinds = {}
    for p in sorted(glob.glob(os.path.join(ROOT, "k8s", "*.yaml"))):
        for d in _docs(p):
            assert d.get("apiVersion") and d.get("kind") and d.get("metadata", {}).get("name"), p
            kinds.setdefault(d["kind"], []).append(d)
    assert {"Deployment", "Service", "ScaledObject", "HorizontalPodAutoscaler", "Job"} <= set(kinds)
    for dep in kinds["Deployment"]:
        c = dep["spec"]["template"]["spec"]["containers"][0]
        limits = c.get("resources", {}).get("limits", {})
        assert "amd.com/gpu" in limits, dep["metadata"]["name"]
        if "api" in dep["metadata"]["name"]:
            assert c["readinessProbe"]["httpGet"]["path"] == "/health"
            assert c["livenessProbe"]["httpGet"]["path"] == "/status"
    so = kinds["ScaledObject"][0]
    assert any("fdx_task_queue" in str(t) or "fdx_queue_depth" in str(t) for t in so["spec"]["triggers"])
    hpa = kinds["HorizontalPodAutoscaler"][0]
    assert hpa["spec"]["minReplicas"] <= hpa["spec"]["maxReplicas"]


def test_chart_templates_reference_existing_values():
    chart = os.path.join(ROOT, "charts", "fraud-detection-amd")
    with open(os.path.join(chart, "values.yaml")) as f:
        values = yaml.safe_load(f)
    with open(os.path.join(chart, "Chart.yaml")) as f:
        meta = yaml.safe_load(f)
    assert meta["apiVersion"] == "v2" and meta["name"] and meta["version"]
    for t in glob.glob(os.path.join(chart, "templates", "*.yaml")):
        src = open(t).read()
        assert src.count("{{") == src.count("}}"), t
        for ref in re.findall(r"\.Values\.([A-Za-z0-9_.]+)", src):
            node = values
            for k in ref.split("."):
                assert isinstance(node, dict) and k in node, f"{os.path.basename(t)}: .Values.{ref} not in values.yaml"
                node = node[k]
