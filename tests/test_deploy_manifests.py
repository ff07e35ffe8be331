"""Deployment packaging lint without helm / kustomize binaries:

* every Gateway provider overlay under deploy/gateway renders (a small
  kustomize subset: resources + JSON6902 ``add`` patches) to the
  ``llm-d-inference-gateway`` Gateway with its provider's class;
* every ``.Values.<path>`` the Helm templates read exists in values.yaml, and
  every values layer (base, features, guides) only sets keys the chart
  defines - a typo in a guide's values file would otherwise be silently
  ignored by helm;
* every EndpointPickerConfig embedded in a values layer loads with the
  router's config loader.
"""
import glob
import os
import re

import pytest
import yaml

from llmd_amd.router.config import load_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GW = os.path.join(ROOT, "deploy/gateway")
CHART = os.path.join(ROOT, "deploy/helm/llmd-amd")


def _kustomize(d: str) -> list[dict]:
    with open(os.path.join(d, "kustomization.yaml")) as f:
        k = yaml.safe_load(f)
    objs = []
    for r in k.get("resources", []):
        p = os.path.normpath(os.path.join(d, r))
        if os.path.isdir(p):
            objs += _kustomize(p)
        else:
            with open(p) as f:
                objs += [o for o in yaml.safe_load_all(f) if o]
    for pt in k.get("patches", []):
        tgt = pt["target"]
        ops = yaml.safe_load(pt["patch"])
        hit = [o for o in objs if o["kind"] == tgt["kind"] and o["metadata"]["name"] == tgt.get("name", o["metadata"]["name"])]
        assert hit, (d, tgt)
        for o in hit:
            for op in ops:
                assert op["op"] == "add", op
                parts = op["path"].strip("/").split("/")
                cur = o
                for q in parts[:-1]:
                    cur = cur.setdefault(q, {})
                cur[parts[-1]] = op["value"]
    return objs


PROVIDERS = {"istio": "istio", "agentgateway": "agentgateway", "agentgateway-openshift": "agentgateway",
             "gke-l7-rilb": "gke-l7-rilb", "gke-l7-regional-external-managed": "gke-l7-regional-external-managed"}


@pytest.mark.parametrize("provider", sorted(PROVIDERS))
def test_gateway_overlays_render(provider):
    objs = _kustomize(os.path.join(GW, provider))
    gws = [o for o in objs if o["kind"] == "Gateway"]
    assert len(gws) == 1 and gws[0]["metadata"]["name"] == "llm-d-inference-gateway"
    assert gws[0]["spec"]["gatewayClassName"] == PROVIDERS[provider]
    assert gws[0]["spec"]["listeners"][0]["port"] == 80
    if provider == "agentgateway-openshift":
        ref = gws[0]["spec"]["infrastructure"]["parametersRef"]
        assert any(o["kind"] == ref["kind"] and o["metadata"]["name"] == ref["name"] for o in objs)


def _values() -> dict:
    with open(os.path.join(CHART, "values.yaml")) as f:
        return yaml.safe_load(f)


def _has(d, path: list[str]) -> bool:
    for p in path:
        if not isinstance(d, dict) or p not in d:
            return False
        d = d[p]
    return True


def test_templates_read_only_defined_values():
    vals = _values()
    missing = set()
    for t in glob.glob(os.path.join(CHART, "templates/*")):
        with open(t) as f:
            text = f.read()
        for m in re.finditer(r"\.Values((?:\.[A-Za-z_][A-Za-z0-9_]*)+)", text):
            path = m.group(1).strip(".").split(".")
            if not _has(vals, path):
                missing.add((os.path.basename(t), ".".join(path)))
    assert not missing, sorted(missing)


# maps whose keys are free-form (resource names, env, labels, nested vendor config)
FREE = {"resources", "limits", "requests", "env", "labels", "annotations", "haLeaseVolume", "gate",
        "scalingConfig", "nodeSelector", "tolerations", "extraEnv"}


def _unknown(layer, ref, path=()) -> list[str]:
    out = []
    if not isinstance(layer, dict):
        return out
    for k, v in layer.items():
        if k in FREE:
            continue
        if not isinstance(ref, dict) or k not in ref:
            out.append(".".join(path + (k,)))
        elif isinstance(v, dict) and isinstance(ref[k], dict):
            out += _unknown(v, ref[k], path + (k,))
    return out


LAYERS = sorted(glob.glob(os.path.join(ROOT, "deploy/values/**/*.values.yaml"), recursive=True))


@pytest.mark.parametrize("layer", LAYERS, ids=[os.path.relpath(p, ROOT) for p in LAYERS])
def test_values_layers_set_only_chart_keys(layer):
    with open(layer) as f:
        v = yaml.safe_load(f) or {}
    assert _unknown(v, _values()) == []
    conf = (v.get("router") or {}).get("pluginsConfig")
    if conf:
        load_config(conf)
