"""EndpointPickerConfig loader, validator and defaulting (SURVEY C04/C05;
docs/architecture/core/router/epp/configuration.md, docs/api-reference/
endpointpickerconfig.md).

Accepts the reference's config text verbatim, either as a bare
``EndpointPickerConfig`` document or embedded in router Helm values
(``router.epp.pluginsCustomConfig[<pluginsConfigFile>]``).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field
from typing import Any, Optional

import yaml

from .plugins import base as pb

log = logging.getLogger("llmd.router.config")

API_VERSION = "llm-d.ai/v1alpha1"
KIND = "EndpointPickerConfig"
KNOWN_GATES = {"flowControl"}


class ConfigError(ValueError):
    pass


@dataclass
class Profile:
    name: str
    filters: list = field(default_factory=list)
    scorers: list = field(default_factory=list)  # (Scorer, weight)
    picker: Any = None


@dataclass
class EPPConfig:
    plugins: dict
    profiles: dict  # name -> Profile (ordered)
    profile_handler: Any
    parser: Any
    feature_gates: set
    flow_control: Optional[dict]
    saturation_detector: Any
    admitters: list
    producers: list
    pre_request: list
    response_processors: list
    data_sources: list  # (source, [extractors])
    raw: dict

    @property
    def flow_control_enabled(self) -> bool:
        return "flowControl" in self.feature_gates


def extract_config_text(text: str) -> dict:
    """Return the EndpointPickerConfig dict from raw text or Helm values."""
    docs = [d for d in yaml.safe_load_all(text) if d]
    for d in docs:
        if d.get("kind") == KIND:
            return d
        epp = ((d.get("router") or {}).get("epp") or {}) if isinstance(d, dict) else {}
        custom = epp.get("pluginsCustomConfig") or {}
        if custom:
            fname = epp.get("pluginsConfigFile") or next(iter(custom))
            inner = custom.get(fname) or next(iter(custom.values()))
            return extract_config_text(inner)
    raise ConfigError("no EndpointPickerConfig document found")


def _load_plugin_modules():
    # importing registers every plugin type
    from . import datalayer, flow_control  # noqa: F401
    from .plugins import parsers, producers, scheduling  # noqa: F401


def load_config(text_or_dict, ctx=None) -> EPPConfig:
    _load_plugin_modules()
    raw = extract_config_text(text_or_dict) if isinstance(text_or_dict, str) else dict(text_or_dict)
    if raw.get("apiVersion", API_VERSION) != API_VERSION:
        raise ConfigError(f"apiVersion must be {API_VERSION}")
    if raw.get("kind", KIND) != KIND:
        raise ConfigError(f"kind must be {KIND}")
    gates = set(raw.get("featureGates") or [])
    for g in gates - KNOWN_GATES:
        log.warning("unknown feature gate %s ignored", g)
    # ---------------------------------------------------------- plugins
    plugins: dict[str, pb.Plugin] = {}
    for spec in raw.get("plugins") or []:
        t = spec.get("type")
        if not t:
            raise ConfigError("plugin entry without type")
        name = spec.get("name") or t
        if name in plugins:
            raise ConfigError(f"duplicate plugin name {name!r}")
        if t in pb.DEPRECATED_ALIASES:
            log.warning("plugin type %s is deprecated, use %s", t, pb.DEPRECATED_ALIASES[t])
        try:
            plugins[name] = pb.create(t, name, spec.get("parameters") or {}, ctx)
        except ValueError as e:
            raise ConfigError(str(e)) from e

    def ref(r, role: Optional[str] = None):
        if r not in plugins:
            raise ConfigError(f"reference to undefined plugin {r!r}")
        p = plugins[r]
        if role and role not in pb.roles(p):
            raise ConfigError(f"plugin {r!r} is not a {role}")
        return p

    # a prefix scorer without any prefix producer: auto-instantiate the approximate one
    has_prefix_scorer = any(p.plugin_type == "prefix-cache-scorer" for p in plugins.values())
    has_prefix_producer = any(p.plugin_type in ("approx-prefix-cache-producer", "precise-prefix-cache-producer")
                              for p in plugins.values())
    if has_prefix_scorer and not has_prefix_producer:
        plugins["approx-prefix-cache-producer"] = pb.create("approx-prefix-cache-producer", None, {}, ctx)

    # ---------------------------------------------------------- profiles
    profiles: dict[str, Profile] = {}
    sp = raw.get("schedulingProfiles")
    if sp is None:
        # tier 1: a default profile referencing every filter/scorer/picker
        sp = [{"name": "default", "plugins": [{"pluginRef": n} for n, p in plugins.items()
                                              if pb.roles(p) & {"filter", "scorer", "picker"}]}]
    for prof in sp:
        pname = prof.get("name")
        if not pname:
            raise ConfigError("scheduling profile without name")
        if pname in profiles:
            raise ConfigError(f"duplicate scheduling profile {pname!r}")
        P = Profile(pname)
        for ent in prof.get("plugins") or []:
            p = ref(ent.get("pluginRef"))
            rs = pb.roles(p)
            if "filter" in rs:
                P.filters.append(p)
            if "scorer" in rs:
                w = ent.get("weight", 1.0)
                P.scorers.append((p, float(1.0 if w is None else w)))
            if "picker" in rs:
                if P.picker is not None:
                    raise ConfigError(f"profile {pname!r} references more than one picker")
                P.picker = p
            if not rs & {"filter", "scorer", "picker"}:
                # e.g. a data producer listed for readability: auto-wired elsewhere, no role here
                log.debug("plugin %s has no scheduling role in profile %s", p.name, pname)
        if P.picker is None:  # tier 3
            P.picker = pb.create("max-score-picker", "max-score-picker", {"maxNumOfEndpoints": 1}, ctx)
        profiles[pname] = P
    if not profiles:
        raise ConfigError("no scheduling profiles")
    handlers = [p for p in plugins.values() if "profile-handler" in pb.roles(p)]
    if len(handlers) > 1:
        raise ConfigError("only one profile handler plugin is allowed")
    if handlers:
        handler = handlers[0]
    else:
        if len(profiles) > 1:
            raise ConfigError("multiple scheduling profiles require a profile handler plugin")
        handler = pb.create("single-profile-handler", "single-profile-handler", {}, ctx)
    # ---------------------------------------------------------- parser
    # parser: top-level ``parser.pluginRef``, or ``requestHandler.parser.pluginRef`` /
    # ``requestHandler.parsers[].pluginRef`` (docs/api-reference/epp-grpc-apis.md:16-33)
    rh = raw.get("requestHandler") or {}
    pref = ((raw.get("parser") or {}).get("pluginRef") or (rh.get("parser") or {}).get("pluginRef")
            or next((p.get("pluginRef") for p in (rh.get("parsers") or []) if isinstance(p, dict)), None))
    parser = ref(pref, "parser") if pref else pb.create("openai-parser", "openai-parser", {}, ctx)
    # ---------------------------------------------------------- flow control
    fc = raw.get("flowControl")
    if fc is not None and "flowControl" not in gates:
        log.warning("flowControl section present but the flowControl feature gate is off")
    sd_ref = (raw.get("saturationDetector") or {}).get("pluginRef")
    if sd_ref:
        detector = ref(sd_ref, "saturation-detector")
    else:
        existing = [p for p in plugins.values() if p.plugin_type == "utilization-detector"]
        detector = existing[0] if existing else pb.create("utilization-detector", "utilization-detector", {}, ctx)
    if fc:
        for b in [fc.get("defaultPriorityBand") or {}] + list(fc.get("priorityBands") or []):
            for k in ("orderingPolicyRef", "fairnessPolicyRef"):
                if b.get(k):
                    ref(b[k], "ordering" if k.startswith("ordering") else "fairness")
        prios = [b.get("priority") for b in fc.get("priorityBands") or []]
        if any(p is None for p in prios):
            raise ConfigError("priorityBands entries require a priority")
        if len(set(prios)) != len(prios):
            raise ConfigError("duplicate priority band")
    # ---------------------------------------------------------- auto-wired roles
    admitters = [p for p in plugins.values() if "admitter" in pb.roles(p)]
    producers = [p for p in plugins.values() if "data-producer" in pb.roles(p)]
    # producer ordering: tokenization first, then prefix/inflight, then predictions
    order = {"token-producer": 0, "inflight-load-producer": 1, "approx-prefix-cache-producer": 2,
             "precise-prefix-cache-producer": 2, "predicted-latency-producer": 5}
    producers.sort(key=lambda p: order.get(p.plugin_type, 3))
    pre = [p for p in plugins.values() if "pre-request" in pb.roles(p)]
    resp = [p for p in plugins.values() if "response-processor" in pb.roles(p)]
    # ---------------------------------------------------------- data layer
    dl = raw.get("dataLayer") or {}
    sources = []
    for s in dl.get("sources") or []:
        src = ref(s.get("pluginRef"), "data-source")
        exs = []
        for x in s.get("extractors") or []:
            xp = ref(x.get("pluginRef"))
            # Extractor, or an EndpointExtractor (endpoint lifecycle hooks)
            if "extractor" not in pb.roles(xp) and not hasattr(xp, "on_endpoint_added"):
                raise ConfigError(f"plugin {xp.name!r} is not an extractor")
            exs.append(xp)
        sources.append((src, exs))
    _check_extractor_dag(dl)
    inject = dl.get("injectDefaults", True)
    if inject and not any(s.plugin_type == "metrics-data-source" for s, _ in sources):
        src = pb.create("metrics-data-source", "metrics-data-source", {}, ctx)
        ex = pb.create("core-metrics-extractor", "core-metrics-extractor", {}, ctx)
        sources.append((src, [ex]))
    return EPPConfig(plugins, profiles, handler, parser, gates, fc, detector, admitters, producers, pre, resp,
                     sources, raw)


def _check_extractor_dag(dl: dict):
    """Extractors may declare `dependsOn` other extractors: must be acyclic."""
    deps = {}
    for s in dl.get("sources") or []:
        for x in s.get("extractors") or []:
            deps[x.get("pluginRef")] = list(x.get("dependsOn") or [])
    state = {}

    def visit(n):
        if state.get(n) == 1:
            raise ConfigError(f"extractor dependency cycle at {n!r}")
        if state.get(n) == 2:
            return
        state[n] = 1
        for m in deps.get(n, []):
            visit(m)
        state[n] = 2

    for n in deps:
        visit(n)
