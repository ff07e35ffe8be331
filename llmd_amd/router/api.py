"""Control-plane API objects: InferencePool,
InferenceObjective, InferenceModelRewrite, loaded from YAML manifests
(the same documents the reference applies as CRDs, docs/api-reference/*.md).
"""
from __future__ import annotations

import random
from dataclasses import dataclass, field
from typing import Optional

import yaml


@dataclass
class InferencePool:
    name: str
    namespace: str = "default"
    selector: dict = field(default_factory=dict)      # matchLabels (<= 64)
    target_ports: list = field(default_factory=lambda: [8000])  # <= 8, each a distinct endpoint
    app_protocol: str = "http"
    epp_ref: Optional[str] = None
    failure_mode: str = "FailClose"

    @classmethod
    def from_doc(cls, d: dict) -> "InferencePool":
        md, spec = d.get("metadata", {}), d.get("spec", {})
        sel = spec.get("selector", {})
        sel = sel.get("matchLabels", sel)
        if len(sel) > 64:
            raise ValueError("selector: at most 64 matchLabels")
        ports = [p["number"] if isinstance(p, dict) else int(p) for p in spec.get("targetPorts", [{"number": 8000}])]
        if not 1 <= len(ports) <= 8:
            raise ValueError("targetPorts: 1..8 entries")
        ep = spec.get("endpointPickerRef") or {}
        fm = ep.get("failureMode", "FailClose")
        if fm not in ("FailOpen", "FailClose"):
            raise ValueError("failureMode must be FailOpen or FailClose")
        return cls(md.get("name", "pool"), md.get("namespace", "default"), dict(sel), ports,
                   spec.get("appProtocol", "http"), ep.get("name"), fm)


@dataclass
class InferenceObjective:
    name: str
    priority: int = 0
    pool: Optional[str] = None

    @classmethod
    def from_doc(cls, d):
        spec = d.get("spec", {})
        return cls(d.get("metadata", {}).get("name"), int(spec.get("priority", 0) or 0),
                   (spec.get("poolRef") or {}).get("name"))


@dataclass
class RewriteRule:
    matches: list      # [{"model": {"type": "Exact", "value": "x"}}] ; empty = match all
    targets: list      # [{"modelRewrite": "y", "weight": 50}]


@dataclass
class InferenceModelRewrite:
    name: str
    rules: list
    creation: float = 0.0
    pool: Optional[str] = None

    @classmethod
    def from_doc(cls, d, order: float = 0.0):
        spec = d.get("spec", {})
        rules = [RewriteRule(r.get("matches") or [], r.get("targets") or []) for r in spec.get("rules", [])]
        md = d.get("metadata", {})
        ts = md.get("creationTimestamp")
        return cls(md.get("name"), rules, float(order if ts is None else hash(ts) % 10**9),
                   (spec.get("poolRef") or {}).get("name"))


class ControlPlane:
    """Holds objectives and rewrites; resolves priority and model rewrites."""

    def __init__(self):
        self.pools: dict[str, InferencePool] = {}
        self.objectives: dict[str, InferenceObjective] = {}
        self.rewrites: list[InferenceModelRewrite] = []
        self._order = 0

    def load_yaml(self, text: str):
        for d in yaml.safe_load_all(text):
            if not d:
                continue
            self.apply(d)

    def apply(self, d: dict):
        kind = d.get("kind")
        if kind == "InferencePool":
            p = InferencePool.from_doc(d)
            self.pools[p.name] = p
        elif kind == "InferenceObjective":
            o = InferenceObjective.from_doc(d)
            self.objectives[o.name] = o
        elif kind == "InferenceModelRewrite":
            self._order += 1
            self.rewrites.append(InferenceModelRewrite.from_doc(d, self._order))
        else:
            raise ValueError(f"unsupported kind {kind!r}")

    def priority_of(self, objective: Optional[str]) -> int:
        if not objective:
            return 0
        o = self.objectives.get(objective)
        return o.priority if o is not None else 0

    def rewrite(self, model: str) -> tuple[str, Optional[str]]:
        """Precedence: Exact match beats generic (match-all) rules; ties go to
        the oldest resource, then the first rule. Weighted target split."""
        exact, generic = [], []
        for rw in sorted(self.rewrites, key=lambda r: r.creation):
            for i, rule in enumerate(rw.rules):
                if not rule.matches:
                    generic.append((rw, rule))
                    continue
                for m in rule.matches:
                    mm = m.get("model") or {}
                    if mm.get("type", "Exact") == "Exact" and mm.get("value") == model:
                        exact.append((rw, rule))
                        break
        chosen = exact[0] if exact else (generic[0] if generic else None)
        if chosen is None:
            return model, None
        rw, rule = chosen
        if not rule.targets:
            return model, rw.name
        tot = sum(float(t.get("weight", 1)) for t in rule.targets)
        r = random.random() * tot
        acc = 0.0
        for t in rule.targets:
            acc += float(t.get("weight", 1))
            if r <= acc:
                return t.get("modelRewrite", model), rw.name
        return rule.targets[-1].get("modelRewrite", model), rw.name
