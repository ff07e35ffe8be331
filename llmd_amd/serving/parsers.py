"""Reasoning and tool-call output parsers for chat completions (the engine
side of the agentic-serving / gpt-oss guides: ``--reasoning-parser``,
``--enable-auto-tool-choice --tool-call-parser``; e.g.
guides/tiered-prefix-cache/modelserver/gpu/vllm/base/patch-vllm-gpt-oss-120b.yaml:18-20).

A parser splits the generated text into ``reasoning_content``, ``content``
and OpenAI ``tool_calls``. Every parser has a one-shot form (``extract``) for
non-streaming responses and an incremental form (``Streamer.feed`` /
``Streamer.finish``) that emits OpenAI chat-chunk deltas: reasoning and
content stream as they are generated (a possibly partial marker at the end
of the buffer is held back), tool calls are emitted whole once the
generation ends (clients accumulate ``tool_calls`` deltas by index either
way).

Reasoning parsers
  deepseek_r1     ``...</think>`` (the ``<think>`` opener is in the prompt)
  qwen3           ``<think>...</think>`` (optional block at the start)
  openai_gptoss   harmony channels: ``analysis`` -> reasoning, ``final`` ->
                  content (also handles ``commentary`` tool calls)
Tool parsers
  hermes          ``<tool_call>{"name": ..., "arguments": {...}}</tool_call>``
  llama3_json     a JSON object (or ``;``-separated objects) with ``name`` and
                  ``parameters``/``arguments``, optionally after ``<|python_tag|>``
  mistral         ``[TOOL_CALLS] [{"name": ..., "arguments": {...}}, ...]``
  pythonic        ``[get_weather(city="SF"), f(x=1)]``
  openai          harmony ``<|channel|>commentary to=functions.NAME ...<|message|>{json}<|call|>``
"""
from __future__ import annotations

import ast
import json
import re
import uuid
from typing import Optional


def _call(name: str, args) -> dict:
    if not isinstance(args, str):
        args = json.dumps(args if args is not None else {}, ensure_ascii=False)
    return {"id": f"chatcmpl-tool-{uuid.uuid4().hex[:24]}", "type": "function",
            "function": {"name": name, "arguments": args}}


# ------------------------------------------------------------------ reasoning
class ThinkReasoning:
    """``<think>`` ... ``</think>``; ``implicit_start``: the generation starts
    inside the block (DeepSeek-R1 templates put ``<think>`` in the prompt)."""

    def __init__(self, start="<think>", end="</think>", implicit_start=False):
        self.start, self.end, self.implicit = start, end, implicit_start

    def extract(self, text: str) -> tuple[Optional[str], str]:
        t = text
        if t.lstrip().startswith(self.start):
            t = t.lstrip()[len(self.start):]
        elif not self.implicit:
            return None, text
        k = t.find(self.end)
        if k < 0:  # still thinking (truncated): all of it is reasoning
            return t, ""
        return t[:k], t[k + len(self.end):].lstrip("\n")


class HarmonyParser:
    """gpt-oss harmony messages: ``[<|start|>assistant]<|channel|>CH[ to=functions.F][ <|constrain|>json]
    <|message|>BODY(<|end|>|<|call|>|<|return|>)``."""

    MSG = re.compile(r"(?:<\|start\|>assistant)?<\|channel\|>(\w+)([^<]*?)(?:<\|constrain\|>\s*\w+\s*)?"
                     r"<\|message\|>(.*?)(?:<\|end\|>|<\|call\|>|<\|return\|>|$)", re.S)

    def parse(self, text: str) -> tuple[Optional[str], str, list]:
        reasoning, content, calls = [], [], []
        matched = False
        for m in self.MSG.finditer(text):
            matched = True
            ch, hdr, body = m.group(1), m.group(2), m.group(3)
            to = re.search(r"to=functions\.([\w.-]+)", hdr)
            if to:
                calls.append(_call(to.group(1), body.strip()))
            elif ch == "analysis":
                reasoning.append(body)
            else:  # final (or commentary text to the user)
                content.append(body)
        if not matched:
            if "<|channel|>" in text or text.startswith("<|"):  # a header still being generated
                return None, "", []
            return None, text, []
        return ("".join(reasoning) or None), "".join(content), calls

    def extract(self, text):
        r, c, _ = self.parse(text)
        return r, c


REASONING_PARSERS = {
    "deepseek_r1": lambda: ThinkReasoning(implicit_start=True),
    "qwen3": lambda: ThinkReasoning(),
    "granite": lambda: ThinkReasoning("Here is my thought process:", "Here is my response:"),
    "openai_gptoss": HarmonyParser,
}


# ------------------------------------------------------------------ tools
def _json_objects(s: str) -> list:
    """Every top-level JSON value in ``s`` (objects / arrays), in order."""
    dec, out, i = json.JSONDecoder(), [], 0
    while i < len(s):
        j = min([k for k in (s.find("{", i), s.find("[", i)) if k >= 0], default=-1)
        if j < 0:
            break
        try:
            v, end = dec.raw_decode(s, j)
        except json.JSONDecodeError:
            i = j + 1
            continue
        out.append(v)
        i = end
    return out


class HermesTools:
    marker = "<tool_call>"
    RE = re.compile(r"<tool_call>\s*(.*?)\s*(?:</tool_call>|$)", re.S)

    def extract(self, text: str) -> tuple[str, list]:
        k = text.find(self.marker)
        if k < 0:
            return text, []
        calls = []
        for m in self.RE.finditer(text[k:]):
            for v in _json_objects(m.group(1))[:1]:
                if isinstance(v, dict) and "name" in v:
                    calls.append(_call(v["name"], v.get("arguments", v.get("parameters", {}))))
        return (text[:k].rstrip() if calls else text), calls


class Llama3JsonTools:
    marker = "<|python_tag|>"

    def extract(self, text: str) -> tuple[str, list]:
        s = text.replace(self.marker, "").strip()
        if not s.startswith("{"):
            return text, []
        calls = []
        for v in _json_objects(s):
            if isinstance(v, dict) and "name" in v:
                calls.append(_call(v["name"], v.get("parameters", v.get("arguments", {}))))
        return ("" if calls else text), calls


class MistralTools:
    marker = "[TOOL_CALLS]"

    def extract(self, text: str) -> tuple[str, list]:
        k = text.find(self.marker)
        if k < 0:
            return text, []
        calls = []
        for v in _json_objects(text[k + len(self.marker):])[:1]:
            for c in (v if isinstance(v, list) else [v]):
                if isinstance(c, dict) and "name" in c:
                    calls.append(_call(c["name"], c.get("arguments", {})))
        return (text[:k].rstrip() if calls else text), calls


class PythonicTools:
    marker = "["

    def extract(self, text: str) -> tuple[str, list]:
        s = text.strip()
        if not (s.startswith("[") and s.endswith("]")):
            return text, []
        try:
            tree = ast.parse(s, mode="eval")
        except SyntaxError:
            return text, []
        if not isinstance(tree.body, ast.List):
            return text, []
        calls = []
        for e in tree.body.elts:
            if not (isinstance(e, ast.Call) and isinstance(e.func, (ast.Name, ast.Attribute))):
                return text, []
            name = e.func.id if isinstance(e.func, ast.Name) else ast.unparse(e.func)
            try:
                args = {kw.arg: ast.literal_eval(kw.value) for kw in e.keywords}
            except ValueError:
                return text, []
            calls.append(_call(name, args))
        return "", calls


class HarmonyTools:
    marker = "to=functions."

    def extract(self, text: str) -> tuple[str, list]:
        _, content, calls = HarmonyParser().parse(text)
        return (content if calls else text), calls


TOOL_PARSERS = {"hermes": HermesTools, "llama3_json": Llama3JsonTools, "mistral": MistralTools,
                "pythonic": PythonicTools, "openai": HarmonyTools}


# ------------------------------------------------------------------ combined
class ChatOutputParser:
    """Reasoning first, then tool calls on the remaining content."""

    def __init__(self, reasoning: Optional[str] = None, tools: Optional[str] = None):
        if reasoning is not None and reasoning not in REASONING_PARSERS:
            raise ValueError(f"unknown reasoning parser {reasoning!r}; known: {sorted(REASONING_PARSERS)}")
        if tools is not None and tools not in TOOL_PARSERS:
            raise ValueError(f"unknown tool-call parser {tools!r}; known: {sorted(TOOL_PARSERS)}")
        self.reasoning = REASONING_PARSERS[reasoning]() if reasoning else None
        self.tools = TOOL_PARSERS[tools]() if tools else None
        self.harmony = isinstance(self.reasoning, HarmonyParser) or isinstance(self.tools, HarmonyTools)

    def extract(self, text: str, use_tools: bool = True) -> tuple[Optional[str], Optional[str], list]:
        if self.harmony:
            r, c, calls = HarmonyParser().parse(text)
            if self.reasoning is None:
                r = None
            if not (use_tools and self.tools is not None):
                calls = []
            return r, (c if c or not calls else None), calls
        r, c = (None, text) if self.reasoning is None else self.reasoning.extract(text)
        calls = []
        if use_tools and self.tools is not None:
            c, calls = self.tools.extract(c)
        return r, (c if c or not calls else None), calls

    def streamer(self, use_tools: bool = True) -> "Streamer":
        return Streamer(self, use_tools)


class Streamer:
    """Incremental deltas from the cumulative generated text."""

    def __init__(self, parser: ChatOutputParser, use_tools: bool):
        self.p = parser
        self.use_tools = use_tools and parser.tools is not None
        self.sent_r = 0   # chars of reasoning already emitted
        self.sent_c = 0   # chars of content already emitted
        self.text = ""

    def _markers(self) -> list[str]:
        ms = []
        if self.p.reasoning is not None and not self.p.harmony:
            ms += [self.p.reasoning.start, self.p.reasoning.end]
        if self.use_tools and not self.p.harmony:
            ms.append(self.p.tools.marker)
        if self.p.harmony:
            ms += ["<|channel|>", "<|message|>", "<|end|>", "<|start|>", "<|call|>", "<|return|>", "<|constrain|>"]
        return ms

    def _held(self, s: str) -> int:
        """Length of a suffix of ``s`` that may be the start of a marker."""
        best = 0
        for m in self._markers():
            for n in range(min(len(m) - 1, len(s)), 0, -1):
                if s.endswith(m[:n]):
                    best = max(best, n)
                    break
        return best

    def feed(self, text: str) -> list[dict]:
        self.text = text
        safe = text[:len(text) - self._held(text)]
        r, c, calls = self.p.extract(safe, use_tools=self.use_tools)
        out = []
        if r and len(r) > self.sent_r:
            out.append({"reasoning_content": r[self.sent_r:]})
            self.sent_r = len(r)
        c = c or ""
        if self.use_tools and not self.p.harmony:
            k = safe.find(self.p.tools.marker)
            if k >= 0 or (isinstance(self.p.tools, (Llama3JsonTools, PythonicTools)) and
                          safe.strip()[:1] in ("{", "[")):
                c = c[:self.sent_c]  # inside a tool call: hold content until the end
        if calls and self.p.harmony:
            c = c[:self.sent_c]
        if len(c) > self.sent_c:
            out.append({"content": c[self.sent_c:]})
            self.sent_c = len(c)
        return out

    def finish(self) -> tuple[list[dict], bool]:
        """Remaining deltas at the end of generation; True if tool calls were made."""
        r, c, calls = self.p.extract(self.text, use_tools=self.use_tools)
        out = []
        if r and len(r) > self.sent_r:
            out.append({"reasoning_content": r[self.sent_r:]})
        c = c or ""
        if len(c) > self.sent_c:
            out.append({"content": c[self.sent_c:]})
        if calls:
            out.append({"tool_calls": [dict(tc, index=i) for i, tc in enumerate(calls)]})
        return out, bool(calls)
