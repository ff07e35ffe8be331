"""Chat prompt rendering: the model's own Jinja chat template when its
tokenizer_config.json has one (rendered in a sandbox, with ``tools``,
``add_generation_prompt``, ``bos_token`` / ``eos_token``, as HF does), else a
built-in template per model family: ``llama3``, ``chatml`` (Qwen; hermes
tool block), ``harmony`` (gpt-oss), ``deepseek`` (DeepSeek-V3/R1).

Built-in templates render tool definitions, assistant ``tool_calls`` and
``tool`` results so a multi-turn agentic conversation round-trips, and so the
render endpoints (and hence the router's precise prefix keys) see the same
tokens the engine prefills.
"""
from __future__ import annotations

import json
import os
from datetime import datetime
from typing import Optional


def _text(content) -> str:
    if isinstance(content, list):
        return "".join(p.get("text", "") for p in content if isinstance(p, dict))
    return content or ""


def _tool_defs(tools) -> list[dict]:
    out = []
    for t in tools or []:
        f = t.get("function", t) if isinstance(t, dict) else {}
        if f.get("name"):
            out.append({"name": f["name"], "description": f.get("description", ""),
                        "parameters": f.get("parameters", {})})
    return out


def _calls(m) -> list[tuple[str, str]]:
    out = []
    for tc in m.get("tool_calls") or []:
        f = tc.get("function", {})
        args = f.get("arguments", {})
        out.append((f.get("name", ""), args if isinstance(args, str) else json.dumps(args)))
    return out


def _llama3(messages, add_gen, tools) -> str:
    out = ["<|begin_of_text|>"]
    defs = _tool_defs(tools)
    if defs:
        sys = "Environment: ipython\n\nYou have access to the following functions. To call a function, respond " \
              "with JSON {\"name\": function name, \"parameters\": {argument: value}}.\n\n" + \
              "\n\n".join(json.dumps({"type": "function", "function": d}) for d in defs)
        out.append(f"<|start_header_id|>system<|end_header_id|>\n\n{sys}<|eot_id|>")
    for m in messages:
        role = "ipython" if m["role"] == "tool" else m["role"]
        body = _text(m.get("content"))
        calls = _calls(m)
        if calls:
            body = "<|python_tag|>" + "; ".join(json.dumps({"name": n, "parameters": json.loads(a or "{}")})
                                                for n, a in calls)
        out.append(f"<|start_header_id|>{role}<|end_header_id|>\n\n{body}<|eot_id|>")
    if add_gen:
        out.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
    return "".join(out)


def _chatml(messages, add_gen, tools) -> str:
    out = []
    defs = _tool_defs(tools)
    msgs = list(messages)
    if defs:
        block = "# Tools\n\nYou may call one or more functions to assist with the user query.\n\n" \
                "You are provided with function signatures within <tools></tools> XML tags:\n<tools>\n" + \
                "\n".join(json.dumps({"type": "function", "function": d}) for d in defs) + \
                "\n</tools>\n\nFor each function call, return a json object with function name and arguments " \
                "within <tool_call></tool_call> XML tags."
        if msgs and msgs[0]["role"] == "system":
            msgs[0] = dict(msgs[0], content=_text(msgs[0].get("content")) + "\n\n" + block)
        else:
            msgs.insert(0, {"role": "system", "content": block})
    for m in msgs:
        body = _text(m.get("content"))
        if m["role"] == "tool":
            out.append(f"<|im_start|>user\n<tool_response>\n{body}\n</tool_response><|im_end|>\n")
            continue
        for n, a in _calls(m):
            body += f"\n<tool_call>\n{{\"name\": \"{n}\", \"arguments\": {a}}}\n</tool_call>"
        out.append(f"<|im_start|>{m['role']}\n{body}<|im_end|>\n")
    if add_gen:
        out.append("<|im_start|>assistant\n")
    return "".join(out)


def _harmony(messages, add_gen, tools) -> str:
    today = datetime.now().strftime("%Y-%m-%d")
    out = [f"<|start|>system<|message|>You are ChatGPT, a large language model trained by OpenAI.\n"
           f"Knowledge cutoff: 2024-06\nCurrent date: {today}\n\nReasoning: medium\n\n"
           f"# Valid channels: analysis, commentary, final. Channel must be included for every message."
           + (" Calls to these tools must go to the commentary channel: 'functions'." if tools else "")
           + "<|end|>"]
    defs = _tool_defs(tools)
    dev = [_text(m.get("content")) for m in messages if m["role"] in ("system", "developer")]
    if dev or defs:
        body = ("# Instructions\n\n" + "\n\n".join(dev) + "\n\n") if dev else ""
        if defs:
            body += "# Tools\n\n## functions\n\nnamespace functions {\n\n" + "\n\n".join(
                f"// {d['description']}\ntype {d['name']} = (_: {json.dumps(d['parameters'])}) => any;"
                for d in defs) + "\n\n} // namespace functions"
        out.append(f"<|start|>developer<|message|>{body}<|end|>")
    last_fn = None
    for m in messages:
        r = m["role"]
        if r in ("system", "developer"):
            continue
        if r == "tool":
            out.append(f"<|start|>functions.{m.get('name') or last_fn or 'tool'} to=assistant<|channel|>commentary"
                       f"<|message|>{_text(m.get('content'))}<|end|>")
            continue
        if r == "assistant":
            if m.get("reasoning_content"):
                out.append(f"<|start|>assistant<|channel|>analysis<|message|>{m['reasoning_content']}<|end|>")
            for n, a in _calls(m):
                last_fn = n
                out.append(f"<|start|>assistant<|channel|>commentary to=functions.{n} <|constrain|>json"
                           f"<|message|>{a}<|call|>")
            if _text(m.get("content")):
                out.append(f"<|start|>assistant<|channel|>final<|message|>{_text(m.get('content'))}<|end|>")
            continue
        out.append(f"<|start|>{r}<|message|>{_text(m.get('content'))}<|end|>")
    if add_gen:
        out.append("<|start|>assistant")
    return "".join(out)


def _deepseek(messages, add_gen, tools) -> str:
    out = ["<｜begin▁of▁sentence｜>"]
    sys = [_text(m.get("content")) for m in messages if m["role"] == "system"]
    defs = _tool_defs(tools)
    if defs:
        sys.append("## Tools\n\n" + "\n".join(json.dumps(d) for d in defs))
    out.append("\n\n".join(sys))
    for m in messages:
        r = m["role"]
        if r == "system":
            continue
        if r == "user":
            out.append(f"<｜User｜>{_text(m.get('content'))}")
        elif r == "tool":
            out.append(f"<｜tool▁output▁begin｜>{_text(m.get('content'))}<｜tool▁output▁end｜>")
        else:
            calls = "".join(f"<｜tool▁call▁begin｜>function<｜tool▁sep｜>{n}\n```json\n{a}\n```<｜tool▁call▁end｜>"
                            for n, a in _calls(m))
            if calls:
                calls = f"<｜tool▁calls▁begin｜>{calls}<｜tool▁calls▁end｜>"
            out.append(f"<｜Assistant｜>{_text(m.get('content'))}{calls}<｜end▁of▁sentence｜>")
    if add_gen:
        out.append("<｜Assistant｜>")
    return "".join(out)


def render_tools(body: dict, enable_auto_tool_choice: bool) -> Optional[list]:
    """The tools a chat request renders into its prompt (vLLM semantics, shared
    by the engine and the render sidecar so their token ids agree): none for
    ``tool_choice: none``; an omitted tool_choice means ``auto`` only when the
    server runs with --enable-auto-tool-choice."""
    tools = body.get("tools")
    if not tools:
        return None
    tc = body.get("tool_choice")
    if tc == "none" or (tc is None and not enable_auto_tool_choice):
        return None
    return tools


BUILTIN = {"llama3": _llama3, "chatml": _chatml, "harmony": _harmony, "deepseek": _deepseek}


def style_for(model_type: str) -> str:
    return {"llama": "llama3", "llava": "llama3", "gpt_oss": "harmony", "deepseek": "deepseek"}.get(model_type, "chatml")


class ChatTemplate:
    def __init__(self, style: str = "chatml", model_dir: Optional[str] = None, template: Optional[str] = None):
        self.style = style
        self.jinja = None
        self.bos = self.eos = ""
        src = template
        if src and os.path.exists(src):
            with open(src) as f:
                src = f.read()
        if src is None and model_dir:
            p = os.path.join(model_dir, "tokenizer_config.json")
            if os.path.exists(p):
                with open(p) as f:
                    tc = json.load(f)
                ct = tc.get("chat_template")
                if isinstance(ct, list):  # [{name, template}]: the default one
                    ct = next((x["template"] for x in ct if x.get("name") == "default"), ct[0]["template"])
                src = ct
                self.bos = _tok_str(tc.get("bos_token"))
                self.eos = _tok_str(tc.get("eos_token"))
        if src:
            self.jinja = _compile(src)

    def render(self, messages: list[dict], add_generation_prompt: bool = True, tools=None, **kw) -> str:
        if self.jinja is not None:
            return self.jinja.render(messages=messages, tools=tools or None,
                                     add_generation_prompt=add_generation_prompt,
                                     bos_token=self.bos, eos_token=self.eos, **kw)
        return BUILTIN[self.style](messages, add_generation_prompt, tools)


def _tok_str(t) -> str:
    if isinstance(t, dict):
        return t.get("content", "")
    return t or ""


def _compile(src: str):
    from jinja2.exceptions import TemplateError
    from jinja2.sandbox import ImmutableSandboxedEnvironment

    def raise_exception(msg):
        raise TemplateError(msg)

    env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
    env.filters["tojson"] = lambda x, indent=None, ensure_ascii=False, separators=None, sort_keys=False: \
        json.dumps(x, indent=indent, ensure_ascii=ensure_ascii, separators=separators, sort_keys=sort_keys)
    env.globals["raise_exception"] = raise_exception
    env.globals["strftime_now"] = lambda fmt: datetime.now().strftime(fmt)
    return env.from_string(src)
