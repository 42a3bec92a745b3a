"""Chat-template rendering.

The reference sends `[system?, user]` messages to llama-server, which applies the GGUF
`tokenizer.chat_template` (`runtime/src/inference.rs:363-376`).  We render that Jinja template
in a sandbox; known formats are also available by name for files without a template:
zephyr (TinyLlama), mistral ([INST], no system role -> folded into the first user turn),
llama3 and chatml (Qwen).
"""
from __future__ import annotations

from typing import Dict, List, Optional

from jinja2.exceptions import TemplateError
from jinja2.sandbox import ImmutableSandboxedEnvironment

BUILTIN = {
    "zephyr": (
        "{% for m in messages %}{{ '<|' + m['role'] + '|>\n' + m['content'] + eos_token + '\n' }}{% endfor %}"
        "{% if add_generation_prompt %}{{ '<|assistant|>\n' }}{% endif %}"
    ),
    "mistral": (
        "{{ bos_token }}{% for m in messages %}{% if m['role'] == 'user' %}{{ '[INST] ' + m['content'] + ' [/INST]' }}"
        "{% elif m['role'] == 'assistant' %}{{ m['content'] + eos_token }}{% endif %}{% endfor %}"
    ),
    "llama3": (
        "{{ bos_token }}{% for m in messages %}{{ '<|start_header_id|>' + m['role'] + '<|end_header_id|>\n\n' + "
        "m['content'] | trim + '<|eot_id|>' }}{% endfor %}"
        "{% if add_generation_prompt %}{{ '<|start_header_id|>assistant<|end_header_id|>\n\n' }}{% endif %}"
    ),
    "chatml": (
        "{% for m in messages %}{{ '<|im_start|>' + m['role'] + '\n' + m['content'] + '<|im_end|>\n' }}{% endfor %}"
        "{% if add_generation_prompt %}{{ '<|im_start|>assistant\n' }}{% endif %}"
    ),
}


def _raise(msg):
    raise TemplateError(msg)


class ChatTemplate:
    def __init__(self, template: str, bos_token: str = "<s>", eos_token: str = "</s>", name: str = "custom"):
        self.name = name
        self.source = BUILTIN.get(template, template)
        self.supports_system = "system" in self.source or template in ("zephyr", "llama3", "chatml")
        if template == "mistral":
            self.supports_system = False
        env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
        env.globals["raise_exception"] = _raise
        self._tmpl = env.from_string(self.source)
        self.bos, self.eos = bos_token, eos_token

    def render(self, messages: List[Dict[str, str]], add_generation_prompt: bool = True) -> str:
        msgs = [dict(m) for m in messages]
        if not self.supports_system and msgs and msgs[0]["role"] == "system":
            sys_msg = msgs.pop(0)["content"]
            if msgs and msgs[0]["role"] == "user":
                msgs[0]["content"] = f"{sys_msg}\n\n{msgs[0]['content']}"
            else:
                msgs.insert(0, {"role": "user", "content": sys_msg})
        try:
            return self._tmpl.render(messages=msgs, add_generation_prompt=add_generation_prompt,
                                     bos_token=self.bos, eos_token=self.eos)
        except TemplateError:
            if self.name == "fallback":
                raise
            return ChatTemplate("chatml", self.bos, self.eos, name="fallback").render(messages,
                                                                                      add_generation_prompt)


def build_messages(prompt: str, system_prompt: Optional[str]) -> List[Dict[str, str]]:
    """[system?, user] exactly like the reference (`runtime/src/inference.rs:363-376`)."""
    msgs = []
    if system_prompt:
        msgs.append({"role": "system", "content": system_prompt})
    msgs.append({"role": "user", "content": prompt})
    return msgs


def for_model(reader_or_template, tokenizer=None) -> ChatTemplate:
    tmpl = reader_or_template
    if hasattr(reader_or_template, "get"):
        tmpl = reader_or_template.get("tokenizer.chat_template") or "zephyr"
    bos = tokenizer.tokens[tokenizer.bos_id] if tokenizer is not None and tokenizer.bos_id >= 0 else "<s>"
    eos = tokenizer.tokens[tokenizer.eos_id] if tokenizer is not None and tokenizer.eos_id >= 0 else "</s>"
    return ChatTemplate(tmpl, bos, eos, name=tmpl if tmpl in BUILTIN else "gguf")
