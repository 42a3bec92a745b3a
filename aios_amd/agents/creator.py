"""CreatorAgent: scaffolds projects, generates code, initialises repositories (reference
`aios_agent/agents/creator.py:24-323`; tools code.*, git.init/add/commit; think(TACTICAL) for a
project spec, think(STRATEGIC) for full projects)."""
from __future__ import annotations

import os
import re
from typing import Any, Dict

from .base import BaseAgent, IntelligenceLevel, main_for

WORKSPACE = os.environ.get("AIOS_WORKSPACE", "/var/lib/aios/workspace")
LANGS = ("python", "rust", "cpp", "hip", "node", "go", "bash")
EXT = {"python": "py", "rust": "rs", "cpp": "cpp", "hip": "hip", "node": "js", "go": "go", "bash": "sh"}
AUTHOR = "aiOS creator <creator@aios.local>"  # git needs 'Name <email>'


def gen_path(directory: str, stem: str, lang: str) -> str:
    return os.path.join(directory, f"{slug(stem) or 'generated'}.{EXT.get(lang, 'txt')}")


def slug(text: str) -> str:
    m = re.search(r"(?:called|named)\s+([A-Za-z0-9_-]+)", text)
    if m:
        return m.group(1).lower()
    words = re.findall(r"[a-z0-9]+", text.lower())
    return "-".join(w for w in words if w not in ("a", "an", "the", "create", "new", "project", "scaffold")
                    )[:40] or "project"


class CreatorAgent(BaseAgent):
    AGENT_TYPE = "creator"
    CAPABILITIES = ("creator.scaffold", "creator.generate_code", "creator.init_repo", "creator.full_project",
                    "code.scaffold", "code.generate", "git.init", "git.add", "git.commit", "fs.write")
    ACTIONS = ((("full project", "complete project", "application"), "full_project"),
               (("scaffold", "new project", "skeleton"), "scaffold"),
               (("repo", "git init"), "init_repo"),
               (("generate", "write code", "implement", "function", "class"), "generate_code"))

    def _lang(self, text: str) -> str:
        t = text.lower()
        return next((l for l in LANGS if l in t), "python")

    async def scaffold(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp, d = task.get("input") or {}, task.get("description", "")
        name = inp.get("name") or slug(d)
        return await self.call_tool("code.scaffold", {"name": name, "project_type": inp.get("project_type",
                                                                                             self._lang(d)),
                                                      "path": inp.get("path", WORKSPACE)})

    async def generate_code(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp, d = task.get("input") or {}, task.get("description", "")
        lang = inp.get("language") or self._lang(d)
        spec = await self.think_json(f"Write {lang} code for: {d}. JSON: {{\"filename\": \"...\", \"code\": \"...\"}}",
                                     IntelligenceLevel.TACTICAL, max_tokens=2048)
        if isinstance(spec, dict) and spec.get("code"):
            path = os.path.join(inp.get("path", WORKSPACE), os.path.basename(spec.get("filename") or f"generated.{lang}"))
            r = await self.call_tool("fs.write", {"path": path, "content": spec["code"]})
            return {"success": r["success"], "path": path, **({} if r["success"] else {"error": r["error"]})}
        # no model available: the tool writes a documented skeleton
        fp = inp.get("file_path") or gen_path(inp.get("path", WORKSPACE), d[:40], lang)
        return await self.call_tool("code.generate", {"file_path": fp, "description": d, "language": lang,
                                                      "create_dirs": True})

    async def init_repo(self, task: Dict[str, Any]) -> Dict[str, Any]:
        path = (task.get("input") or {}).get("path") or os.path.join(WORKSPACE, slug(task.get("description", "")))
        r = await self.call_tool("git.init", {"path": path})
        if not r["success"]:
            return r
        try:
            empty = not [n for n in os.listdir(path) if n != ".git"]
        except OSError:
            empty = False
        if empty:  # a new repository: the initial commit carries a README
            await self.call_tool("fs.write", {"path": os.path.join(path, "README.md"),
                                              "content": f"# {os.path.basename(path)}\n\n{task.get('description', '')}\n"})
        await self.call_tool("git.add", {"repo_path": path, "all": True})
        c = await self.call_tool("git.commit", {"repo_path": path, "message": "Initial commit", "author": AUTHOR})
        return {"success": c["success"], "path": path, "commit": c.get("output", {}).get("commit_hash") if c["success"]
                else None, **({} if c["success"] else {"error": c.get("error")})}

    async def full_project(self, task: Dict[str, Any]) -> Dict[str, Any]:
        d = task.get("description", "")
        plan = await self.think_json(f"Design a small project for: {d}. JSON: {{\"name\": \"...\", \"language\": "
                                     "\"python\", \"files\": [{\"path\": \"...\", \"purpose\": \"...\"}]}",
                                     IntelligenceLevel.STRATEGIC)
        name = (plan or {}).get("name") or slug(d) if isinstance(plan, dict) else slug(d)
        lang = (plan or {}).get("language", self._lang(d)) if isinstance(plan, dict) else self._lang(d)
        sc = await self.call_tool("code.scaffold", {"name": name, "project_type": lang, "path": WORKSPACE})
        if not sc["success"]:
            return sc
        root = sc["output"].get("path", os.path.join(WORKSPACE, name))
        files = plan.get("files", []) if isinstance(plan, dict) else []
        made = []
        for f in files[:10]:
            rel = f.get("path") or gen_path("", f.get("purpose", "module"), lang)
            r = await self.call_tool("code.generate", {"file_path": os.path.join(root, rel.lstrip("/")),
                                                       "description": f.get("purpose", ""), "language": lang,
                                                       "create_dirs": True})
            if r["success"]:
                made.append(f.get("path"))
        repo = await self.init_repo({"input": {"path": root}})
        return {"success": True, "path": root, "files_generated": made, "repo": repo.get("success")}


if __name__ == "__main__":
    main_for(CreatorAgent)
