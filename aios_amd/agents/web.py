"""WebAgent: browse / scrape, search, API interaction, URL monitoring, webhook notification
(reference `aios_agent/agents/web.py:24-382`; tools web.scrape / http_request / api_call /
webhook; think(OPERATIONAL) to summarise pages and to shape API calls)."""
from __future__ import annotations

import json
import os
import re
import time
from typing import Any, Dict
from urllib.parse import quote_plus

from .base import BaseAgent, IntelligenceLevel, main_for

URL_MONITOR_INTERVAL_S = 60.0
_URL = re.compile(r"https?://[^\s\"'<>]+")


class WebAgent(BaseAgent):
    AGENT_TYPE = "web"
    CAPABILITIES = ("web.browse", "web.search", "web.api_interact", "web.monitor_url", "web.notify", "web.scrape",
                    "web.http_request", "web.api_call", "web.webhook", "web.download")
    ACTIONS = ((("webhook", "notify", "alert"), "notify"),
               (("monitor", "watch", "uptime of"), "monitor_url"),
               (("search", "look up", "google"), "search"),
               (("api", "endpoint", "post ", "json"), "api_interact"),
               (("download",), "download"),
               (("browse", "scrape", "fetch", "read page", "http"), "browse"))

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.watched: Dict[str, Dict[str, Any]] = {}

    def _url(self, task):
        inp = task.get("input") or {}
        if inp.get("url"):
            return inp["url"]
        m = _URL.search(task.get("description", ""))
        return m.group(0).rstrip(".,)") if m else ""

    async def browse(self, task: Dict[str, Any]) -> Dict[str, Any]:
        url = self._url(task)
        if not url:
            return {"success": False, "error": "no URL in task"}
        r = await self.call_tool("web.scrape", {"url": url})
        if r["success"] and (task.get("input") or {}).get("summarize", True):
            text = str(r["output"].get("text", ""))[:4000]
            summary = await self.think_json(f"Summarise this page in JSON {{\"summary\": \"...\"}}:\n{text}",
                                            IntelligenceLevel.OPERATIONAL)
            if isinstance(summary, dict):
                r["summary"] = summary.get("summary")
        return r

    async def search(self, task: Dict[str, Any]) -> Dict[str, Any]:
        q = (task.get("input") or {}).get("query") or re.sub(r"^(search|look up)( for)?\s+", "",
                                                             task.get("description", ""), flags=re.I)
        return await self.call_tool("web.scrape", {"url": f"https://duckduckgo.com/html/?q={quote_plus(q)}"})

    async def api_interact(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp = task.get("input") or {}
        url = self._url(task)
        if not url:
            return {"success": False, "error": "no URL in task"}
        method = inp.get("method", "GET")
        r = await self.call_tool("web.api_call", {"url": url, "method": method,
                                                  "body": inp.get("body"), "headers": inp.get("headers", {}),
                                                  "query_params": inp.get("query_params", {})})
        if r["success"] and inp.get("interpret"):
            # the model's reading of the response when asked for (reference web.py:234)
            out = r.get("output", {})
            body = json.dumps(out.get("data", out.get("body", {})), default=str)[:3000]
            r["interpretation"] = await self.analyze(
                f"Interpret this API response:\nURL: {url}\nMethod: {method}\n"
                f"Status: {out.get('status', 'unknown')}\nResponse: {body}\n\n"
                "Provide a brief interpretation of what this response means.", IntelligenceLevel.OPERATIONAL)
        return r

    async def download(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp = task.get("input") or {}
        url = self._url(task)
        if not url:
            return {"success": False, "error": "no URL in task"}
        name = os.path.basename(url.split("?")[0].rstrip("/")) or "download"
        dst = inp.get("destination") or os.path.join(inp.get("path", "/var/lib/aios/downloads"), name)
        return await self.call_tool("web.download", {"url": url, "destination": dst, "create_dirs": True})

    async def monitor_url(self, task: Dict[str, Any]) -> Dict[str, Any]:
        url = self._url(task)
        if not url:
            return {"success": False, "error": "no URL in task"}
        t0 = time.time()
        r = await self.call_tool("web.http_request", {"url": url, "method": "GET"})
        status = r.get("output", {}).get("status", 0) if r["success"] else 0
        up = r["success"] and 200 <= int(status or 0) < 400
        prev = self.watched.get(url, {}).get("up")
        self.watched[url] = {"up": up, "status": status, "latency_ms": int((time.time() - t0) * 1000),
                             "checked": int(time.time())}
        if prev is not None and prev != up:
            try:
                await self.push_event("web.url_state_changed", {"url": url, "up": up}, critical=not up)
            except Exception:
                pass
        return {"success": True, "url": url, **self.watched[url]}

    async def notify(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp = task.get("input") or {}
        url = self._url(task)
        if not url:
            return {"success": False, "error": "no webhook URL"}
        return await self.call_tool("web.webhook", {"url": url, "payload": inp.get("payload",
                                                                                  {"text": task.get("description")})})

    async def background(self):
        async def recheck():
            for url in list(self.watched):
                await self.monitor_url({"input": {"url": url}})
        return [self.periodic(URL_MONITOR_INTERVAL_S, recheck)]


if __name__ == "__main__":
    main_for(WebAgent)
