"""Management console: REST + WebSocket + single-page dashboard on :9090.

Reference: `agent-core/src/management.rs` -- routes `:43-55` (/api/status, /api/goals GET/POST,
/api/goals/{id}/tasks, /api/goals/{id}/messages GET/POST, /api/chat, /api/agents, /api/health,
/ws, /), posting a message resumes awaiting_input tasks (`:251-289`), chat builds a live-state
system prompt and calls the gateway (`:292-473`), goal submission stores the preferred provider
in the goal metadata (`:475-512`), the WebSocket pushes full state every 2 s and honours
`subscribe_goal` (`:565-713`).  Extra here: /api/gpus (amdgpu telemetry), /api/decisions,
/api/schedules, /api/metrics (Prometheus text).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time

from aiohttp import WSMsgType, web

from ..utils import sysinfo
from .state import OrchestratorState

log = logging.getLogger("aios.management")


def _uptime(s: float) -> str:
    s = int(s)
    return f"{s // 3600}h {(s % 3600) // 60}m" if s >= 3600 else f"{s // 60}m {s % 60}s"


class ManagementConsole:
    def __init__(self, st: OrchestratorState, host: str = "0.0.0.0", port: int = 9090):
        self.st, self.host, self.port = st, host, port
        self.app = web.Application()
        r = self.app.router
        r.add_get("/", self.dashboard)
        r.add_get("/api/status", self.status)
        r.add_get("/api/goals", self.list_goals)
        r.add_post("/api/goals", self.submit_goal)
        r.add_get("/api/goals/{goal_id}/tasks", self.goal_tasks)
        r.add_get("/api/goals/{goal_id}/messages", self.goal_messages)
        r.add_post("/api/goals/{goal_id}/messages", self.post_message)
        r.add_post("/api/chat", self.chat)
        r.add_get("/api/agents", self.agents)
        r.add_get("/api/health", self.health)
        r.add_get("/api/gpus", self.gpus)
        r.add_get("/api/decisions", self.decisions)
        r.add_get("/api/schedules", self.schedules)
        r.add_get("/api/events", self.events)
        r.add_post("/api/events", self.publish_event)
        r.add_post("/api/events/subscriptions", self.subscribe_event)
        r.add_get("/api/metrics", self.metrics)
        r.add_get("/ws", self.ws)
        self.runner = None

    async def start(self):
        self.runner = web.AppRunner(self.app, access_log=None)
        await self.runner.setup()
        site = web.TCPSite(self.runner, self.host, self.port)
        await site.start()
        log.info("management console on http://%s:%d", self.host, self.port)

    async def stop(self):
        if self.runner:
            await self.runner.cleanup()

    # ------------------------------------------------------------------ state
    def state_dict(self) -> dict:
        st = self.st
        c = st.goal_engine.counts()
        used, total = sysinfo.memory_mb()
        goals, _ = st.goal_engine.list("", 50, 0)
        lat = sorted(st.plan_latency_ms[-200:])
        return {
            "status": {**c, "active_agents": st.router.healthy_count(), "uptime": _uptime(time.time() - st.started),
                       "cpu_percent": sysinfo.cpu_percent(), "memory_used_mb": used, "memory_total_mb": total,
                       "disk_percent": sysinfo.disk_percent("/"), "autonomy_level": st.autonomy_level,
                       "loaded_models": st.loaded_models,
                       "plan_latency_p50_ms": lat[len(lat) // 2] if lat else None},
            "goals": [{k: g[k] for k in ("id", "description", "priority", "status", "source", "created_at")}
                      | {"progress": st.goal_engine.progress(g["id"])} for g in goals],
            "agents": st.router.list(),
            "health": st.health.status() if st.health else [],
            "gpus": sysinfo.amd_gpus(),
        }

    # ------------------------------------------------------------------ REST
    async def status(self, req):
        return web.json_response(self.state_dict()["status"])

    async def list_goals(self, req):
        goals, total = self.st.goal_engine.list(req.query.get("status", ""), int(req.query.get("limit", 50)),
                                                int(req.query.get("offset", 0)))
        for g in goals:
            g["progress"] = self.st.goal_engine.progress(g["id"])
        return web.json_response({"goals": goals, "total": total})

    async def submit_goal(self, req):
        body = await req.json()
        desc = str(body.get("description", "")).strip()
        if not desc:
            return web.json_response({"error": "description required"}, status=400)
        provider = str(body.get("provider", ""))
        meta = json.dumps({"preferred_provider": provider}).encode() if provider else b""
        g = await self.st.submit_goal(desc, int(body.get("priority", 5)), "management-console", [], meta)
        return web.json_response({"goal_id": g["id"]})

    async def goal_tasks(self, req):
        return web.json_response(self.st.goal_engine.tasks_for_goal(req.match_info["goal_id"]))

    async def goal_messages(self, req):
        return web.json_response(self.st.goal_engine.messages(req.match_info["goal_id"], 200))

    async def post_message(self, req):
        gid = req.match_info["goal_id"]
        ge = self.st.goal_engine
        if not ge.goal(gid):
            return web.json_response({"error": "goal not found"}, status=404)
        content = str((await req.json()).get("content", ""))
        ge.add_message(gid, "user", content)
        resumed = [t["id"] for t in ge.tasks_for_goal(gid) if t["status"] == "awaiting_input"]
        for tid in resumed:
            ge.update_task({"id": tid, "status": "pending"})
        if resumed:
            log.info("resumed %d awaiting tasks for goal %s", len(resumed), gid)
        return web.json_response({"sender": "user", "content": content, "timestamp": int(time.time() * 1000),
                                  "resumed_tasks": resumed})

    def system_context(self) -> str:
        s = self.state_dict()["status"]
        h = self.st.health.status() if self.st.health else []
        lines = ["You are aiOS, an AI-native operating system running on AMD Instinct MI355X GPUs.",
                 f"Uptime: {s['uptime']}. Active goals: {s['active_goals']}. Pending tasks: {s['pending_tasks']}.",
                 f"CPU {s['cpu_percent']:.1f}%, memory {s['memory_used_mb']:.0f}/{s['memory_total_mb']:.0f} MB, "
                 f"disk {s['disk_percent']:.1f}%.",
                 "Services: " + ", ".join(f"{x['name']}={'up' if x['healthy'] else 'down'}" for x in h),
                 "Agents: " + ", ".join(a["agent_id"] + f"({a.get('status', '')})" for a in self.st.router.list()),
                 "Loaded models: " + ", ".join(self.st.loaded_models or ["none"])]
        for g in self.st.goal_engine.list("", 10, 0)[0]:
            lines.append(f"- goal {g['id'][:8]} [{g['status']}] {g['description'][:100]}")
        return "\n".join(lines)

    async def chat(self, req):
        body = await req.json()
        t0 = time.time()
        r = await self.st.clients.gateway_infer(str(body.get("message", "")), self.system_context(), 4096, 0.7,
                                                provider=str(body.get("provider", "")), agent="chat-console")
        if r is None:
            r = await self.st.clients.runtime_infer(str(body.get("message", "")), self.system_context(), 1024, 0.7,
                                                    level="tactical", agent="chat-console")
        if r is None:
            return web.json_response({"reply": "AI backend error: no inference backend reachable.", "model": "error",
                                      "tokens": 0, "latency_ms": 0})
        return web.json_response({"reply": r.text, "model": r.model_used, "tokens": r.tokens_used,
                                  "latency_ms": int((time.time() - t0) * 1000)})

    async def agents(self, req):
        return web.json_response(self.st.router.list())

    async def health(self, req):
        return web.json_response({"healthy": True, "services": self.st.health.status() if self.st.health else []})

    async def gpus(self, req):
        return web.json_response(sysinfo.amd_gpus())

    async def decisions(self, req):
        return web.json_response(self.st.decisions.recent(int(req.query.get("n", 50))))

    async def events(self, req):
        return web.json_response(self.st.events.recent(int(req.query.get("n", 50))))

    async def publish_event(self, req):
        """External producers (agents, scripts) push events into the bus."""
        b = await req.json()
        if not b.get("event_type"):
            return web.json_response({"error": "event_type required"}, status=400)
        ok = self.st.emit(b["event_type"], b.get("source", "api"), b.get("data") or {}, b.get("severity", "info"))
        return web.json_response({"queued": ok})

    async def subscribe_event(self, req):
        b = await req.json()
        if not b.get("event_pattern") or not b.get("goal_template"):
            return web.json_response({"error": "event_pattern and goal_template required"}, status=400)
        sid = self.st.events.subscribe(b["event_pattern"], b.get("min_severity", "info"), b["goal_template"],
                                       int(b.get("priority", 5)))
        return web.json_response({"subscription_id": sid})

    async def schedules(self, req):
        return web.json_response(self.st.schedules.list())

    async def metrics(self, req):
        s = self.state_dict()["status"]
        out = [f"aios_active_goals {s['active_goals']}", f"aios_pending_tasks {s['pending_tasks']}",
               f"aios_active_agents {s['active_agents']}", f"aios_cpu_percent {s['cpu_percent']:.2f}",
               f"aios_memory_used_mb {s['memory_used_mb']:.1f}"]
        if s["plan_latency_p50_ms"] is not None:
            out.append(f"aios_plan_latency_p50_ms {s['plan_latency_p50_ms']:.3f}")
        for g in sysinfo.amd_gpus():
            out.append(f'aios_gpu_busy_percent{{card="{g["card"]}"}} {g["busy_percent"]}')
            out.append(f'aios_gpu_vram_used_mb{{card="{g["card"]}"}} {g["vram_used_mb"]:.1f}')
            out.append(f'aios_gpu_ecc_uncorrectable{{card="{g["card"]}"}} {g["ecc_ue"]}')
            out.append(f'aios_gpu_ecc_correctable{{card="{g["card"]}"}} {g["ecc_ce"]}')
            out.append(f'aios_gpu_xgmi_uncorrectable{{card="{g["card"]}"}} {g["xgmi_ue"]}')
            out.append(f'aios_gpu_pcie_replays{{card="{g["card"]}"}} {g["pcie_replays"]}')
            for k, v in g.items():
                if k.startswith("temp_") or k == "power_w":
                    out.append(f'aios_gpu_{k}{{card="{g["card"]}"}} {v:.1f}')
        return web.Response(text="\n".join(out) + "\n", content_type="text/plain")

    # ------------------------------------------------------------------ websocket
    async def ws(self, req):
        ws = web.WebSocketResponse(heartbeat=30)
        await ws.prepare(req)
        sub = {"goal": ""}

        async def pusher():
            while not ws.closed:
                msg = {"type": "state", **self.state_dict()}
                if sub["goal"]:
                    msg["goal_detail"] = {"tasks": self.st.goal_engine.tasks_for_goal(sub["goal"]),
                                          "messages": self.st.goal_engine.messages(sub["goal"], 100)}
                await ws.send_json(msg)
                await asyncio.sleep(2.0)

        task = asyncio.ensure_future(pusher())
        try:
            async for m in ws:
                if m.type != WSMsgType.TEXT:
                    continue
                try:
                    d = json.loads(m.data)
                except ValueError:
                    continue
                if d.get("type") == "subscribe_goal":
                    sub["goal"] = str(d.get("goal_id", ""))
        finally:
            task.cancel()
        return ws

    async def dashboard(self, req):
        return web.Response(text=DASHBOARD_HTML, content_type="text/html")


DASHBOARD_HTML = """<!doctype html><html><head><meta charset="utf-8"><title>aiOS · MI355X</title>
<style>body{font-family:system-ui,sans-serif;margin:0;background:#0f1115;color:#e6e6e6}
header{padding:10px 16px;background:#161a22;display:flex;gap:16px;align-items:center}
header b{color:#ed1c24}nav button{background:none;border:0;color:#aaa;padding:6px 10px;cursor:pointer}
nav button.on{color:#fff;border-bottom:2px solid #ed1c24}main{padding:16px}.tab{display:none}.tab.on{display:block}
table{border-collapse:collapse;width:100%}td,th{border-bottom:1px solid #2a2f3a;padding:4px 8px;text-align:left;font-size:13px}
input,select,textarea{background:#1c212b;color:#eee;border:1px solid #333;padding:6px}button.go{background:#ed1c24;color:#fff;border:0;padding:6px 12px}
#log{height:340px;overflow:auto;background:#151922;padding:8px;white-space:pre-wrap}.kv{display:grid;grid-template-columns:220px 1fr;gap:4px}
</style></head><body><header><b>aiOS</b><span>MI355X agent OS console</span>
<nav><button data-t="chat" class="on">Chat</button><button data-t="goals">Goals &amp; Tasks</button><button data-t="sys">System</button></nav></header>
<main><section id="chat" class="tab on"><div id="log"></div><p><select id="cprov"><option value="">auto</option><option>local</option>
<option>claude</option><option>openai</option><option>qwen3</option></select> <input id="msg" size="80" placeholder="Ask aiOS...">
<button class="go" onclick="chat()">Send</button></p></section>
<section id="goals" class="tab"><p><input id="goal" size="70" placeholder="New goal"> <select id="gprov"><option value="">auto</option>
<option>local</option><option>claude</option><option>openai</option><option>qwen3</option></select>
<button class="go" onclick="submitGoal()">Submit</button></p><table id="gt"></table><div id="detail"></div></section>
<section id="sys" class="tab"><div class="kv" id="kv"></div><h4>Services</h4><table id="ht"></table><h4>Agents</h4><table id="at"></table>
<h4>GPUs</h4><table id="gpu"></table></section></main>
<script>
const $=id=>document.getElementById(id);let sel="";
document.querySelectorAll('nav button').forEach(b=>b.onclick=()=>{document.querySelectorAll('nav button,.tab').forEach(e=>e.classList.remove('on'));b.classList.add('on');$(b.dataset.t).classList.add('on')});
async function chat(){const m=$('msg').value;if(!m)return;$('log').textContent+='\\n> '+m;$('msg').value='';
const r=await fetch('/api/chat',{method:'POST',headers:{'Content-Type':'application/json'},body:JSON.stringify({message:m,provider:$('cprov').value})});
const j=await r.json();$('log').textContent+='\\n['+j.model+', '+j.latency_ms+' ms] '+j.reply;$('log').scrollTop=1e9}
async function submitGoal(){const d=$('goal').value;if(!d)return;await fetch('/api/goals',{method:'POST',headers:{'Content-Type':'application/json'},body:JSON.stringify({description:d,priority:5,provider:$('gprov').value})});$('goal').value=''}
function row(c,h){return '<tr>'+c.map(x=>(h?'<th>':'<td>')+x+(h?'</th>':'</td>')).join('')+'</tr>'}
function pick(id){sel=id;ws.send(JSON.stringify({type:'subscribe_goal',goal_id:id}))}
const ws=new WebSocket((location.protocol=='https:'?'wss://':'ws://')+location.host+'/ws');
ws.onmessage=e=>{const s=JSON.parse(e.data);$('gt').innerHTML=row(['goal','status','prio','progress','source'],1)+s.goals.map(g=>
row(['<a href="#" onclick="pick(\\''+g.id+'\\')">'+g.description.slice(0,80)+'</a>',g.status,g.priority,g.progress.toFixed(0)+'%',g.source])).join('');
$('kv').innerHTML=Object.entries(s.status).map(([k,v])=>'<div>'+k+'</div><div>'+JSON.stringify(v)+'</div>').join('');
$('ht').innerHTML=row(['service','healthy','failures'],1)+s.health.map(h=>row([h.name,h.healthy,h.consecutive_failures])).join('');
$('at').innerHTML=row(['agent','type','status'],1)+s.agents.map(a=>row([a.agent_id,a.agent_type,a.status])).join('');
$('gpu').innerHTML=row(['card','busy %','VRAM MB'],1)+s.gpus.map(g=>row([g.card,g.busy_percent,g.vram_used_mb.toFixed(0)+' / '+g.vram_total_mb.toFixed(0)])).join('');
if(s.goal_detail){$('detail').innerHTML='<h4>Tasks</h4><table>'+row(['task','status','agent','error'],1)+s.goal_detail.tasks.map(t=>row([t.description,t.status,t.assigned_agent,t.error])).join('')+
'</table><h4>Conversation</h4><pre>'+s.goal_detail.messages.map(m=>'['+m.sender+'] '+m.content).join('\\n')+'</pre>'}}
</script></body></html>"""
