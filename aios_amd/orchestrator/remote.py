"""Remote execution on other cluster nodes (reference: `agent-core/src/remote_exec.rs:11-107`).

`RemoteExecutor` keeps one lazily-connected gRPC channel per remote address (the shared channel
cache of `aios_amd.rpc.client`, so node mTLS applies when AIOS_TLS_DIR is set) and offers the
reference's two operations:

* `submit_remote_goal(address, description, priority, source)` -> remote goal id: the autonomy
  loop's cluster route (`autonomy.rs:436-450`);
* `execute_remote_tool(tools_address, tool, agent_id, task_id, input_json)` ->
  (success, output_json, error): a tool call executed by ANOTHER node's tool service.  The
  reference defines it but never calls it; here the autonomy loop uses it for tool calls that
  name a target node (`{"tool": ..., "input": ..., "node": "<node_id>"}`), e.g. "check disk
  usage on worker-2" planned on the coordinator.

A node's tool-service address comes from its registration metadata (`tools_address`), else the
host of its orchestrator address with the tool service's port (AIOS_TOOLS_PORT, default 50052).
"""
from __future__ import annotations

import logging
import os
from typing import Dict, Optional, Tuple

log = logging.getLogger("aios.orchestrator.remote")

TOOLS_PORT = int(os.environ.get("AIOS_TOOLS_PORT", "50052"))


def tools_address_of(node: dict) -> str:
    md = node.get("metadata") or {}
    if md.get("tools_address"):
        return md["tools_address"]
    addr = node.get("address", "")
    host = addr.rsplit(":", 1)[0] if ":" in addr else addr
    return f"{host}:{TOOLS_PORT}"


class RemoteExecutor:
    def __init__(self, timeout: float = 60.0, connect_timeout: float = 5.0):
        self.timeout = timeout
        self.connect_timeout = connect_timeout
        self.channels: Dict[str, object] = {}

    def _stub(self, address: str, service: str):
        from ..rpc.client import Stub, channel

        ch = self.channels.get(address)
        if ch is None:
            ch = channel(address)
            self.channels[address] = ch
            log.info("connected to remote node at %s", address)
        return Stub(ch, service, timeout=self.timeout)

    async def submit_remote_goal(self, address: str, description: str, priority: int = 5,
                                 source: str = "cluster") -> str:
        from ..rpc.schema import pb

        stub = self._stub(address, "aios.orchestrator.Orchestrator")
        r = await stub.SubmitGoal(pb.orchestrator.SubmitGoalRequest(description=description, priority=priority,
                                                                    source=source), timeout=min(10.0, self.timeout))
        log.info("submitted goal to remote node %s: %s", address, r.id)
        return r.id

    async def execute_remote_tool(self, tools_address: str, tool_name: str, agent_id: str, task_id: str,
                                  input_json: bytes) -> Tuple[bool, bytes, str]:
        from ..rpc.schema import pb

        stub = self._stub(tools_address, "aios.tools.ToolRegistry")
        r = await stub.Execute(pb.tools.ExecuteRequest(tool_name=tool_name, agent_id=agent_id, task_id=task_id,
                                                       input_json=input_json,
                                                       reason="Remote execution from cluster"))
        return bool(r.success), bytes(r.output_json), r.error

    def close_all(self):
        # channels are shared with the process-wide cache (rpc.client.close_all closes them)
        self.channels.clear()


def find_node(cluster, node_id: str) -> Optional[dict]:
    for n in cluster.list(False):
        if n.get("node_id") == node_id:
            return n
    return None
