"""Tensor parallelism for the local "strategic" tier (BASELINE config 5).

One process per GPU.  Every rank holds a shard of the model (column-parallel Q/K/V and gate/up,
row-parallel attn_output / ffn_down, replicated embeddings / norms / lm_head; see
`aios_amd/runtime/loader.py:shard_tensor`) and an `XgmiComm` whose one-shot all-reduce (HIP,
`aios_amd/csrc/kernels/allreduce.hip`) is fused with the residual add and runs inside the
engine's captured hipGraph -- 2 collectives per layer, no host involvement per collective.

After each all-reduce every rank holds the identical residual stream, so the replicated lm_head
and the on-device sampler produce identical tokens on every rank: no token broadcast is needed,
only the *commands* (prefill / decode / decode_loop ...) that rank 0 -- the serving leader --
issues.  `TPEngine` is a drop-in for the native Engine on the leader (the runtime scheduler
drives it unchanged); `worker_loop` executes the same calls on ranks 1..N-1.

The bootstrap (IPC handle exchange) and the command channel use a gloo process group, so the
data plane never depends on RCCL; this also lets TP run with several ranks on ONE GPU (how the
numerics tests exercise it on a single-GPU box), which RCCL refuses.
"""
from __future__ import annotations

import logging
import os
from typing import Any, List, Optional

log = logging.getLogger("aios.tp")

# largest all-reduce: a prefill chunk of the engine's 64-row workspace at d_model
DEFAULT_PREFILL_ROWS = 64


def comm_capacity(d_model: int, max_batch: int = 8, prefill_rows: int = DEFAULT_PREFILL_ROWS) -> int:
    return max(max_batch, prefill_rows) * d_model


def create_comm(rank: int, world: int, device: int, cap_floats: int, group=None):
    """XgmiComm connected to every rank of `group` (default: the default process group)."""
    import torch.distributed as dist

    from ..runtime import native

    m = native.require()
    comm = m.XgmiComm(rank, world, device, cap_floats)
    if world > 1:
        handles: List[Any] = [None] * world
        dist.all_gather_object(handles, comm.ipc_handle(), group=group)
        comm.connect(handles)
    return comm


class TPEngine:
    """Leader-side proxy: forwards each engine call to the workers, then runs it locally.

    Workers block in `worker_loop`; `close()` releases them.  Attribute reads (config,
    weight_bytes, ...) are served from the local shard."""

    _FORWARD = {"prefill", "decode", "resample", "last_logits", "decode_loop_prepare", "decode_loop_run",
                "decode_loop_history", "synchronize", "reset_graphs", "copy_slot"}

    def __init__(self, engine, comm, group=None):
        self._eng = engine
        self._comm = comm
        self._group = group
        self._closed = False

    def _bcast(self, msg):
        import torch.distributed as dist

        obj = [msg]
        dist.broadcast_object_list(obj, src=0, group=self._group)

    def __getattr__(self, name):
        attr = getattr(self._eng, name)
        if name not in self._FORWARD or not callable(attr):
            return attr

        def call(*args, **kw):
            self._bcast((name, args, kw))
            out = attr(*args, **kw)
            if self._comm.error():
                raise RuntimeError("TP all-reduce timed out (a rank stopped participating)")
            return out
        return call

    def close(self):
        if not self._closed:
            self._closed = True
            self._bcast(("__exit__", (), {}))


def worker_loop(engine, comm, group=None):
    """Ranks 1..N-1: execute the leader's engine calls until it sends __exit__."""
    import torch.distributed as dist

    while True:
        obj = [None]
        dist.broadcast_object_list(obj, src=0, group=group)
        name, args, kw = obj[0]
        if name == "__exit__":
            return
        getattr(engine, name)(*args, **kw)
        if comm.error():
            log.error("TP all-reduce timed out on this worker")


def build_tp_engine(cfg, rank: int, world: int, device: int, recipe: str = "Q4_K_M", path: Optional[str] = None,
                    seed: int = 0, max_ctx: int = 4096, max_slots: int = 4, max_batch: int = 8, group=None,
                    act_q8: bool = True):
    """This rank's shard (from a GGUF file, or random-init) with its XgmiComm attached."""
    from ..runtime.loader import load_engine, random_engine

    if path:
        eng, cfg, _ = load_engine(path, max_ctx=max_ctx, max_slots=max_slots, max_batch=max_batch, device=device,
                                  tp_rank=rank, tp_size=world, act_q8=act_q8)
    else:
        eng = random_engine(cfg, recipe, seed=seed, max_ctx=max_ctx, max_slots=max_slots, max_batch=max_batch,
                            device=device, tp_rank=rank, tp_size=world, act_q8=act_q8)
    comm = create_comm(rank, world, device, comm_capacity(cfg.d_model, max_batch), group)
    eng.set_comm(comm)
    return eng, comm


def local_device(local_rank: int) -> int:
    """GPU for this rank: one per rank when there are enough GPUs, else ranks share (tests)."""
    import torch

    n = torch.cuda.device_count()
    return local_rank % max(n, 1)


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))
