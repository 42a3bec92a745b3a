"""TP worker process (ranks 1..N-1 of a runtime-hosted strategic model; see tp.launch_tp)."""
from __future__ import annotations

import argparse
import logging
import os


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--leader", required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--spec", required=True)
    ap.add_argument("--max-ctx", type=int, default=4096)
    ap.add_argument("--max-slots", type=int, default=4)
    ap.add_argument("--max-batch", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--q8", type=int, default=1)
    ap.add_argument("--kv", default="bf16")
    a = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("AIOS_LOG", "INFO"))
    import torch  # noqa: F401  (loads the HIP runtime the extension links against)

    from ..runtime import native
    from .channel import WorkerChannel
    from .tp import (_shard, channel_allgather, comm_capacity, comm_kind, reconcile_tp_fuse, share_prefill_plans,
                     worker_loop, xgmi_handshake)

    ch = WorkerChannel(a.leader, a.rank, os.environ.pop("AIOS_TP_TOKEN", ""))
    eng, cfg = _shard(a.spec, a.rank, a.world, a.device, a.max_ctx, a.max_slots, a.max_batch, a.seed, bool(a.q8),
                      a.kv)
    if comm_kind() == "rccl":  # the leader broadcasts the ncclUniqueId; the init is collective
        comm = native.require().RcclComm(a.rank, a.world, a.device, ch.recv())
    else:
        comm = native.require().XgmiComm(a.rank, a.world, a.device, comm_capacity(cfg.d_model, a.max_batch))
        ch.send(comm.ipc_handle())
        comm.connect(ch.recv())
        xgmi_handshake(comm, a.rank, a.world, a.device, channel_allgather(ch, False))
    eng.set_comm(comm)
    share_prefill_plans(channel_allgather(ch, False))
    if comm_kind() != "rccl":
        reconcile_tp_fuse(eng, channel_allgather(ch, False))
    # per-step commands arrive through the leader's shared-memory ring (ring.py); the TCP channel
    # only carried the authenticated setup
    from .ring import CommandRing

    ring = CommandRing(a.world, name=str(ch.recv()["ring"]), worker=a.rank)
    try:
        worker_loop(eng, comm, recv=ring.recv)
    except ConnectionError:
        pass
    finally:
        ring.close()
        ch.close()


if __name__ == "__main__":
    main()
