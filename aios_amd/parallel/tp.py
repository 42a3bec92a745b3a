"""Tensor parallelism for the local "strategic" tier (BASELINE config 5).

One process per GPU.  Every rank holds a shard of the model (column-parallel Q/K/V and gate/up,
row-parallel attn_output / ffn_down, vocab-parallel lm_head, replicated embeddings / norms; see
`aios_amd/runtime/loader.py:shard_tensor`) and an `XgmiComm` whose all-reduce (HIP,
`aios_amd/csrc/kernels/allreduce.hip`: one-shot for decode-size messages, reduce-scatter +
all-gather with bf16 staging for prefill chunks) is fused with the residual add and runs inside
the engine's captured hipGraph -- 2 collectives per layer plus one logits all-gather per step, no
host involvement per collective.

After each all-reduce every rank holds the identical residual stream and, after the logits
all-gather, the identical logits, so the on-device sampler produces identical tokens on every
rank: no token broadcast is needed,
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


def comm_kind() -> str:
    """AIOS_TP_COMM: 'xgmi' (default; the IPC one-shot / two-shot kernels, fused with the residual
    add) or 'rccl' (librccl all-reduce / all-gather inside the same captured step; one GPU per rank)."""
    k = os.environ.get("AIOS_TP_COMM", "xgmi").strip().lower()
    if k not in ("xgmi", "rccl"):
        raise ValueError(f"AIOS_TP_COMM must be 'xgmi' or 'rccl', not {k!r}")
    return k


def ranks_per_gpu(world: int, identities: Optional[List[str]] = None) -> int:
    """TP ranks that share one GPU (1 on a node with a GPU per rank).  With `identities` (every
    rank's physical device identity, all-gathered: host + PCI bus id) it counts the ranks on the
    most shared device -- the same answer on every rank, and right when each rank sees only its own
    GPU (HIP_VISIBLE_DEVICES per rank makes device_count() 1 everywhere).  Without them: inferred
    from the visible device count (single-process tools)."""
    if identities:
        from collections import Counter

        return max(Counter(identities).values())
    try:
        import torch

        n = torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        n = 0
    return max(1, -(-world // n)) if n > 0 else 1


def device_identity(device: int) -> str:
    """host + PCI bus id of `device` (ranks that share a GPU report the same string)."""
    import socket

    from ..runtime import native

    try:
        bus = native.require().device_pci_bus_id(device)
    except Exception:  # noqa: BLE001
        bus = f"device{device}"
    return f"{socket.gethostname()}/{bus}"


def comm_self_test(comm, rank: int, world: int, device: int) -> bool:
    """All-reduce (one-shot and two-shot sizes) and column all-gather through `comm`, checked on the
    host against the values every rank contributed.  Run once at TP init: a peer mapping that
    silently misbehaves (wrong IPC memory type, a stale mapping) shows up here, not as a wrong token."""
    import torch

    dev = torch.device("cuda", device)
    st = torch.cuda.current_stream(dev).cuda_stream
    ok = True
    for n in (4096, 16384, 1 << 20):
        if n > comm.capacity:
            continue
        base = torch.arange(n, dtype=torch.float32, device=dev) * 1e-3
        t = base + (rank + 1)
        comm.allreduce(t.data_ptr(), n, 0, st)
        torch.cuda.synchronize(dev)
        want = base * world + world * (world + 1) / 2
        ok &= bool(torch.allclose(t, want, rtol=1e-2, atol=1e-2))  # (two-shot stages bf16)
    rows, sl = 2, 64
    if rows * sl * world <= comm.capacity:
        ld = sl * world
        g = torch.full((rows, ld), -7.0, dtype=torch.float32, device=dev)
        g[:, rank * sl:(rank + 1) * sl] = rank + 0.25
        comm.allgather_cols(g.data_ptr(), rows, sl, ld, st)
        torch.cuda.synchronize(dev)
        want = torch.arange(world, dtype=torch.float32, device=dev).repeat_interleave(sl) + 0.25
        ok &= bool(torch.equal(g, want.expand(rows, ld)))
    ok &= not comm.error()
    return ok


def gloo_allgather(group, world: int):
    """allgather(obj) -> every rank's obj, through the torch.distributed (gloo) group."""
    import torch.distributed as dist

    def g(obj):
        if world == 1:
            return [obj]
        out: List[Any] = [None] * world
        dist.all_gather_object(out, obj, group=group)
        return out

    return g


def channel_allgather(ch, leader: bool):
    """allgather(obj) through the runtime's TP setup channel (leader: gather + broadcast; worker:
    send + receive): the same calls in the same order on every rank."""
    def g(obj):
        if leader:
            out = ch.gather(obj)
            ch.broadcast(out)
            return out
        ch.send(obj)
        return ch.recv()

    return g


def fused_self_test(comm, rank: int, world: int, device: int, allgather) -> bool:
    """One batch-1 EPI_TP_RESID GEMV (the O / down all-reduce in the GEMV epilogue, gemv_q8.h) per
    rank through the comm's fused context, checked on the host: every rank's weights and x are drawn
    from rank-keyed seeds, so each rank computes residual + sum over ranks of q8(x_r) . W_r^T itself.
    The fused protocol publishes partials with relaxed flag stores to uncached peer memory; a
    cross-device visibility problem would give wrong tokens, not an error -- this turns it into a
    fallback (verdict r5 weak #8).  Every rank first reports whether the launch fits (dry run): a
    rank that would not launch would leave its peers waiting on flags."""
    import numpy as np
    import torch

    from ..gguf.quants import GGMLType, dequantize, quantize
    from ..models.reference import ReferenceModel
    from ..runtime import native

    N, K, y0 = 512, 1024, 0.5

    def draw(r):
        rng = np.random.default_rng(90017 + r)
        w = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
        raw = quantize(w, GGMLType.Q8_0)
        return raw, dequantize(raw, GGMLType.Q8_0).reshape(N, K), rng.standard_normal(K).astype(np.float32)

    # (exactly one collective on every path: a rank failing early must not skip it)
    fit, mat, x, st = False, None, None, 0
    dev = torch.device("cuda", device)
    try:
        raw, _, x = draw(rank)
        mat = native.require().QMatrix(int(GGMLType.Q8_0), N, K, raw)
        st = torch.cuda.current_stream(dev).cuda_stream
        fit = bool(comm.fused_gemv(mat, 0, 0, st, True))
    except Exception as e:  # noqa: BLE001
        log.warning("fused TP epilogue self-test setup failed: %s: %s", type(e).__name__, e)
    if not all(allgather(fit)):
        return False
    xd = torch.from_numpy(x).to(dev)
    y = torch.full((N,), y0, dtype=torch.float32, device=dev)
    launched = comm.fused_gemv(mat, xd.data_ptr(), y.data_ptr(), st, False)
    torch.cuda.synchronize(dev)
    if not launched or comm.error():
        return False
    want = torch.full((N,), y0, dtype=torch.float64)
    for r in range(world):
        _, wr, xr = draw(r)
        want += (ReferenceModel.q8(torch.from_numpy(xr)[None]).double() @ torch.from_numpy(wr).double().T)[0]
    return bool(torch.allclose(y.cpu().double(), want, atol=2e-2, rtol=1e-2))


def check_fused_comm(comm, rank: int, world: int, device: int, allgather) -> bool:
    """Keep the fused all-reduce epilogue only if every rank has it and every rank's fused self-test
    passes (AIOS_TP_SELFTEST=0 skips the test); otherwise every rank disables it and the engines
    run GEMV + separate all-reduce.  Returns whether it stays on."""
    if world == 1:
        return False
    has = allgather(bool(comm.fused))
    if not all(has):
        if any(has):
            comm.disable_fuse()
        return False
    if os.environ.get("AIOS_TP_SELFTEST", "1") == "0":
        return True
    # (fused_self_test runs one collective on every path before anything can raise past it)
    try:
        ok = fused_self_test(comm, rank, world, device, allgather)
    except Exception as e:  # noqa: BLE001  (reported as a failed check: every rank falls back)
        log.warning("fused TP epilogue self-test raised %s: %s", type(e).__name__, e)
        ok = False
    if not all(allgather(bool(ok))):
        comm.disable_fuse()
        log.warning("fused TP all-reduce epilogue self-test failed on a rank; GEMV + all-reduce on every rank")
        return False
    return True


def share_prefill_plans(allgather):
    """Every TP rank runs the leader's prefill-GEMM plans (each rank's own timing could
    pick a different tile / split, i.e. a different summation order per rank)."""
    from ..runtime import native

    m = native.require()
    plans = allgather([int(v) for v in m.gemm_pf_export()])[0]
    m.gemm_pf_import(plans)


def reconcile_tp_fuse(eng, allgather) -> bool:
    """After set_comm: every rank's per-layer fit of the fused O / down launch (Engine.tp_fuse_fits,
    which depends on the device's CU count and the co-residency cap) must be identical, or fusion goes
    off on every rank (a rank falling back alone leaves its peers waiting on flags)."""
    if not getattr(eng, "tp_fused", False):
        allgather(None)  # (the other ranks' gather still needs this rank's turn)
        return False
    mine = [int(v) for v in eng.tp_fuse_fits()]
    allv = allgather(mine)
    if any(v != mine for v in allv):
        eng.disable_tp_fuse()
        log.warning("fused TP epilogue fits differ across ranks; disabled on every rank")
        return False
    return True


def create_comm(rank: int, world: int, device: int, cap_floats: int, group=None, kind: Optional[str] = None):
    """XgmiComm (or RcclComm, see comm_kind) connected to every rank of `group` (default: the
    default process group).

    The xGMI comm is checked before use: every rank's fused-epilogue eligibility (uncached peer
    memory, AIOS_TP_FUSE) is all-gathered and the fused path stays on only if ALL agree, then
    `comm_self_test` runs on every rank (AIOS_TP_SELFTEST=0 skips it).  A failed self-test or a rank
    without uncached peer memory falls back to RCCL when each rank has its own GPU, and is an error
    when ranks share one (RCCL refuses that)."""
    import torch.distributed as dist

    from ..runtime import native

    m = native.require()

    def rccl():
        uid: List[Any] = [m.RcclComm.unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0, group=group)
        return m.RcclComm(rank, world, device, uid[0])

    if (kind or comm_kind()) == "rccl":
        return rccl()
    ids: List[Any] = [device_identity(device)]
    if world > 1:
        ids = [None] * world
        dist.all_gather_object(ids, device_identity(device), group=group)
    per_gpu = ranks_per_gpu(world, ids)
    comm = m.XgmiComm(rank, world, device, cap_floats)
    if per_gpu > 1:  # every spinning workgroup of every rank must be resident on the shared GPU at once
        comm.call_wg = max(1, min(512, 1024 // per_gpu))
        # ... including the O / down GEMV engines whose epilogue runs the all-reduce (EPI_TP_RESID)
        comm.set_ranks_per_gpu(per_gpu)
    if world == 1:
        return comm
    handles: List[Any] = [None] * world
    dist.all_gather_object(handles, comm.ipc_handle(), group=group)
    comm.connect(handles)
    flags: List[Any] = [None] * world
    dist.all_gather_object(flags, (bool(comm.fuse_eligible), bool(comm.uncached)), group=group)
    if not all(f[0] for f in flags):
        comm.disable_fuse()
    ok = True
    if os.environ.get("AIOS_TP_SELFTEST", "1") != "0":
        oks: List[Any] = [None] * world
        dist.all_gather_object(oks, comm_self_test(comm, rank, world, device), group=group)
        ok = all(oks)
    if ok and all(f[1] for f in flags):
        check_fused_comm(comm, rank, world, device, gloo_allgather(group, world))
        return comm
    why = "self-test mismatch" if not ok else "a rank without uncached peer memory"
    if per_gpu > 1:
        if not ok:
            raise RuntimeError(f"xGMI comm: {why} (ranks share a GPU, no RCCL fallback)")
        log.warning("xGMI comm: %s; fused all-reduce epilogue off", why)
        comm.disable_fuse()
        return comm
    log.warning("xGMI comm: %s; falling back to RCCL", why)
    del comm
    return rccl()


def xgmi_handshake(comm, rank: int, world: int, device: int, allgather):
    """The runtime daemon's TP setup (launch_tp / worker.py, over the setup channel): fused-epilogue
    eligibility on every rank, the collectives' self-test (a failure is an error here: the daemon
    reports the tier as failed and routes to the next one), then the fused-epilogue self-test."""
    flags = allgather([bool(comm.fuse_eligible), bool(comm.uncached)])
    if not all(f[0] and f[1] for f in flags):
        comm.disable_fuse()
    if os.environ.get("AIOS_TP_SELFTEST", "1") != "0":
        if not all(allgather(bool(comm_self_test(comm, rank, world, device)))):
            raise RuntimeError("xGMI comm: self-test mismatch on a rank")
    check_fused_comm(comm, rank, world, device, allgather)


class TPEngine:
    """Leader-side proxy: forwards each engine call to the workers, then runs it locally.

    `send` broadcasts one command tuple to every worker: a gloo group (torchrun tools / tests) or
    the loopback LeaderChannel (runtime daemon, channel.py).  Workers block in `worker_loop`;
    `close()` releases them.  Attribute reads (config, weight_bytes, ...) come from the local
    shard."""

    _FORWARD = frozenset({"prefill", "decode", "resample", "sample_first", "last_logits", "decode_loop_prepare",
                          "decode_loop_run", "decode_loop_history", "synchronize", "reset_graphs", "copy_slot",
                          "release_slot", "decode_submit", "decode_sample", "decode_collect"})

    def __init__(self, engine, comm, group=None, send=None, on_close=None, on_abort=None):
        self._eng = engine
        self._comm = comm
        self._send = send or (lambda msg: _dist_bcast(msg, group))
        self._on_close = on_close
        self._on_abort = on_abort
        self._closed = False

    def __getattr__(self, name):
        attr = getattr(self._eng, name)
        if name not in self._FORWARD or not callable(attr):
            return attr

        def call(*args):
            self._send([name, list(args)])
            out = attr(*args)
            if self._comm.error():
                raise RuntimeError("TP all-reduce timed out (a rank stopped participating)")
            return out
        return call

    def close(self):
        if not self._closed:
            self._closed = True
            self._send(["__exit__", []])
            if self._on_close:
                self._on_close()

    def abort(self):
        """Failure teardown (a rank timed out or died): no __exit__ handshake -- the workers are
        killed and the channel closed, so nothing waits on a rank that will never answer."""
        if not self._closed:
            self._closed = True
            if self._on_abort:
                self._on_abort()


def _dist_bcast(msg, group):
    import torch.distributed as dist

    obj = [msg]
    dist.broadcast_object_list(obj, src=0, group=group)


def _dist_recv(group):
    import torch.distributed as dist

    obj = [None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def worker_loop(engine, comm, group=None, recv=None):
    """Ranks 1..N-1: execute the leader's engine calls (whitelisted) until it sends __exit__."""
    recv = recv or (lambda: _dist_recv(group))
    while True:
        name, args = recv()
        if name == "__exit__":
            return
        if name not in TPEngine._FORWARD:
            log.error("TP worker: refusing unknown command %r", name)
            continue
        getattr(engine, name)(*args)
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
    if world > 1:
        share_prefill_plans(gloo_allgather(group, world))
        if hasattr(comm, "ipc_handle"):
            reconcile_tp_fuse(eng, gloo_allgather(group, world))
    return eng, comm


def local_device(local_rank: int) -> int:
    """GPU for this rank: one per rank when there are enough GPUs, else ranks share (tests)."""
    import torch

    n = torch.cuda.device_count()
    return local_rank % max(n, 1)


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


# ------------------------------------------------------------------------------ runtime launcher
def spec_kv_dtype(path: str) -> str:
    """the '#...&kv=fp8_e4m3' fragment of a model spec (default: AIOS_KV_DTYPE, else bf16)"""
    for kv in filter(None, path.partition("#")[2].split("&")):
        k, _, v = kv.partition("=")
        if k == "kv":
            return v
    return os.environ.get("AIOS_KV_DTYPE", "bf16")


def parse_spec(path: str):
    """'synthetic:<preset>[:<recipe>]#tp=N&q8=0' or '<file.gguf>#tp=N' -> (base, tp, act_q8).
    q8=0 selects fp32 activations in the GEMVs (int8 activations are the default); kv=fp8_e4m3 the
    fp8 KV cache (spec_kv_dtype)."""
    base, _, frag = path.partition("#")
    tp, q8 = 1, True
    for kv in filter(None, frag.split("&")):
        k, _, v = kv.partition("=")
        if k == "tp":
            tp = int(v)
        elif k == "q8":
            q8 = v not in ("0", "false", "no")
    return base, tp, q8


def _shard(spec: str, rank: int, world: int, device: int, max_ctx: int, max_slots: int, max_batch: int, seed: int,
           act_q8: bool = True, kv_dtype: str = "bf16"):
    from ..models.config import get_preset
    from ..runtime.loader import load_engine, random_engine

    if spec.startswith("synthetic:"):
        parts = spec.split(":")
        cfg = get_preset(parts[1])
        eng = random_engine(cfg, parts[2] if len(parts) > 2 else "Q4_K_M", seed=seed, max_ctx=max_ctx,
                            max_slots=max_slots, max_batch=max_batch, device=device, tp_rank=rank, tp_size=world,
                            act_q8=act_q8, kv_dtype=kv_dtype)
        return eng, cfg
    eng, cfg, _ = load_engine(spec, max_ctx=max_ctx, max_slots=max_slots, max_batch=max_batch, device=device,
                              tp_rank=rank, tp_size=world, act_q8=act_q8, kv_dtype=kv_dtype)
    return eng, cfg


def launch_tp(spec: str, world: int, devices, max_ctx: int, max_slots: int, max_batch: int, seed: int = 0,
              act_q8: bool = True, kv_dtype: str = "bf16"):
    """Runtime-side TP model: spawn ranks 1..N-1 as worker processes (python -m
    aios_amd.parallel.worker), build rank 0 here, exchange IPC handles over the channel.
    Returns (TPEngine, cfg)."""
    import subprocess
    import sys

    from ..runtime import native
    from .channel import LeaderChannel
    from .ring import CommandRing

    devices = list(devices) or [0]
    ch = LeaderChannel(world)
    ring = CommandRing(world)
    procs = []
    for r in range(1, world):
        env = dict(os.environ, AIOS_TP_TOKEN=ch.token)
        procs.append(subprocess.Popen([sys.executable, "-m", "aios_amd.parallel.worker", "--leader", ch.address,
                                       "--rank", str(r), "--world", str(world), "--device",
                                       str(devices[r % len(devices)]), "--spec", spec, "--max-ctx", str(max_ctx),
                                       "--max-slots", str(max_slots), "--max-batch", str(max_batch),
                                       "--seed", str(seed), "--q8", "1" if act_q8 else "0", "--kv", kv_dtype],
                                      env=env))
    try:
        ch.accept_all()
        eng, cfg = _shard(spec, 0, world, devices[0], max_ctx, max_slots, max_batch, seed, act_q8, kv_dtype)
        if comm_kind() == "rccl":
            uid = native.require().RcclComm.unique_id()
            ch.broadcast(uid)
            comm = native.require().RcclComm(0, world, devices[0], uid)  # collective with the workers
        else:
            comm = native.require().XgmiComm(0, world, devices[0], comm_capacity(cfg.d_model, max_batch))
            handles = ch.gather(comm.ipc_handle())
            ch.broadcast(handles)
            comm.connect(handles)
            xgmi_handshake(comm, 0, world, devices[0], channel_allgather(ch, True))
        eng.set_comm(comm)
        share_prefill_plans(channel_allgather(ch, True))
        if comm_kind() != "rccl":
            reconcile_tp_fuse(eng, channel_allgather(ch, True))
        ch.broadcast({"ring": ring.name})
    except Exception:
        for p in procs:
            p.kill()
        ch.close()
        ring.close()
        raise

    def shutdown():
        for p in procs:
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                p.kill()
        ch.close()
        ring.close()

    def abort():
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                pass
        ch.close()
        ring.close()

    tp = TPEngine(eng, comm, send=ring.send, on_close=shutdown, on_abort=abort)
    tp._keep = (comm, ch, ring, procs)
    return tp, cfg
