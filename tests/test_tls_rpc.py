"""Optional node mTLS on the gRPC contract (AIOS_TLS_DIR): certificates from the native TlsManager,
server requires a client certificate signed by the node CA; plaintext and certificate-less
clients are refused."""
import asyncio

import grpc
import pytest

from aios_amd.rpc.client import Stub, channel
from aios_amd.rpc.schema import pb
from aios_amd.rpc.server import RpcServer


def test_mtls_tool_registry(tmp_path):
    from aios_amd.tools.service import ToolRegistryService

    certs = str(tmp_path / "certs")

    async def run():
        svc = ToolRegistryService(str(tmp_path / "data"))
        srv = RpcServer("127.0.0.1:0", {"aios.tools.ToolRegistry": svc}, tls_dir=certs)
        assert srv.tls
        await srv.start()
        addr = f"127.0.0.1:{srv.port}"
        try:
            ok = Stub(channel(addr, fresh=True, tls_dir=certs), "aios.tools.ToolRegistry", timeout=10)
            r = await ok.ListTools(pb.tools.ListToolsRequest())
            assert len(r.tools) >= 88
            plain = Stub(channel(addr, fresh=True, tls_dir=""), "aios.tools.ToolRegistry", timeout=3)
            with pytest.raises(grpc.aio.AioRpcError):
                await plain.ListTools(pb.tools.ListToolsRequest())
            # server-authenticated only (no client certificate): refused by require_client_auth
            ca = open(f"{certs}/ca.crt", "rb").read()
            ch = grpc.aio.secure_channel(addr, grpc.ssl_channel_credentials(root_certificates=ca),
                                         options=[("grpc.ssl_target_name_override", "aios")])
            anon = Stub(ch, "aios.tools.ToolRegistry", timeout=3)
            with pytest.raises(grpc.aio.AioRpcError):
                await anon.ListTools(pb.tools.ListToolsRequest())
            await ch.close()
        finally:
            await srv.stop()
            svc.close()

    asyncio.run(run())


def _gen(d, q):
    from aios_amd.core import load as load_core

    mgr = load_core().TlsManager(d)
    q.put(bool(mgr.generate_self_signed("aios")["generated"]))


def test_concurrent_service_starts_share_one_ca(tmp_path):
    """services started together each ran generate_self_signed; without a lock they
    could create different CAs and overwrite each other's files.  Now exactly one process
    generates, the others find a complete, consistent set, and the keys are 0600."""
    import multiprocessing as mp
    import os
    import stat

    from aios_amd.core import load as load_core

    d = str(tmp_path / "certs")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gen, args=(d, q)) for _ in range(6)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(60)
    gens = [q.get(timeout=5) for _ in procs]
    assert sum(gens) == 1, gens
    v = load_core().TlsManager(d).verify()
    assert v["ok"], v
    for k in ("ca.key", "server.key"):
        assert stat.S_IMODE(os.stat(os.path.join(d, k)).st_mode) == 0o600
    assert not [f for f in os.listdir(d) if ".tmp." in f]
