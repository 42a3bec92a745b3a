"""bench.py's --gpus contract on the CPU (multi-process, gloo): `--gpus N` without torchrun spawns N
ranks itself, each seeing WORLD_SIZE=N; under torchrun a mismatching --gpus is refused."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    e = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    return e


def test_gpus_n_spawns_n_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 for d in lines)
    assert all(d["ranks_share_gpu"] for d in lines)  # no GPU here: both ranks share "one"


def test_gpus_mismatch_is_refused():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_gpus_8_through_torchrun_dry_run():
    """the driver's 8-GPU scaling launch shape (torch.distributed.run, 8 ranks, 127.0.0.1) on the CPU:
    every rank joins the process group and reports WORLD_SIZE 8"""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(d["rank"] for d in lines) == list(range(8))
    assert all(d["world"] == 8 for d in lines)


def test_gpus_8_one_device_per_rank():
    """the 8-GPU node shape: with 8 devices visible every rank gets its own (share False -> RCCL
    process group, the XgmiComm / self-test path, the persistent kernels on), device = LOCAL_RANK"""
    env = _env()
    env["AIOS_BENCH_DEVICES"] = "8"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(d["rank"] for d in lines) == list(range(8))
    assert not any(d["ranks_share_gpu"] for d in lines)
    assert sorted(d["device"] for d in lines) == list(range(8))


def test_ranks_per_gpu_from_device_identity():
    """sharing is counted from the physical device identity, not device_count() (each
    rank may see only its own GPU)"""
    from aios_amd.parallel.tp import ranks_per_gpu

    assert ranks_per_gpu(8, [f"node/0000:{i:02x}:00.0" for i in range(8)]) == 1
    assert ranks_per_gpu(4, ["node/0000:05:00.0"] * 4) == 4
    assert ranks_per_gpu(4, ["n/a", "n/a", "n/b", "n/b"]) == 2
