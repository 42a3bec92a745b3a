"""L0 distro assets (reference: scripts/build-{kernel,initramfs,rootfs,iso}.sh, run-qemu.sh,
rootfs/boot/grub/grub.cfg, rootfs/etc/apparmor.d): every build script parses and dry-runs its
plan without network or root; the kernel fragment carries the MI355X compute stack (amdgpu, KFD,
HMM, P2P, IOMMU passthrough) and the boot/security features; the AppArmor profile lets the runtime
reach /dev/kfd and the render nodes and nothing of the control-plane state."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = ["build-kernel.sh", "build-rootfs.sh", "build-initramfs.sh", "build-iso.sh", "run-qemu.sh",
           "build-all.sh", "install.sh", "first-boot.sh", "create-release.sh"]


@pytest.mark.parametrize("name", SCRIPTS)
def test_script_parses(name):
    subprocess.run(["bash", "-n", os.path.join(ROOT, "scripts", name)], check=True)


def test_iso_build_dry_run(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "build-iso.sh"), "--dry-run", "--out", str(tmp_path),
                        "--iso", str(tmp_path / "a.iso")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    for step in ("merge_config.sh", "bzImage", "debootstrap", "mksquashfs", "cpio", "grub-mkrescue"):
        assert step in out, step
    assert "-volid AIOS" in out


def test_kernel_fragment_has_compute_stack():
    frag = open(os.path.join(ROOT, "distro", "kernel", "aios-mi355x.config")).read()
    for opt in ("CONFIG_DRM_AMDGPU=m", "CONFIG_HSA_AMD=y", "CONFIG_HSA_AMD_SVM=y", "CONFIG_HMM_MIRROR=y",
                "CONFIG_PCI_P2PDMA=y", "CONFIG_IOMMU_DEFAULT_PASSTHROUGH=y", "CONFIG_SECURITY_APPARMOR=y",
                "CONFIG_SQUASHFS=y", "CONFIG_OVERLAY_FS=y", "CONFIG_BLK_DEV_NVME=y"):
        assert opt in frag, opt


def test_grub_and_apparmor():
    grub = open(os.path.join(ROOT, "deploy", "boot", "grub", "grub.cfg")).read()
    assert grub.count("menuentry") == 3 and "iommu=pt" in grub and "aios.runtime_device=cpu" in grub
    prof = open(os.path.join(ROOT, "deploy", "etc", "apparmor.d", "aios-runtime")).read()
    assert "/dev/kfd rw," in prof and "/dev/dri/renderD* rw," in prof
    assert "deny /var/lib/aios/data/** w," in prof


def test_first_boot_initialises_a_node(tmp_path):
    """scripts/first-boot.sh on an empty data dir: identity keys, every service schema, system-agent
    state, certificates, hardware inventory, flag removed; a second run is idempotent."""
    import json
    import sqlite3
    import subprocess

    data = tmp_path / "var"
    data.mkdir()
    (data / ".first-boot").write_text("")
    env = dict(os.environ, AIOS_DATA_DIR=str(data), AIOS_ETC=str(tmp_path / "etc"), AIOS_LOG_DIR=str(tmp_path / "log"),
               AIOS_CONFIG=str(tmp_path / "none.toml"))
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "first-boot.sh"), "--no-network"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    rep = json.loads((data / "first-boot.json").read_text())
    assert all(v["ok"] for v in rep.values()), rep
    assert not (data / ".first-boot").exists() and (data / ".first-boot-done").exists()
    assert oct((data / "keys" / "node.key").stat().st_mode & 0o777) == "0o600"
    assert (data / "keys" / "node.pub").read_text().startswith("-----BEGIN PUBLIC KEY-----")
    tables = lambda p: {t for (t,) in sqlite3.connect(p).execute("SELECT name FROM sqlite_master WHERE type='table'")}
    assert "usage" in tables(data / "data" / "gateway_usage.db")
    assert {"agent_states", "goals", "patterns"} <= tables(data / "memory" / "working.db")
    st = sqlite3.connect(data / "memory" / "working.db").execute(
        "SELECT state_json FROM agent_states WHERE agent_name = 'system-agent'").fetchone()
    assert json.loads(st[0])["first_boot"] is True
    assert rep["tls"]["verify"] and os.path.exists(rep["tls"]["paths"]["ca_cert"])
    hw = json.loads((data / "hardware.json").read_text())
    assert hw["cpus"] > 0 and hw["mem_kb"] > 0 and isinstance(hw["amd_gpus"], list)
    node_id = (data / "node_id").read_text()
    r2 = subprocess.run(["bash", os.path.join(ROOT, "scripts", "first-boot.sh"), "--no-network"], env=env,
                        capture_output=True, text=True, timeout=120)
    assert r2.returncode == 0 and (data / "node_id").read_text() == node_id
