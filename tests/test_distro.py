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


def test_cpio_newc_roundtrip(tmp_path):
    """aios_amd.utils.cpio: a tree (dirs, files with modes, a symlink) -> newc -> the same entries back,
    root-owned, deterministic (two writes are byte-identical), /dev/console declared"""
    from aios_amd.utils.cpio import read_newc, write_newc

    root = tmp_path / "t"
    (root / "a" / "b").mkdir(parents=True)
    (root / "a" / "b" / "x.txt").write_text("hello")
    (root / "run.sh").write_text("#!/bin/sh\n")
    os.chmod(root / "run.sh", 0o755)
    os.symlink("a/b/x.txt", root / "link")
    data = write_newc(str(root))
    assert data == write_newc(str(root)) and len(data) % 4 == 0
    ents = {n: (m, b) for n, m, _, b in read_newc(data)}
    assert ents["a/b/x.txt"][1] == b"hello" and ents["run.sh"][0] == 0o100755
    assert ents["link"] == (0o120777, b"a/b/x.txt") and ents["a"][0] == 0o40755
    assert ents["dev/console"][0] == 0o20600


def test_initramfs_builds_offline(tmp_path):
    """scripts/build-initramfs.sh without busybox, cpio or root: a static /init (distro/initramfs/init.c)
    in a gzip newc image; the packed /init, run with --plan on the build host, prints the boot plan ending in
    switch_root into aios-init"""
    import shutil
    import stat

    from aios_amd.utils.cpio import read_newc

    if not shutil.which("gcc"):
        pytest.skip("no C compiler")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "build-initramfs.sh"), "--out", str(tmp_path)],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "cannot find -lc" in r.stderr:
        pytest.skip("no static libc")
    assert r.returncode == 0, r.stderr
    ents = {n: (m, b) for n, m, _, b in read_newc((tmp_path / "initramfs.img").read_bytes())}
    for d in ("proc", "sys", "dev", "mnt/medium", "mnt/ro", "mnt/rw", "newroot", "lib/modules"):
        assert stat.S_ISDIR(ents[d][0]), d
    mode, init = ents["init"]
    assert stat.S_ISREG(mode) and mode & 0o111 and init[:4] == b"\x7fELF"
    import struct

    phoff, = struct.unpack_from("<Q", init, 0x20)
    phentsize, phnum = struct.unpack_from("<HH", init, 0x36)
    ptypes = [struct.unpack_from("<I", init, phoff + i * phentsize)[0] for i in range(phnum)]
    assert 3 not in ptypes  # static: no PT_INTERP program header
    exe = tmp_path / "init_plan"
    exe.write_bytes(init)
    exe.chmod(0o755)
    plan = subprocess.run([str(exe), "--plan"], capture_output=True, text=True, timeout=30)
    assert plan.returncode == 0, plan.stderr
    lines = plan.stdout.splitlines()
    assert lines[0] == "mount -t proc proc /proc" and "squashfs" in plan.stdout and "overlay" in plan.stdout
    assert lines[-1] == "switch_root /newroot /usr/sbin/aios-init"


def test_overlay_rootfs_builds_offline(tmp_path):
    """scripts/build-rootfs.sh --overlay-only: the aiOS layer (package with its built extensions, aios-init,
    configs, environment) as an ext4 image built without root (mkfs.ext4 -d)"""
    import shutil

    mkfs = shutil.which("mkfs.ext4") or ("/usr/sbin/mkfs.ext4" if os.path.exists("/usr/sbin/mkfs.ext4") else None)
    if not mkfs:
        pytest.skip("no mkfs.ext4")
    env = dict(os.environ, PATH=os.environ.get("PATH", "") + ":/usr/sbin:/sbin")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "build-rootfs.sh"), "--out", str(tmp_path),
                        "--overlay-only"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    img = tmp_path / "aios-overlay.ext4"
    assert img.exists() and img.stat().st_size > 1 << 20
    o = tmp_path / "overlay"
    assert (o / "usr/lib/aios/aios_amd/__init__.py").exists() and (o / "etc/aios/config.toml").exists()
    assert "PYTHONPATH=/usr/lib/aios" in (o / "etc/aios/environment").read_text()
    assert not list(o.rglob("__pycache__"))
    debugfs = shutil.which("debugfs", path=env["PATH"])
    if debugfs:
        ls = subprocess.run([debugfs, "-R", "ls /usr/lib/aios/aios_amd", str(img)], capture_output=True, text=True)
        assert "__init__.py" in ls.stdout


def test_iso9660_writer_roundtrip(tmp_path):
    """aios_amd.utils.iso9660: nested directories, an empty file, sizes across sector boundaries and a
    directory whose records span several sectors; read back by our parser, the volume id where the early
    init looks for it (sector 16, offset 40), and by util-linux's blkid when present"""
    import shutil

    from aios_amd.utils.iso9660 import read_iso, write_iso

    src = tmp_path / "src"
    want = {}
    for rel, size in [("boot/vmlinuz", 5000), ("boot/grub/grub.cfg", 30), ("rootfs.squashfs", 2048),
                      ("empty.txt", 0), ("aios-overlay.ext4", 4097)] + [(f"a/b/c/file_number_{i}.dat", i) for i in range(90)]:
        p = src / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        body = os.urandom(size)
        p.write_bytes(body)
        want[rel.replace("-", "_")] = body
    iso = tmp_path / "a.iso"
    n = write_iso(str(src), str(iso), "AIOS")
    assert n == iso.stat().st_size and n % 2048 == 0
    volid, files = read_iso(str(iso))
    assert volid == "AIOS" and files == want
    raw = iso.read_bytes()
    assert raw[16 * 2048 + 1:16 * 2048 + 6] == b"CD001" and raw[16 * 2048 + 40:16 * 2048 + 44] == b"AIOS"
    assert write_iso(str(src), str(tmp_path / "b.iso")) == n and (tmp_path / "b.iso").read_bytes() == raw  # deterministic
    blkid = shutil.which("blkid") or ("/usr/sbin/blkid" if os.path.exists("/usr/sbin/blkid") else None)
    if blkid:
        r = subprocess.run([blkid, "-p", "-o", "export", str(iso)], capture_output=True, text=True)
        assert "TYPE=iso9660" in r.stdout and "LABEL=AIOS" in r.stdout, r.stdout + r.stderr


def test_data_medium_builds_offline(tmp_path):
    """scripts/build-iso.sh --data: the initramfs (built offline) on an ISO 9660 medium labelled AIOS"""
    import shutil

    from aios_amd.utils.iso9660 import read_iso

    if not shutil.which("gcc"):
        pytest.skip("no C compiler")
    iso = tmp_path / "aios.iso"
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "build-iso.sh"), "--data", "--out", str(tmp_path),
                        "--iso", str(iso)], capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "cannot find -lc" in r.stderr:
        pytest.skip("no static libc")
    assert r.returncode == 0, r.stderr
    volid, files = read_iso(str(iso))
    assert volid == "AIOS" and files["boot/initramfs.img"] == (tmp_path / "initramfs.img").read_bytes()


def test_root_image_from_base_tree_offline(tmp_path):
    """scripts/build-rootfs.sh --base DIR: a userland tree with the aiOS layer over it, packed as rootfs.ext4
    (the early init's root image when the medium has no squashfs), then put on the data medium"""
    import shutil

    from aios_amd.utils.iso9660 import read_iso

    mkfs = shutil.which("mkfs.ext4") or ("/usr/sbin/mkfs.ext4" if os.path.exists("/usr/sbin/mkfs.ext4") else None)
    if not mkfs or not shutil.which("gcc"):
        pytest.skip("no mkfs.ext4 / C compiler")
    base = tmp_path / "base"
    (base / "bin").mkdir(parents=True)
    (base / "etc").mkdir()
    (base / "bin" / "sh").write_text("#!/bin/false\n")
    (base / "etc" / "os-release").write_text('NAME="Ubuntu"\nVERSION_ID="22.04"\n')
    env = dict(os.environ, PATH=os.environ.get("PATH", "") + ":/usr/sbin:/sbin")
    out = tmp_path / "out"
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "build-rootfs.sh"), "--out", str(out), "--base", str(base)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    img = out / "rootfs.ext4"
    assert img.exists() and not (out / "rootfs-stage").exists()
    debugfs = shutil.which("debugfs", path=env["PATH"])
    if debugfs:
        for path, want in (("/etc", "os-release"), ("/usr/sbin", "aios-init"), ("/etc/aios", "config.toml")):
            ls = subprocess.run([debugfs, "-R", f"ls {path}", str(img)], capture_output=True, text=True)
            assert want in ls.stdout, (path, ls.stdout)
    iso = tmp_path / "aios.iso"
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "build-iso.sh"), "--data", "--out", str(out), "--iso", str(iso)],
                       capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0 and "cannot find -lc" in r.stderr:
        pytest.skip("no static libc")
    assert r.returncode == 0, r.stderr
    _, files = read_iso(str(iso))
    assert files["rootfs.ext4"] == img.read_bytes() and "boot/initramfs.img" in files
