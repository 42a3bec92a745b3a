"""GPU health telemetry from a fake amdgpu sysfs tree (aios_amd/utils/sysinfo.py): RAS counters
(HBM ECC = umc, xGMI = xgmi_wafl), PCIe replays, hwmon temperatures / power; the verdict feeds the
proactive goal generator and the runtime metrics (SURVEY §5 failure detection)."""
import os

from aios_amd.utils import sysinfo


def _card(root, n, ras=None, temp_mc=None, power_uw=None, busy="7"):
    dev = root / "sys" / "class" / "drm" / f"card{n}" / "device"
    (dev / "ras").mkdir(parents=True)
    (dev / "vendor").write_text("0x1002\n")
    (dev / "device").write_text("0x75a3\n")
    (dev / "gpu_busy_percent").write_text(busy + "\n")
    (dev / "mem_info_vram_used").write_text(str(2 << 30) + "\n")
    (dev / "mem_info_vram_total").write_text(str(288 << 30) + "\n")
    (dev / "pcie_replay_count").write_text("0\n")
    for block, (ue, ce) in (ras or {}).items():
        (dev / "ras" / f"{block}_err_count").write_text(f"ue: {ue}\nce: {ce}\n")
    hw = dev / "hwmon" / "hwmon3"
    hw.mkdir(parents=True)
    if temp_mc is not None:
        (hw / "temp2_input").write_text(f"{temp_mc}\n")
        (hw / "temp2_label").write_text("junction\n")
    if power_uw is not None:
        (hw / "power1_average").write_text(f"{power_uw}\n")
    return dev


def test_counters_and_verdict(tmp_path):
    _card(tmp_path, 0, ras={"umc": (0, 4), "xgmi_wafl": (0, 0)}, temp_mc=61000, power_uw=812000000)
    _card(tmp_path, 1, ras={"umc": (2, 9), "gfx": (0, 1)}, temp_mc=70000)
    _card(tmp_path, 2, ras={"xgmi_wafl": (1, 0)}, temp_mc=97500)
    g = {x["card"]: x for x in sysinfo.amd_gpus(str(tmp_path))}
    assert g["card0"]["ecc_ce"] == 4 and g["card0"]["ecc_ue"] == 0 and g["card0"]["temp_junction_c"] == 61.0
    assert abs(g["card0"]["power_w"] - 812.0) < 1e-9 and g["card0"]["vram_total_mb"] == 288 * 1024
    assert g["card1"]["ras"]["umc"] == {"ue": 2, "ce": 9} and g["card1"]["ecc_ce"] == 10
    h = sysinfo.gpu_health(str(tmp_path))
    kinds = {(p["card"], p["kind"]) for p in h["problems"]}
    assert kinds == {("card1", "uncorrectable_ecc"), ("card2", "xgmi_link_errors"), ("card2", "overtemperature"),
                     ("card2", "uncorrectable_ecc")}
    assert not h["healthy"] and h["ecc_ue_total"] == 3 and h["gpus"] == 3
    _card(tmp_path / "ok", 0, ras={"umc": (0, 0)}, temp_mc=50000)
    assert sysinfo.gpu_health(str(tmp_path / "ok"))["healthy"]


def test_proactive_goals_from_gpu_health(tmp_path):
    from aios_amd.orchestrator.loops import ProactiveConfig, proactive_candidates
    from aios_amd.orchestrator.state import OrchestratorState

    _card(tmp_path / "sys1", 4, ras={"umc": (5, 0)})
    st = OrchestratorState(str(tmp_path / "orch"), in_memory=True)
    cfg = ProactiveConfig(network_probe=False, etc_probe=False, sysfs_root=str(tmp_path / "sys1"),
                          cert_path=str(tmp_path / "none"), log_path=str(tmp_path / "none.log"),
                          cpu_threshold=101, memory_threshold=101, disk_threshold=101)
    c = proactive_candidates(st, cfg)
    assert any("card4" in d and "uncorrectable ECC" in d and prio == 9 for d, prio in c), c
