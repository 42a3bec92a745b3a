"""First-boot identity keys survive a crash mid-generation: an empty or truncated key
left by an interrupted run is regenerated, a valid one is kept."""
import shutil

import pytest

from aios_amd.utils.first_boot import FirstBoot, _valid_key

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl not installed")


def test_empty_key_is_regenerated_valid_key_kept(tmp_path, monkeypatch):
    fb = FirstBoot(str(tmp_path), str(tmp_path / "etc"), str(tmp_path / "log"), probe_network=False)
    fb.directories()
    key = tmp_path / "keys" / "node.key"
    key.write_text("")  # what a crash between create and openssl used to leave
    out = fb.identity()
    assert _valid_key(str(key)) and out["keys"]["node"] == str(key)
    before = key.read_bytes()
    fb.identity()
    assert key.read_bytes() == before  # valid: untouched
    assert not list((tmp_path / "keys").glob("*.tmp.*"))
