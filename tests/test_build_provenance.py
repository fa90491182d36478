"""Build provenance (ops/build.py): every native artefact carries the hash of the sources it
was built from; a library built from other sources is detected at import."""
import shutil

import pytest

from yoda_scheduler_amd.ops import build
from yoda_scheduler_amd.ops.native import core


def test_loaded_modules_match_this_tree():
    from yoda_scheduler_amd.kube.native import module
    assert core().build_id() == build.source_hash("core")
    assert module().build_id() == build.source_hash("kube")
    for name in ("core", "kube", "fakeapi"):
        assert build.recorded_id(name) == build.source_hash(name)


def test_touched_source_is_detected_as_stale(tmp_path, monkeypatch):
    """Copy the sources, touch one file's contents: the loaded module's id no longer
    matches (verify_loaded raises), and the pre-import check refuses (or would rebuild)."""
    native = tmp_path / "native"
    shutil.copytree(build.NATIVE, native)
    loaded = core().build_id()
    build.verify_loaded("core", loaded, native)              # identical copy: fine
    with open(native / "core" / "engine.cpp", "a") as f:
        f.write("\n// touched\n")
    with pytest.raises(build.StaleArtefact):
        build.verify_loaded("core", loaded, native)
    # the pre-import check sees the recorded id of the artefact as stale against the
    # touched tree: refuse mode raises instead of loading it
    monkeypatch.setattr(build, "NATIVE", native)
    monkeypatch.setenv("YODA_BUILD_CHECK", "refuse")
    assert build._stale("core") and not build._stale("kube")
    with pytest.raises(build.StaleArtefact):
        build.ensure_fresh("core")
    build.ensure_fresh("kube")                                  # untouched: loads


def test_recipe_change_changes_identity(monkeypatch):
    before = build.source_hash("core")
    monkeypatch.setitem(build.ARTEFACTS["core"], "recipe", build.ARTEFACTS["core"]["recipe"] + " -DX")
    assert build.source_hash("core") != before


def test_binaries_report_their_build_id():
    import subprocess
    exe = build.out_path("fakeapi")
    out = subprocess.run([str(exe), "--build-id"], capture_output=True, text=True, timeout=30).stdout.strip()
    assert out == build.source_hash("fakeapi")
