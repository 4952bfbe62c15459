"""Fresh-checkout build (CPU): the tree the driver pushes holds tracked files only (the .so and
build/ are git-ignored), so the entry points must build the library themselves. This copies the
git-tracked files of the working tree into a temp dir, runs the same hook conftest.py / bench.py /
__graft_entry__.smoke() run (build_lib.ensure_built), and checks that the library appears there and
exports every entry point include/b2p_hip.h declares. Cold build: ~80 s on 8 cores."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "b2p_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(b2p_[a-z0-9_]+)\s*\(", src)))


@pytest.mark.skipif(shutil.which("git") is None, reason="git not available")
def test_tracked_tree_builds_its_library(tmp_path):
    files = subprocess.run(["git", "ls-files", "-z"], cwd=ROOT, capture_output=True, check=True).stdout
    files = [f for f in files.decode().split("\0") if f]
    for f in files:
        src = os.path.join(ROOT, f)
        if not os.path.exists(src):        # deleted in the working tree, not yet committed
            continue
        dst = tmp_path / f
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy2(src, dst)
    so = tmp_path / "wav2vec2forbrain_amd" / "libb2p_hip.so"
    assert not so.exists() and not (tmp_path / "build").exists()
    r = subprocess.run([sys.executable, "-c", "from wav2vec2forbrain_amd import build_lib; build_lib.ensure_built()"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert so.exists()
    nm = subprocess.run(["nm", "-D", "--defined-only", str(so)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (b2p_[a-z0-9_]+)$", nm, flags=re.M))
    missing = [n for n in _declared() if n not in exported]
    assert not missing, missing
