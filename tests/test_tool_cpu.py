"""zdb-integrity-check (0-db_amd/tools) against the reference tool's captured
stdout / stderr / exit code (tests/golden/datafiles/*), with the explicitly
selected scalar engine (--engine=cpu).  The GPU engine is checked by the
same comparison in tests/test_gpu.py."""
from __future__ import annotations

import os
import re
import shutil
import subprocess
from pathlib import Path

import pytest

from conftest import GOLDEN, ROOT

TOOL = ROOT / "0-db_amd" / "bin" / "zdb-integrity-check"
TIMELOG = re.compile(r"\[\s*\d+\.\d{6}\]")
CASES = ["mixed", "zipf_small", "fixed_4k", "corrupt_payload", "corrupt_crc", "multi_errors",
         "truncated_payload", "truncated_header", "bad_magic", "bad_version", "header_only"]


def run_tool(name: str, tmp: Path, engine: str):
    d = tmp / name
    d.mkdir()
    shutil.copy(GOLDEN / "datafiles" / f"{name}.d0", d / "d0")
    os.symlink("d0", d / "zdb-data-0")
    env = dict(os.environ, TZ="UTC")
    p = subprocess.run([str(TOOL), f"--engine={engine}", str(d / "zdb-data-0")], capture_output=True,
                       env=env, timeout=120)
    norm = lambda s: TIMELOG.sub("[T]", s.decode().replace(str(d), "@DIR@"))
    return norm(p.stdout), norm(p.stderr), p.returncode


def expected(name: str):
    norm = lambda s: TIMELOG.sub("[T]", s)
    return (norm((GOLDEN / "datafiles" / f"{name}.stdout").read_text()),
            norm((GOLDEN / "datafiles" / f"{name}.stderr").read_text()))


@pytest.mark.parametrize("name", CASES)
def test_tool_matches_reference_cpu_engine(tmp_path, datafile_cases, name):
    out, err, code = run_tool(name, tmp_path, "cpu")
    eout, eerr = expected(name)
    assert out == eout
    assert err == eerr
    assert code == {c["name"]: c for c in datafile_cases}[name]["exit"]


def test_tool_argument_errors(tmp_path):
    p = subprocess.run([str(TOOL)], capture_output=True)
    assert p.returncode == 1 and b"Usage:" in p.stderr
    p = subprocess.run([str(TOOL), str(tmp_path / "nothing")], capture_output=True)
    assert p.returncode == 1 and p.stderr.decode().endswith("invalid target file\n")
    f = tmp_path / "d0"
    f.write_bytes(b"DAT0")
    p = subprocess.run([str(TOOL), str(f)], capture_output=True)
    assert p.returncode == 1 and b"data filename seems wrong" in p.stderr
    # name accepted but <dir>/d<id> missing (data.c:135)
    (tmp_path / "zdb-data-5").write_bytes(b"")
    p = subprocess.run([str(TOOL), "--engine=cpu", str(tmp_path / "zdb-data-5")], capture_output=True)
    assert p.returncode == 1
    assert b"d5: No such file or directory" in p.stderr
    assert p.stderr.endswith(b"[-] data file inconsistency: 1 error(s)\n")


def test_default_engine_is_auto(tmp_path, datafile_cases):
    """No --engine: the auto engine, which checks a small store on the scalar
    engine without starting the GPU runtime -- so the reference's command line
    gives the reference's report here too (this container has no GPU: the hip
    engine would exit 1 with "GPU engine unavailable")."""
    d = tmp_path / "mixed"
    d.mkdir()
    shutil.copy(GOLDEN / "datafiles" / "mixed.d0", d / "d0")
    os.symlink("d0", d / "zdb-data-0")
    p = subprocess.run([str(TOOL), str(d / "zdb-data-0")], capture_output=True, timeout=120,
                       env=dict(os.environ, TZ="UTC", ZDBCRC_TOOL_TRACE="1"))
    norm = lambda s: TIMELOG.sub("[T]", s.decode().replace(str(d), "@DIR@"))
    eout, eerr = expected("mixed")
    assert norm(p.stdout) == eout
    err = "".join(ln + "\n" for ln in norm(p.stderr).splitlines() if not ln.startswith("[trace]"))
    assert err == eerr
    assert p.returncode == {c["name"]: c for c in datafile_cases}["mixed"]["exit"]
    assert "auto engine" in p.stderr.decode() and "engine cpu" in p.stderr.decode()
