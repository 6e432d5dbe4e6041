"""The host code (datafile walk and encoders, scalar engine, GF(2) table
builder, the integrity tool's report and worker logic, the SET harness's
parser / index / datafile writer) built with AddressSanitizer +
UndefinedBehaviorSanitizer (`make -C 0-db_amd sanitize`) and run on every
golden datafile (valid, corrupt, truncated, malformed) and on pipelined SET
streams: no sanitizer report, and the same output as the regular build."""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import pytest

from conftest import GOLDEN, ROOT
from test_tool_cpu import CASES, TIMELOG, expected

SAN = ROOT / "0-db_amd" / "bin" / "san"
ENV = dict(os.environ, TZ="UTC", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-C", str(ROOT / "0-db_amd"), "sanitize"], check=True, capture_output=True)


@pytest.mark.parametrize("jobs", [1, 4])
def test_sanitized_integrity_tool(tmp_path, datafile_cases, jobs):
    exits = {c["name"]: c["exit"] for c in datafile_cases}
    for name in CASES:
        d = tmp_path / f"{jobs}_{name}"
        d.mkdir()
        shutil.copy(GOLDEN / "datafiles" / f"{name}.d0", d / "d0")
        os.symlink("d0", d / "zdb-data-0")
        p = subprocess.run([str(SAN / "zdb-integrity-check"), "--engine=cpu", f"--jobs={jobs}", str(d / "zdb-data-0")],
                           capture_output=True, env=ENV, timeout=120)
        err = p.stderr.decode()
        assert "Sanitizer" not in err and "runtime error" not in err, err[-3000:]
        norm = lambda s: TIMELOG.sub("[T]", s.replace(str(d), "@DIR@"))
        eout, eerr = expected(name)
        assert norm(p.stdout.decode()) == eout
        assert norm(err) == eerr
        assert p.returncode == exits[name]


def test_sanitized_multi_file_scan(tmp_path):
    from test_tool_multi import MULTI, stage
    dirs = stage(MULTI * 2, tmp_path)
    p = subprocess.run([str(SAN / "zdb-integrity-check"), "--engine=cpu", "--jobs=5"] + [str(d / "zdb-data-0") for d in dirs],
                       capture_output=True, env=ENV, timeout=300)
    err = p.stderr.decode()
    assert "Sanitizer" not in err and "runtime error" not in err, err[-3000:]
    assert p.returncode not in (98, 99)


@pytest.mark.parametrize("batch", [1, 37, 4096])
def test_sanitized_set_pipeline(tmp_path, batch):
    from test_set_pipeline import build_stream
    stream, _ = build_stream(21)
    outs = {}
    for tag, exe in (("san", SAN / "zdb-set-pipeline"), ("std", ROOT / "0-db_amd" / "bin" / "zdb-set-pipeline")):
        p = subprocess.run([str(exe), "--engine=cpu", "--datasize=600000", f"--batch={batch}", str(tmp_path / tag)],
                           input=stream, capture_output=True, env=ENV, timeout=300)
        err = p.stderr.decode()
        assert "Sanitizer" not in err and "runtime error" not in err, err[-3000:]
        assert p.returncode == 0
        outs[tag] = p.stdout
    assert outs["san"] == outs["std"]


def test_sanitized_index_verify(tmp_path):
    from test_index_verify import NAMESPACES, make_ns
    for name, files in NAMESPACES.items():
        ns = make_ns(tmp_path / name, files)
        outs = []
        for exe in (SAN / "zdb-index-verify", ROOT / "0-db_amd" / "bin" / "zdb-index-verify"):
            p = subprocess.run([str(exe), "--engine=cpu", "--list", str(ns)], capture_output=True, env=ENV,
                               timeout=120)
            err = p.stderr.decode()
            assert "Sanitizer" not in err and "runtime error" not in err, err[-3000:]
            outs.append((p.stdout, p.returncode))
        assert outs[0] == outs[1]
