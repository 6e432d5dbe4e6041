"""SURVEY §8(d) C4 workload: the synthetic datafiles bench.py scans are
reference-valid -- the reference integrity-check tool (compiled from its
sources, oracle/_ref) accepts a C4 file with every crc matching, our tool
prints the same report, and zdb_datafile_walk finds exactly the layout."""
from __future__ import annotations

import os
import re
import subprocess

import numpy as np
import pytest

import bench
import oracle
import zdbcrc
from conftest import ROOT

TOOL = ROOT / "0-db_amd" / "bin" / "zdb-integrity-check"
TIMELOG = re.compile(r"\[\s*\d+\.\d{6}\]")


@pytest.fixture(scope="module")
def c4_file0(reference):
    """Datafile 0 of the rank-0 C4 shard (256 MiB), crcs by the reference."""
    lay = bench.c4_layout(0)
    sel = lay["file_of"] == 0
    end = int(lay["file_off"][0] + lay["file_size"][0])
    raw = zdbcrc.synth_fill(end, bench.C4_SEED)
    crcs = np.zeros(len(lay["lens"]), np.uint32)
    crcs[sel] = reference.batch(raw, lay["payload_off"][sel].astype(np.uint64),
                                lay["lens"][sel].astype(np.uint32), threads=8)
    img = bench.c4_image_host(lay, bench.C4_SEED, crcs, files=1)
    return lay, sel, crcs, img


def test_c4_layout_shape():
    lay = bench.c4_layout(0)
    assert len(lay["file_off"]) == bench.C4_FILES
    assert lay["file_size"].max() <= bench.C4_FILE_CAP
    assert 15.5 * 2**30 < lay["lens"].sum() < 16 * 2**30
    # payloads never overlap headers: entries are back to back inside a file
    e = lay["entry_off"]
    nxt = e + bench.ENTRY_HDR + bench.C4_KEY + lay["lens"]
    same = lay["file_of"][1:] == lay["file_of"][:-1]
    np.testing.assert_array_equal(nxt[:-1][same], e[1:][same])


def test_c4_file_walk(c4_file0):
    lay, sel, crcs, img = c4_file0
    recs, status = zdbcrc.datafile_walk(img)
    assert status == 0
    np.testing.assert_array_equal(recs["header_offset"], lay["entry_off"][sel])
    np.testing.assert_array_equal(recs["payload_offset"], lay["payload_off"][sel])
    np.testing.assert_array_equal(recs["datalength"], lay["lens"][sel])
    np.testing.assert_array_equal(recs["integrity"], crcs[sel])
    np.testing.assert_array_equal(recs["previous"], lay["prev"][sel])


def test_c4_file_accepted_by_reference_tool(tmp_path, c4_file0):
    lay, sel, crcs, img = c4_file0
    d = tmp_path / "c4"
    d.mkdir()
    img.tofile(d / "d0")  # the tools resolve zdb-data-<id> to <dir>/d<id>, as in test_tool_cpu
    os.symlink("d0", d / "zdb-data-0")
    env = dict(os.environ, TZ="UTC")
    ref = subprocess.run([str(oracle.REF_INTEGRITY), str(d / "zdb-data-0")], capture_output=True, env=env,
                         timeout=300)
    assert ref.returncode == 0, ref.stderr[-500:]
    assert ref.stdout.count(b"data crc       : ok, match") == int(sel.sum())
    assert b"[-]" not in ref.stderr
    ours = subprocess.run([str(TOOL), "--engine=cpu", str(d / "zdb-data-0")], capture_output=True, env=env,
                          timeout=300)
    norm = lambda b: TIMELOG.sub("[T]", b.decode())
    assert norm(ours.stdout) == norm(ref.stdout)
    assert norm(ours.stderr) == norm(ref.stderr)
    assert ours.returncode == ref.returncode
