"""f4: zdb-index-verify (the index-rebuild scan plus the payload check
index-rebuild.c:94 leaves out) against the REFERENCE index-rebuild and
index-dump, compiled from their sources (oracle/Makefile `indextools`): on
namespaces assembled from the golden datafiles (overwrites, deletions,
corrupt payloads and crcs, a payload cut by the end of a file, a bad file
that ends the rebuild), the live keys this tool reports -- key, datafile,
offset, length, stored crc -- are exactly the entries the reference's
rebuilt index holds (index-dump, not flagged deleted), and the ones it
reports corrupt are exactly the live entries whose payload fails its crc."""
from __future__ import annotations

import re
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
import zdbcrc
from conftest import GOLDEN, ROOT

REF = Path(oracle.__file__).resolve().parent / "_ref"
TOOL = ROOT / "0-db_amd" / "bin" / "zdb-index-verify"

def damaged(name: str, payload_flips=(), crc_flips=()) -> bytes:
    """a golden datafile with payload bytes / stored crcs of some records flipped"""
    img = bytearray((GOLDEN / "datafiles" / f"{name}.d0").read_bytes())
    recs, _ = zdbcrc.datafile_walk(bytes(img))
    live = recs[recs["datalength"] > 0]
    for k in payload_flips:
        img[int(live["payload_offset"][k]) + int(live["datalength"][k]) // 2] ^= 0x10
    for k in crc_flips:
        img[int(live["header_offset"][k]) + 9] ^= 0x01
    return bytes(img)


NAMESPACES = {
    "clean": ["mixed", "zipf_small", "fixed_4k"],
    "damaged": ["mixed", "corrupt_payload", damaged("zipf_small", (3, 11, 19)), damaged("fixed_4k", (), (5, 60))],
    "cut": ["zipf_small", "mixed", "truncated_payload"],
    "stops_at_bad_file": ["fixed_4k", "bad_magic", "mixed"],
}


def make_ns(tmp: Path, files) -> Path:
    d = tmp / "data" / "ns"
    d.mkdir(parents=True)
    for i, name in enumerate(files):
        if isinstance(name, bytes):
            (d / f"d{i}").write_bytes(name)
        else:
            shutil.copy(GOLDEN / "datafiles" / f"{name}.d0", d / f"d{i}")
    return d


def reference_live(tmp: Path, ns: Path, tlimit: int = 0) -> set:
    idx = tmp / "index"
    args = [str(REF / "index-rebuild"), "--data", str(ns.parent), "--index", str(idx), "--namespace", "ns",
            "--mode", "user"] + (["--time", str(tlimit)] if tlimit else [])
    subprocess.run(args, capture_output=True, timeout=120, check=True)
    out = subprocess.run([str(REF / "index-dump"), str(idx / "ns")], capture_output=True, timeout=120)
    text = out.stdout.decode(errors="replace")
    live = set()
    for block in text.split("[+] index entry: ")[1:]:
        f = dict(re.findall(r"\[\+\]\s+([a-z ]+?)\s*: (.*)", block))
        if int(f["entry flags"], 16) & 1:
            continue  # superseded or deleted (INDEX_ENTRY_DELETED, index.h:73)
        live.add((f["entry key"].strip(), int(f["data fileid"]), int(f["data offset"]), int(f["data length"]),
                  f["data crc"].strip()))
    return live


def tool_live(ns: Path, engine: str = "cpu", tlimit: int = 0):
    args = [str(TOOL), f"--engine={engine}", "--list"] + ([f"--time={tlimit}"] if tlimit else []) + [str(ns)]
    p = subprocess.run(args, capture_output=True, timeout=120)
    live, corrupt = set(), set()
    for ln in p.stdout.decode().splitlines():
        if ln.startswith("live "):
            _, key, fid, off, ln_, crc, st = ln.split()
            row = (key, int(fid), int(off), int(ln_), crc)
            live.add(row)
            if st == "CORRUPT":
                corrupt.add(row)
    return live, corrupt, p


def oracle_corrupt(ns: Path, live: set) -> set:
    """live entries whose payload crc (the oracle's) differs from the stored one"""
    orc, bad = oracle.Oracle(), set()
    for row in live:
        key, fid, off, length, crc = row
        img = np.fromfile(ns / f"d{fid}", dtype=np.uint8)
        p = off + 18 + int(img[off])
        if p + length > len(img) or orc.crc32(img[p:p + length]) != int(crc, 16):
            bad.add(row)
    return bad


needs_ref = pytest.mark.skipif(not (REF / "index-rebuild").exists(), reason="make -C oracle indextools")


@needs_ref
@pytest.mark.parametrize("name", sorted(NAMESPACES))
def test_index_verify_matches_reference_rebuild(tmp_path, name):
    ns = make_ns(tmp_path, NAMESPACES[name])
    want = reference_live(tmp_path, ns)
    live, corrupt, p = tool_live(ns)
    assert live == want
    assert corrupt == oracle_corrupt(ns, live)
    assert p.returncode == len(corrupt)
    if name == "damaged":
        assert corrupt
    if name == "clean":
        assert not corrupt and live


@needs_ref
def test_index_verify_time_limit(tmp_path):
    ns = make_ns(tmp_path, NAMESPACES["clean"])
    recs, _ = zdbcrc.datafile_walk((ns / "d1").read_bytes())
    t = int(np.median(recs["timestamp"]))
    want = reference_live(tmp_path, ns, t)
    live, _, _ = tool_live(ns, "cpu", t)
    assert live == want


def test_index_verify_short_header_is_fatal(tmp_path):
    ns = make_ns(tmp_path, ["mixed", "truncated_header"])
    _, _, p = tool_live(ns)
    assert p.returncode == 1 and b"data header read failed" in p.stderr
