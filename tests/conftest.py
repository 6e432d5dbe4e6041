"""Shared test setup.

Markers: ``gpu`` -- needs an MI355X (run on the GPU box with ``-m gpu``);
everything else runs on the CPU-only build container.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
for p in (ROOT / "0-db_amd", ROOT / "oracle", ROOT / "tests", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP) -- run with -m gpu")


@pytest.fixture(scope="session")
def oracle_c():
    import oracle
    return oracle.Oracle()


@pytest.fixture(scope="session")
def reference():
    import oracle
    if not oracle.Reference.available():
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    return oracle.Reference()


@pytest.fixture(scope="session")
def kats():
    return json.loads((GOLDEN / "kat.json").read_text())


def kat_bytes(entry) -> bytes:
    if "hex" in entry:
        return bytes.fromhex(entry["hex"])
    return bytes([int(entry["fill"], 16)]) * entry["length"]


@pytest.fixture(scope="session")
def vectors():
    d = np.load(GOLDEN / "vectors.npz")
    return d["lengths"], d["seeds"], d["crcs"]


@pytest.fixture(scope="session")
def datafile_cases():
    return json.loads((GOLDEN / "datafiles.json").read_text())


@pytest.fixture(scope="session")
def digests():
    p = GOLDEN / "digests.json"
    if not p.exists():
        pytest.skip("digests.json not generated")
    return json.loads(p.read_text())
