#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REAL
reference, built from /root/reference by oracle/Makefile into oracle/_ref/:

  kat.json            known-answer vectors: zdb_crc32 (libzdb/crc32.c) on
                      fixed strings, including the test payloads of the
                      reference's own suite (tests/zdb_payload.c:13-33,
                      tests/zdb_default.c:66, examples/zdb-example.c:20,
                      tests/pipeline/pipeline.c:32)
  vectors.npz         (length, seed, crc) for splitmix64 buffers of lengths
                      0..1100, a sweep to 4160 and 7 large sizes; the data is
                      regenerated from (length, seed) by oracle.splitmix_bytes
  datafiles/*.d0      small real datafiles written through the reference
                      libzdb (oracle/gen_datafile_ref.c), some corrupted on
                      purpose, each with the reference integrity-check's
                      stdout / stderr / exit code (TZ=UTC)
  digests.json        count / XOR / order-sensitive crc of the per-record
                      crcs of the full-size bench datasets (C2, C3, C4 shard 0), so the GPU
                      can be checked bit-exact at BASELINE sizes

Run in the build container (needs /root/reference):
    make -C oracle all ref && make -C 0-db_amd && python tests/golden/make_golden.py
Inputs of the large datasets come from the product's zdb_synth_fill /
zdb_synth_zipf_lengths (tests/test_oracle.py pins zdb_synth_fill to
oracle.splitmix_bytes); every expected OUTPUT here comes from the reference.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "0-db_amd"))
import oracle  # noqa: E402

OUT = ROOT / "tests" / "golden"
DF = OUT / "datafiles"

VECTOR_SEED_BASE = 0x5EED0000
C2_SEED = 0x5A0DB5EED
C3_SEED = 0x5A0DB5EED + 3
C3_LEN_SEED = 0xC3C3C3
MAX_SEED = 0x5A0DB5EED + 9


def kats(ref: oracle.Reference) -> list[dict]:
    cases = [
        ("empty", b""),
        ("digits", b"123456789"),
        ("world", b"world"),                          # SET hello world (tests/zdb_default.c:66)
        ("hello_world", b"Hello World !"),            # examples/zdb-example.c:20
        ("pipeline", b"THISISMYDATAHELLOYEAHWORKS"),  # tests/pipeline/pipeline.c:32
        ("byte01", b"\x01"),
        ("byte80", b"\x80"),
        ("ff32", b"\xff" * 32),
        ("zeros4096", b"\x00" * 4096),
        ("ascii_a_1000", b"a" * 1000),
        ("seq256", bytes(range(256))),
    ]
    # tests/zdb_payload.c:13-33: 0x42-filled payloads 512 B .. 8 MiB
    for size in (512, 1024, 4096, 65536, 512 * 1024, 1 << 20, 2 << 20, 4 << 20, 8 << 20):
        cases.append((f"x42_{size}", b"\x42" * size))
    out = []
    for name, data in cases:
        entry = {"name": name, "length": len(data), "crc": f"{ref.crc32(data):08x}"}
        if len(data) <= 4096 and name != "seq256":
            entry["hex"] = data.hex()
        elif name == "seq256":
            entry["hex"] = data.hex()
        else:
            entry["fill"] = f"{data[0]:02x}"
        out.append(entry)
    return out


def vector_lengths() -> np.ndarray:
    lens = list(range(0, 1101)) + list(range(1101, 4161, 7)) + [4160]
    lens += [8191, 8192, 65535, 65536, 262144, 1048575, 1048576]
    return np.array(sorted(set(lens)), dtype=np.int64)


def vectors(ref: oracle.Reference):
    lens = vector_lengths()
    seeds = (VECTOR_SEED_BASE + lens).astype(np.uint64)
    crcs = np.zeros(len(lens), dtype=np.uint32)
    for i, (n, s) in enumerate(zip(lens, seeds)):
        crcs[i] = ref.crc32(oracle.splitmix_bytes(int(n), int(s)))
    np.savez_compressed(OUT / "vectors.npz", lengths=lens, seeds=seeds, crcs=crcs)
    return len(lens)


def run_ref_tool(d0: Path) -> tuple[str, str, int]:
    with tempfile.TemporaryDirectory() as td:
        shutil.copy(d0, Path(td) / "d0")
        os.symlink("d0", Path(td) / "zdb-data-0")
        env = dict(os.environ, TZ="UTC")
        p = subprocess.run([str(oracle.REF_INTEGRITY), f"{td}/zdb-data-0"], capture_output=True,
                           env=env, cwd=td)
        out = p.stdout.decode().replace(td, "@DIR@")
        err = p.stderr.decode().replace(td, "@DIR@")
        return out, err, p.returncode


def gen_datafile(mode: str, count: int, seed: int, size: int) -> bytes:
    with tempfile.TemporaryDirectory() as td:
        subprocess.run([str(oracle.REF_GEN), td, mode, str(count), str(seed), str(size)], check=True,
                       capture_output=True)
        return (Path(td) / "data" / "default" / "d0").read_bytes()


def datafiles() -> list[dict]:
    DF.mkdir(parents=True, exist_ok=True)
    for f in DF.iterdir():
        f.unlink()
    base = gen_datafile("mixed", 100, 7, 0)
    zipf = gen_datafile("zipf", 1000, 11, 600_000)
    fixed = gen_datafile("fixed", 64, 13, 4096)
    orc = oracle.Oracle()
    recs, errors, fatal = orc.integrity_scan(base)
    assert errors == 0 and fatal == 0
    live = [r for r in recs if r["datalength"] > 0]

    def flip_payload(img: bytes, rec, delta=0x5A) -> bytes:
        b = bytearray(img)
        b[int(rec["payload_offset"]) + int(rec["datalength"]) // 2] ^= delta
        return bytes(b)

    def flip_crc(img: bytes, rec) -> bytes:
        b = bytearray(img)
        b[int(rec["header_offset"]) + 9] ^= 0x01
        return bytes(b)

    last = recs[-1]
    cases = {
        "mixed": base,
        "zipf_small": zipf,
        "fixed_4k": fixed,
        "corrupt_payload": flip_payload(base, live[7]),
        "corrupt_crc": flip_crc(base, live[3]),
        "multi_errors": flip_payload(flip_crc(flip_payload(base, live[1]), live[10]), live[20]),
        "truncated_payload": base[: int(last["payload_offset"]) + int(last["datalength"]) // 2],
        "truncated_header": base[: int(last["header_offset"]) + 7],
        "bad_magic": b"DAT1" + base[4:],
        "bad_version": base[:4] + (2).to_bytes(4, "little") + base[8:],
        "header_only": base[:28],
    }
    meta = []
    for name, img in cases.items():
        path = DF / f"{name}.d0"
        path.write_bytes(img)
        out, err, code = run_ref_tool(path)
        (DF / f"{name}.stdout").write_text(out)
        (DF / f"{name}.stderr").write_text(err)
        meta.append({"name": name, "bytes": len(img), "exit": code})
        print(f"  datafile {name}: {len(img)} B, exit {code}")
    return meta


def digest(ref: oracle.Reference, crcs: np.ndarray) -> dict:
    return {
        "count": int(len(crcs)),
        "xor": f"{int(np.bitwise_xor.reduce(crcs)) if len(crcs) else 0:08x}",
        "crc_of_crcs": f"{ref.crc32(crcs.astype('<u4').tobytes()):08x}",
    }


def digests(ref: oracle.Reference) -> dict:
    import zdbcrc
    out = {}
    # C2: 1 Mi x 4 KiB, record i at 4096*i
    n2 = 1 << 20
    arena = zdbcrc.synth_fill(n2 * 4096, C2_SEED)
    offs = np.arange(n2, dtype=np.uint64) * 4096
    lens = np.full(n2, 4096, dtype=np.uint32)
    c2 = ref.batch(arena, offs, lens, threads=8)
    out["C2"] = {"seed": C2_SEED, "records": n2, "record_bytes": 4096, **digest(ref, c2)}
    del arena
    # C3: Zipf 64 B..1 MiB, packed back to back (any byte alignment), ~4 GiB
    lens = zdbcrc.zipf_lengths(4 << 30, C3_LEN_SEED)
    offs = np.zeros(len(lens), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum(dtype=np.uint64))
    arena = zdbcrc.synth_fill(total, C3_SEED)
    c3 = ref.batch(arena, offs, lens, threads=8)
    out["C3"] = {"seed": C3_SEED, "len_seed": C3_LEN_SEED, "target": 4 << 30, "total_bytes": total,
                 **digest(ref, c3)}
    del arena
    out["C2u"] = c2u_digest(ref)
    out["C4"] = digest_c4(ref)
    out["MAX"] = max_digest(ref)
    return out


def digest_c4(ref: oracle.Reference) -> dict:
    """C4 shard of rank 0 (bench.c4_layout): 64 reference-valid datafiles,
    ~16 GiB; payload crcs by the reference over the synthetic image bytes
    (headers never overlap payloads, so they need not be written here)."""
    import zdbcrc
    sys.path.insert(0, str(ROOT))
    import bench
    lay = bench.c4_layout(0)
    arena = zdbcrc.synth_fill(lay["total"], bench.C4_SEED)
    c4 = ref.batch(arena, lay["payload_off"].astype(np.uint64), lay["lens"].astype(np.uint32), threads=8)
    return {"seed": bench.C4_SEED, "len_seed": bench.C4_LEN_SEED, "files": len(lay["file_off"]),
            "image_bytes": lay["total"], "payload_bytes": int(lay["lens"].sum()), **digest(ref, c4)}


def max_case() -> tuple[int, np.ndarray, np.ndarray]:
    """the size limits of the interface on a 4.5 GiB arena: a record of the
    largest length (2^32 - 1, u32), one of 0-db's largest payload (8 MiB,
    data.h:6) past the 4 GiB offset mark, one straddling that mark, an empty
    one, one ending at the arena's last byte, and 5,000 small ones beyond
    4 GiB (tests/test_gpu.py::test_max_sizes_digest)"""
    total = (9 << 29) + 1000
    rng = np.random.default_rng(MAX_SEED)
    offs = [100, (1 << 32) + 7, (1 << 32) - 8, (1 << 32) + 3, total - 4999]
    lens = [(1 << 32) - 1, 8 << 20, 64, 0, 4999]
    small = rng.integers(0, 70_000, 5000)
    offs += [int(rng.integers(1 << 32, total - int(l))) for l in small]
    lens += [int(l) for l in small]
    return total, np.array(offs, np.uint64), np.array(lens, np.uint32)


def max_digest(ref: oracle.Reference) -> dict:
    import zdbcrc
    total, offs, lens = max_case()
    arena = zdbcrc.synth_fill(total, MAX_SEED)
    crcs = ref.batch(arena, offs, lens, threads=8)
    return {"seed": MAX_SEED, "total_bytes": total, "first": [f"{int(c):08x}" for c in crcs[:5]],
            **digest(ref, crcs)}


def c3_shard_digest(ref: oracle.Reference, rank: int, target: int) -> dict:
    """bench.make_dataset("zipf", target, rank): rank r's C3 shard"""
    import zdbcrc
    sys.path.insert(0, str(ROOT))
    import bench
    offs, lens, seed, _ = bench.make_dataset("zipf", target, rank)
    total = int(offs[-1] + lens[-1])
    arena = zdbcrc.synth_fill(total, seed)
    crcs = ref.batch(arena, offs.astype(np.uint64), lens.astype(np.uint32), threads=8)
    return {"rank": rank, "seed": seed, "target": target, "total_bytes": total, **digest(ref, crcs)}


def c4_shard_digest(ref: oracle.Reference, rank: int) -> dict:
    import zdbcrc
    sys.path.insert(0, str(ROOT))
    import bench
    lay = bench.c4_layout(rank)
    arena = zdbcrc.synth_fill(lay["total"], bench.C4_SEED + rank)
    c4 = ref.batch(arena, lay["payload_off"].astype(np.uint64), lay["lens"].astype(np.uint32), threads=8)
    return {"rank": rank, "seed": bench.C4_SEED + rank, "files": len(lay["file_off"]), "image_bytes": lay["total"],
            "payload_bytes": int(lay["lens"].sum()), **digest(ref, c4)}


def c2u_digest(ref: oracle.Reference) -> dict:
    """bench.make_dataset("c2u", 4 GiB, 0): the C2 payload count (1 Mi x 4 KiB)
    laid out as a datafile image, payload i at 28 + i * 4122 + 26 (SURVEY
    §8(d) C2u), bytes from splitmix64(C2_SEED) over the whole image"""
    import zdbcrc
    sys.path.insert(0, str(ROOT))
    import bench
    offs, lens, seed, _ = bench.make_dataset("c2u", 4 << 30, 0)
    total = int(offs[-1] + lens[-1])
    arena = zdbcrc.synth_fill(total, seed)
    crcs = ref.batch(arena, offs.astype(np.uint64), lens.astype(np.uint32), threads=8)
    return {"seed": seed, "records": len(lens), "record_bytes": 4096, "first_offset": int(offs[0]),
            "stride": int(offs[1] - offs[0]), "total_bytes": total, **digest(ref, crcs)}


def rank_digests(ref: oracle.Reference, ranks: int = 8) -> dict:
    """every rank's shard of a multi-GPU bench run (bench.py --gpus N, N <= 8):
    the full-size C3 (4 GiB) and C4 (64 datafiles) shards, and the 16 MiB C3
    shards the CPU-mode plumbing test (tests/test_dist.py) runs"""
    out = {"C3_ranks": [], "C4_ranks": [], "C3_16MiB_ranks": []}
    for r in range(ranks):
        out["C3_16MiB_ranks"].append(c3_shard_digest(ref, r, 16 << 20))
        out["C3_ranks"].append(c3_shard_digest(ref, r, 4 << 30))
        out["C4_ranks"].append(c4_shard_digest(ref, r))
        print(f"  rank {r}: C3 {out['C3_ranks'][-1]['xor']} C4 {out['C4_ranks'][-1]['xor']}", flush=True)
    return out


def main():
    ref = oracle.Reference()
    assert ref.engine() == "sse42", ref.engine()
    OUT.mkdir(parents=True, exist_ok=True)
    if "--only-rank-digests" in sys.argv:  # add / refresh the per-rank shard digests
        d = json.loads((OUT / "digests.json").read_text())
        d.update(rank_digests(ref))
        (OUT / "digests.json").write_text(json.dumps(d, indent=1) + "\n")
        return
    if "--only-max" in sys.argv:  # add / refresh the size-limit digest only
        d = json.loads((OUT / "digests.json").read_text())
        d["MAX"] = max_digest(ref)
        (OUT / "digests.json").write_text(json.dumps(d, indent=1) + "\n")
        print("digests.json MAX:", d["MAX"])
        return
    if "--only-c2u" in sys.argv:  # add / refresh the C2u digest only
        d = json.loads((OUT / "digests.json").read_text())
        d["C2u"] = c2u_digest(ref)
        (OUT / "digests.json").write_text(json.dumps(d, indent=1) + "\n")
        print("digests.json C2u:", d["C2u"])
        return
    if "--only-c4" in sys.argv:  # add / refresh the C4 digest only
        d = json.loads((OUT / "digests.json").read_text())
        d["C4"] = digest_c4(ref)
        (OUT / "digests.json").write_text(json.dumps(d, indent=1) + "\n")
        print("digests.json C4:", d["C4"])
        return
    if "--only-digests" in sys.argv:
        d = digests(ref)
        (OUT / "digests.json").write_text(json.dumps(d, indent=1) + "\n")
        print("digests.json:", d)
        return
    (OUT / "kat.json").write_text(json.dumps(kats(ref), indent=1) + "\n")
    print("kat.json written")
    print(f"vectors.npz: {vectors(ref)} lengths")
    meta = datafiles()
    (OUT / "datafiles.json").write_text(json.dumps(meta, indent=1) + "\n")
    if "--no-digests" not in sys.argv:
        d = digests(ref)
        (OUT / "digests.json").write_text(json.dumps(d, indent=1) + "\n")
        print("digests.json:", d)


if __name__ == "__main__":
    main()
