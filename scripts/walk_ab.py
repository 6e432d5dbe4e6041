#!/usr/bin/env python3
"""A/B of f3 walk variants selected by environment (diagnostic library):
each variant runs scripts/walk_probe.py in its own process, variants
alternate for R rounds.  Args: rounds chunk_bytes NAME=ENV1=V1,ENV2=V2 ..."""
import json, os, subprocess, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
rounds, chunk = int(sys.argv[1]), sys.argv[2]
variants = []
for a in sys.argv[3:]:
    name, _, envs = a.partition("=")
    env = dict(kv.split(":", 1) for kv in envs.split(",") if kv)
    variants.append((name, env))
for r in range(rounds):
    for name, env in variants:
        e = dict(os.environ, ZDBCRC_LIB=str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"), **env)
        out = subprocess.run([sys.executable, "-u", str(ROOT / "scripts" / "walk_probe.py"), chunk], env=e,
                             capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"variant": name, "env": env, "round": r,
                          "res": json.loads(line[-1]) if line else out.stderr[-500:]}), flush=True)
