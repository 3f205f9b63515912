#!/usr/bin/env python3
"""the send path over a real socket.  Builds the config-5 file
set on tmpfs (100 k files, log-uniform 4 KiB-4 MiB; also a text-like set),
then runs tools/wire/hbx_wire_e2e (a child process: it owns the GPU) which
stores the files with hbx_store_paths_z and sends every chunk through the
allo/READ/writ/ACKN exchange to a loopback sink that re-verifies every write
like the server.  Prints one JSON line per file set.

Run on the GPU box: python tools/bench_wire.py [--files 100000]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=100_000)
    ap.add_argument("--dir", default="/dev/shm/hbx_wire")
    ap.add_argument("--window", type=int, default=4096)
    ap.add_argument("--timeout", type=int, default=500)
    ap.add_argument("--verify-threads", type=int, default=8)
    ap.add_argument("--sampled", action="store_true", help="also the one-in-64 sampled run (second figure)")
    a = ap.parse_args()
    from bench_config5 import make_files
    exe = os.path.join(ROOT, "tools", "wire", "hbx_wire_e2e")
    shutil.rmtree(a.dir, ignore_errors=True)
    try:
        paths, _ = make_files(a.dir, a.files, 5)
        lst = os.path.join(a.dir, "list.txt")
        with open(lst, "w") as fh:
            fh.write("\n".join(paths))
        # every write verified before its ACKN (server.go:180-182), then, as a
        # labelled second figure only, one write in 64
        for every, label in ((1, "every write verified (server.go:182)"),
                             (64, "sampled: one write in 64 verified (not the reference's behaviour)")):
            if every != 1 and not a.sampled:
                continue
            r = subprocess.run([exe, lst, "16", str(a.window), str(every), str(a.verify_threads)],
                               capture_output=True, text=True, timeout=a.timeout)
            sys.stderr.write(r.stderr[-2000:])
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            out = json.loads(line[-1]) if line else {"error": r.returncode}
            out["returncode"] = r.returncode
            out["set"] = "config-5 sizes, random pool (incompressible)"
            out["verification"] = label
            print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
