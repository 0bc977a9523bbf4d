#!/usr/bin/env python3
"""Expected output of the reference's own test programs (tests/golden/ref_programs.json).

Runs oracle/_ref/test_{dct,quantization,entropy}_cpu -- the reference's
tests/test_*.c linked against its own src/*.c, built from /root/reference by
oracle/Makefile -- and records exit code + stdout.  The drop-in test
(tests/test_gpu_parity.py::test_reference_programs_relinked) runs the same
programs linked against libdct_amd.so on the GPU and requires identical output.
"""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TESTS = ["dct", "quantization", "entropy"]


def run(kind, t):
    exe = os.path.join(ROOT, "oracle", "_ref", f"test_{t}_{kind}")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    return {"rc": out.returncode, "stdout": out.stdout}


if __name__ == "__main__":
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True, capture_output=True)
    res = {t: run("cpu", t) for t in TESTS}
    json.dump(res, open(os.path.join(ROOT, "tests", "golden", "ref_programs.json"), "w"), indent=1)
    print({t: (r["rc"], len(r["stdout"].splitlines())) for t, r in res.items()})
