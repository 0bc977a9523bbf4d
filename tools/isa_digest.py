"""Per-kernel digest of the gfx950 machine code in a library (CPU only).

    python tools/isa_digest.py [lib] > digest.json
    python tools/isa_digest.py --diff a.json b.json

Extracts every embedded gfx950 code object (llvm-objdump --offloading),
disassembles it, drops addresses and encodings, and hashes each kernel's
instruction text.  A source change that must not change the kernels (folding a
compile-time knob into a constant, deleting an ablation branch that is off in
the product) is checked by an empty --diff.
"""
import glob
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def digest(lib):
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        local = os.path.join(tmp, os.path.basename(lib))
        shutil.copy(lib, local)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", local], cwd=tmp, check=True,
                       capture_output=True)
        for obj in sorted(glob.glob(local + ".*gfx950")):
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn",
                                  "--no-leading-addr", obj], capture_output=True, text=True, check=True).stdout
            name, body = None, []
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]* ?<(.+)>:$", line.strip())
                if m:
                    if name:
                        out[name] = hashlib.sha256("\n".join(body).encode()).hexdigest()[:16]
                    name, body = m.group(1), []
                elif name and line.strip():
                    # branch targets carry addresses: keep the mnemonic and operands' shape only
                    body.append(re.sub(r"\s*//.*$", "", re.sub(r"0x[0-9a-f]+", "X", line.strip())))
            if name:
                out[name] = hashlib.sha256("\n".join(body).encode()).hexdigest()[:16]
    return out


if __name__ == "__main__":
    if sys.argv[1:2] == ["--diff"]:
        a, b = (json.load(open(p)) for p in sys.argv[2:4])
        diff = sorted(k for k in set(a) | set(b) if a.get(k) != b.get(k))
        print("\n".join(diff) if diff else "identical")
        sys.exit(1 if diff else 0)
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "dct_amd", "libdct_amd.so")
    print(json.dumps(digest(lib), indent=1, sort_keys=True))
